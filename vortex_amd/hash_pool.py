"""Host-side mirror of vortex's hashing-pool boundary, backed by the HIP engine.

The reference has no trait for this path; its "interface" is three call sites
(SURVEY.md §8b), mirrored here under the reference's own names:

===============================  ==============================================
reference                        here
===============================  ==============================================
``scope.spawn(hash closure)``    :meth:`HashPool.spawn`
  peer_connection.rs:1139-1158     (index, conn_id, buffer, piece_len, expected)
``downloaded_piece_rc.try_recv`` :meth:`HashPool.try_recv` → ``DownloadedPiece``
  torrent.rs:415-442
``DownloadedPiece``              :class:`DownloadedPiece` (piece_selector.rs:311-317)
``par_iter().map(check).collect``:func:`verify_pieces` → ``list[bool]``
  torrent.rs:724-740
===============================  ==============================================

Semantics kept from the reference:
* a hash mismatch is a value (``hash_matched=False``), never an exception;
* the buffer is moved into the job and handed back in ``DownloadedPiece``
  (the caller must return it to its pool, buf_pool.rs:21-30);
* the digest covers exactly ``buffer[:piece_len]`` (peer_connection.rs:1148) —
  pool buffers are reused without zeroing, bytes past piece_len are ignored;
* completions arrive in batch-completion order, not submission order.

All hashing runs in libvortex_amd.so on the GPU; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Any, Optional, Sequence

from . import _lib
from ._lib import CONFIG_OPTIONS, VxError, check, lib, vx_completion, vx_config, vx_stats


@dataclass
class DownloadedPiece:
    """piece_selector.rs:311-317."""

    index: int
    conn_id: int
    hash_matched: bool
    buffer: Any
    digest: bytes = b""


def _addr_of(buf) -> tuple[int, Any]:
    """Stable address of a writable or read-only buffer plus a keep-alive."""
    if isinstance(buf, (bytes,)):
        keep = ctypes.create_string_buffer(buf, len(buf))
        return ctypes.addressof(keep), keep
    try:
        import numpy as np

        if isinstance(buf, np.ndarray):
            return buf.ctypes.data, buf
    except ImportError:  # pragma: no cover
        pass
    mv = memoryview(buf)
    if mv.readonly:
        keep = ctypes.create_string_buffer(mv.tobytes(), mv.nbytes)
        return ctypes.addressof(keep), keep
    c = (ctypes.c_uint8 * mv.nbytes).from_buffer(mv)
    return ctypes.addressof(c), (c, mv)


class HashPool:
    """The GPU engine behind vortex's spawn / try_recv hash boundary.

    ``piece_length`` is the torrent's piece_length (the BufferPool buffer
    size, torrent.rs:344).  One HashPool per torrent, used from one thread.
    ``options`` set the other vx_config fields (include/vx_hash.h, ABI 2):
    zero_copy, direct_io, batch_chunk, verify_chunk, verify_cold_chunk,
    verify_ramp; unset ones keep vx_config_default's values (each must fit
    the field's uint32: negative or >= 2**32 values are refused here, ctypes
    would wrap them silently).  ``hooks=True`` creates the context in the
    test build libvortex_amd_tuning.so, for fault injection
    (include/vx_tuning.h); ``self.lib`` is the library holding the context.
    """

    def __init__(self, piece_length: int, device: int = 0, slots: Optional[int] = None,
                 batch_pieces: Optional[int] = None, slot_bytes: Optional[int] = None, hooks: bool = False,
                 **options):
        L = _lib.tuning() if hooks else lib()
        self.lib = L
        cfg = vx_config()
        L.vx_config_default(ctypes.byref(cfg), piece_length)
        cfg.device = device
        if slots is not None:
            cfg.slots = slots
        if slot_bytes is not None:
            cfg.slot_bytes = slot_bytes
        if batch_pieces is not None:
            cfg.batch_pieces = batch_pieces
        for name, value in options.items():
            if name not in CONFIG_OPTIONS:
                raise TypeError(f"HashPool: unknown option {name!r} (vx_config has {', '.join(CONFIG_OPTIONS)})")
            if not 0 <= int(value) < 1 << 32:
                raise ValueError(f"HashPool: option {name}={value} outside the uint32 range of vx_config")
            setattr(cfg, name, int(value))
        h = ctypes.c_void_p()
        check(L.vx_create(ctypes.byref(cfg), ctypes.byref(h)), "vx_create", L)
        self._h = h
        self.config = cfg
        self._next_tag = 0
        self._inflight: dict[int, tuple[int, int, Any, Any]] = {}
        self._cbuf = (vx_completion * 1024)()
        self._registered: dict[int, tuple[int, Any, Any]] = {}  # id(buf) -> (address, keep-alive, buf)

    # -- lifecycle ---------------------------------------------------------
    def close(self) -> None:
        if self._h:
            check(self.lib.vx_destroy(self._h), "vx_destroy", self.lib)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    # -- buffer pinning (buf_pool.rs / buf_ring.rs AnonymousMmap) -----------
    def register_buffer(self, buf) -> None:
        """Pin a pool buffer (an mmap, bytearray or numpy array) for direct
        DMA.  Read-only objects such as ``bytes`` are refused: pinning them
        would pin a private copy that no later piece points into.  The
        registration is keyed by the object, so ``unregister_buffer`` must be
        given the same object."""
        mv = memoryview(buf)
        if mv.readonly:
            raise ValueError("register_buffer needs a writable buffer (e.g. an mmap or bytearray), not a read-only one")
        if id(buf) in self._registered:
            raise ValueError("buffer is already registered with this pool")
        addr, keep = _addr_of(buf)
        check(self.lib.vx_register_host_buffer(self._h, addr, mv.nbytes), "vx_register_host_buffer", self.lib)
        self._registered[id(buf)] = (addr, keep, buf)

    def unregister_buffer(self, buf) -> None:
        ent = self._registered.get(id(buf))
        if ent is None or ent[2] is not buf:
            raise ValueError("buffer was not registered with this pool")
        check(self.lib.vx_unregister_host_buffer(self._h, ent[0]), "vx_unregister_host_buffer", self.lib)
        del self._registered[id(buf)]

    # -- download path -------------------------------------------------------
    def spawn(self, index: int, conn_id: int, buffer, piece_len: int, expected_hash: Optional[bytes] = None) -> None:
        """peer_connection.rs:1145-1158: hash buffer[:piece_len] against
        expected_hash (or, when None, against row `index` of the table given
        to set_piece_table); the result comes back from try_recv().

        Ownership (include/vx_hash.h): the piece is taken iff the submit
        returns 0.  Otherwise this raises VxError whose ``refused`` is
        ``(index, conn_id, buffer)``: the piece was not taken, no result will
        ever carry it, it is not in take_unfinished(), and the caller hashes
        it on its own pool.  On VX_EDEVICE the pool is dead: collect the rest
        with try_iter() until it raises, then take_unfinished()."""
        if expected_hash is not None and len(expected_hash) != 20:
            raise ValueError("expected_hash must be 20 bytes")
        addr, keep = _addr_of(buffer)
        if piece_len > memoryview(buffer).nbytes:
            raise ValueError("piece_len exceeds buffer size")
        tag = self._next_tag
        self._next_tag += 1
        if expected_hash is None:
            rc, where = self.lib.vx_submit_piece(self._h, tag, addr, piece_len, index), "vx_submit_piece"
        else:
            exp = ctypes.create_string_buffer(bytes(expected_hash), 20)
            rc, where = self.lib.vx_submit(self._h, tag, addr, piece_len, exp), "vx_submit"
        if rc != 0:
            try:
                check(rc, where, self.lib)
            except VxError as e:
                e.refused = (index, conn_id, buffer)
                raise
        self._inflight[tag] = (index, conn_id, buffer, keep)

    def set_piece_table(self, pieces: bytes) -> None:
        """Upload the torrent's `pieces` string (n x 20 B) once; afterwards
        spawn(..., expected_hash=None) compares on the device by index."""
        if len(pieces) % 20:
            raise ValueError("pieces table must be a multiple of 20 bytes")
        buf = ctypes.create_string_buffer(bytes(pieces), max(1, len(pieces)))
        check(self.lib.vx_set_piece_table(self._h, buf, len(pieces) // 20), "vx_set_piece_table", self.lib)

    def flush(self) -> None:
        """Launch everything queued; call once per event-loop turn."""
        check(self.lib.vx_flush(self._h), "vx_flush", self.lib)

    def _poll(self, max_items: int) -> list[DownloadedPiece]:
        k = check(self.lib.vx_poll(self._h, self._cbuf, min(max_items, len(self._cbuf))), "vx_poll", self.lib)
        out = []
        for j in range(k):
            r = self._cbuf[j]
            index, conn_id, buffer, _keep = self._inflight.pop(r.tag)
            out.append(DownloadedPiece(index, conn_id, bool(r.matched), buffer, bytes(r.digest)))
        return out

    def try_recv(self) -> Optional[DownloadedPiece]:
        """torrent.rs:418 `downloaded_piece_rc.try_recv()`: non-blocking."""
        got = self._poll(1)
        return got[0] if got else None

    def try_iter(self) -> list[DownloadedPiece]:
        """Everything completed so far (the `while let Ok(..) = try_recv()` loop)."""
        out = []
        while True:
            try:
                got = self._poll(len(self._cbuf))
            except VxError:
                if out:  # hand out what was already taken off the engine; the error is sticky
                    return out  # and the next call raises it
                raise
            out.extend(got)
            if len(got) < len(self._cbuf):
                return out

    def take_unfinished(self) -> list[tuple[int, int, Any]]:
        """After a device error (a VxError from spawn / try_recv / try_iter):
        (index, conn_id, buffer) of every TAKEN piece whose result never came
        back, for the caller to hash on its own pool (INTEGRATION.md "Device
        failure").  A spawn that raised did not take its piece (it is in the
        exception's ``refused``), so it is not listed here.  Close the pool
        before reusing those buffers: that waits for the device to stop
        reading them."""
        out = [(index, conn_id, buffer) for index, conn_id, buffer, _keep in self._inflight.values()]
        self._inflight.clear()
        return out

    def drain(self, timeout_ms: int = 0) -> None:
        """Flush and wait for all in-flight pieces (the scope join of
        event_loop.rs:385-602); results stay queued for try_recv."""
        check(self.lib.vx_drain(self._h, timeout_ms), "vx_drain", self.lib)

    @property
    def pending(self) -> int:
        return int(self.lib.vx_pending(self._h))

    # -- observability (vx_get_stats) -------------------------------------------
    def stats(self) -> dict:
        """The engine's counters (include/vx_hash.h vx_stats) as a dict; the
        latency histogram is a list of VX_STATS_HIST log2 buckets in us."""
        st = vx_stats()
        check(self.lib.vx_get_stats(self._h, ctypes.byref(st)), "vx_get_stats", self.lib)
        out = {name: int(getattr(st, name)) for name, _ in vx_stats._fields_ if name != "batch_latency_hist"}
        out["batch_latency_hist"] = [int(x) for x in st.batch_latency_hist]
        return out

    def reset_stats(self) -> None:
        check(self.lib.vx_reset_stats(self._h), "vx_reset_stats", self.lib)

    def last_verify(self) -> dict:
        """Where the last verify_files call spent its time (vx_hash.h
        vx_last_verify), plus the derived rates bench.py records: the
        readers' pread rate, the data copies' GPU-timed rate, and the fraction
        of the copy span the copy engine was busy."""
        t = _lib.vx_verify_trace()
        check(self.lib.vx_last_verify(self._h, ctypes.byref(t)), "vx_last_verify", self.lib)
        d = {name: getattr(t, name) for name, _ in _lib.vx_verify_trace._fields_}
        gib = float(1 << 30)
        d["read_GiBps_per_thread"] = t.read_bytes / gib / (t.read_busy_ms * 1e-3) if t.read_busy_ms else None
        d["read_GiBps"] = t.read_bytes / gib / (t.read_span_ms * 1e-3) if t.read_span_ms else None
        d["copy_GiBps"] = t.copy_bytes / gib / (t.copy_busy_ms * 1e-3) if t.copy_busy_ms else None
        d["copy_busy_frac"] = t.copy_busy_ms / t.copy_span_ms if t.copy_span_ms else None
        return d

    def last_verify_rounds(self) -> list[dict]:
        """The last verify_files call's round timeline (vx_last_verify_rounds):
        per chunk round, ms from the call's start — reads queued / done, copy
        enqueued, the GPU's copy start / end and kernel end — with its bytes,
        chunk offset, lanes and VX_ROUND_* flags.  Empty on the whole-piece
        path."""
        n = check(self.lib.vx_last_verify_rounds(self._h, None, 0), "vx_last_verify_rounds", self.lib)
        arr = (_lib.vx_verify_round * max(1, n))()
        n = check(self.lib.vx_last_verify_rounds(self._h, arr, n), "vx_last_verify_rounds", self.lib)
        return [{name: getattr(arr[k], name) for name, _ in _lib.vx_verify_round._fields_} for k in range(n)]

    # -- bulk verify -----------------------------------------------------------
    def sha1_batch(self, pieces: Sequence) -> list[bytes]:
        n = len(pieces)
        ptrs, lens, keep = _ptr_arrays(pieces)
        out = ctypes.create_string_buffer(20 * max(n, 1))
        check(self.lib.vx_sha1_batch(self._h, ptrs, lens, n, out), "vx_sha1_batch", self.lib)
        raw = out.raw
        return [raw[20 * i: 20 * i + 20] for i in range(n)]

    def verify_files(self, paths: Sequence[str], file_lengths: Sequence[int], piece_length: int,
                     expected: bytes, io_threads: int = 0, first: int = 0,
                     count: int | None = None) -> tuple[list[bool], int]:
        """State::from_metadata_and_root's bulk re-verify (torrent.rs:716-761):
        pieces read from the torrent's files (file_store.rs:228-303 byte
        ranges) and verified on the GPU.  Returns (verdicts, pieces with I/O
        errors).  `expected` is the torrent's `pieces` string (n*20 bytes).
        first/count restrict it to pieces [first, first+count) (one rank's
        shard, vx_verify_files_range); the verdicts then cover that range."""
        return _verify_files(self, paths, file_lengths, piece_length, expected, io_threads, first, count)

    def verify_files_split(self, paths: Sequence[str], file_lengths: Sequence[int], piece_length: int,
                           expected: bytes, split: "Split", io_threads: int = 0) -> int:
        """The engine's side of a split re-verify (vx_verify_files_split):
        verifies the pieces it claims from `split` while the caller's pool
        claims the others, writes their verdicts into split.matched and
        returns how many of its pieces hit an I/O error.  Blocks; run the pool
        on other threads (ctypes drops the GIL for the call)."""
        arr = (ctypes.c_char_p * max(1, len(paths)))(*[os.fsencode(p) for p in paths])
        lens = (ctypes.c_uint64 * max(1, len(file_lengths)))(*file_lengths)
        exp = ctypes.create_string_buffer(bytes(expected), max(1, len(expected)))
        rc = self.lib.vx_verify_files_split(self._h, arr, lens, len(paths), piece_length, exp, len(expected) // 20,
                                            ctypes.byref(split.s), split.matched, io_threads)
        return int(check(rc, "vx_verify_files_split", self.lib))

    def verify_batch(self, pieces: Sequence, expected: Sequence[bytes]) -> tuple[list[bool], list[bytes]]:
        n = len(pieces)
        if len(expected) != n:
            raise ValueError("expected must have one digest per piece")
        ptrs, lens, keep = _ptr_arrays(pieces)
        exp = ctypes.create_string_buffer(b"".join(bytes(e) for e in expected), 20 * max(n, 1))
        matched = ctypes.create_string_buffer(max(n, 1))
        dig = ctypes.create_string_buffer(20 * max(n, 1))
        check(self.lib.vx_verify_batch(self._h, ptrs, lens, exp, n, matched, dig), "vx_verify_batch", self.lib)
        raw = dig.raw
        return [bool(b) for b in matched.raw[:n]], [raw[20 * i: 20 * i + 20] for i in range(n)]


def _verify_files(pool: "HashPool", paths: Sequence[str], file_lengths: Sequence[int], piece_length: int,
                  expected: bytes, io_threads: int = 0, first: int = 0,
                  count: int | None = None) -> tuple[list[bool], int]:
    n = len(expected) // 20
    if count is None:
        count = n - first
    arr = (ctypes.c_char_p * max(1, len(paths)))(*[os.fsencode(p) for p in paths])
    lens = (ctypes.c_uint64 * max(1, len(file_lengths)))(*file_lengths)
    exp = ctypes.create_string_buffer(bytes(expected), max(1, len(expected)))
    out = ctypes.create_string_buffer(max(1, count))
    if first == 0 and count == n:
        rc = pool.lib.vx_verify_files(pool._h, arr, lens, len(paths), piece_length, exp, n, out, io_threads)
    else:
        rc = pool.lib.vx_verify_files_range(pool._h, arr, lens, len(paths), piece_length, exp, n, first, count, out,
                                         io_threads)
    bad = check(rc, "vx_verify_files", pool.lib)
    return [bool(b) for b in out.raw[:count]], int(bad)


class Split:
    """One bulk re-verify shared at once by the engine and the caller's pool,
    with no plan (include/vx_hash.h vx_split / vx_verify_files_split): the
    pool's threads take pieces from the head with claim() and report each
    finished one with done(); the engine (HashPool.verify_files_split) takes
    groups from the top, sized from both sides' rates measured as it goes.
    `matched` holds every verdict once both sides have returned: entries
    [0, boundary - first) are the pool's to write, the rest the engines'.
    claim_fn / done_fn / arg are the C addresses a native pool calls."""

    def __init__(self, first: int, end: int, cpu_threads: int = 0, cpu_thread_rate: float = 0.0):
        self._bind(_lib.vx_split(), ctypes.create_string_buffer(max(1, end - first)), first, end)
        self._init(cpu_threads, cpu_thread_rate, 1)

    @classmethod
    def attach(cls, buf, first: int, end: int, init: bool, cpu_threads: int = 0, cpu_thread_rate: float = 0.0,
               engines: int = 1) -> "Split":
        """A split living in a shared buffer (e.g. a MAP_SHARED mmap of a
        /dev/shm file, one per node): the vx_split at offset 0, the end - first
        verdict bytes after it, so engines in several processes (one per GPU)
        and the pool claim from one word and write one verdict array.  One
        process inits (init=True) before the others attach."""
        self = cls.__new__(cls)
        self._bind(_lib.vx_split.from_buffer(buf, 0),
                   (ctypes.c_char * max(1, end - first)).from_buffer(buf, ctypes.sizeof(_lib.vx_split)), first, end)
        if init:
            self._init(cpu_threads, cpu_thread_rate, engines)
        return self

    def _bind(self, s, matched, first: int, end: int) -> None:
        self.lib = lib()
        self.s, self.matched = s, matched
        self.first, self.end = first, end
        self.arg = ctypes.addressof(self.s)
        self.claim_fn = ctypes.cast(self.lib.vx_split_claim, ctypes.c_void_p).value
        self.done_fn = ctypes.cast(self.lib.vx_split_done, ctypes.c_void_p).value

    def _init(self, cpu_threads: int, cpu_thread_rate: float, engines: int) -> None:
        check(self.lib.vx_split_init(ctypes.byref(self.s), self.first, self.end, cpu_threads, cpu_thread_rate),
              "vx_split_init", self.lib)
        self.s.engines = engines

    def claim(self) -> int:
        """The next piece for the pool, or -1 when none is left."""
        return int(self.lib.vx_split_claim(ctypes.byref(self.s)))

    def done(self, pieces: int = 1) -> None:
        self.lib.vx_split_done(ctypes.byref(self.s), pieces)

    @property
    def boundary(self) -> int:
        """The engine's lowest piece (end when it took none)."""
        return int(self.lib.vx_split_boundary(ctypes.byref(self.s)))

    @property
    def pool_done(self) -> int:
        return int(self.s.pool_done)

    def verdicts(self) -> list[bool]:
        return [bool(b) for b in bytes(self.matched)[:self.end - self.first]]


def verify_files_multi(pools: Sequence["HashPool"], paths: Sequence[str], file_lengths: Sequence[int],
                       piece_length: int, expected: bytes, io_threads: int = 0) -> tuple[list[bool], int]:
    """In-process multi-GPU re-verify (vx_verify_files_multi): one HashPool
    per GPU (or several on one), pieces split into contiguous ranges across
    them, each range verified on its own host thread.  Same result as
    HashPool.verify_files on one pool: (verdicts, pieces with I/O errors)."""
    if not pools:
        raise ValueError("need at least one pool")
    L = pools[0].lib
    if any(p.lib is not L for p in pools):
        raise ValueError("verify_files_multi: every pool must come from the same library (hooks)")
    n = len(expected) // 20
    ctxs = (ctypes.c_void_p * len(pools))(*[p._h.value for p in pools])
    arr = (ctypes.c_char_p * max(1, len(paths)))(*[os.fsencode(p) for p in paths])
    lens = (ctypes.c_uint64 * max(1, len(file_lengths)))(*file_lengths)
    exp = ctypes.create_string_buffer(bytes(expected), max(1, len(expected)))
    out = ctypes.create_string_buffer(max(1, n))
    rc = L.vx_verify_files_multi(ctxs, len(pools), arr, lens, len(paths), piece_length, exp, n, out, io_threads)
    bad = check(rc, "vx_verify_files_multi", L)
    return [bool(b) for b in out.raw[:n]], int(bad)


def verify_files_split_multi(pools: Sequence["HashPool"], paths: Sequence[str], file_lengths: Sequence[int],
                             piece_length: int, expected: bytes, split: "Split", io_threads: int = 0) -> int:
    """The split over several GPUs (vx_verify_files_split_multi): every pool
    is one engine claiming from `split` on its own host thread, beside the
    caller's pool on split.claim().  Verdicts land in split.matched; returns
    the engines' pieces with I/O errors.  Blocks; run the pool on other
    threads."""
    if not pools:
        raise ValueError("need at least one pool")
    L = pools[0].lib
    if any(p.lib is not L for p in pools):
        raise ValueError("verify_files_split_multi: every pool must come from the same library (hooks)")
    ctxs = (ctypes.c_void_p * len(pools))(*[p._h.value for p in pools])
    arr = (ctypes.c_char_p * max(1, len(paths)))(*[os.fsencode(p) for p in paths])
    lens = (ctypes.c_uint64 * max(1, len(file_lengths)))(*file_lengths)
    exp = ctypes.create_string_buffer(bytes(expected), max(1, len(expected)))
    rc = L.vx_verify_files_split_multi(ctxs, len(pools), arr, lens, len(paths), piece_length, exp,
                                       len(expected) // 20, ctypes.byref(split.s), split.matched, io_threads)
    return int(check(rc, "vx_verify_files_split_multi", L))


def _ptr_arrays(pieces: Sequence):
    n = len(pieces)
    keep = []
    ptrs = (ctypes.c_void_p * max(n, 1))()
    lens = (ctypes.c_uint32 * max(n, 1))()
    for i, p in enumerate(pieces):
        addr, k = _addr_of(p if len(p) else b"\0")
        keep.append(k)
        ptrs[i] = addr
        lens[i] = len(p)
    return ptrs, lens, keep


def verify_pieces(pieces: Sequence, expected: Sequence[bytes], device: int = 0,
                  piece_length: Optional[int] = None) -> list[bool]:
    """torrent.rs:724-740: one verdict per piece, in piece order."""
    plen = piece_length or max((len(p) for p in pieces), default=1) or 1
    with HashPool(plen, device=device) as pool:
        matched, _ = pool.verify_batch(pieces, expected)
    return matched


def piece_len(index: int, num_pieces: int, piece_length: int, total_length: int) -> int:
    """PieceSelector::piece_len with the last-piece rule (piece_selector.rs:63-69, 291-298)."""
    last = total_length % piece_length or piece_length
    return last if index == num_pieces - 1 else piece_length


__all__ = ["DownloadedPiece", "HashPool", "verify_pieces", "verify_files_multi", "piece_len", "plan_verify",
           "plan_verify_split"]


def plan_verify(n_pieces: int, piece_length: int, total_length: int, cpu_threads: int = 0,
                cpu_thread_rate: float = 0.0, n_gpus: int = 1) -> dict:
    """Where a bulk verify should run (include/vx_hash.h vx_plan_verify_gpus,
    host-only, no GPU): the predicted seconds of the GPU path over n_gpus
    contexts and of the caller's pool of cpu_threads (torrent.rs:724-740), and
    use_gpu.  0 threads / rate = 16 threads at 2.2e9 B/s (SHA-NI)."""
    p = _lib.vx_plan()
    check(lib().vx_plan_verify_gpus(n_pieces, piece_length, total_length, cpu_threads, cpu_thread_rate, n_gpus,
                                    ctypes.byref(p)), "vx_plan_verify_gpus")
    out = {name: getattr(p, name) for name, _ in _lib.vx_plan._fields_ if not name.startswith("_")}
    out["use_gpu"] = bool(out["use_gpu"])
    return out


def plan_verify_split(n_pieces: int, piece_length: int, total_length: int, cpu_threads: int = 0,
                      cpu_thread_rate: float = 0.0, n_gpus: int = 1) -> dict:
    """Split one bulk verify between the GPUs and the caller's own pool run
    at once (include/vx_hash.h vx_plan_verify_split, host-only): the GPUs take
    pieces [gpu_first, n_pieces), the pool the rest; the plan's predicted
    times for both sides.  gpu_count 0 = keep the pool alone."""
    p = _lib.vx_plan()
    first, count = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().vx_plan_verify_split(n_pieces, piece_length, total_length, cpu_threads, cpu_thread_rate, n_gpus,
                                     ctypes.byref(first), ctypes.byref(count), ctypes.byref(p)),
          "vx_plan_verify_split")
    out = {name: getattr(p, name) for name, _ in _lib.vx_plan._fields_ if not name.startswith("_")}
    out["use_gpu"] = bool(out["use_gpu"])
    out["gpu_first"], out["gpu_count"] = int(first.value), int(count.value)
    return out
