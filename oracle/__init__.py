"""CPU oracle for the SHA-1 piece-verification path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker (or, for the bench, as the
timed CPU baseline).  The product package ``vortex_amd`` never imports it.

Contents
--------
* ``sha1`` / ``sha1_backend``: FIPS 180-4 SHA-1 restated in C (oracle/sha1_oracle.c),
  standing in for the external ``sha1`` 0.11.0 crate that vortex calls at
  bittorrent/src/peer_comm/peer_connection.rs:1146-1149 and
  bittorrent/src/file_store.rs:235-302.  Backends: 0 auto (SHA-NI when present,
  as ``cpufeatures`` selects), 1 scalar, 2 SHA-NI.
* ``pool_verify`` / ``pool_digest_synth``: the rayon-pool + mpsc restatement
  (oracle/pool_oracle.cpp; peer_connection.rs:1145-1158, torrent.rs:415-442,
  torrent.rs:724-740).
* ``gen_piece``: CPU twin of the device synthetic-piece generator.
* ``piece_len`` / ``piece_ranges`` / ``check_piece_hash_sync``: pure-Python
  restatements of the piece length rule (piece_selector.rs:57-69, 291-298) and
  of the multi-file byte-range mapping used by bulk re-verify
  (file_store.rs:108-165 layout, file_store.rs:228-303 read + hash).

Parity pinning: tests/test_oracle.py checks every function here against the
FIPS vectors, hashlib-generated fixtures (tests/golden/, made by
tests/golden/make_golden.py) and the reference's implicit known answers
(SURVEY.md §8c).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.vxo_sha1_backend.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
        L.vxo_sha1_backend.restype = None
        L.vxo_has_shani.restype = ctypes.c_int
        L.vxo_gen_piece.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_void_p]
        L.vxo_gen_piece.restype = None
        L.vxo_pool_verify.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.vxo_pool_verify.restype = ctypes.c_int
        L.vxo_pool_digest_synth.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32,
                                            ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_void_p]
        L.vxo_pool_digest_synth.restype = ctypes.c_int
        L.vxo_pool_verify_files.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_void_p]
        L.vxo_pool_verify_files.restype = ctypes.c_int
        L.vxo_pool_verify_files_claim.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.vxo_pool_verify_files_claim.restype = ctypes.c_int64
        L.vxo_sha1_ctx_size.restype = ctypes.c_size_t
        L.vxo_sha1_init.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.vxo_sha1_update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.vxo_sha1_final.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        del u8p
        _lib = L
    return _lib


NO_LAST = (1 << 64) - 1


def has_shani() -> bool:
    return bool(lib().vxo_has_shani())


def sha1_backend(data: bytes, backend: int = 0) -> bytes:
    out = ctypes.create_string_buffer(20)
    buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data if data else b"\0")
    lib().vxo_sha1_backend(buf, len(data), out, backend)
    return out.raw


def sha1(data: bytes) -> bytes:
    return sha1_backend(data, 0)


class Sha1Stream:
    """Sha1::new / update / finalize, for multi-segment pieces."""

    def __init__(self, backend: int = 0):
        self._ctx = ctypes.create_string_buffer(lib().vxo_sha1_ctx_size())
        lib().vxo_sha1_init(self._ctx, backend)

    def update(self, data: bytes) -> None:
        if data:
            buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
            lib().vxo_sha1_update(self._ctx, buf, len(data))

    def finalize(self) -> bytes:
        out = ctypes.create_string_buffer(20)
        lib().vxo_sha1_final(self._ctx, out)
        return out.raw


def gen_piece(seed: int, piece: int, length: int, corrupt_every: int = 0) -> bytes:
    out = ctypes.create_string_buffer(max(1, length))
    lib().vxo_gen_piece(seed, piece, length, corrupt_every, out)
    return out.raw[:length]


def is_corrupt(piece: int, corrupt_every: int) -> bool:
    return bool(corrupt_every) and piece % corrupt_every == corrupt_every - 1


def pool_verify(pieces, expected: bytes | None = None, threads: int = 1, backend: int = 0):
    """Hash a list of bytes objects on the pool restatement.

    Returns (digests: bytes[n*20], matched: list[bool] | None)."""
    n = len(pieces)
    keep = [(ctypes.c_uint8 * max(1, len(p))).from_buffer_copy(p if p else b"\0") for p in pieces]
    ptrs = (ctypes.c_void_p * max(1, n))(*[ctypes.addressof(k) for k in keep])
    lens = (ctypes.c_uint32 * max(1, n))(*[len(p) for p in pieces])
    dig = ctypes.create_string_buffer(20 * max(1, n))
    matched = ctypes.create_string_buffer(max(1, n)) if expected is not None else None
    exp = ctypes.create_string_buffer(expected, len(expected)) if expected is not None else None
    lib().vxo_pool_verify(ptrs, lens, exp, n, threads, backend, matched, dig)
    return dig.raw[: 20 * n], ([bool(b) for b in matched.raw[:n]] if matched is not None else None)


def pool_verify_ptrs(ptrs_arr, lens_arr, n: int, expected_buf, threads: int, backend: int, matched_buf,
                     digests_buf) -> None:
    """Zero-copy form for the bench: ctypes arrays / buffers prepared by the caller."""
    lib().vxo_pool_verify(ptrs_arr, lens_arr, expected_buf, n, threads, backend, matched_buf, digests_buf)


def pool_digest_synth(seed: int, first: int, n: int, piece_len: int, last_index: int = NO_LAST,
                      last_len: int = 0, corrupt_every: int = 0, threads: int = 1, backend: int = 0) -> bytes:
    out = ctypes.create_string_buffer(20 * max(1, n))
    lib().vxo_pool_digest_synth(seed, first, n, piece_len, last_index, last_len, corrupt_every, threads,
                                backend, out)
    return out.raw[: 20 * n]


def pool_verify_files(paths, file_lengths, piece_length: int, expected: bytes, threads: int = 1,
                      backend: int = 0) -> list:
    """C++ restatement of the bulk re-verify (torrent.rs:724-740 over
    file_store.rs:228-303); the CPU baseline for config 5."""
    n = len(expected) // 20
    arr = (ctypes.c_char_p * max(1, len(paths)))(*[p.encode() for p in paths])
    lens = (ctypes.c_uint64 * max(1, len(file_lengths)))(*file_lengths)
    exp = ctypes.create_string_buffer(expected, max(1, len(expected)))
    out = ctypes.create_string_buffer(max(1, n))
    lib().vxo_pool_verify_files(arr, lens, len(paths), piece_length, exp, n, threads, backend, out)
    return [bool(b) for b in out.raw[:n]]


def pool_verify_files_claim(paths, file_lengths, piece_length: int, expected: bytes, threads: int, claim_fn: int,
                            done_fn: int, arg: int, base: int, out, backend: int = 0) -> int:
    """The pool beside the engine's split (vx_verify_files_split): `threads`
    threads take pieces from claim_fn(arg) until it returns -1 — vortex's
    rayon threads calling vx_split_claim — verify each as
    check_piece_hash_sync does, write out[i - base] and call done_fn(arg, 1).
    claim_fn / done_fn / arg are C addresses (the engine's vx_split_claim /
    vx_split_done and its vx_split).  Returns the pieces the pool took."""
    arr = (ctypes.c_char_p * max(1, len(paths)))(*[p.encode() for p in paths])
    lens = (ctypes.c_uint64 * max(1, len(file_lengths)))(*file_lengths)
    exp = ctypes.create_string_buffer(expected, max(1, len(expected)))
    return lib().vxo_pool_verify_files_claim(arr, lens, len(paths), piece_length, exp, threads, backend, claim_fn,
                                             done_fn, arg, base, out)


# ---------------------------------------------------------------- geometry
def piece_len(index: int, num_pieces: int, piece_length: int, total_length: int) -> int:
    """PieceSelector::piece_len (piece_selector.rs:291-298) with the last-piece
    rule of PieceSelector::new (piece_selector.rs:63-69)."""
    last = total_length % piece_length
    if last == 0:
        last = piece_length
    return last if index == num_pieces - 1 else piece_length


def file_layout(file_lengths, piece_length: int):
    """FileStore::new's per-file (start_piece, start_offset, end_piece, end_offset)
    (file_store.rs:126-160)."""
    out = []
    start_piece, start_offset = 0, 0
    for flen in file_lengths:
        num_pieces = (flen + start_offset) // piece_length
        offset = (flen + start_offset) % piece_length
        f = (start_piece, start_offset, start_piece + num_pieces, offset, flen)
        out.append(f)
        start_piece, start_offset = f[2], f[3]
    return out


def piece_segments(piece_index: int, file_lengths, piece_length: int):
    """(file_idx, offset_in_file, length) segments that make up a piece, in the
    order FileStore::check_piece_hash_sync reads them (file_store.rs:240-298)."""
    segs = []
    total_read = 0
    for fi, (sp, so, ep, eo, flen) in enumerate(file_layout(file_lengths, piece_length)):
        if not (sp <= piece_index <= ep):
            continue
        file_index = piece_index - sp
        file_offset = file_index * piece_length - so
        off = file_offset + total_read
        assert off >= 0
        if piece_index == ep:
            to_read = eo - total_read
        else:
            to_read = min(piece_length - total_read, flen)
        if to_read == 0:
            continue
        segs.append((fi, off, to_read))
        total_read += to_read
    return segs


def check_piece_hash_sync(paths, file_lengths, piece_length: int, piece_index: int, expected: bytes) -> bool:
    """FileStore::check_piece_hash_sync (file_store.rs:228-303): pread each
    overlapping segment and hash; raises OSError like the reference's io::Error."""
    h = Sha1Stream()
    for fi, off, n in piece_segments(piece_index, file_lengths, piece_length):
        with open(paths[fi], "rb") as f:
            f.seek(off)
            data = f.read(n)
        if len(data) != n:
            raise EOFError("unexpected EOF while reading file")
        h.update(data)
    return h.finalize() == expected
