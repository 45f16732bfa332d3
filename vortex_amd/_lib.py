"""ctypes binding of libvortex_amd.so (the C ABI declared in include/vx_hash.h).

The library is the product: there is no CPU or PyTorch fallback.  If it is
missing, loading raises ``ImportError`` (fail loudly, never silently degrade).

``lib()`` is the release library vortex links (vx_hash.h only).  ``tuning()``
is libvortex_amd_tuning.so, the same sources built with the test hooks: it
also exports include/vx_tuning.h (kernel-variant pins, fault injection, clock
stamps) and include/vx_synth.h (the synthetic-piece generator) for tests and
bench.py.  A context lives in the library that created it: pass a handle
only to functions of that same library (HashPool(hooks=True) creates its
context in tuning()).

``torch`` is imported before the library is loaded on purpose: torch ships its
own ``libamdhip64.so`` (same soname ``libamdhip64.so.7``) and loading it first
makes our library bind to that single HIP runtime instead of pulling in a
second one from /opt/rocm.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libvortex_amd.so")
TUNING_PATH = os.path.join(_HERE, "libvortex_amd_tuning.so")

VX_OK = 0
VX_EINVAL = -22
VX_ENOMEM = -12
VX_ERANGE = -34
VX_ENODEV = -19
VX_EDEVICE = -5
VX_EBUSY = -16

# Every function include/vx_hash.h declares: what libvortex_amd.so exports,
# and all it exports (tests/test_abi.py checks the headers and both libraries'
# dynamic symbols against these lists).
EXPORTS = (
    "vx_abi_version", "vx_last_error", "vx_strerror", "vx_device_count", "vx_config_default",
    "vx_create", "vx_destroy", "vx_register_host_buffer", "vx_unregister_host_buffer",
    "vx_submit", "vx_flush", "vx_poll", "vx_drain", "vx_pending", "vx_set_piece_table", "vx_submit_piece",
    "vx_sha1_batch", "vx_verify_batch", "vx_verify_files", "vx_verify_files_range", "vx_verify_files_multi",
    "vx_sha1_device_uniform", "vx_sha1_device_ragged", "vx_sha1_device_ragged_hint", "vx_sort_order",
    "vx_plan_verify", "vx_plan_verify_gpus", "vx_plan_verify_split", "vx_get_stats", "vx_reset_stats",
    "vx_last_verify", "vx_last_verify_rounds",
    "vx_split_init", "vx_split_claim", "vx_split_done", "vx_split_boundary", "vx_verify_files_split",
    "vx_verify_files_split_multi",
)
# ... plus include/vx_tuning.h and include/vx_synth.h: libvortex_amd_tuning.so only.
TUNING_EXPORTS = (
    "vx_synth_fill", "vx_sha1_device_uniform_variant", "vx_sha1_device_ragged_variant",
    "vx_tuning_zero_copy_plan", "vx_tuning_zero_copy_kernel", "vx_tuning_plan_ragged", "vx_tuning_chunk_schedule",
    "vx_tuning_fail_submit_after", "vx_tuning_fail_launch_after", "vx_tuning_verify_copy_stream", "vx_tuning_stage_huge",
    "vx_tuning_split_rules", "vx_tuning_clock_stamp",
    "vx_tuning_wall_clock_khz", "vx_tuning_device_identity", "vx_tuning_split_take_tail",
    "vx_tuning_last_split",
)


class VxError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where} failed: {code} ({msg})")
        self.code = code
        # HashPool.spawn: (index, conn_id, buffer) of a piece the engine did not take
        self.refused = None


class vx_completion(ctypes.Structure):
    _fields_ = [("tag", ctypes.c_uint64), ("matched", ctypes.c_uint8), ("digest", ctypes.c_uint8 * 20),
                ("_pad", ctypes.c_uint8 * 3)]


ABI_VERSION = 3

# vx_config fields a caller may set beyond the pool geometry (ABI 2; include/vx_hash.h)
CONFIG_OPTIONS = ("zero_copy", "direct_io", "batch_chunk", "verify_chunk", "verify_cold_chunk", "verify_ramp",
                  "refuse_when_full")


class vx_config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("max_piece_len", ctypes.c_uint32), ("batch_pieces", ctypes.c_uint32),
                ("slots", ctypes.c_uint32), ("slot_bytes", ctypes.c_uint64)] + \
        [(name, ctypes.c_uint32) for name in CONFIG_OPTIONS]


class vx_plan(ctypes.Structure):
    _fields_ = [("gpu_s", ctypes.c_double), ("gpu_chain_s", ctypes.c_double), ("gpu_transfer_s", ctypes.c_double),
                ("cpu_s", ctypes.c_double), ("piece_latency_s", ctypes.c_double),
                ("cpu_piece_latency_s", ctypes.c_double), ("use_gpu", ctypes.c_int32), ("_pad", ctypes.c_uint32)]


VX_STATS_HIST = 24


class vx_stats(ctypes.Structure):
    _fields_ = [(name, ctypes.c_uint64) for name in (
        "pieces_completed", "pieces_mismatched", "bytes_completed", "batches", "chunk_rounds", "gather_tiles",
        "staged_bytes", "io_errors", "submit_stall_ns", "batch_latency_count", "batch_latency_sum_us",
        "batch_latency_max_us")] + [("batch_latency_hist", ctypes.c_uint64 * VX_STATS_HIST)] + [
        (name, ctypes.c_uint64) for name in ("zero_copy_slots", "zero_copy_loader_slots", "submits_refused")]


class vx_verify_trace(ctypes.Structure):
    _fields_ = [(name, ctypes.c_double) for name in (
        "wall_ms", "read_busy_ms", "read_span_ms", "first_read_ms", "copy_busy_ms", "copy_span_ms", "tail_ms")] + [
        ("read_bytes", ctypes.c_uint64), ("copy_bytes", ctypes.c_uint64), ("readers", ctypes.c_uint32),
        ("rounds", ctypes.c_uint32), ("direct_bytes", ctypes.c_uint64),
        ("chunk_bytes", ctypes.c_uint64)]


VX_ROUND_NEW_WINDOW, VX_ROUND_HEAD_RAMP, VX_ROUND_TAIL_RAMP = 1, 2, 4


class vx_verify_round(ctypes.Structure):
    _fields_ = [(name, ctypes.c_double) for name in (
        "read_submit_ms", "read_done_ms", "enqueue_ms", "copy_start_ms", "copy_end_ms", "kernel_end_ms")] + [
        ("bytes", ctypes.c_uint64), ("offset", ctypes.c_uint64), ("lanes", ctypes.c_uint32),
        ("flags", ctypes.c_uint32)]


class vx_split(ctypes.Structure):
    """The split's claim word and the pool's progress (include/vx_hash.h)."""
    _fields_ = [("word", ctypes.c_uint64), ("pool_done", ctypes.c_uint64), ("start_ns", ctypes.c_uint64),
                ("first", ctypes.c_uint64), ("end", ctypes.c_uint64), ("cpu_threads", ctypes.c_uint32),
                ("engines", ctypes.c_uint32), ("cpu_thread_rate", ctypes.c_double),
                ("pool_last_ns", ctypes.c_uint64)]


_lib = None
_tuning = None
_lock = threading.Lock()


def _declare(L: ctypes.CDLL, tuning: bool = False) -> None:
    c = ctypes
    vp = c.c_void_p
    sig = {
        "vx_abi_version": ([], c.c_int),
        "vx_last_error": ([], c.c_char_p),
        "vx_strerror": ([c.c_int], c.c_char_p),
        "vx_device_count": ([], c.c_int),
        "vx_config_default": ([c.POINTER(vx_config), c.c_uint32], None),
        "vx_create": ([c.POINTER(vx_config), c.POINTER(vp)], c.c_int),
        "vx_destroy": ([vp], c.c_int),
        "vx_register_host_buffer": ([vp, vp, c.c_size_t], c.c_int),
        "vx_unregister_host_buffer": ([vp, vp], c.c_int),
        "vx_submit": ([vp, c.c_uint64, vp, c.c_uint32, vp], c.c_int),
        "vx_flush": ([vp], c.c_int),
        "vx_set_piece_table": ([vp, vp, c.c_uint32], c.c_int),
        "vx_submit_piece": ([vp, c.c_uint64, vp, c.c_uint32, c.c_uint32], c.c_int),
        "vx_poll": ([vp, c.POINTER(vx_completion), c.c_size_t], c.c_int64),
        "vx_drain": ([vp, c.c_uint32], c.c_int),
        "vx_pending": ([vp], c.c_uint64),
        "vx_get_stats": ([vp, c.POINTER(vx_stats)], c.c_int),
        "vx_reset_stats": ([vp], c.c_int),
        "vx_sha1_batch": ([vp, vp, vp, c.c_size_t, vp], c.c_int),
        "vx_verify_batch": ([vp, vp, vp, vp, c.c_size_t, vp, vp], c.c_int),
        "vx_verify_files": ([vp, vp, vp, c.c_size_t, c.c_uint32, vp, c.c_size_t, vp, c.c_uint32], c.c_int64),
        "vx_verify_files_range": ([vp, vp, vp, c.c_size_t, c.c_uint32, vp, c.c_size_t, c.c_size_t, c.c_size_t, vp,
                                   c.c_uint32], c.c_int64),
        "vx_verify_files_multi": ([vp, c.c_size_t, vp, vp, c.c_size_t, c.c_uint32, vp, c.c_size_t, vp, c.c_uint32],
                                  c.c_int64),
        "vx_sha1_device_uniform": ([vp, c.c_uint64, c.c_uint32, c.c_uint32, vp, vp, vp, vp], c.c_int),
        "vx_sha1_device_ragged": ([vp, vp, vp, vp, c.c_uint32, vp, vp, vp, vp], c.c_int),
        "vx_sha1_device_ragged_hint": ([vp, vp, vp, vp, c.c_uint32, c.c_uint32, c.c_uint64, vp, vp, vp, vp],
                                       c.c_int),
        "vx_sort_order": ([vp, c.c_uint32, vp], c.c_int),
        "vx_last_verify": ([vp, c.POINTER(vx_verify_trace)], c.c_int),
        "vx_last_verify_rounds": ([vp, c.POINTER(vx_verify_round), c.c_size_t], c.c_int64),
        "vx_plan_verify": ([c.c_uint64, c.c_uint32, c.c_uint64, c.c_uint32, c.c_double, c.POINTER(vx_plan)], c.c_int),
        "vx_plan_verify_gpus": ([c.c_uint64, c.c_uint32, c.c_uint64, c.c_uint32, c.c_double, c.c_uint32,
                                 c.POINTER(vx_plan)], c.c_int),
        "vx_plan_verify_split": ([c.c_uint64, c.c_uint32, c.c_uint64, c.c_uint32, c.c_double, c.c_uint32,
                                  c.POINTER(c.c_uint64), c.POINTER(c.c_uint64), c.POINTER(vx_plan)], c.c_int),
        "vx_split_init": ([c.POINTER(vx_split), c.c_uint64, c.c_uint64, c.c_uint32, c.c_double], c.c_int),
        "vx_split_claim": ([c.POINTER(vx_split)], c.c_int64),
        "vx_split_done": ([c.POINTER(vx_split), c.c_uint64], None),
        "vx_split_boundary": ([c.POINTER(vx_split)], c.c_uint64),
        "vx_verify_files_split": ([vp, vp, vp, c.c_size_t, c.c_uint32, vp, c.c_size_t, c.POINTER(vx_split), vp,
                                   c.c_uint32], c.c_int64),
        "vx_verify_files_split_multi": ([vp, c.c_size_t, vp, vp, c.c_size_t, c.c_uint32, vp, c.c_size_t,
                                         c.POINTER(vx_split), vp, c.c_uint32], c.c_int64),
    }
    if tuning:
        sig.update({
            "vx_sha1_device_uniform_variant": ([vp, c.c_uint64, c.c_uint32, c.c_uint32, vp, vp, vp, vp, c.c_int],
                                               c.c_int),
            "vx_sha1_device_ragged_variant": ([vp, vp, vp, vp, c.c_uint32, vp, vp, vp, vp, c.c_int], c.c_int),
            "vx_tuning_zero_copy_plan": ([c.c_uint32, c.c_uint64], c.c_int),
            "vx_tuning_zero_copy_kernel": ([vp, vp, c.c_uint32, vp, vp, vp, c.c_int, vp], c.c_int),
            "vx_tuning_fail_submit_after": ([vp, c.c_int64], None),
            "vx_tuning_fail_launch_after": ([vp, c.c_int64], None),
            "vx_tuning_verify_copy_stream": ([vp, c.c_int], None),
            "vx_tuning_stage_huge": ([vp, c.c_int], None),
            "vx_tuning_split_rules": ([vp, c.c_int, c.c_uint64, c.c_int, c.c_int], None),
            "vx_tuning_clock_stamp": ([vp, c.c_uint32, vp], c.c_int),
            "vx_tuning_wall_clock_khz": ([c.c_int], c.c_int),
            "vx_tuning_device_identity": ([c.c_int, c.c_char_p, c.c_size_t, c.c_char_p], c.c_int),
            "vx_tuning_plan_ragged": ([c.c_uint32, c.c_uint32, c.c_uint64], c.c_int),
            "vx_tuning_split_take_tail": ([c.POINTER(vx_split), c.c_uint64, c.POINTER(c.c_uint64)], c.c_uint64),
            "vx_tuning_last_split": ([vp, c.POINTER(c.c_double), c.c_size_t], c.c_size_t),
            "vx_tuning_chunk_schedule": ([c.c_uint64, c.c_uint64, c.c_int, c.c_int, c.POINTER(c.c_uint64),
                                          c.c_size_t], c.c_size_t),
            "vx_synth_fill": ([vp, c.c_uint64, c.c_uint32, c.c_uint32, c.c_uint64, c.c_uint64, c.c_uint32, vp],
                              c.c_int),
        })
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res


def _load(path: str, tuning: bool) -> ctypes.CDLL:
    import torch  # noqa: F401  (single HIP runtime, see module doc)

    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: the HIP engine is not built. Run "
            "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C vortex_amd/csrc`).")
    L = ctypes.CDLL(path)
    _declare(L, tuning)
    if L.vx_abi_version() != ABI_VERSION:
        raise ImportError(f"{os.path.basename(path)} ABI version mismatch")
    return L


def lib() -> ctypes.CDLL:
    """Load libvortex_amd.so once; raise ImportError if it was never built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            _lib = _load(LIB_PATH, False)
    return _lib


def tuning() -> ctypes.CDLL:
    """Load libvortex_amd_tuning.so once (tests, bench.py; vx_tuning.h)."""
    global _tuning
    if _tuning is not None:
        return _tuning
    with _lock:
        if _tuning is None:
            _tuning = _load(TUNING_PATH, True)
    return _tuning


def check(rc: int, where: str, L: ctypes.CDLL | None = None) -> int:
    """Raise VxError for a negative code; the message is the thread-local
    vx_last_error of the library that failed (L, default lib())."""
    if rc < 0:
        msg = (L or lib()).vx_last_error().decode(errors="replace")
        raise VxError(rc, where, msg)
    return rc
