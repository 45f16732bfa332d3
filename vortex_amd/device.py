"""Device-resident batch API (the hot path): torch tensors in, digests out.

PyTorch is only plumbing here — it owns the HBM allocations and the stream;
the hashing is the HIP kernels in libvortex_amd.so, called through the C ABI
(``vx_sha1_device_uniform`` / ``vx_sha1_device_ragged``).

Layout (DESIGN.md "Data layout in HBM"): one uint8 tensor holds all pieces;
piece i starts at ``i * stride`` (uniform) or ``offsets[i]`` (ragged), every
start 16-byte aligned.  Digests are ``[n, 20]`` uint8 (big-endian SHA-1),
verdicts ``[n]`` uint8 (0/1).
"""
from __future__ import annotations

from typing import Optional

import torch

from ._lib import check, lib


def _stream_ptr(stream: Optional[torch.cuda.Stream], device: torch.device) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return int(s.cuda_stream)


def _req(t: torch.Tensor, name: str, dtype=torch.uint8) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def sha1_uniform(data: torch.Tensor, n: int, piece_len: int, stride: Optional[int] = None,
                 expected: Optional[torch.Tensor] = None, digests: Optional[torch.Tensor] = None,
                 matched: Optional[torch.Tensor] = None, want_digests: bool = True,
                 stream: Optional[torch.cuda.Stream] = None, variant: int = 0):
    """Hash n pieces of piece_len bytes at data[i*stride : i*stride+piece_len].

    Returns (digests [n,20] or None, matched [n] or None).  Enqueue-only.
    variant: 0 = default kernel; 1/2 pin a variant (include/vx_tuning.h)."""
    _req(data, "data")
    stride = piece_len if stride is None else stride
    if n and (n - 1) * stride + piece_len > data.numel():
        raise ValueError("batch exceeds data tensor")
    dev = data.device
    if want_digests and digests is None:
        digests = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    if expected is not None:
        _req(expected, "expected")
        if expected.numel() < 20 * n:
            raise ValueError("expected must hold n*20 bytes")
        if matched is None:
            matched = torch.empty((n,), dtype=torch.uint8, device=dev)
    rc = lib().vx_sha1_device_uniform_variant(
        data.data_ptr(), stride, piece_len, n,
        digests.data_ptr() if (want_digests and digests is not None) else None,
        expected.data_ptr() if expected is not None else None,
        matched.data_ptr() if expected is not None else None,
        _stream_ptr(stream, dev), variant)
    check(rc, "vx_sha1_device_uniform")
    return (digests if want_digests else None), (matched if expected is not None else None)


def sha1_ragged(data: torch.Tensor, offsets: torch.Tensor, lens: torch.Tensor,
                order: Optional[torch.Tensor] = None, expected: Optional[torch.Tensor] = None,
                digests: Optional[torch.Tensor] = None, matched: Optional[torch.Tensor] = None,
                stream: Optional[torch.cuda.Stream] = None, variant: int = 0, plan=None):
    """Hash piece i = data[offsets[i] : offsets[i]+lens[i]] for all i.

    offsets: int64 device tensor (16-byte aligned values); lens: int32 device
    tensor; order: optional int32 permutation (see :func:`length_order`).
    variant: 0 = default kernel; 1 lane / 2 split pin one (vx_tuning.h).
    plan: (max_len, total_bytes) of the batch, known on the host when it is
    laid out (see :func:`ragged_plan`); with variant 0 the engine then picks
    the kernel whose time bound is lower (vx_sha1_device_ragged_hint,
    DESIGN.md §3.4)."""
    _req(data, "data")
    _req(offsets, "offsets", torch.int64)
    _req(lens, "lens", torch.int32)
    n = offsets.numel()
    if lens.numel() != n:
        raise ValueError("offsets and lens differ in length")
    dev = data.device
    if digests is None:
        digests = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    if expected is not None:
        _req(expected, "expected")
        if matched is None:
            matched = torch.empty((n,), dtype=torch.uint8, device=dev)
    if order is not None:
        _req(order, "order", torch.int32)
    exp_p = expected.data_ptr() if expected is not None else None
    m_p = matched.data_ptr() if expected is not None else None
    order_p = order.data_ptr() if order is not None else None
    if variant == 0 and plan is not None:
        max_len, total = plan
        rc = lib().vx_sha1_device_ragged_hint(data.data_ptr(), offsets.data_ptr(), lens.data_ptr(), order_p, n,
                                              int(max_len), int(total), digests.data_ptr(), exp_p, m_p,
                                              _stream_ptr(stream, dev))
    else:
        rc = lib().vx_sha1_device_ragged_variant(data.data_ptr(), offsets.data_ptr(), lens.data_ptr(), order_p, n,
                                                 digests.data_ptr(), exp_p, m_p, _stream_ptr(stream, dev), variant)
    check(rc, "vx_sha1_device_ragged")
    return digests, matched


def ragged_plan(lens_host) -> tuple[int, int]:
    """(longest piece, total bytes) of a ragged batch: the `plan` argument of
    :func:`sha1_ragged`."""
    import numpy as np

    arr = np.asarray(lens_host, dtype=np.uint64)
    return (int(arr.max()) if arr.size else 0), int(arr.sum())


def length_order(lens_host) -> torch.Tensor:
    """Permutation sorting pieces by descending length (vx_sort_order), as
    an int32 CPU tensor; move it to the device for sha1_ragged."""
    import ctypes

    import numpy as np

    arr = np.ascontiguousarray(np.asarray(lens_host, dtype=np.uint32))
    out = np.empty_like(arr)
    check(lib().vx_sort_order(arr.ctypes.data, arr.size, out.ctypes.data), "vx_sort_order")
    del ctypes
    return torch.from_numpy(out.astype(np.int32))


def synth_fill(data: torch.Tensor, n: int, piece_len: int, stride: Optional[int] = None, first: int = 0,
               seed: int = 0x5EED0002, corrupt_every: int = 0,
               stream: Optional[torch.cuda.Stream] = None) -> None:
    """Fill n synthetic pieces on the device (DESIGN.md "Synthetic pieces")."""
    _req(data, "data")
    stride = piece_len if stride is None else stride
    rc = lib().vx_synth_fill(data.data_ptr(), stride, piece_len, n, first, seed, corrupt_every,
                             _stream_ptr(stream, data.device))
    check(rc, "vx_synth_fill")
