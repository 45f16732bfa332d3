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

from ._lib import check, lib, tuning


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
    variant: 0 = the default kernel (vx_sha1_device_uniform, the release
    library); others pin a variant through the tuning build (vx_tuning.h)."""
    _req(data, "data")
    stride = piece_len if stride is None else stride
    if n and (n - 1) * stride + piece_len > data.numel():
        raise ValueError("batch exceeds data tensor")
    dev = data.device
    if want_digests and digests is None:
        digests = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    elif want_digests:
        _req(digests, "digests")
        if digests.numel() < 20 * n or digests.device != dev:
            raise ValueError("digests must hold n*20 bytes on the data's device")
    if expected is not None:
        _req(expected, "expected")
        if expected.numel() < 20 * n or expected.device != dev:
            raise ValueError("expected must hold n*20 bytes on the data's device")
        if matched is None:
            matched = torch.empty((n,), dtype=torch.uint8, device=dev)
        else:
            _req(matched, "matched")
            if matched.numel() < n or matched.device != dev:
                raise ValueError("matched must hold n bytes on the data's device")
    args = (data.data_ptr(), stride, piece_len, n,
            digests.data_ptr() if (want_digests and digests is not None) else None,
            expected.data_ptr() if expected is not None else None,
            matched.data_ptr() if expected is not None else None,
            _stream_ptr(stream, dev))
    if variant == 0:
        check(lib().vx_sha1_device_uniform(*args), "vx_sha1_device_uniform")
    else:
        check(tuning().vx_sha1_device_uniform_variant(*args, variant), "vx_sha1_device_uniform_variant", tuning())
    return (digests if want_digests else None), (matched if expected is not None else None)


def _check_ragged_layout(data: torch.Tensor, offsets: torch.Tensor, lens: torch.Tensor,
                         order: Optional[torch.Tensor]) -> None:
    """The kernels trust their offsets (vx_hash.h: the raw device entries do
    not validate device-resident metadata), so check here what an
    out-of-range batch would otherwise turn into reads of arbitrary HBM:
    every offset 16-byte aligned and >= 0, every length >= 0, every piece
    inside `data`, and `order` a set of indices in [0, n).  One small
    reduction on the device and one 4-value copy back (a sync)."""
    n = offsets.numel()
    if n == 0:
        return
    ends = offsets + lens.to(torch.int64)
    stats = torch.stack([
        (offsets & 15).ne(0).any().to(torch.int64),
        offsets.min().lt(0).to(torch.int64) + lens.min().lt(0).to(torch.int64),
        ends.max(),
        (order.min().lt(0) | order.max().ge(n)).to(torch.int64) if order is not None else offsets.new_zeros(()),
    ]).cpu().tolist()
    if stats[0]:
        raise ValueError("sha1_ragged: every offset must be a multiple of 16 (the kernels load 16 bytes per lane)")
    if stats[1]:
        raise ValueError("sha1_ragged: negative offset or length")
    if stats[2] > data.numel():
        raise ValueError(f"sha1_ragged: a piece ends at byte {stats[2]}, past the data tensor ({data.numel()} bytes)")
    if stats[3]:
        raise ValueError("sha1_ragged: order holds an index outside [0, n)")


def sha1_ragged(data: torch.Tensor, offsets: torch.Tensor, lens: torch.Tensor,
                order: Optional[torch.Tensor] = None, expected: Optional[torch.Tensor] = None,
                digests: Optional[torch.Tensor] = None, matched: Optional[torch.Tensor] = None,
                stream: Optional[torch.cuda.Stream] = None, variant: int = 0, plan=None,
                validate: bool = True):
    """Hash piece i = data[offsets[i] : offsets[i]+lens[i]] for all i.

    offsets: int64 device tensor (16-byte aligned values); lens: int32 device
    tensor; order: optional int32 permutation (see :func:`length_order`).
    variant: 0 = default kernel; 1 lane / 2 split pin one (vx_tuning.h).
    plan: (max_len, total_bytes) of the batch, known on the host when it is
    laid out (see :func:`ragged_plan`); with variant 0 the engine then picks
    the kernel whose time bound is lower (vx_sha1_device_ragged_hint,
    DESIGN.md §3.4).
    validate: check alignment and bounds of offsets/lens/order first (a
    device reduction and a sync; see :func:`_check_ragged_layout`).  Pass
    False only for a layout built by trusted code, e.g. a timed loop over a
    batch that was validated once."""
    _req(data, "data")
    _req(offsets, "offsets", torch.int64)
    _req(lens, "lens", torch.int32)
    n = offsets.numel()
    if lens.numel() != n:
        raise ValueError("offsets and lens differ in length")
    if order is not None:
        _req(order, "order", torch.int32)
        if order.numel() != n:
            raise ValueError("order must hold n indices")
    dev = data.device
    for name, t in (("offsets", offsets), ("lens", lens), ("order", order), ("expected", expected),
                    ("digests", digests), ("matched", matched)):
        if t is not None and t.device != dev:
            raise ValueError(f"{name} is on {t.device}, data on {dev}")
    if validate:
        _check_ragged_layout(data, offsets, lens, order)
    if digests is None:
        digests = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    elif digests.dtype != torch.uint8 or not digests.is_contiguous() or digests.numel() < 20 * n:
        raise ValueError("digests must be a contiguous uint8 tensor of n*20 bytes")
    if expected is not None:
        _req(expected, "expected")
        if expected.numel() < 20 * n:
            raise ValueError("expected must hold n*20 bytes")
        if matched is None:
            matched = torch.empty((n,), dtype=torch.uint8, device=dev)
        elif matched.dtype != torch.uint8 or not matched.is_contiguous() or matched.numel() < n:
            raise ValueError("matched must be a contiguous uint8 tensor of n bytes")
    exp_p = expected.data_ptr() if expected is not None else None
    m_p = matched.data_ptr() if expected is not None else None
    order_p = order.data_ptr() if order is not None else None
    if variant == 0 and plan is not None:
        max_len, total = plan
        rc = lib().vx_sha1_device_ragged_hint(data.data_ptr(), offsets.data_ptr(), lens.data_ptr(), order_p, n,
                                              int(max_len), int(total), digests.data_ptr(), exp_p, m_p,
                                              _stream_ptr(stream, dev))
        check(rc, "vx_sha1_device_ragged_hint")
    elif variant == 0:
        rc = lib().vx_sha1_device_ragged(data.data_ptr(), offsets.data_ptr(), lens.data_ptr(), order_p, n,
                                         digests.data_ptr(), exp_p, m_p, _stream_ptr(stream, dev))
        check(rc, "vx_sha1_device_ragged")
    else:
        rc = tuning().vx_sha1_device_ragged_variant(data.data_ptr(), offsets.data_ptr(), lens.data_ptr(), order_p, n,
                                                    digests.data_ptr(), exp_p, m_p, _stream_ptr(stream, dev), variant)
        check(rc, "vx_sha1_device_ragged_variant", tuning())
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
    """Fill n synthetic pieces on the device (DESIGN.md "Synthetic pieces";
    include/vx_synth.h, a test/bench generator: tuning build only)."""
    _req(data, "data")
    stride = piece_len if stride is None else stride
    rc = tuning().vx_synth_fill(data.data_ptr(), stride, piece_len, n, first, seed, corrupt_every,
                                _stream_ptr(stream, data.device))
    check(rc, "vx_synth_fill", tuning())
