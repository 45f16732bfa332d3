"""Multi-GPU sharding of a piece batch.

Pieces are independent, so a batch is split by piece index with no exchange
during hashing: one process per GPU hashes its shard, then ONE collective
gathers the per-piece verdicts to every rank (RCCL over xGMI on MI355X
nodes — torch.distributed's "nccl" backend is RCCL on ROCm — and gloo in the
CPU tests).  At 65,536 pieces per GPU the verdicts are 64 KiB per rank: a
latency-bound gather that is never on the throughput-critical path.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous piece-index range [start, start+count) of `rank`:
    n_total // world each, the remainder going to the LAST ranks."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, rem = divmod(n_total, world)
    extra_from = world - rem  # ranks >= extra_from get one more piece
    start = rank * base + max(0, rank - extra_from)
    count = base + (1 if rank >= extra_from else 0)
    return start, count


def blocks(length: int) -> int:
    """SHA-1 compressions for a piece of `length` bytes (incl. padding)."""
    return (length + 9 + 63) // 64


def shard_ragged(lens: Sequence[int], world: int) -> List[List[int]]:
    """Balance a ragged batch by compression count, not piece count:
    longest-first greedy onto the least-loaded rank (LPT).  Each rank's list
    is returned in descending-length order (what the ragged kernel wants)."""
    order = sorted(range(len(lens)), key=lambda i: (-lens[i], i))
    load = [0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(i)
        load[r] += blocks(lens[i])
    return out


def gather_verdicts(matched_local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather every rank's contiguous-shard verdicts into one [n_total]
    uint8 tensor, in global piece order, on every rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [shard_range(n_total, world, r)[1] for r in range(world)]
    width = max(counts)
    if matched_local.numel() != counts[rank]:
        raise ValueError("local verdicts do not match this rank's shard")
    # gloo (CPU tests, single-GPU rehearsals) gathers host tensors; RCCL gathers
    # device tensors in place over xGMI.
    dev = matched_local.device
    on_host = dist.get_backend(group) == "gloo"
    work_dev = torch.device("cpu") if on_host else dev
    padded = torch.zeros(width, dtype=torch.uint8, device=work_dev)
    padded[: counts[rank]] = matched_local.to(work_dev)
    out = torch.empty(world * width, dtype=torch.uint8, device=work_dev)
    dist.all_gather_into_tensor(out, padded, group=group)
    parts = [out[r * width: r * width + counts[r]] for r in range(world)]
    return torch.cat(parts).to(dev)


def verify_files_sharded(pool, paths: Sequence[str], file_lengths: Sequence[int], piece_length: int,
                         expected: bytes, group=None, io_threads: int = 0) -> Tuple[List[bool], int]:
    """Multi-GPU bulk re-verify (torrent.rs:716-761 split across ranks): each
    rank's HashPool reads and verifies only its contiguous piece range
    (vx_verify_files_range; its own GPU's PCIe link carries only its bytes),
    then the verdicts are all-gathered and the I/O-error counts summed.
    Every rank returns the whole torrent's verdicts."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = len(expected) // 20
    first, count = shard_range(n, world, rank)
    local, bad = pool.verify_files(paths, file_lengths, piece_length, expected, io_threads=io_threads,
                                   first=first, count=count)
    on_host = dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if on_host else torch.device("cuda", torch.cuda.current_device())
    matched = torch.tensor(local, dtype=torch.uint8, device=dev) if count else torch.zeros(0, dtype=torch.uint8,
                                                                                            device=dev)
    allv = gather_verdicts(matched, n, group=group)
    nbad = torch.tensor([bad], dtype=torch.int64, device=dev)
    dist.all_reduce(nbad, group=group)
    return [bool(x) for x in allv.cpu().tolist()], int(nbad.item())
