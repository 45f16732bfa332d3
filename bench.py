#!/usr/bin/env python3
"""bench.py — device-resident SHA-1 piece hashing on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: hash every piece of the
GPU's shard (65,536 x 256 KiB = 16 GiB by default, BASELINE config 2),
compare each digest with the expected table (DownloadedPiece::hash_matched),
and — on N > 1 GPUs — all-gather the verdicts over RCCL (the only exchange the
path has; vortex_amd/shard.py).  Inputs are resident in HBM before the timed
region.  Weak scaling: every GPU hashes its own 65,536 pieces
(global index r*65536 + i, BASELINE config 4 at N=8).

Extra fields (DESIGN.md "Measurement"):
  roofline      dominant kernel's achieved algorithmic bytes per launch / its
                HIP-event duration on the launch stream, vs 8 TB/s HBM3E;
                traffic = corrected PMC FETCH bytes from profiles/ when a
                profile of this workload is committed, else null.
  cpu_baseline  the oracle's restatement of vortex's rayon+SHA-NI pool
                (oracle/pool_oracle.cpp, kind "port") on this host's cores,
                rank 0 at N=1 only, bounded sample of config 1.
  e2e           host-resident pieces through the C-ABI host path (pinned
                H2D + kernel + D2H of digests/verdicts), N=1 only.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
(N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import mmap
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s SHA-1 piece hashing (device-resident), 256 KiB pieces, 1/2/4/8 MI355X"
HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md)
GiB = float(1 << 30)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_share() -> int:
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def load_traffic(workload: str, pieces: int, plen: int):
    """Corrected HBM bytes per launch from a committed PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    ent = d.get(f"{pieces}x{plen}")
    return ent.get("hbm_bytes_per_launch") if ent else None


def cpu_baseline(seconds: float, plen: int):
    """vortex's pool restated (oracle/pool_oracle.cpp): one task per piece on
    `threads` workers, SHA-NI when the CPU has it, results over an MPSC queue.
    Sample: config 1 = 4,096 x 256 KiB pieces (1 GiB) in host memory, passes
    repeated until about `seconds` of CPU-thread time."""
    import oracle

    threads = cpu_share()
    n = 4096
    buf = mmap.mmap(-1, n * plen)
    base = ctypes.addressof(ctypes.c_char.from_buffer(buf))
    for i in range(n):
        oracle.lib().vxo_gen_piece(0x5EED0001, i, plen, 0, ctypes.c_void_p(base + i * plen))
    ptrs = (ctypes.c_void_p * n)(*[base + i * plen for i in range(n)])
    lens = (ctypes.c_uint32 * n)(*([plen] * n))
    dig = ctypes.create_string_buffer(20 * n)
    matched = ctypes.create_string_buffer(n)
    oracle.pool_verify_ptrs(ptrs, lens, n, None, threads, 0, None, dig)  # warm + expected table
    exp = ctypes.create_string_buffer(dig.raw, 20 * n)
    passes, t0 = 0, time.perf_counter()
    while True:
        oracle.pool_verify_ptrs(ptrs, lens, n, exp, threads, 0, matched, dig)
        passes += 1
        el = time.perf_counter() - t0
        if el * threads >= seconds or el > 60:
            break
    assert matched.raw[:n] == b"\x01" * n
    del ptrs
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(passes * n * plen / el / GiB, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{passes} pass(es) over 4096 x {plen // 1024} KiB host pieces (config 1), "
                      f"{el:.2f} s wall, sha_ni={bool(oracle.has_shani())}, cpu='{model}'"}


def e2e_rate(plen: int, n: int = 8192):
    """Host-resident pieces through the C ABI's vx_verify_batch with the
    pieces in a registered (pinned) mmap: H2D + kernel + D2H of verdicts and
    digests, PCIe-inclusive.  Argument arrays are built before the timed call
    (the Rust caller would hand over its own pointer table)."""
    import torch

    import oracle
    from vortex_amd._lib import check, lib
    from vortex_amd.hash_pool import HashPool

    buf = mmap.mmap(-1, n * plen)
    base = ctypes.addressof(ctypes.c_char.from_buffer(buf))
    for i in range(n):
        oracle.lib().vxo_gen_piece(0x5EED0001, i, plen, 0, ctypes.c_void_p(base + i * plen))
    exp = ctypes.create_string_buffer(oracle.pool_digest_synth(0x5EED0001, 0, n, plen, threads=cpu_share()), 20 * n)
    ptrs = (ctypes.c_void_p * n)(*[base + i * plen for i in range(n)])
    lens = (ctypes.c_uint32 * n)(*([plen] * n))
    matched = ctypes.create_string_buffer(n)
    digests = ctypes.create_string_buffer(20 * n)
    with HashPool(plen, slots=4, slot_bytes=256 << 20, batch_pieces=1024) as pool:
        pool.register_buffer(buf)
        check(lib().vx_verify_batch(pool._h, ptrs, lens, exp, 256, matched, digests), "warm")
        runs = []  # three timed calls (one 2 GiB call is ~40 ms); the median is reported
        for _ in range(3):
            ctypes.memset(matched, 0, n)
            t0 = time.perf_counter()
            check(lib().vx_verify_batch(pool._h, ptrs, lens, exp, n, matched, digests), "vx_verify_batch")
            runs.append(time.perf_counter() - t0)
            assert matched.raw[:n] == b"\x01" * n
        pool.unregister_buffer(buf)
    el = sorted(runs)[1]
    # plain pinned H2D copy of the same byte count, for context (PCIe Gen5 x16)
    host = torch.empty(n * plen, dtype=torch.uint8, pin_memory=True)
    dev_t = torch.empty(n * plen, dtype=torch.uint8, device="cuda")
    dev_t.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    dev_t.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    h2d = n * plen / (time.perf_counter() - t1) / GiB
    del dev_t, host
    return {"value": round(n * plen / el / GiB, 3), "unit": "GiB/s", "pinned_h2d_copy_GiBps": round(h2d, 2),
            "runs_GiBps": [round(n * plen / r / GiB, 2) for r in runs],
            "sample": f"{n} x {plen // 1024} KiB from a registered host mmap via vx_verify_batch "
                      f"(H2D + kernel + D2H), median of 3 calls, {el * 1e3:.1f} ms"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pieces", type=int, default=65536, help="pieces per GPU")
    ap.add_argument("--piece-len", type=int, default=262144)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-thread seconds for the baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm, the real path) or gloo (single-GPU multi-rank rehearsal)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank uses cuda:0 (with --dist-backend gloo)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from vortex_amd import device as vdev
    from vortex_amd.shard import gather_verdicts

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    n, plen = args.pieces, args.piece_len
    stride = (plen + 15) // 16 * 16
    first = rank * n  # weak scaling: global piece index shard
    seed = 0x5EED0002
    data = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    # Expected table = digests of the clean batch; then 1% of pieces get a flipped byte.
    vdev.synth_fill(data, n, plen, stride=stride, first=first, seed=seed)
    expected, _ = vdev.sha1_uniform(data, n, plen, stride=stride)
    torch.cuda.synchronize()
    import oracle  # checker only

    exp_host = expected.cpu().numpy().tobytes()
    sample = sorted({0, n - 1, n // 2, *range(0, n, max(1, n // 29))})
    for i in sample:
        want = oracle.sha1(oracle.gen_piece(seed, first + i, plen))
        assert exp_host[20 * i:20 * i + 20] == want, f"rank {rank}: digest of piece {first + i} differs from oracle"
    corrupt_every = 100
    vdev.synth_fill(data, n, plen, stride=stride, first=first, seed=seed, corrupt_every=corrupt_every)
    matched = torch.empty(n, dtype=torch.uint8, device=dev)
    n_total = n * world

    def step():
        vdev.sha1_uniform(data, n, plen, stride=stride, expected=expected, matched=matched, want_digests=False,
                          stream=stream)

    for _ in range(args.warmup):
        step()
        if world > 1:
            gather_verdicts(matched, n_total)
    torch.cuda.synchronize()

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    verdicts = None
    for k in range(args.steps):
        evs[k][0].record(stream)
        step()
        evs[k][1].record(stream)
        if world > 1:
            verdicts = gather_verdicts(matched, n_total)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    # Verdicts: exactly the corrupted pieces mismatch (checked on the gathered
    # table when N > 1, else locally).
    m = (verdicts if verdicts is not None else matched).cpu().numpy()
    g0 = 0 if verdicts is not None else first
    bad = [i for i in range(len(m)) if not m[i]]
    want_bad = [i for i in range(len(m)) if oracle.is_corrupt(g0 + i, corrupt_every)]
    assert bad == want_bad, f"rank {rank}: verdicts differ from the expected mismatch set"

    total_bytes = n_total * plen
    value = total_bytes / elapsed * args.steps / GiB
    achieved = n * plen / (kern_ms * 1e-3)
    # Integer-VALU ceiling (DESIGN.md "Roofline"): 613.5 VALU per 64-byte block
    # (measured SQ_INSTS_VALU / waves / blocks), 16 lanes/clk per SIMD for
    # these VOP3 integer ops, 1,024 SIMDs, nominal 2.4 GHz.
    valu_ops = n * ((plen + 9 + 63) // 64) * 613.5 / (kern_ms * 1e-3)
    valu_peak = 256 * 4 * 16 * 2.4e9
    workload = f"{n} x {plen // 1024} KiB pieces per GPU"
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: counter-based splitmix64 pieces generated in HBM, 1% with one flipped byte",
        "config": {"workload": workload + " (BASELINE config 2; config 4 at N=8), SHA-1 + verify vs expected table"
                               + (", RCCL all-gather of verdicts" if world > 1 else ""),
                   "pieces_per_gpu": n, "piece_len": plen, "total_GiB": round(total_bytes / GiB, 2),
                   "parallelism": f"piece-index shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4),
                     "traffic": load_traffic(workload, n, plen),
                     "kernel": "sha1_uniform_kernel", "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_launch": n * plen,
                     "valu": {"achieved_Tops": round(valu_ops / 1e12, 2), "peak_Tops_at_2.4GHz": round(valu_peak / 1e12, 2),
                              "frac": round(valu_ops / valu_peak, 4),
                              "note": "the kernel is integer-VALU bound; see DESIGN.md Roofline"}},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args.cpu_seconds, plen)
    if rank == 0 and world == 1 and not args.no_e2e:
        del data
        torch.cuda.empty_cache()
        res["e2e"] = e2e_rate(plen)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
