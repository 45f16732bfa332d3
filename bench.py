#!/usr/bin/env python3
"""bench.py — device-resident SHA-1 piece hashing on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: hash every piece of the
GPU's shard (65,536 x 256 KiB = 16 GiB by default, BASELINE config 2),
compare each digest with the expected table (DownloadedPiece::hash_matched),
and — on N > 1 GPUs — all-gather the verdicts over RCCL (the only exchange the
path has; vortex_amd/shard.py).  Inputs are resident in HBM before the timed
region.  Weak scaling: every GPU hashes its own 65,536 pieces
(global index r*65536 + i, BASELINE config 4 at N=8).

Extra fields (DESIGN.md §7 "Measurement"; all but roofline at N=1 only):
  roofline       dominant kernel's achieved algorithmic bytes per launch / its
                 HIP-event duration on the launch stream, vs 8 TB/s HBM3E
                 (the metric's fraction); traffic = corrected PMC FETCH bytes
                 from profiles/; bound = the VALU-issue roof it really hits,
                 with fractions in roofline.valu.
  cpu_baseline   the oracle's restatement of vortex's rayon+SHA-NI pool
                 (oracle/pool_oracle.cpp, kind "port") on this host's cores,
                 bounded sample of config 1.
  ragged         config 3 (16 GiB ragged mix), device-resident, with the
                 per-block chain time against its floor.
  e2e            8,192 x 256 KiB host pieces in 8,192 separately registered
                 mmaps (vortex's BufferPool layout) via vx_verify_batch.
  e2e_async      the same pieces through vx_submit/vx_flush/vx_poll; `paced`:
                 the download loop at 1/4/16/40 GB/s arrivals (loop-thread
                 time in the engine, submit stall, submit-to-poll latency).
  e2e_contiguous the same pieces in one registered mmap (best-case layout).
  reverify       config 5: linux-mint-geometry re-verify from an fsync'd,
                 page-cache-warm file via vx_verify_files, with the CPU pool
                 on the same file, and each call's read / copy budget.
  reverify_cold  the same with the file's pages evicted before every call
                 (fsync + POSIX_FADV_DONTNEED): reads from the disk.
At N > 1 (every rank takes part):
  ranks          every rank's step / kernel / verdict-gather time, shader
                 clock, and identity (device index, PCI bus id, UUID, the
                 world size RCCL reported); distinct_devices must hold unless
                 --same-device (a rehearsal).
  reverify_multi (opt-in, --reverify-multi) config 5 split over the N GPUs by
                 piece index, warm and cold, the slowest rank's time, beside
                 the CPU pool on every node CPU.
roofline.valu.clock_run: the shader clock of each XCC over the timed steps
(s_memtime / s_memrealtime stamps, vortex_amd/csrc/vx_clock.hip) and the
kernel's issue fraction at that clock.

Output: stdout carries ONE compact JSON line of at most 8 KB (compact_line:
the headline, config, roofline scalars, cpu_baseline, parity, per-rank
scalars, each leg's scalars); the full record — traces, timelines, the split
sweep, the nested roofline.valu block, rank identities — goes to the side
file the line names in `detail` (bench_detail.json beside bench.py, or
--detail PATH).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1: either launched by the driver as
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
or started plainly, in which case bench.py starts the N ranks itself (a
child torch.distributed.run, before any GPU call) and relays rank 0's line
and exit code.  --gpus must equal WORLD_SIZE when one is set, and a run that
cannot get N ranks fails: it never prints a one-GPU line for --gpus N.
Whenever it runs under torch.distributed (even WORLD_SIZE=1) the process
group is real and the line reports its world_size and backend.
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


def node_cpus(cpu_max: str = "/sys/fs/cgroup/cpu.max") -> int:
    """CPUs this process may really use on the node: its affinity set, capped by
    a cgroup v2 CPU quota (cpu.max "quota period") when one is set.  Unlike
    cpu_share() it ignores OMP_NUM_THREADS, which torch.distributed.run sets
    to 1 for every rank of a multi-rank launch."""
    n = len(os.sched_getaffinity(0))
    try:
        with open(cpu_max) as f:
            quota, period = f.read().split()[:2]
        if quota != "max" and int(period) > 0:
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return max(1, n)


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


def _register_all(pool, bufs):
    for b in bufs:
        pool.register_buffer(b)


def _unregister_all(pool, bufs):
    for b in bufs:
        pool.unregister_buffer(b)


def e2e_contiguous(plen: int, n: int = 8192):
    """Secondary e2e figure: all n pieces in ONE registered mmap at a constant
    stride, so vx_verify_batch takes the strided hipMemcpy2DAsync chunk path
    (vx_engine.hip batch_chunked).  vortex never lays its buffers out like
    this (one AnonymousMmap per buffer, buf_pool.rs:92-98): see e2e_batch."""
    import torch

    import oracle
    from vortex_amd._lib import check
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
        check(pool.lib.vx_verify_batch(pool._h, ptrs, lens, exp, 256, matched, digests), "warm")
        runs = []
        for _ in range(3):
            ctypes.memset(matched, 0, n)
            t0 = time.perf_counter()
            check(pool.lib.vx_verify_batch(pool._h, ptrs, lens, exp, n, matched, digests), "vx_verify_batch")
            runs.append(time.perf_counter() - t0)
            assert matched.raw[:n] == b"\x01" * n
        pool.unregister_buffer(buf)
    del ptrs
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
            "sample": f"{n} x {plen // 1024} KiB in ONE registered host mmap via vx_verify_batch "
                      f"(strided 2-D copy path; H2D + kernel + D2H), median of 3 calls, {el * 1e3:.1f} ms"}


def e2e_batch(plen: int, n: int = 8192):
    """Host-resident pieces in vortex's own buffer layout — one registered
    mmap per buffer (BufferPool, buf_pool.rs:92-98) — verified by
    vx_verify_batch (the bulk verify of torrent.rs:724-740 over host
    buffers): the gather kernel pulls each piece over PCIe through its
    buffer's device mapping, then the hash kernels run; verdicts and digests
    come back (PCIe-inclusive end to end)."""
    import oracle
    from vortex_amd._lib import check
    from vortex_amd.hash_pool import HashPool

    bufs = [mmap.mmap(-1, plen) for _ in range(n)]
    addrs = [ctypes.addressof(ctypes.c_char.from_buffer(b)) for b in bufs]
    for i, a in enumerate(addrs):
        oracle.lib().vxo_gen_piece(0x5EED0001, i, plen, 0, ctypes.c_void_p(a))
    exp = ctypes.create_string_buffer(oracle.pool_digest_synth(0x5EED0001, 0, n, plen, threads=cpu_share()), 20 * n)
    ptrs = (ctypes.c_void_p * n)(*addrs)
    lens = (ctypes.c_uint32 * n)(*([plen] * n))
    matched = ctypes.create_string_buffer(n)
    digests = ctypes.create_string_buffer(20 * n)
    with HashPool(plen, slots=4, slot_bytes=256 << 20, batch_pieces=1024) as pool:
        t0 = time.perf_counter()
        _register_all(pool, bufs)
        t_reg = time.perf_counter() - t0
        check(pool.lib.vx_verify_batch(pool._h, ptrs, lens, exp, 256, matched, digests), "warm")
        pool.reset_stats()
        runs = []
        for _ in range(3):
            ctypes.memset(matched, 0, n)
            t0 = time.perf_counter()
            check(pool.lib.vx_verify_batch(pool._h, ptrs, lens, exp, n, matched, digests), "vx_verify_batch")
            runs.append(time.perf_counter() - t0)
            assert matched.raw[:n] == b"\x01" * n
        st = pool.stats()
        # one call over the same buffers 4 times (8 GiB): the head and tail of a bulk verify weigh 4x less
        n4 = 4 * n
        ptrs4 = (ctypes.c_void_p * n4)(*(addrs * 4))
        lens4 = (ctypes.c_uint32 * n4)(*([plen] * n4))
        exp4 = ctypes.create_string_buffer(exp.raw * 4, 20 * n4)
        matched4 = ctypes.create_string_buffer(n4)
        t0 = time.perf_counter()
        check(pool.lib.vx_verify_batch(pool._h, ptrs4, lens4, exp4, n4, matched4, None), "vx_verify_batch x4")
        el4 = time.perf_counter() - t0
        assert matched4.raw[:n4] == b"\x01" * n4
        _unregister_all(pool, bufs)
    del ptrs, addrs
    el = sorted(runs)[1]
    return {"value": round(n * plen / el / GiB, 3), "unit": "GiB/s",
            "runs_GiBps": [round(n * plen / r / GiB, 2) for r in runs],
            "register_s": round(t_reg, 3),
            "batch_4x": {"GiBps": round(4 * n * plen / el4 / GiB, 3), "GiB": round(4 * n * plen / GiB, 3),
                         "note": "one vx_verify_batch over the same buffers 4 times, verdicts only"},
            "engine": {k: st[k] for k in ("pieces_completed", "batches", "chunk_rounds", "gather_tiles", "staged_bytes")},
            "sample": f"{n} x {plen // 1024} KiB, one registered mmap per piece (buf_pool.rs:92-98), "
                      f"vx_verify_batch (gather kernel + hash + D2H), median of 3 calls, {el * 1e3:.1f} ms"}


def e2e_async(plen: int, n: int = 8192, cpu_thread_GiBps: float | None = None):
    """The download path end to end: tools/native/async_probe (C++, built by
    build()) submits n pieces from n separately registered mmaps in shuffled
    order with vx_submit, flushes every 64 submits and polls like the event
    loop (peer_connection.rs:1145-1158, event_loop.rs:554-557); every
    completion must match.  Run as a child process (no exec)."""
    import subprocess

    exe = os.path.join(ROOT, "tools", "native", "async_probe")
    if not os.path.exists(exe):
        return {"error": "tools/native/async_probe not built"}
    total_gib = n * plen / GiB
    p = subprocess.run([exe, str(plen), str(n), f"{total_gib:.6f}", "64", "2"], capture_output=True, text=True,
                       timeout=240)
    if p.returncode != 0:
        return {"error": f"async_probe rc={p.returncode}: {p.stderr[-300:]}"}
    d = json.loads(p.stdout.strip().splitlines()[-1])
    # the same buffers streamed 4 times over (8 GiB): a download never stops after
    # 2 GiB, and the first gather and last chain weigh 4x less
    p4 = subprocess.run([exe, str(plen), str(n), f"{4 * total_gib:.6f}", "64", "2"], capture_output=True, text=True,
                        timeout=240)
    d4 = json.loads(p4.stdout.strip().splitlines()[-1]) if p4.returncode == 0 else {"error": p4.stderr[-300:]}
    # the same burst with refuse_when_full = 1: a submit that finds every slot in flight is refused at
    # once and the piece goes to a CPU pool (vortex's own, as INTEGRATION.md's call site does; here the
    # oracle's SHA-NI on cpu_share() - 1 threads, the loop thread being the last): no loop stall, and
    # the burst is hashed by both sides
    ot = max(1, cpu_share() - 1)
    po = subprocess.run([exe, str(plen), str(n), f"{total_gib:.6f}", "64", "2", "0", "4", str(ot)],
                        capture_output=True, text=True, timeout=240)
    if po.returncode == 0:
        do = json.loads(po.stdout.strip().splitlines()[-1])
        overflow = {"GiBps": do["GiBps"], "pool_threads": ot, "backlog_cap": do.get("backlog_cap"),
                    "refusals": do["refused"], "cpu_pieces": do["cpu_pieces"], "gpu_pieces": do["polled"],
                    "mismatched": do["mismatched"], "submit_stall_ms": do["engine"]["submit_stall_ms"],
                    "blocking_GiBps": d["GiBps"],
                    "note": "vx_config.refuse_when_full = 1: a refused piece goes to the CPU pool (the CPU pool "
                            "restatement's SHA-1, vortex's pool stand-in, kind port) while the pool's backlog is "
                            "under one GPU batch latency of work (vx_plan_verify piece_latency_s / "
                            "cpu_piece_latency_s x threads), else the loop polls and offers it again; every "
                            "verdict checked (DESIGN.md §6.5)"}
    else:
        overflow = {"error": f"async_probe overflow rc={po.returncode}: {po.stderr[-300:]}"}
    return {"value": d["GiBps"], "unit": "GiB/s", "mismatched": d["mismatched"], "polled": d["polled"],
            "engine": d.get("engine"), "overflow": overflow,
            "stream_4x": {"GiBps": d4.get("GiBps"), "GiB": round(4 * total_gib, 3), "mismatched": d4.get("mismatched"),
                          "polled": d4.get("polled"), "error": d4.get("error")},
            "paced": paced_leg(plen, cpu_thread_GiBps=cpu_thread_GiBps),
            "sample": f"{d['pieces']} x {plen // 1024} KiB from {n} separately registered mmaps, shuffled, "
                      f"vx_submit + vx_flush every 64 + vx_poll (tools/native/async_probe)"}


def paced_leg(plen: int, rates=(1, 4, 16, 40), seconds: float = 1.0, cpu_thread_GiBps: float | None = None):
    """The download path at network-realistic arrival rates
    (tools/native/paced_probe): pieces arrive at R GB/s into a pool of 8,192
    registered buffers; every 1 ms loop turn submits what arrived, flushes
    once and polls (peer_connection.rs:1145-1158, event_loop.rs:554-557).
    Per rate: the loop thread's time inside the engine per second of wall
    time, vx_stats' submit stall per second, and submit-to-poll latency
    percentiles; every verdict checked.  vortex's loop waits at most 150 ms
    per turn (event_loop.rs:438-439).  Beside it, one pool thread's time for
    one piece (rayon runs a piece per task): plen / the per-thread rate of
    the CPU baseline measured in this run (or 2.2e9 B/s, SHA-NI, if absent)."""
    import subprocess

    exe = os.path.join(ROOT, "tools", "native", "paced_probe")
    if not os.path.exists(exe):
        return {"error": "tools/native/paced_probe not built"}
    out = {}
    for r in rates:
        p = subprocess.run([exe, str(plen), str(r), str(seconds), "1000", "8192"], capture_output=True, text=True,
                           timeout=120)
        if p.returncode != 0:
            out[f"{r}GBps"] = {"error": f"paced_probe rc={p.returncode}: {p.stderr[-300:]}"}
            continue
        d = json.loads(p.stdout.strip().splitlines()[-1])
        out[f"{r}GBps"] = {k: d[k] for k in ("achieved_GBps", "pieces", "loop_ms_per_s", "submit_ms_per_s",
                                              "flush_ms_per_s", "poll_ms_per_s", "max_call_ms",
                                              "submit_stall_ms_per_s", "batches", "latency_ms", "pool_waits",
                                              "mismatched_verdicts")}
    rate = cpu_thread_GiBps * GiB if cpu_thread_GiBps else 2.2e9
    out["cpu_pool_piece_ms"] = {"value": round(plen / rate * 1e3, 4),
                                "source": "cpu_baseline per-thread rate" if cpu_thread_GiBps else "2.2e9 B/s (SHA-NI)"}
    out["note"] = ("1 ms loop turns, one vx_flush per turn, 8,192 registered 256 KiB buffers; loop_ms_per_s is the "
                   "event-loop thread's time inside vx_submit/vx_flush/vx_poll per second")
    return out


def ragged_leg(dev, stream, steps: int = 5):
    """BASELINE config 3, device-resident: 262,144 x 16 KiB + 16,384 x 256 KiB
    + 4,096 x 1 MiB + 1,024 x 4 MiB (4 GiB per class, 16 GiB), shuffled
    (seed 0x5EED0003), lanes in longest-first order, verified against the
    expected table by the kernel the planner picks (vx_sha1_device_ragged_hint).
    The batch is bound by its longest piece's chain (65,537 dependent
    compressions of a 4 MiB piece), reported against the rounds-only floor."""
    import numpy as np
    import torch

    import oracle
    from vortex_amd import device as vdev
    from vortex_amd._lib import tuning

    classes = [(16384, 262144), (262144, 16384), (1 << 20, 4096), (4 << 20, 1024)]
    seed_base = 0x5EED0003
    total = sum(L * k for L, k in classes)
    data = torch.empty(total, dtype=torch.uint8, device=dev)
    offs, lens, o = [], [], 0
    for c, (L, k) in enumerate(classes):
        vdev.synth_fill(data[o:o + L * k], k, L, seed=seed_base + c, stream=stream)
        offs.append(np.arange(k, dtype=np.int64) * L + o)
        lens.append(np.full(k, L, dtype=np.int32))
        o += L * k
    offs, lens = np.concatenate(offs), np.concatenate(lens)
    perm = np.random.default_rng(seed_base).permutation(len(offs))
    offs, lens = offs[perm], lens[perm]
    n = len(lens)
    d_off = torch.from_numpy(offs).to(dev)
    d_len = torch.from_numpy(lens).to(dev)
    order = vdev.length_order(lens).to(dev)
    plan = vdev.ragged_plan(lens)
    variant = int(tuning().vx_tuning_plan_ragged(n, plan[0], plan[1]))
    with torch.cuda.stream(stream):
        dig, _ = vdev.sha1_ragged(data, d_off, d_len, order=order, plan=plan, stream=stream)  # validates the layout
    torch.cuda.synchronize()
    inv = np.empty(n, dtype=np.int64)
    inv[perm] = np.arange(n)
    raw = dig.cpu().numpy().tobytes()
    starts = np.cumsum([0] + [k for _, k in classes])
    for c, (L, k) in enumerate(classes):  # spot-check every class against the CPU oracle
        for j in sorted({0, 1, k // 2, k - 1}):
            p = int(inv[starts[c] + j])
            assert raw[20 * p:20 * p + 20] == oracle.sha1(oracle.gen_piece(seed_base + c, j, L)), (L, j)
    expected = dig.reshape(-1).clone()
    matched = torch.empty(n, dtype=torch.uint8, device=dev)
    times = []
    for k in range(steps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        vdev.sha1_ragged(data, d_off, d_len, order=order, expected=expected, digests=dig, matched=matched,
                         stream=stream, plan=plan, validate=False)
        e1.record(stream)
        torch.cuda.synchronize()
        if k:
            times.append(e0.elapsed_time(e1))
    assert int(matched.sum()) == n
    ms = sorted(times)[len(times) // 2]
    blocks = (max(int(x) for x in lens) + 9 + 63) // 64
    per_block_us = ms * 1e3 / blocks
    floor_valu_us = 405 * 4 / 2.4e9 * 1e6     # rounds only: 405 VALU at one wave's 4-cycle issue, 2.4 GHz
    floor_inst_us = 425 * 4 / 2.4e9 * 1e6     # + the consumer's 20 ds_read_b128 issue slots
    # the generated consumer alone (no producer, no barriers) with its 20-read burst per block:
    # 1,775 cycles (round-2 pair probe, no_barriers_idle_producer: profiles/r02/consumer_asm/, EXPERIMENTS.md §3.2)
    floor_reads_us = 1775.4 / 2.4e9 * 1e6
    del data, d_off, d_len, order, dig, expected, matched
    torch.cuda.empty_cache()
    return {"value": round(total / (ms * 1e-3) / GiB, 2), "unit": "GiB/s", "kernel_ms_median": round(ms, 3),
            "kernel_ms_runs": [round(t, 3) for t in times], "pieces": n, "bytes": total,
            "kernel": {1: "lane", 2: "split", 5: "split, one pair per CU"}.get(variant, str(variant)),
            "hbm_frac": round(total / (ms * 1e-3) / HBM_PEAK, 4),
            "chain": {"longest_piece_blocks": blocks, "us_per_block": round(per_block_us, 4),
                      "floor_405_valu_us": round(floor_valu_us, 4), "floor_425_inst_us": round(floor_inst_us, 4),
                      "frac_of_valu_floor": round(floor_valu_us / per_block_us, 4),
                      "frac_of_inst_floor": round(floor_inst_us / per_block_us, 4),
                      "floor_consumer_with_reads_us": round(floor_reads_us, 4),
                      "frac_of_consumer_with_reads": round(floor_reads_us / per_block_us, 4),
                      "note": "one 4 MiB piece is a chain of 65,537 dependent compressions in one lane; "
                              "floors at nominal 2.4 GHz: 405 VALU / 425 instructions at one wave's 4-cycle "
                              "issue, and the measured consumer stream with its LDS reads (the pair's real "
                              "floor: barriers and the producer add < 1 %, DESIGN.md §3.2.1)"},
            "sample": "config 3: 262,144 x 16 KiB + 16,384 x 256 KiB + 4,096 x 1 MiB + 1,024 x 4 MiB, shuffled, "
                      "device-resident, verify vs expected table, median of %d launches" % steps}


def fs_type(path: str) -> str:
    """Filesystem type of the mount holding `path` (longest /proc/mounts prefix)."""
    best, kind = "", "?"
    try:
        with open("/proc/mounts") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 3 and (path == parts[1] or path.startswith(parts[1].rstrip("/") + "/")) \
                        and len(parts[1]) > len(best):
                    best, kind = parts[1], parts[2]
    except OSError:
        pass
    return kind


def resident_fraction(path: str) -> float | None:
    """Fraction of the file's pages in the page cache (mmap + mincore; maps
    without touching the pages)."""
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    libc.mincore.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    size = os.path.getsize(path)
    if size == 0:
        return None
    fd = os.open(path, os.O_RDONLY)
    try:
        addr = libc.mmap(None, size, mmap.PROT_READ, mmap.MAP_SHARED, fd, 0)
        if addr in (None, ctypes.c_void_p(-1).value):
            return None
        try:
            pages = (size + mmap.PAGESIZE - 1) // mmap.PAGESIZE
            vec = (ctypes.c_ubyte * pages)()
            if libc.mincore(addr, size, vec) != 0:
                return None
            return sum(b & 1 for b in bytes(vec)) / pages
        finally:
            libc.munmap(addr, size)
    finally:
        os.close(fd)


def drop_cache(path: str) -> float | None:
    """Write back and evict the file's pages (fsync + POSIX_FADV_DONTNEED; no
    privilege needed), return the resident fraction left."""
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    finally:
        os.close(fd)
    return resident_fraction(path)


def disk_direct_rate(path: str, total: int, threads: int, bs: int = 1 << 20) -> float | None:
    """The disk's own O_DIRECT read rate over the (evicted) file: `threads`
    threads, one bs-byte read in flight each, no copy and no hash (the cold
    leg's reference for what the disk gives; tools/disk_qd_probe.py).  None
    where the filesystem refuses O_DIRECT."""
    import mmap
    from concurrent.futures import ThreadPoolExecutor

    try:
        fd = os.open(path, os.O_RDONLY | os.O_DIRECT)
    except OSError:
        return None
    n = (total + bs - 1) // bs

    def work(t: int) -> int:
        buf = mmap.mmap(-1, bs)  # page-aligned, as O_DIRECT needs
        return sum(os.preadv(fd, [buf], i * bs) for i in range(t, n, threads))

    try:
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            got = sum(ex.map(work, range(threads)))
        el = time.perf_counter() - t0
    except OSError:
        return None
    finally:
        os.close(fd)
    return got / el / GiB if got == total else None


def reverify_dir() -> str:
    """Where the config-5 file goes: the first candidate on a disk-backed
    filesystem (a 'cold' read from tmpfs would still be a memory copy)."""
    cands = [os.environ.get("TMPDIR", ""), "/var/tmp", "/tmp", os.path.join(ROOT, "gpurun_out"), ROOT]
    for d in cands:
        if d and os.path.isdir(d) and os.access(d, os.W_OK) and fs_type(d) not in ("tmpfs", "ramfs"):
            return d
    return next(d for d in cands if d and os.path.isdir(d) and os.access(d, os.W_OK))


def copy_gaps(rounds: list, min_ms: float = 0.02) -> dict:
    """Where the copy engine sat idle inside one re-verify call, from its round
    timeline (HashPool.last_verify_rounds, vx_last_verify_rounds).  For every
    gap between round k-1's copy end and round k's copy start: "read" when
    round k's reads finished after round k-1's copy had ended (the readers
    were late), "hand-off" when they had finished but round k was enqueued
    after it (the loop thread was waiting elsewhere: an earlier round's
    reads, a free slot), else "device" (enqueued in time, started late:
    stream order).  ramp: round k is a shortened head/tail round."""
    from vortex_amd._lib import VX_ROUND_HEAD_RAMP, VX_ROUND_TAIL_RAMP

    gaps = []
    for k in range(1, len(rounds)):
        a, b = rounds[k - 1], rounds[k]
        if not a["copy_end_ms"] or not b["copy_start_ms"]:
            continue
        g = b["copy_start_ms"] - a["copy_end_ms"]
        if g <= min_ms:
            continue
        cause = "read" if b["read_done_ms"] > a["copy_end_ms"] else (
            "hand-off" if b["enqueue_ms"] > a["copy_end_ms"] else "device")
        gaps.append({"round": k, "gap_ms": round(g, 3), "cause": cause,
                     "ramp": bool(b["flags"] & (VX_ROUND_HEAD_RAMP | VX_ROUND_TAIL_RAMP)),
                     "read_late_ms": round(b["read_done_ms"] - a["copy_end_ms"], 3),
                     "enqueue_late_ms": round(b["enqueue_ms"] - a["copy_end_ms"], 3)})
    by = {}
    for g in gaps:
        by[g["cause"]] = round(by.get(g["cause"], 0.0) + g["gap_ms"], 3)
    first = rounds[0]["copy_start_ms"] if rounds and rounds[0]["copy_start_ms"] else None
    return {"gap_ms": round(sum(g["gap_ms"] for g in gaps), 3), "by_cause": by,
            "ramp_gap_ms": round(sum(g["gap_ms"] for g in gaps if g["ramp"]), 3),
            "worst": sorted(gaps, key=lambda g: -g["gap_ms"])[:3], "rounds": len(rounds),
            "first_copy_start_ms": None if first is None else round(first, 3)}


def split_call(pool, paths: list, lens: list, n: int, pl: int, exp: bytes, first: int, io_threads: int,
               cpu_threads: int) -> dict:
    """One bulk re-verify split between the GPU and vortex's pool, both at
    once (INTEGRATION.md "Split"): the engine verifies pieces [first, n)
    with vx_verify_files_range while the CPU restatement of vortex's own
    re-verify (oracle/pool_oracle.cpp, the par_iter of torrent.rs:724-740;
    the pool's stand-in, kind "port", as in `cpu_pool`) verifies [0, first)
    on cpu_threads threads.  ctypes drops the GIL in both calls, so they run
    concurrently.  Returns wall time, each side's time, whether every
    verdict matched, and the merged verdicts (pool's head + engine's tail:
    the one Box<[bool]> of torrent.rs:727-740)."""
    import threading

    import oracle

    res, errs = {}, []

    def gpu():
        try:
            t0 = time.perf_counter()
            got, bad = pool.verify_files(paths, lens, pl, exp, io_threads=io_threads, first=first, count=n - first)
            res["gpu"] = (all(got) and bad == 0, time.perf_counter() - t0, got)
        except Exception as e:  # noqa: BLE001  (raised below, on the calling thread)
            errs.append(e)

    def cpu():
        try:
            t0 = time.perf_counter()
            ok = oracle.pool_verify_files(paths, lens, pl, exp[:20 * first], threads=cpu_threads)
            res["cpu"] = (all(ok) and len(ok) == first, time.perf_counter() - t0, ok)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = ([threading.Thread(target=gpu)] if first < n else []) + ([threading.Thread(target=cpu)] if first else [])
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    if errs:
        raise errs[0]
    ok = all(v[0] for v in res.values())
    merged = list(res.get("cpu", (0, 0, []))[2]) + list(res.get("gpu", (0, 0, []))[2])
    return {"s": wall, "gpu_s": res.get("gpu", (True, 0.0))[1], "cpu_s": res.get("cpu", (True, 0.0))[1], "ok": ok,
            "matched": merged}


def balanced_call(pool, paths: list, lens: list, n: int, pl: int, exp: bytes, io_threads: int, cpu_threads: int,
                  cpu_thread_rate: float) -> dict:
    """One bulk re-verify shared by the engine and vortex's pool with no plan
    (vx_verify_files_split, INTEGRATION.md "The split"): the pool stand-in
    (oracle/pool_oracle.cpp's claim pool, kind "port": vortex's rayon threads
    calling vx_split_claim) takes pieces from the head while the engine takes
    groups from the top, sized from both sides' rates as measured in the call.
    Returns wall time, each side's time, the boundary, and the verdicts."""
    import threading

    import oracle
    from vortex_amd.hash_pool import Split

    sp = Split(0, n, cpu_threads, cpu_thread_rate)
    res, errs = {}, []

    def gpu():
        try:
            t0 = time.perf_counter()
            res["gpu_bad"] = pool.verify_files_split(paths, lens, pl, exp, sp, io_threads=io_threads)
            res["gpu_s"] = time.perf_counter() - t0
            # the engine's own end (its last kernel), not the call's return: the
            # call may wait for the pool's last verdicts (vx_hash.h)
            ends = [r["kernel_end_ms"] for r in pool.last_verify_rounds() if r["kernel_end_ms"] > 0]
            if ends:
                res["gpu_s"] = min(res["gpu_s"], max(ends) * 1e-3)
        except Exception as e:  # noqa: BLE001  (raised below, on the calling thread)
            errs.append(e)

    def cpu():
        try:
            t0 = time.perf_counter()
            res["taken"] = oracle.pool_verify_files_claim(paths, lens, pl, exp, cpu_threads, sp.claim_fn, sp.done_fn,
                                                          sp.arg, 0, sp.matched)
            res["cpu_s"] = time.perf_counter() - t0
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=gpu), threading.Thread(target=cpu)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    if errs:
        raise errs[0]
    got = sp.verdicts()
    return {"s": wall, "gpu_s": res["gpu_s"], "cpu_s": res["cpu_s"], "ok": all(got) and res["gpu_bad"] == 0,
            "boundary": sp.boundary, "pool_pieces": res["taken"], "matched": got}


def reverify_leg(reps: int = 5, cold_reps: int = 3, split_reps: int = 11):
    """BASELINE config 5: full re-verify of a torrent's data from disk with
    the linux-mint geometry (cli/linux-mint.torrent: 2,907,832,320 B, 2 MiB
    pieces, last 1,179,648 B) through vx_verify_files (pread into pinned
    stages -> H2D -> kernel -> verdicts back), next to the CPU restatement of
    vortex's own re-verify (par_iter over check_piece_hash_sync,
    oracle/pool_oracle.cpp) on the same file and host cores.  The ISO is
    not available offline: a synthetic file of identical geometry is written
    first, then fsync'd so no writeback overlaps the timed calls.

    Two legs, each GPU and CPU pool alternating per rep:
      warm  the file's pages in the page cache (vortex re-verifying data it
            just wrote or read);
      cold  every call preceded by fsync + POSIX_FADV_DONTNEED, so the reads
            go to the disk (vortex starting up on a torrent whose data is not
            cached); the resident fraction before each call is recorded, and
            the disk alone (disk_direct_rate: O_DIRECT reads of the evicted
            file by as many threads, no copy, no hash) alternates with both.
    Each GPU call's time budget (vx_tuning_last_verify: reader busy time and
    rate, GPU-timed copy busy fraction) goes into the record."""
    import oracle
    from vortex_amd.hash_pool import HashPool, plan_verify_split

    pl = 2097152
    threads = cpu_share()
    d = reverify_dir()
    path = os.path.join(d, f"vx_bench_linuxmint_{os.getpid()}.iso")
    t0 = time.perf_counter()

    def trace_of(pool):
        tr = pool.last_verify()
        keep = ("wall_ms", "read_busy_ms", "read_span_ms", "first_read_ms", "copy_busy_ms", "copy_span_ms", "tail_ms",
                "read_GiBps", "read_GiBps_per_thread", "copy_GiBps", "copy_busy_frac", "rounds", "readers",
                "direct_bytes", "chunk_bytes")
        out = {k: (round(tr[k], 3) if isinstance(tr[k], float) else tr[k]) for k in keep}
        rounds = pool.last_verify_rounds()
        out["copy_gaps"] = copy_gaps(rounds)
        out["timeline"] = [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()} for r in rounds]
        return out

    try:
        total, n, last = write_linuxmint_file(path)
        t_write = time.perf_counter() - t0
        exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
        legs = {}
        with HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=4096) as pool:
            got, bad = pool.verify_files([path], [total], pl, exp, io_threads=threads)  # warm (stages, rows, cache)
            assert all(got) and bad == 0
            pool.reset_stats()
            for leg in ("warm", "cold"):
                gpu_t, cpu_t, traces, resident, disk = [], [], [], [], []
                for _ in range(reps if leg == "warm" else cold_reps):
                    if leg == "cold":
                        resident.append(drop_cache(path))
                    else:
                        resident.append(resident_fraction(path))
                    t0 = time.perf_counter()
                    got, bad = pool.verify_files([path], [total], pl, exp, io_threads=threads)
                    gpu_t.append(time.perf_counter() - t0)
                    assert all(got) and bad == 0
                    traces.append(trace_of(pool))
                    if leg == "cold":
                        resident.append(drop_cache(path))
                    t0 = time.perf_counter()
                    cpu = oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
                    cpu_t.append(time.perf_counter() - t0)
                    assert all(cpu)
                    if leg == "cold":  # the disk alone, same file, same readers, evicted again
                        drop_cache(path)
                        disk.append(disk_direct_rate(path, total, threads))
                legs[leg] = (gpu_t, cpu_t, traces, resident, disk)
            st = pool.stats()
            # the split (vx_plan_verify_split with the pool's per-thread rate just measured), warm
            for _ in range(2):
                resident_fraction(path)  # cached again after the cold leg: read it once through
                oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
            # The pool beside the engine gets 3/4 of the threads, the engine 8 readers (half):
            # a full-size pool beside them oversubscribed the host and ran bimodal, 38-71 ms a
            # call; 12 + 8 ran 48 +- 0.5 ms (profiles/r05/split/sweep.json)
            cw = sorted(legs["warm"][1])[len(legs["warm"][1]) // 2]
            rate = total / cw / threads
            pool_t, io_t = max(1, threads * 3 // 4), max(2, threads // 2)
            plan = plan_verify_split(n, pl, total, cpu_threads=pool_t, cpu_thread_rate=rate)
            split = {"plan": {k: (round(v, 5) if isinstance(v, float) else v) for k, v in plan.items()},
                     "configs": []}
            # the planner's split point and one either side (10 % more / fewer GPU pieces)
            k0 = plan["gpu_count"]
            points = sorted({n - k0, n - int(k0 * 0.9), max(0, n - int(k0 * 1.1))}) if k0 else [n]
            # The points alternate call by call with the GPU alone (all readers) and the pool
            # alone (all threads) as references, so a box's drift lands on all of them alike.
            cfgs = [(first, io_t, pool_t) for first in points] + [(0, threads, threads), (n, threads, threads)]
            by_cfg = {c: [] for c in cfgs}
            # The balanced split's first group starts from what the last split calls on
            # the context measured: three untimed calls first, as a
            # long-lived context has them (keep one context)
            for _ in range(3):
                assert balanced_call(pool, [path], [total], n, pl, exp, io_t, pool_t, rate)["ok"]
            bal = []  # the self-balancing split (no plan), in the same alternation
            for _ in range(split_reps):
                for c in cfgs:
                    by_cfg[c].append(split_call(pool, [path], [total], n, pl, exp, c[0], c[1], c[2]))
                bal.append(balanced_call(pool, [path], [total], n, pl, exp, io_t, pool_t, rate))
            assert all(b["ok"] for b in bal), "balanced split: a verdict differs from the expected table"
            bm = sorted(bal, key=lambda b: b["s"])[len(bal) // 2]
            # each side's own rate in the median call: the engine's pieces
            # [boundary, n) over its time, the pool's [0, boundary) over its
            eng_bytes = total - bm["boundary"] * pl
            split["balanced"] = {"io_threads": io_t, "cpu_threads": pool_t, "value": round(total / bm["s"] / GiB, 2),
                                 "s_runs": [round(b["s"], 4) for b in bal],
                                 "gpu_first_runs": [b["boundary"] for b in bal],
                                 "gpu_s": round(bm["gpu_s"], 4), "cpu_s": round(bm["cpu_s"], 4),
                                 "gpu_first": bm["boundary"],
                                 "engine_GiBps": round(eng_bytes / bm["gpu_s"] / GiB, 2) if bm["gpu_s"] else None,
                                 "pool_GiBps": round((total - eng_bytes) / bm["cpu_s"] / GiB, 2) if bm["cpu_s"] else None}
            for (first, io_c, pool_c), calls in by_cfg.items():
                assert all(c["ok"] for c in calls), "split re-verify: a verdict differs from the expected table"
                med = sorted(calls, key=lambda c: c["s"])[len(calls) // 2]
                entry = {"io_threads": io_c, "cpu_threads": pool_c, "gpu_first": first,
                         "planned": first == n - k0 and io_c == io_t, "value": round(total / med["s"] / GiB, 2),
                         "s_runs": [round(c["s"], 4) for c in calls],
                         "gpu_s": round(med["gpu_s"], 4), "cpu_s": round(med["cpu_s"], 4)}
                if first in (0, n) and io_c == threads:
                    split["gpu_alone" if first == 0 else "pool_alone"] = entry
                else:
                    split["configs"].append(entry)
    finally:
        if os.path.exists(path):
            os.unlink(path)

    def record(leg):
        gpu_t, cpu_t, traces, resident, disk = legs[leg]
        g, c = sorted(gpu_t)[len(gpu_t) // 2], sorted(cpu_t)[len(cpu_t) // 2]
        dk = sorted(x for x in disk if x)
        dmed = dk[len(dk) // 2] if dk else None
        # the median call's copy-engine gaps by cause (its full timeline stays in gpu_traces)
        med_trace = traces[sorted(range(len(gpu_t)), key=lambda i: gpu_t[i])[len(gpu_t) // 2]]
        # what bound this box's calls: the H2D copies busy nearly all
        # the time = PCIe; otherwise the cause that left the copy engine idle longest in
        # the median call's round timeline (the reads, the hand-off, or the device)
        cb = sorted(t["copy_busy_frac"] for t in traces if t.get("copy_busy_frac") is not None)
        cbm = cb[len(cb) // 2] if cb else None
        causes = (med_trace.get("copy_gaps") or {}).get("by_cause") or {}
        top = max(causes, key=causes.get) if causes else "read"
        what = {"read": f"host reads (waiting on {'the disk' if leg == 'cold' else 'page-cache reads'})",
                "hand-off": "the hand-off (reads done, round enqueued late)",
                "device": "the device (copies enqueued in time, started late)"}[top]
        bound = None if cbm is None else (
            "pcie (H2D copies busy >= 0.95 of the call)" if cbm >= 0.95 else
            f"{what}; H2D copies busy {cbm:.2f}, median call's idle copy engine {causes.get(top, 0):.1f} ms by this "
            f"cause")
        for t in traces:  # one full timeline (the median call's) is enough for the record
            if t is not med_trace:
                t.pop("timeline", None)
        if leg == "cold" and dmed:
            bound = (bound or "") + f"; the disk alone (O_DIRECT, {threads} threads, 1 MiB) {dmed:.1f} GiB/s"
        out = {"value": round(total / g / GiB, 2), "unit": "GiB/s", "bound": bound,
                "copy_gaps": med_trace.get("copy_gaps"),
                "gpu_s_runs": [round(t, 4) for t in gpu_t],
                "cpu_pool": {"value": round(total / c / GiB, 2), "unit": "GiB/s", "cores": threads, "kind": "port",
                             "s_runs": [round(t, 4) for t in cpu_t]},
                "gpu_over_cpu": round(c / g, 3),
                "resident_before_calls": [None if r is None else round(r, 4) for r in resident],
                "gpu_traces": traces}
        if leg == "cold":
            out["disk_direct"] = {"value": None if dmed is None else round(dmed, 2), "unit": "GiB/s",
                                  "runs": [None if x is None else round(x, 2) for x in disk],
                                  "gpu_frac_of_disk": None if not dmed else round(total / g / GiB / dmed, 3)}
        return out

    warm, cold = record("warm"), record("cold")
    best = max(split["configs"], key=lambda c: c["value"])
    planned = [c for c in split["configs"] if c["planned"]]
    # `value` is the self-balancing split's (vx_verify_files_split: no plan, the
    # boundary found at run time); the planner's point and the best of the three
    # fixed points stay beside it, so the record shows how far either is off
    pv = max(c["value"] for c in planned) if planned else best["value"]
    bv = split["balanced"]["value"]
    either = max(split["gpu_alone"]["value"], split["pool_alone"]["value"], warm["value"], warm["cpu_pool"]["value"])
    split.update({"value": bv, "unit": "GiB/s", "kind": "balanced (vx_verify_files_split)",
                  "balanced_vs_best_fixed": round(bv / best["value"], 4),
                  "planned_value": pv, "planned_vs_best_fixed": round(pv / best["value"], 4),
                  "best_value": best["value"], "best_gpu_first": best["gpu_first"],
                  "best_io_threads": best["io_threads"], "balanced_gpu_first": split["balanced"]["gpu_first"],
                  "balanced_engine_GiBps": split["balanced"]["engine_GiBps"],
                  "balanced_pool_GiBps": split["balanced"]["pool_GiBps"],
                  "gpu_only": split["gpu_alone"]["value"], "pool_only": split["pool_alone"]["value"],
                  # against the better of each side's two figures: in the alternation and in the legs above
                  "beats_both": bv > either, "planned_beats_both": pv > either,
                  "best_beats_both": best["value"] > either,
                  "pool_kind": "port",
                  "sample": f"the warm file shared by the engine and the CPU pool restatement (vortex's par_iter "
                            f"stand-in, 3/4 of the {threads} threads) at once: balanced = vx_verify_files_split "
                            f"(the pool claims from the head, the engine sizes its groups from the rates it "
                            f"measures; after 3 untimed calls); fixed points = vx_verify_files_range over "
                            f"[first, {n}) with the pool on [0, first), first = vx_plan_verify_split's {split['plan']['gpu_first']} and 10 % "
                            f"fewer / more GPU pieces; engine readers at half the threads; alternating call by "
                            f"call with the GPU alone and the pool alone (gpu_only / pool_only); median of "
                            f"{split_reps} per config; every verdict checked"})
    warm["split"] = split
    where = {"dir": d, "fs": fs_type(d)}
    warm.update({"write_s": round(t_write, 2), "file": where,
                 "engine": {k: st[k] for k in ("pieces_completed", "bytes_completed", "batches", "chunk_rounds",
                                               "io_errors")},
                 "sample": f"re-verify {n} x 2 MiB pieces ({total} B, linux-mint geometry, synthetic data) from one "
                           f"fsync'd, page-cache-warm file: vx_verify_files e2e vs the CPU pool restatement, "
                           f"alternating, median of {reps}"})
    cold.update({"file": where,
                 "sample": f"the same file with fsync + POSIX_FADV_DONTNEED before every call (reads from "
                           f"{where['fs']}), GPU and CPU pool alternating, median of {cold_reps}"})
    return warm, cold


def write_linuxmint_file(path: str, scale: float = 1.0):
    """The config-5 torrent's data (linux-mint geometry: 2 MiB pieces, last
    piece 1,179,648 B; `scale` < 1 keeps the piece length and shrinks the
    piece count, for rehearsals), synthetic, fsync'd.  Returns (total, n, last)."""
    import oracle  # the checker: generates the bytes and, below, the expected table

    pl, total = 2097152, 2907832320
    if scale < 1.0:
        total = max(2, int((total // pl) * scale)) * pl + 1179648
    n = (total + pl - 1) // pl
    last = total - (n - 1) * pl
    buf = ctypes.create_string_buffer(pl)
    with open(path, "wb") as f:
        for i in range(n):
            L = last if i == n - 1 else pl
            oracle.lib().vxo_gen_piece(0x5EED0005, i, L, 0, buf)
            f.write(memoryview(buf)[:L])
        f.flush()
        os.fsync(f.fileno())  # writeback done before anything is timed
    return total, n, last


def reverify_multi_leg(rank: int, world: int, local: int, dev, backend: str, same_device: bool, scale: float = 1.0,
                       reps: int = 3, cold_reps: int = 2) -> dict | None:
    """BASELINE config 5 across the N GPUs of the node: rank 0
    writes the linux-mint-geometry file; every rank re-verifies its contiguous
    piece range (shard.shard_range, vx_verify_files_range) on its own GPU,
    reading its bytes over its own PCIe link, warm (page cache) and cold
    (rank 0 evicts the file before each call: fsync + POSIX_FADV_DONTNEED).
    A call's time is the slowest rank's; every verdict is gathered and checked
    on rank 0.  Beside it, rank 0 times the CPU restatement of vortex's
    re-verify (oracle/pool_oracle.cpp, the par_iter of torrent.rs:724-740)
    with every CPU of the node, while the GPU ranks wait.  Returns the record
    on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    import oracle
    from vortex_amd import shard
    from vortex_amd.hash_pool import HashPool, plan_verify

    ncpu = node_cpus()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    io_threads = max(2, min(16, ncpu // max(1, local_world)))

    # Every step that can fail on one rank only is caught there and agreed on
    # by all ranks before the next collective, so the ranks fail together and
    # none waits in a collective the others never reach.
    def agree(ok: bool) -> bool:
        flags = [None] * world
        dist.all_gather_object(flags, bool(ok))
        return all(flags)

    obj = [None]
    if rank == 0:
        try:
            d = reverify_dir()
            path = os.path.join(d, f"vx_bench_multi_linuxmint_{os.getpid()}.iso")
            t0 = time.perf_counter()
            total, n, last = write_linuxmint_file(path, scale)
            exp = oracle.pool_digest_synth(0x5EED0005, 0, n, 2097152, last_index=n - 1, last_len=last,
                                           threads=min(ncpu, 64))
            obj = [{"path": path, "dir": d, "total": total, "n": n, "exp": exp, "write_s": time.perf_counter() - t0}]
        except Exception as e:  # noqa: BLE001  (reported to every rank)
            obj = [{"error": f"rank 0 could not write the torrent file: {type(e).__name__}: {e}"}]
    dist.broadcast_object_list(obj, src=0)
    spec = obj[0]
    if "error" in spec:
        raise RuntimeError(spec["error"])
    path, total, n, exp = spec["path"], spec["total"], spec["n"], spec["exp"]
    pl = 2097152
    first, count = shard.shard_range(n, world, rank)
    vdev = torch.device("cpu") if backend == "gloo" else dev
    legs = {"warm": [], "cold": []}
    traces = {"warm": [], "cold": []}
    cpu = {"warm": [], "cold": []}
    cpu_ok = True
    pool = None
    split = balanced = None
    try:
        try:
            pool = HashPool(pl, device=local, slots=4, slot_bytes=512 << 20, batch_pieces=4096)
            got, bad = pool.verify_files([path], [total], pl, exp, io_threads=io_threads, first=first, count=count)
            ok = all(got) and bad == 0
        except Exception as e:  # noqa: BLE001
            log(f"rank {rank}: re-verify setup failed: {type(e).__name__}: {e}")
            ok = False
        if not agree(ok):
            raise RuntimeError("multi-GPU re-verify: a rank failed to open its context or its warm-up verdicts "
                               "differ from the expected table")
        for leg, k in (("warm", reps), ("cold", cold_reps)):
            for _ in range(k):
                if leg == "cold" and rank == 0:
                    try:
                        drop_cache(path)
                    except OSError:
                        pass
                dist.barrier()
                try:
                    t0 = time.perf_counter()
                    got, bad = pool.verify_files([path], [total], pl, exp, io_threads=io_threads, first=first,
                                                 count=count)
                    el = time.perf_counter() - t0
                    tr = pool.last_verify()
                    ok = True
                except Exception as e:  # noqa: BLE001
                    log(f"rank {rank}: re-verify call failed: {type(e).__name__}: {e}")
                    ok = False
                if not agree(ok):
                    raise RuntimeError("multi-GPU re-verify: a rank's vx_verify_files_range call failed")
                verdicts = shard.gather_verdicts(torch.tensor(got, dtype=torch.uint8, device=vdev), n)
                times = [None] * world
                dist.all_gather_object(times, {"s": el, "bad": bad, "read_GiBps": tr["read_GiBps"],
                                               "copy_busy_frac": tr["copy_busy_frac"],
                                               "direct_bytes": tr["direct_bytes"]})
                if int(verdicts.sum()) != n or any(t["bad"] for t in times):  # the same on every rank
                    raise RuntimeError("multi-GPU re-verify: verdicts differ from the expected table")
                if rank == 0:
                    legs[leg].append(max(t["s"] for t in times))
                    traces[leg].append([{k2: (round(v, 3) if isinstance(v, float) else v) for k2, v in t.items()}
                                        for t in times])
                    # the CPU pool on the whole node, the GPU ranks idle at the barrier below
                    try:
                        if leg == "cold":
                            drop_cache(path)
                        t0 = time.perf_counter()
                        okc = oracle.pool_verify_files([path], [total], pl, exp, threads=ncpu)
                        cpu[leg].append(time.perf_counter() - t0)
                        cpu_ok = cpu_ok and all(okc)
                    except Exception as e:  # noqa: BLE001  (recorded; the GPU figures stand)
                        log(f"CPU pool re-verify failed: {type(e).__name__}: {e}")
                        cpu_ok = False
                dist.barrier()
        split = multi_split(rank, world, pool, path, total, n, exp, io_threads, ncpu, cpu, agree, reps)
        balanced = multi_balanced(rank, world, pool, path, total, n, exp, io_threads, ncpu, cpu, agree, reps)
    finally:
        if pool is not None:
            pool.close()
        dist.barrier()
        if rank == 0 and os.path.exists(path):
            os.unlink(path)
    if rank != 0:
        return None

    def med(v):
        return sorted(v)[len(v) // 2]

    out = {}
    for leg in ("warm", "cold"):
        g = med(legs[leg])
        c = med(cpu[leg]) if cpu[leg] else None
        out[leg] = {"value": round(total / g / GiB, 2), "unit": "GiB/s", "s_runs": [round(t, 4) for t in legs[leg]],
                    "cpu_pool": None if c is None else {
                        "value": round(total / c / GiB, 2), "unit": "GiB/s", "cores": ncpu, "kind": "port",
                        "s_runs": [round(t, 4) for t in cpu[leg]]},
                    "gpu_over_cpu": None if c is None else round(c / g, 3), "rank_traces": traces[leg]}
    # What vx_plan_verify_gpus predicts for this split, with the pool's measured
    # per-thread rate: each rank's pieces are one lane each, so a 2 MiB piece's
    # chain (~25 ms) floors a call however many GPUs share the file.
    cw = med(cpu["warm"]) if cpu["warm"] else None
    p = plan_verify(n, pl, total, cpu_threads=ncpu, cpu_thread_rate=total / cw / ncpu if cw else 0.0, n_gpus=world)
    out["plan"] = {"gpu_s": round(p["gpu_s"], 5), "gpu_chain_s": round(p["gpu_chain_s"], 5),
                   "gpu_transfer_s": round(p["gpu_transfer_s"], 5), "cpu_s": round(p["cpu_s"], 5),
                   "use_gpu": p["use_gpu"], "predicted_GiBps": round(total / p["gpu_s"] / GiB, 2),
                   "model": "vx_plan_verify_gpus (DESIGN.md §6.6), n_gpus = ranks, the CPU pool's measured warm "
                            "rate per thread"}
    if split is not None:
        split["value"] = round(total / split["s"] / GiB, 2)
        split.update({"unit": "GiB/s", "gpu_only": out["warm"]["value"],
                      "pool_only": out["warm"]["cpu_pool"]["value"] if out["warm"]["cpu_pool"] else None})
        split["beats_both"] = split["value"] > max(v for v in (split["gpu_only"], split["pool_only"]) if v)
        out["split"] = split
    if balanced is not None:
        balanced["vs_planned"] = round(balanced["value"] / split["value"], 4) if split else None
        out["split_balanced"] = balanced
    out.update({"ranks": world, "same_device": same_device, "io_threads_per_rank": io_threads,
                "pieces": n, "bytes": total, "write_s": round(spec["write_s"], 2), "cpu_pool_verdicts_ok": cpu_ok,
                "file": {"dir": spec["dir"], "fs": fs_type(spec["dir"])},
                "sample": f"config 5 split over {world} ranks by piece index (vx_verify_files_range per rank, own "
                          f"GPU and PCIe link): {n} x 2 MiB pieces ({total} B, linux-mint geometry, synthetic), "
                          f"warm median of {reps}, cold (evicted) median of {cold_reps}; the slowest rank's time; "
                          f"CPU pool restatement with all {ncpu} node CPUs beside it"})
    return out


def multi_balanced(rank, world, pool, path, total, n, exp, io_threads, ncpu, cpu, agree, reps):
    """The self-balancing split over a node (vx_verify_files_split with one
    engine per rank): one vx_split and one verdict array in a
    /dev/shm mapping every rank shares, declared for `world` engines; every
    rank's engine claims groups from the top on its own GPU while rank 0's CPU
    pool restatement claims pieces from the head.  A call's time is the
    slowest side's; rank 0 checks every verdict in the shared array.  Warm
    only.  Returns the record on rank 0 (None elsewhere)."""
    import mmap
    import threading

    import torch.distributed as dist

    import oracle
    from vortex_amd import _lib
    from vortex_amd.hash_pool import Split

    pl = 2097152
    size = ctypes.sizeof(_lib.vx_split) + n
    name = [None]
    if rank == 0:
        name = [f"/dev/shm/vx_bench_split_{os.getpid()}_{time.time_ns()}"]
        try:
            with open(name[0], "wb") as f:
                f.truncate(size)
        except OSError as e:
            name = [f"error: {e}"]
    dist.broadcast_object_list(name, src=0)
    if name[0].startswith("error"):
        raise RuntimeError(f"multi-GPU balanced split: no shared mapping ({name[0]})")
    mm = None
    try:
        fd = os.open(name[0], os.O_RDWR)
        try:
            mm = mmap.mmap(fd, size)
        finally:
            os.close(fd)
    except OSError as e:
        log(f"rank {rank}: cannot map the shared split: {e}")
    if not agree(mm is not None):  # every rank maps it, or every rank stops here
        if mm is not None:
            mm.close()
        if rank == 0:
            os.unlink(name[0])
        raise RuntimeError("multi-GPU balanced split: a rank could not map the shared split")
    pool_threads = max(1, ncpu * 3 // 4)
    cw = sorted(cpu["warm"])[len(cpu["warm"]) // 2] if cpu["warm"] else None
    rate = total / cw / ncpu if cw else 0.0
    times, ok_all, bounds = [], True, []
    sp = None
    try:
        for _ in range(reps):
            if rank == 0:
                mm[ctypes.sizeof(_lib.vx_split):] = bytes(n)
                sp = Split.attach(mm, 0, n, True, pool_threads, rate, engines=world)
            dist.barrier()
            if rank != 0:
                sp = Split.attach(mm, 0, n, False)
            res, ok = {}, True

            def pool_side():
                try:
                    t0 = time.perf_counter()
                    res["taken"] = oracle.pool_verify_files_claim([path], [total], pl, exp, pool_threads, sp.claim_fn,
                                                                  sp.done_fn, sp.arg, 0, sp.matched)
                    res["cpu_s"] = time.perf_counter() - t0
                except Exception as e:  # noqa: BLE001  (a failed pool is a wrong-verdict run, below)
                    log(f"balanced split: the CPU pool failed: {type(e).__name__}: {e}")

            th = threading.Thread(target=pool_side) if rank == 0 else None
            t0 = time.perf_counter()
            if th:
                th.start()
            try:
                bad = pool.verify_files_split([path], [total], pl, exp, sp, io_threads=io_threads)
            except Exception as e:  # noqa: BLE001
                log(f"rank {rank}: balanced split call failed: {type(e).__name__}: {e}")
                ok, bad = False, 0
            gpu_s = time.perf_counter() - t0
            if th:
                th.join()
            el = time.perf_counter() - t0
            if not agree(ok and bad == 0):
                raise RuntimeError("multi-GPU balanced split: a rank's vx_verify_files_split call failed")
            dist.barrier()  # every engine has written its verdicts
            allt = [None] * world
            dist.all_gather_object(allt, {"s": el, "gpu_s": gpu_s})
            if rank == 0:
                ok_all = ok_all and bytes(sp.matched)[:n] == b"\x01" * n
                bounds.append(sp.boundary)
                times.append({"s": max(t["s"] for t in allt), "gpu_s": max(t["gpu_s"] for t in allt),
                              "cpu_s": res.get("cpu_s", 0.0)})
            sp = None
            dist.barrier()  # rank 0 re-inits the word only after every rank let go of it
    finally:
        sp = None
        mm.close()
        if rank == 0:
            os.unlink(name[0])
    if rank != 0:
        return None
    if not ok_all:
        raise RuntimeError("multi-GPU balanced split: verdicts differ from the expected table")
    med = sorted(times, key=lambda t: t["s"])[len(times) // 2]
    return {"value": round(total / med["s"] / GiB, 2), "unit": "GiB/s", "s": med["s"],
            "gpu_s": round(med["gpu_s"], 4), "cpu_s": round(med["cpu_s"], 4),
            "s_runs": [round(t["s"], 4) for t in times], "gpu_first_runs": bounds, "pool_threads": pool_threads,
            "sample": f"warm; one vx_split and verdict array shared through /dev/shm by the {world} ranks' engines "
                      f"(engines = {world}) and rank 0's CPU pool restatement; no plan; the slowest side's time, "
                      f"median of {reps}; every verdict checked"}


def multi_split(rank, world, pool, path, total, n, exp, io_threads, ncpu, cpu, agree, reps):
    """The split over a node (INTEGRATION.md "The split"): rank
    0 plans with vx_plan_verify_split (n_gpus = ranks, the pool on 3/4 of the
    node's CPUs at the warm rate it just measured); every rank verifies its
    share of the GPU tail [first, n) on its GPU while rank 0's CPU pool
    restatement verifies the head [0, first) beside it.  A call's time is the
    slowest of all; every verdict is gathered and checked.  Warm only.
    Returns the record on rank 0 (None elsewhere)."""
    import threading

    import torch
    import torch.distributed as dist

    import oracle
    from vortex_amd import shard
    from vortex_amd.hash_pool import plan_verify_split

    pl = 2097152
    obj = [None]
    if rank == 0:
        cw = sorted(cpu["warm"])[len(cpu["warm"]) // 2] if cpu["warm"] else None
        rate = total / cw / ncpu if cw else 0.0
        obj = [plan_verify_split(n, pl, total, cpu_threads=max(1, ncpu * 3 // 4), cpu_thread_rate=rate,
                                 n_gpus=world)]
    dist.broadcast_object_list(obj, src=0)
    plan = obj[0]
    first = plan["gpu_first"]
    sub_first, sub_count = shard.shard_range(n - first, world, rank)
    times, head_ok, tail_ok = [], True, True
    for _ in range(reps):
        dist.barrier()
        res = {}

        def head():
            try:
                t0 = time.perf_counter()
                res["head"] = oracle.pool_verify_files([path], [total], pl, exp[:20 * first],
                                                       threads=max(1, ncpu * 3 // 4))
                res["head_s"] = time.perf_counter() - t0
            except Exception as e:  # noqa: BLE001  (a failed head is a wrong-verdict run, below)
                log(f"split: the CPU pool's head failed: {type(e).__name__}: {e}")
                res["head"] = []

        th = threading.Thread(target=head) if rank == 0 and first else None
        ok = True
        try:
            t0 = time.perf_counter()
            if th:
                th.start()
            got, bad = (pool.verify_files([path], [total], pl, exp, io_threads=io_threads, first=first + sub_first,
                                          count=sub_count) if sub_count else ([], 0))
            gpu_s = time.perf_counter() - t0
            if th:
                th.join()
            el = time.perf_counter() - t0
        except Exception as e:  # noqa: BLE001
            log(f"rank {rank}: split call failed: {type(e).__name__}: {e}")
            ok = False
        if not agree(ok):
            raise RuntimeError("multi-GPU split re-verify: a rank's call failed")
        vdev = torch.device("cpu") if dist.get_backend() == "gloo" else torch.device("cuda", torch.cuda.current_device())
        tail = shard.gather_verdicts(torch.tensor(got, dtype=torch.uint8, device=vdev), n - first) if n - first else None
        allt = [None] * world
        dist.all_gather_object(allt, {"s": el, "gpu_s": gpu_s, "bad": bad})
        tail_ok = tail_ok and (tail is None or int(tail.sum()) == n - first) and not any(t["bad"] for t in allt)
        if rank == 0:
            head_ok = head_ok and (not first or (len(res["head"]) == first and all(res["head"])))
            times.append({"s": max(t["s"] for t in allt), "gpu_s": max(t["gpu_s"] for t in allt),
                          "cpu_s": res.get("head_s", 0.0)})
    if not tail_ok:  # the same on every rank
        raise RuntimeError("multi-GPU split re-verify: verdicts differ from the expected table")
    if rank != 0:
        return None
    if not head_ok:
        raise RuntimeError("multi-GPU split re-verify: the pool's head verdicts differ from the expected table")
    med = sorted(times, key=lambda t: t["s"])[len(times) // 2]
    return {"s": med["s"], "gpu_s": round(med["gpu_s"], 4), "cpu_s": round(med["cpu_s"], 4),
            "s_runs": [round(t["s"], 4) for t in times], "gpu_first": first, "gpu_count": n - first,
            "pool_threads": max(1, ncpu * 3 // 4),
            "plan": {k: (round(v, 5) if isinstance(v, float) else v) for k, v in plan.items()},
            "sample": "warm; GPU ranks verify [gpu_first, n) split by index while rank 0's CPU pool restatement "
                      "verifies [0, gpu_first) at once; the slowest side's time, median; every verdict checked"}


def roofline(n: int, plen: int, kern_ms: float, achieved: float, workload: str, clock: dict | None = None,
             steps: int = 1) -> dict:
    """Roofline record of the dominant kernel (sha1_uniform_kernel).

    achieved/peak/frac: algorithmic bytes per launch / HIP-event launch time
    against the 8 TB/s HBM3E peak — the fraction of the HBM roofline the
    metric asks for.  The kernel is NOT bound by HBM (traffic is 1.0007x the
    algorithmic bytes, waits < 1 %): it is bound by integer-VALU issue — 613.5
    VOP3-encoded ops per 64-byte block, one wave per SIMD, each op holding the
    SIMD ~4.1 cycles — at the 2.0-2.4 GHz the chip holds under full VALU load.
    `bound` names that; `valu` gives the fraction against the one-wave issue
    ceiling (4 cycles per op at the nominal 2.4 GHz), the measured VOP3 rate
    per SIMD, the measured whole-chip rate of SHA-1's ops at one wave per SIMD
    (tools/native/energy_probe.hip), the 2-cycle rate only VOP2 ops reach, and
    the PMC cycles per VALU and clock of the committed profile."""
    blocks = (plen + 9 + 63) // 64
    valu_per_block = 613.5  # measured: SQ_INSTS_VALU / waves / blocks (profiles/pmc_traffic.json)
    ops = n * blocks * valu_per_block / (kern_ms * 1e-3)  # lane-ops per second
    simds, f_nom = 1024, 2.4e9

    def peak(cycles_per_inst):
        return simds * 64 / cycles_per_inst * f_nom

    # Measured ceilings of this op mix (tools/native/energy_probe.hip):
    # a VOP3 op (add3/alignbit/bitop3/perm) costs its SIMD ~4.08-4.17 cycles with
    # one or two waves per SIMD (only VOP2 ops reach 2 cycles), and a stream of
    # SHA-1's round ops at one wave per SIMD on all 1,024 SIMDs sustains the
    # chip's wave-op rate at the clock it holds under VALU load (2.17-2.37 GHz).
    vop3_cyc, stream = 4.08, None
    try:
        with open(os.path.join(ROOT, "profiles", "r02", "valu", "energy_probe_run2.json")) as f:
            ep = json.load(f)
        vop3_cyc = ep["add3_2_waves_per_simd"]["cycles_per_op"] / 2
        rates = [ep[k]["chip_Gwaveops_per_s"] for k in ("sha_mix", "sha_mix_again")]
        stream = {"lo": min(rates), "hi": max(rates),
                  "clock_GHz": sorted({ep[k]["clock_GHz"] for k in ("sha_mix", "sha_mix_again")})}
    except (OSError, ValueError, KeyError):
        pass
    wave_ops = ops / 64  # wave-instructions per second, whole chip

    traffic = load_traffic(workload, n, plen)
    pmc = None
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            ent = json.load(f).get(f"{n}x{plen}")
        if ent and ent.get("sq"):
            sq = ent["sq"][-1]
            pmc = {"cycles_per_valu": sq["cycles_per_valu"], "clock_GHz": sq["clock_GHz"],
                   "valu_active_frac": sq["valu_active_frac"], "wait_frac": sq["wait_frac"],
                   "issue_frac_at_measured_clock": round(4.0 / sq["cycles_per_valu"], 4),
                   "source": ent.get("source")}
    except (OSError, ValueError):
        pass
    clock_run = None
    issue_run = None  # the one-wave issue fraction at the measured clock, when the clock is the kernels'
    busy = None
    if clock and clock.get("GHz_mean"):
        f_run = clock["GHz_mean"] * 1e9
        ceil_run = simds * 64 / 4.0 * f_run
        # The stamps bracket the whole timed loop.  At N = 1 that is the hash
        # launches back to back; at N > 1 it also holds the verdict gathers and
        # barrier waits, where the chip idles at a low clock, so the mean then
        # understates the clock the kernels ran at: no issue fraction from it.
        span = clock.get("span_ms")
        busy = min(1.0, steps * kern_ms / span) if span else None
        trusted = busy is not None and busy >= 0.9
        issue_run = round(ops / ceil_run, 4) if trusted else None
        clock_run = dict(clock, kernel_busy_frac=None if busy is None else round(busy, 4),
                         one_wave_issue_at_run_clock={
                             "peak_Tops": round(ceil_run / 1e12, 2), "frac": issue_run,
                             "note": "the one-wave VOP3 issue ceiling (4 cycles per op per SIMD) at the shader clock "
                                     "measured over this run's timed steps; frac near 1 = issue-bound at the clock the "
                                     "chip held.  null when the hash kernels fill < 0.9 of the stamped span (gathers "
                                     "and idle time inside it, N > 1): that mean is not the kernels' clock"})
    elif clock:
        clock_run = clock
    return {"bound": "valu", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK, 4), "traffic": traffic,
            "traffic_ratio": round(traffic / (n * plen), 5) if traffic else None,
            "bound_note": "integer-VALU issue (VOP3 ops, one wave per SIMD), not HBM: frac is the HBM-roofline "
                          "fraction the metric asks for; the binding roof and the kernel's fraction of it are in `valu`",
            "kernel": "sha1_uniform_kernel", "kernel_ms": round(kern_ms, 4),
            "algorithmic_bytes_per_launch": n * plen,
            # the binding-roof evidence as scalars (the driver keeps only scalar fields of roofline)
            "clock_GHz_run": clock.get("GHz_mean") if clock else None,
            "clock_GHz_run_min": clock.get("GHz_min") if clock else None,
            "clock_kernel_busy_frac": None if busy is None else round(busy, 4),
            "valu_Tops": round(ops / 1e12, 2),
            "valu_issue_frac_run_clock": issue_run,
            "valu_issue_frac_nominal": round(ops / peak(4.0), 4),
            "valu": {"achieved_Tops": round(ops / 1e12, 2), "valu_per_block": valu_per_block,
                     "one_wave_issue": {"peak_Tops": round(peak(4.0) / 1e12, 2), "frac": round(ops / peak(4.0), 4)},
                     "vop3_simd_measured": {"cycles_per_op_per_simd": round(vop3_cyc, 3),
                                            "peak_Tops": round(peak(vop3_cyc) / 1e12, 2),
                                            "frac": round(ops / peak(vop3_cyc), 4),
                                            "source": "profiles/r02/valu/energy_probe_run2.json (2 waves/SIMD)"},
                     "multi_wave_mixed_measured": {
                         "peak_Tops": round(peak(3.03) / 1e12, 2), "frac": round(ops / peak(3.03), 4),
                         "source": "profiles/r01/valu/valu.json (4 waves/SIMD)",
                         "note": "that probe's loop, as hipcc compiled it, is half VOP2 (v_xor_b32_e32, "
                                 "v_add_u32_e32), and a VOP2 op takes its SIMD 2 cycles, so the mix beats 4 cycles "
                                 "per op; this kernel's stream is VOP3: see vop3_simd_measured"},
                     "stream_ceiling": None if stream is None else {
                         "achieved_Gwaveops_per_s": round(wave_ops / 1e9, 1),
                         "ceiling_Gwaveops_per_s": [stream["lo"], stream["hi"]],
                         "clock_GHz": stream["clock_GHz"],
                         "frac_vs_fast_clock": round(wave_ops / 1e9 / stream["hi"], 4),
                         "frac_vs_slow_clock": round(wave_ops / 1e9 / stream["lo"], 4),
                         "source": "profiles/r02/valu/energy_probe_run*.json: SHA-1 round ops, 1 wave on each of "
                                   "the 1,024 SIMDs, ~1.5-2 s; the two ceilings are the two clock states the chip "
                                   "ran such streams at. A frac_vs_slow_clock near or above 1 means the kernel ran "
                                   "at (or above) the slow state's clock and is at that clock's ceiling"},
                     "simd32_vop2_only": {"peak_Tops": round(peak(2.0) / 1e12, 2), "frac": round(ops / peak(2.0), 4)},
                     "pmc": pmc,
                     "clock_run": clock_run,
                     "note": "65,536 pieces = exactly one wave per SIMD. Every SHA-1 op but the schedule's "
                             "2-input xor and the feed-forward add is VOP3-only on gfx950, and a VOP3 op holds "
                             "its SIMD ~4.1 cycles however many waves share it, so 2 waves/SIMD (131,072 x "
                             "128 KiB) run no faster (DESIGN.md §4)"}}


LINE_LIMIT = 8192  # bytes: the stdout line the driver parses (a 23 KB line was lost)
LEGS = ("ragged", "e2e", "e2e_async", "e2e_contiguous", "reverify", "reverify_cold", "reverify_multi")
_PROSE = ("sample", "note", "bound_note", "source")  # explanations: the side file keeps them


def _scalars(d: dict, depth: int, prefix: str = "", maxlen: int = 96) -> dict:
    """The scalar fields of `d` (numbers, bools, None, short strings), and of
    its nested dicts down to `depth` more levels as dotted keys; lists of up
    to 8 numbers stay.  Errors are always kept (cut to 240 characters)."""
    out = {}
    for k, v in d.items():
        key = prefix + k
        if k == "error" and v is not None:
            out[key] = str(v)[:240]
        elif k in _PROSE:
            continue
        elif v is None or isinstance(v, (bool, int, float)):
            out[key] = v
        elif isinstance(v, str):
            if len(v) <= maxlen:
                out[key] = v
        elif isinstance(v, list):
            if len(v) <= 8 and all(x is None or isinstance(x, (int, float)) for x in v):
                out[key] = v
        elif isinstance(v, dict) and depth > 0:
            out.update(_scalars(v, depth - 1, key + ".", maxlen))
    return out


def compact_line(res: dict, detail: str | None = None, limit: int = LINE_LIMIT) -> dict:
    """The one stdout line (≤ `limit` bytes of JSON): the headline fields,
    `config`, `roofline` as scalars, `cpu_baseline`, `parity`, the device's
    bus id, per-rank scalars at N > 1, and every extra leg reduced to its
    scalars.  Everything else (traces, timelines, sweeps, the nested `valu`
    block, rank identities) stays in the side file `detail` that bench.py
    writes beside it.  If the legs still overflow, they are cut down in
    steps — nested scalars first, then to value/bound/error — and never the
    headline, roofline, cpu_baseline or parity."""
    keep = {}
    for k, v in res.items():
        if k in LEGS or k in ("roofline", "ranks", "device"):
            continue
        keep[k] = v
    if "roofline" in res:
        keep["roofline"] = _scalars(res["roofline"], 0)
    if "device" in res:
        keep["device"] = {k: res["device"].get(k) for k in ("device_index", "pci_bus_id")}
    if "ranks" in res:
        rk = res["ranks"]
        keep["ranks"] = {k: rk[k] for k in ("step_ms", "kernel_ms", "verdict_gather_ms", "clock_GHz",
                                             "distinct_devices") if k in rk}
        keep["ranks"]["pci_bus_ids"] = [d.get("pci_bus_id") for d in rk.get("devices", [])]
    if detail:
        keep["detail"] = detail
    legs = [k for k in LEGS if k in res]
    for depth in (1, 0, -1):  # -1: value, bound and error only
        line = dict(keep)
        for k in legs:
            v = res[k]
            if not isinstance(v, dict):
                line[k] = v
            elif depth < 0:
                line[k] = {f: v[f] for f in ("value", "unit") if f in v}
                if v.get("error"):
                    line[k]["error"] = str(v["error"])[:240]
            else:
                line[k] = _scalars(v, depth)
        if len(json.dumps(line)) <= limit:
            return line
    for k in legs:  # a pathological leg: drop them whole, the headline must print
        line.pop(k, None)
    if len(json.dumps(line)) > limit:
        raise ValueError(f"bench line {len(json.dumps(line))} B over {limit} B without any leg")
    return line


CLOCK_BLOCKS = 256  # stamp workgroups: 32 per XCC under round-robin dispatch


def clock_from_stamps(before, after, khz: int) -> dict:
    """Mean shader clock per XCC over the stretch two vx_tuning_clock_stamp
    launches bracket (vortex_amd/csrc/vx_clock.hip).  before/after: [blocks,
    3] int arrays of (shader cycles, real-time ticks, XCC id).  Each XCC's
    counters are compared only with its own (the counters of different XCCs
    need not agree), from the mean of its workgroups' stamps on each side."""
    import numpy as np

    b = np.asarray(before, dtype=np.float64).reshape(-1, 3)
    a = np.asarray(after, dtype=np.float64).reshape(-1, 3)
    per = {}
    for x in sorted(set(int(v) for v in b[:, 2]) & set(int(v) for v in a[:, 2])):
        bb, aa = b[b[:, 2] == x], a[a[:, 2] == x]
        d_rt = aa[:, 1].mean() - bb[:, 1].mean()
        d_cy = aa[:, 0].mean() - bb[:, 0].mean()
        if d_rt > 0:
            per[x] = d_cy / d_rt * khz * 1e3 / 1e9
    span_ms = (a[:, 1].max() - b[:, 1].min()) / (khz * 1e3) * 1e3 if len(a) and len(b) else None
    ghz = list(per.values())
    return {"GHz_mean": round(float(np.mean(ghz)), 4) if ghz else None,
            "GHz_per_xcc": {str(k): round(v, 4) for k, v in per.items()},
            "GHz_min": round(min(ghz), 4) if ghz else None, "GHz_max": round(max(ghz), 4) if ghz else None,
            "span_ms": round(span_ms, 3) if span_ms is not None else None, "wall_clock_kHz": khz,
            "source": "s_memtime / s_memrealtime stamps of each XCC before and after the timed steps "
                      "(vx_tuning_clock_stamp, vortex_amd/csrc/vx_clock.hip), same stream"}


class ClockStamps:
    """Two stamp launches on `stream` bracketing the timed steps."""

    def __init__(self, dev, stream):
        import torch

        from vortex_amd._lib import tuning

        self.stream, self.dev = stream, dev
        self.buf = [torch.zeros(3 * CLOCK_BLOCKS, dtype=torch.int64, device=dev) for _ in range(2)]
        self.khz = tuning().vx_tuning_wall_clock_khz(dev.index or 0)

    def stamp(self, k: int) -> None:
        from vortex_amd._lib import check, tuning

        check(tuning().vx_tuning_clock_stamp(self.buf[k].data_ptr(), CLOCK_BLOCKS, self.stream.cuda_stream),
              "vx_tuning_clock_stamp", tuning())

    def result(self) -> dict:
        if self.khz <= 0:
            return {"error": f"wall clock rate unavailable ({self.khz})"}
        return clock_from_stamps(self.buf[0].cpu().numpy(), self.buf[1].cpu().numpy(), self.khz)


def device_identity(local: int) -> dict:
    """Which physical GPU this rank hashed on (PCI bus id, UUID)."""
    from vortex_amd._lib import check, tuning

    bus = ctypes.create_string_buffer(64)
    uuid = ctypes.create_string_buffer(16)
    check(tuning().vx_tuning_device_identity(local, bus, 64, uuid), "vx_tuning_device_identity", tuning())
    return {"device_index": local, "pci_bus_id": bus.value.decode().lower(), "uuid": uuid.raw.hex(),
            "visible_devices": {k: os.environ[k] for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES",
                                                          "CUDA_VISIBLE_DEVICES") if k in os.environ}}


def _free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_cmd(args, argv, port: int) -> list:
    """The child launch of a plain `bench.py --gpus N` (N > 1): one rank per
    GPU on this node through torch.distributed.run, same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(args, argv) -> int:
    """Start args.gpus ranks as a child process group and relay rank 0's JSON
    line and the exit code.  The parent never touches the GPU: it counts
    devices from the KFD topology in sysfs (vortex_amd/topology.py — no HIP,
    no torch), refuses when that count is below --gpus or unreadable, checks
    that no HIP runtime is mapped in it before starting the launcher, and
    never execs."""
    import subprocess

    from vortex_amd import topology

    if not args.same_device:
        ndev = topology.visible_gpus()
        if ndev is None:
            log(f"error: --gpus {args.gpus} but the KFD topology ({topology.KFD_NODES}) is unreadable; "
                "refusing to guess the GPU count")
            return 2
        if ndev < args.gpus:
            log(f"error: --gpus {args.gpus} but only {ndev} GPU(s) visible; refusing to report a smaller run")
            return 2
    if topology.hip_runtime_mapped():
        log("error: the launching process has the HIP runtime mapped; it must not touch the GPU")
        return 3
    cmd = launch_cmd(args, argv, _free_port())
    log("launching", args.gpus, "ranks:", " ".join(cmd))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    import signal

    signal.signal(signal.SIGTERM, lambda *_: sys.exit(143))  # so the handler below runs
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = []
    try:
        for line in p.stdout:  # stream: a long run keeps printing (stderr is inherited)
            sys.stdout.write(line)
            sys.stdout.flush()
            lines.append(line)
        rc = p.wait()
    except BaseException:  # interrupted: take the ranks down with us (the launcher forwards SIGTERM)
        p.terminate()
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
        raise
    if rc != 0:
        log(f"error: the {args.gpus}-rank run failed (rc {rc})")
        return rc
    res = [json.loads(x) for x in lines if x.startswith("{")]
    if len(res) != 1 or res[0].get("n_gpus") != args.gpus or res[0].get("world_size") != args.gpus:
        log(f"error: expected one result line with n_gpus = world_size = {args.gpus}, got {len(res)}")
        return 1
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed steps first: the clock climbs for ~50 ms after the generation kernels")
    ap.add_argument("--pieces", type=int, default=65536, help="pieces per GPU")
    ap.add_argument("--piece-len", type=int, default=262144)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-thread seconds for the baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-ragged", action="store_true", help="skip the config-3 leg")
    ap.add_argument("--no-reverify", action="store_true", help="skip the config-5 legs (N=1 and N>1)")
    ap.add_argument("--reverify-multi-scale", type=float, default=1.0,
                    help="N>1 re-verify leg: fraction of linux-mint's pieces (rehearsals)")
    ap.add_argument("--reverify-multi", action="store_true",
                    help="under torch.distributed (any world size): run the config-5 leg split over the ranks "
                         "(reverify_multi), in place of the N=1 one")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm, the real path) or gloo (single-GPU multi-rank rehearsal)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank uses cuda:0 (with --dist-backend gloo)")
    ap.add_argument("--detail", default=None,
                    help="side file for the full record (traces, sweeps, identities); default bench_detail.json "
                         "beside bench.py.  stdout carries only the compact line (compact_line, <= 8 KB)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    # N ranks or nothing: a plain `bench.py --gpus N` launches its own ranks
    # (before any GPU call); under a launcher, WORLD_SIZE must be N.
    distributed = "WORLD_SIZE" in os.environ
    if not distributed and args.gpus > 1:
        return launch_ranks(args, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE {world}")
        return 2

    import torch
    import torch.distributed as dist

    from vortex_amd import device as vdev
    from vortex_amd.shard import gather_verdicts

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if distributed:  # a real process group, even at WORLD_SIZE=1 (exercises RCCL init and the gather)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
        backend = dist.get_backend()
        assert dist.get_world_size() == world
    else:
        backend = None

    n, plen = args.pieces, args.piece_len
    stride = (plen + 15) // 16 * 16
    first = rank * n  # weak scaling: global piece index shard
    seed = 0x5EED0002
    data = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    # Expected table = vortex's pool over this rank's clean pieces: the CPU
    # restatement (oracle/pool_oracle.cpp, the rayon tasks of torrent.rs:724-740
    # with SHA-NI SHA-1) hashes every piece [first, first+n) from the same
    # generator, before anything is timed.  The device batch is generated with
    # 1 % of its pieces carrying one flipped byte, so a clean piece's verdict is
    # "GPU digest == the pool's digest": the exact-mismatch-set check after the
    # timed steps proves every clean digest bit-exact against the pool.
    import oracle  # checker only

    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    exp_threads = cpu_share() if world == 1 else max(1, node_cpus() // max(1, local_world))
    t_exp = time.perf_counter()
    exp_host = oracle.pool_digest_synth(seed, first, n, plen, threads=exp_threads)
    t_exp = time.perf_counter() - t_exp
    expected = torch.frombuffer(bytearray(exp_host), dtype=torch.uint8).to(dev)
    corrupt_every = 100
    vdev.synth_fill(data, n, plen, stride=stride, first=first, seed=seed, corrupt_every=corrupt_every)
    torch.cuda.synchronize()
    matched = torch.empty(n, dtype=torch.uint8, device=dev)
    n_total = n * world
    # On RCCL each step's verdict all-gather runs on the collective stream while
    # the next step hashes: verdicts alternate between two buffers, and a step
    # waits (on the device) only for the gather that read its buffer two steps
    # before.  Every step is still hashed, verified and gathered.  (gloo gathers
    # host copies synchronously: shard.gather_verdicts.)
    overlap = distributed and backend == "nccl"
    mbuf = [matched, torch.empty_like(matched)]
    gathered = [torch.empty(n_total, dtype=torch.uint8, device=dev) for _ in range(2)] if overlap else None
    works = [None, None]

    def step(buf=None):
        vdev.sha1_uniform(data, n, plen, stride=stride, expected=expected,
                          matched=matched if buf is None else buf, want_digests=False, stream=stream)

    def before_step(k):
        if overlap and works[k % 2] is not None:
            works[k % 2].wait()  # device-side: the gather of step k-2 has read mbuf[k % 2]

    def after_step(k):
        """Start (RCCL) or do (gloo) step k's verdict gather; the gathered table, or None."""
        if overlap:
            works[k % 2] = dist.all_gather_into_tensor(gathered[k % 2], mbuf[k % 2], async_op=True)
            return None
        return gather_verdicts(matched, n_total) if distributed else None

    # everything the timed region needs is set up before the warm-up, so the
    # warm-up runs right up to the first timed step and the clock it raised holds
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    clk = ClockStamps(dev, stream)
    ident = device_identity(local)
    for k in range(args.warmup):
        before_step(k)
        step(mbuf[k % 2] if overlap else None)
        after_step(k)
    for w in works:
        if w is not None:
            w.wait()
    works[:] = [None, None]
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    verdicts = None
    clk.stamp(0)  # two 256-workgroup stamp launches bracket the steps (~10 us each)
    for k in range(args.steps):
        before_step(k)
        evs[k][0].record(stream)
        step(mbuf[k % 2] if overlap else None)
        evs[k][1].record(stream)
        g = after_step(k)
        verdicts = g if g is not None else verdicts
    for w in works:  # the last gathers are part of the timed work
        if w is not None:
            w.wait()
    if overlap:
        verdicts = gathered[(args.steps - 1) % 2]
    clk.stamp(1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if distributed:
        dist.barrier()
    elapsed = t1 - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    clock = clk.result()
    ranks = None
    if distributed:
        # The verdict all-gather alone, after the timed region: what the one
        # collective costs per step (the scaling overhead at N > 1).
        # (wall clock: RCCL runs on its own stream, gloo on the host)
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        for _ in range(args.steps):
            gather_verdicts(matched, n_total)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) / args.steps * 1e3
        # every rank's figures (max over ranks is what `value` uses)
        mine = torch.tensor([elapsed, kern_ms, gather_ms, clock.get("GHz_mean") or 0.0], dtype=torch.float64,
                            device=dev if args.dist_backend == "nccl" else "cpu")
        allr = torch.empty(4 * world, dtype=torch.float64, device=mine.device)
        dist.all_gather_into_tensor(allr, mine)
        per = allr.view(world, 4).cpu().tolist()
        elapsed, kern_ms = max(r[0] for r in per), max(r[1] for r in per)
        # which physical GPU every rank ran on, and the world RCCL reported
        idents = [None] * world
        dist.all_gather_object(idents, dict(ident, rank=rank, world_size=dist.get_world_size()))
        buses = [d["pci_bus_id"] for d in idents]
        distinct = len(set(buses)) == world
        if not args.same_device and not distinct:  # every rank sees the same list: all fail together
            log(f"error: ranks share a GPU (bus ids {buses}); a {world}-GPU line needs {world} distinct devices")
            dist.destroy_process_group()
            return 4
        ranks = {"step_ms": [round(r[0] / args.steps * 1e3, 4) for r in per],
                 "kernel_ms": [round(r[1], 4) for r in per],
                 "verdict_gather_ms": [round(r[2], 4) for r in per],
                 "clock_GHz": [round(r[3], 4) for r in per],
                 "devices": idents, "distinct_devices": distinct}

    # Verdicts: exactly the corrupted pieces mismatch (checked on the gathered
    # table when N > 1, else locally).
    m = (verdicts if verdicts is not None else matched).cpu().numpy()
    g0 = 0 if verdicts is not None else first
    bad = [i for i in range(len(m)) if not m[i]]
    want_bad = [i for i in range(len(m)) if oracle.is_corrupt(g0 + i, corrupt_every)]
    assert bad == want_bad, f"rank {rank}: verdicts differ from the expected mismatch set"
    # every verdict of the (gathered) table checked: clean pieces bit-exact against the pool's digests
    parity = {"checked": len(m), "bit_exact": len(m) - len(want_bad), "corrupt_mismatched": len(want_bad),
              "against": "cpu pool restatement (oracle/pool_oracle.cpp, SHA-NI SHA-1 per piece task)",
              "expected_table_threads": exp_threads, "expected_table_s": round(t_exp, 3)}

    total_bytes = n_total * plen
    value = total_bytes / elapsed * args.steps / GiB
    achieved = n * plen / (kern_ms * 1e-3)
    workload = f"{n} x {plen // 1024} KiB pieces per GPU"
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "world_size": dist.get_world_size() if distributed else 1,
        "backend": backend,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: counter-based splitmix64 pieces generated in HBM, 1% with one flipped byte",
        "config": {"workload": workload + " (BASELINE config 2; config 4 at N=8), SHA-1 + verify vs expected table"
                               + (f", {backend} all-gather of verdicts" if distributed else ""),
                   "pieces_per_gpu": n, "piece_len": plen, "total_GiB": round(total_bytes / GiB, 2),
                   "parallelism": f"piece-index shard x{world}",
                   "parity_checked": parity["checked"], "parity_bit_exact": parity["bit_exact"],
                   "parity_against": "cpu pool restatement"},
        "roofline": roofline(n, plen, kern_ms, achieved, workload, clock, steps=args.steps),
        "parity": parity,
        "device": ident,
    }
    if ranks is not None:
        res["ranks"] = ranks
    # The N>1 re-verify leg is opt-in: it runs collectives over a 2.9 GB file
    # after the headline is measured, and a rank that dies inside it would take
    # the line down with it.  The driver's N>1 runs print only the
    # config-2/4 line; builder runs add --reverify-multi.
    multi = distributed and args.reverify_multi and not args.no_reverify
    extra = rank == 0 and world == 1
    if multi or extra:
        del data, matched, expected
        torch.cuda.empty_cache()
    if multi:
        # config 5 split over the node's GPUs; every rank takes part
        try:
            rm = reverify_multi_leg(rank, world, local, dev, backend, args.same_device, args.reverify_multi_scale)
        except Exception as e:  # noqa: BLE001  (recorded in the line; the checks raise on every rank alike)
            import traceback

            traceback.print_exc()
            rm = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0:
            res["reverify_multi"] = rm
            log("reverify_multi:", {k: rm[k].get("value") for k in ("warm", "cold")} if "warm" in rm else rm)
    if extra:
        # Extra legs (N=1 only): the other BASELINE configs and
        # the host-resident path, each with its own correctness check.  A leg
        # that fails (its check, or the host: disk space, pinning limits) is
        # recorded as {"error": ...} in its key; the metric line still prints.
        log(f"config 2: {value:.1f} GiB/s, kernel {kern_ms:.3f} ms")

        def leg(keys, fn, *a):
            try:
                out = fn(*a)
            except Exception as e:  # noqa: BLE001  (recorded in the line, not swallowed)
                import traceback

                traceback.print_exc()
                out = tuple({"error": f"{type(e).__name__}: {e}"} for _ in keys) if len(keys) > 1 else \
                    {"error": f"{type(e).__name__}: {e}"}
            for k, v in zip(keys, out if len(keys) > 1 else (out,)):
                res[k] = v
                log(f"{k}:", v.get("value", v.get("error")), "GiB/s" if "value" in v else "")
            torch.cuda.empty_cache()

        if not args.no_cpu_baseline:
            leg(("cpu_baseline",), cpu_baseline, args.cpu_seconds, plen)
        if not args.no_ragged:
            leg(("ragged",), ragged_leg, dev, stream)
        if not args.no_e2e:
            leg(("e2e",), e2e_batch, plen)
            cb = res.get("cpu_baseline") or {}
            per_thread = cb["value"] / cb["cores"] if cb.get("value") and cb.get("cores") else None
            leg(("e2e_async",), e2e_async, plen, 8192, per_thread)
            leg(("e2e_contiguous",), e2e_contiguous, plen)
        if not args.no_reverify and not multi:
            leg(("reverify", "reverify_cold"), reverify_leg)
    if rank == 0:
        # the full record to the side file, the compact line (≤ 8 KB) to stdout
        detail = args.detail or os.path.join(ROOT, "bench_detail.json")
        name = os.path.relpath(detail, ROOT) if detail.startswith(ROOT + os.sep) else detail
        try:
            with open(detail, "w") as f:
                json.dump(res, f, indent=1)
        except OSError as e:
            log(f"warning: side file {detail} not written: {e}")
            name = None
        print(json.dumps(compact_line(res, name)), flush=True)
    if distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
