#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) rate of BASELINE config 3's ragged batch held in
host memory: 262,144 x 16 KiB + 16,384 x 256 KiB + 4,096 x 1 MiB + 1,024 x
4 MiB = 16 GiB, order shuffled with seed 0x5EED0003, packed
back to back in one registered host mmap, through vx_verify_batch (H2D +
kernel + D2H of verdicts and digests) — the same timing as bench.e2e_rate.
The CPU pool restatement (oracle/, the checker) hashes the same pieces first,
which gives the expected table and its own rate on the box's CPU share.
Every 100th expected digest is spoiled; verdicts and digests are checked
against the CPU pool.  One JSON line.

usage: python tools/e2e_ragged.py [--scale 1.0] [--reps 3]
"""
import argparse
import ctypes
import json
import mmap
import os
import random
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GiB = float(1 << 30)
SEED = 0x5EED0003


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of config 3's piece counts")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--unregistered", action="store_true", help="plain host memory (pinned-stage path)")
    a = ap.parse_args()
    import torch  # noqa: F401  (loads torch's HIP runtime first, as vortex_amd expects)

    import oracle
    from bench import cpu_share
    from vortex_amd._lib import check, lib
    from vortex_amd.hash_pool import HashPool

    classes = [(16 << 10, 262144), (256 << 10, 16384), (1 << 20, 4096), (4 << 20, 1024)]
    lens = []
    for L, k in classes:
        lens += [L] * max(1, int(k * a.scale))
    random.Random(SEED).shuffle(lens)
    n, total = len(lens), sum(lens)
    offs, o = [], 0
    for L in lens:
        offs.append(o)
        o += L
    buf = mmap.mmap(-1, total)
    base = ctypes.addressof(ctypes.c_char.from_buffer(buf))
    threads = cpu_share()
    t0 = time.perf_counter()

    def fill(r):
        for i in range(r, n, threads):
            oracle.lib().vxo_gen_piece(SEED, i, lens[i], 0, ctypes.c_void_p(base + offs[i]))

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(fill, range(threads)))
    t_gen = time.perf_counter() - t0

    ptrs = (ctypes.c_void_p * n)(*[base + x for x in offs])
    clens = (ctypes.c_uint32 * n)(*lens)
    cpu_dig = ctypes.create_string_buffer(20 * n)
    t0 = time.perf_counter()
    oracle.pool_verify_ptrs(ptrs, clens, n, None, threads, 0, None, cpu_dig)
    t_cpu = time.perf_counter() - t0
    exp = bytearray(cpu_dig.raw)
    for i in range(99, n, 100):
        exp[20 * i] ^= 0xFF
    cexp = ctypes.create_string_buffer(bytes(exp), 20 * n)
    want = bytes(0 if i % 100 == 99 else 1 for i in range(n))

    matched = ctypes.create_string_buffer(n)
    digests = ctypes.create_string_buffer(20 * n)
    runs = []
    with HashPool(max(lens)) as pool:
        t0 = time.perf_counter()
        if not a.unregistered:
            pool.register_buffer(buf)
        t_reg = time.perf_counter() - t0
        check(lib().vx_verify_batch(pool._h, ptrs, clens, cexp, min(n, 4096), matched, digests), "warm")
        for _ in range(a.reps):
            ctypes.memset(matched, 0, n)
            ctypes.memset(digests, 0, 20 * n)
            t0 = time.perf_counter()
            check(lib().vx_verify_batch(pool._h, ptrs, clens, cexp, n, matched, digests), "vx_verify_batch")
            runs.append(time.perf_counter() - t0)
            assert matched.raw[:n] == want, "verdicts differ from the CPU pool"
            assert digests.raw[:20 * n] == cpu_dig.raw[:20 * n], "digests differ from the CPU pool"
        if not a.unregistered:
            pool.unregister_buffer(buf)
    el = sorted(runs)[len(runs) // 2]
    print(json.dumps({
        "workload": f"config 3 ragged mix from host: {n} pieces, {total / GiB:.2f} GiB "
                    f"(16 KiB/256 KiB/1 MiB/4 MiB, equal bytes per class, scale {a.scale})",
        "e2e_GiBps": round(total / el / GiB, 2),
        "runs_GiBps": [round(total / r / GiB, 2) for r in runs],
        "ms": round(el * 1e3, 1),
        "cpu_pool_GiBps": round(total / t_cpu / GiB, 2), "cpu_threads": threads, "sha_ni": bool(oracle.has_shani()),
        "registered": not a.unregistered,
        "register_s": round(t_reg, 2), "gen_s": round(t_gen, 2),
        "checked": "all verdicts and digests equal to the CPU pool restatement",
    }), flush=True)


if __name__ == "__main__":
    main()
