#!/usr/bin/env python3
"""The balanced split on one context alternating page-cached and evicted calls
(GPU, diagnostic).

The split's first group starts from what earlier split calls on the context
measured, kept apart for cached and uncached data.  This
alternates, on the linux-mint-geometry file: a warm balanced call, then
(evicting before each) a cold balanced call, the cold engine alone and the
cold pool alone; every verdict checked.  Prints the medians and boundaries.

usage: python tools/split_cold_mix.py OUT.json [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import oracle  # noqa: E402
from vortex_amd.hash_pool import HashPool  # noqa: E402


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    threads = bench.cpu_share()
    pool_t, io_t = max(1, threads * 3 // 4), max(2, threads // 2)
    pl = 2097152
    path = os.path.join(bench.reverify_dir(), f"vx_cold_mix_{os.getpid()}.iso")
    runs = {"warm_balanced": [], "cold_balanced": [], "cold_engine": [], "cold_pool": []}
    bounds = {"warm_balanced": [], "cold_balanced": []}
    try:
        total, n, last = bench.write_linuxmint_file(path)
        exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
        for _ in range(2):
            oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
        t0 = time.perf_counter()
        oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
        rate = total / (time.perf_counter() - t0) / threads
        with HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=4096) as pool:
            pool.verify_files([path], [total], pl, exp, io_threads=threads)
            for r in range(reps):
                bench.resident_fraction(path)
                oracle.pool_verify_files([path], [total], pl, exp, threads=threads)  # cached again
                c = bench.balanced_call(pool, [path], [total], n, pl, exp, io_t, pool_t, rate)
                assert c["ok"]
                runs["warm_balanced"].append(c["s"])
                bounds["warm_balanced"].append(c["boundary"])
                bench.drop_cache(path)
                c = bench.balanced_call(pool, [path], [total], n, pl, exp, io_t, pool_t, rate)
                assert c["ok"]
                runs["cold_balanced"].append(c["s"])
                bounds["cold_balanced"].append(c["boundary"])
                bench.drop_cache(path)
                t0 = time.perf_counter()
                _, bad = pool.verify_files([path], [total], pl, exp, io_threads=threads)
                runs["cold_engine"].append(time.perf_counter() - t0)
                assert bad == 0
                bench.drop_cache(path)
                t0 = time.perf_counter()
                assert all(oracle.pool_verify_files([path], [total], pl, exp, threads=threads))
                runs["cold_pool"].append(time.perf_counter() - t0)
                print(f"rep {r}: " + " ".join(f"{k} {v[-1] * 1e3:.1f}" for k, v in runs.items())
                      + f" bounds {bounds['warm_balanced'][-1]} {bounds['cold_balanced'][-1]}", flush=True)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    med = {k: sorted(v)[len(v) // 2] for k, v in runs.items()}
    res = {"runs_s": runs, "boundaries": bounds, "median_s": med,
           "median_GiBps": {k: round(total / v / (1 << 30), 2) for k, v in med.items()}}
    print("median GiB/s:", res["median_GiBps"], flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
