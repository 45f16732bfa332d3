#!/usr/bin/env python3
"""The self-balancing split's decisions, call by call (GPU; test build).

Writes the linux-mint-geometry file (bench.write_linuxmint_file), then
alternates, `reps` times, the balanced split (bench.balanced_call, the engine
through vx_verify_files_split beside the oracle's claim pool) with the fixed
split at vx_plan_verify_split's point (bench.split_call).  Per balanced call
it records wall / engine / pool seconds, the boundary, every round's decision
(vx_tuning_last_split: rates, predicted remaining times, the group taken) and
the round timeline's GPU kernel ends, to JSON.

usage: python tools/split_probe.py OUT.json [reps] [pool_threads] [readers] [sweep] [cold]
  sweep: comma-separated scales of the planner's GPU share for the fixed
  points (default 1.0: the planner's point only); "cold" evicts the file
  (fsync + POSIX_FADV_DONTNEED) before every call
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import oracle  # noqa: E402
from vortex_amd.hash_pool import HashPool, plan_verify_split  # noqa: E402

COLS = ("t_ms", "pool_rate", "engine_rate", "block_ns", "t_engine_ms", "t_pool_ms", "unclaimed", "group", "lanes",
        "pool_done", "mode", "measured", "lag_ms")


def decisions(pool):
    n = pool.lib.vx_tuning_last_split(pool._h, None, 0)
    buf = (ctypes.c_double * (len(COLS) * max(1, n)))()
    pool.lib.vx_tuning_last_split(pool._h, buf, n)
    return [{k: round(buf[len(COLS) * i + j], 4) for j, k in enumerate(COLS)} for i in range(n)]


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    threads = bench.cpu_share()
    pool_t = int(sys.argv[3]) if len(sys.argv) > 3 else max(1, threads * 3 // 4)
    io_t = int(sys.argv[4]) if len(sys.argv) > 4 else max(2, threads // 2)
    sweep = [float(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else [1.0]
    cold = len(sys.argv) > 6 and sys.argv[6] == "cold"  # evict the file before every call
    pl = 2097152
    path = os.path.join(bench.reverify_dir(), f"vx_split_probe_{os.getpid()}.iso")
    res = {"pool_threads": pool_t, "readers": io_t, "calls": [], "fixed": []}
    summary_b = []
    try:
        total, n, last = bench.write_linuxmint_file(path)
        exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
        for _ in range(2):
            oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
        t0 = time.perf_counter()
        oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
        rate = total / (time.perf_counter() - t0) / threads
        plan = plan_verify_split(n, pl, total, cpu_threads=pool_t, cpu_thread_rate=rate)
        res["plan_first"] = plan["gpu_first"]
        res["rate_per_thread"] = rate
        with HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=4096, hooks=True) as pool:
            pool.verify_files([path], [total], pl, exp, io_threads=threads)
            def evict():
                if cold:
                    bench.drop_cache(path)

            res["cold"] = cold
            res["alone"] = []
            for r in range(reps):
                evict()
                c = bench.balanced_call(pool, [path], [total], n, pl, exp, io_t, pool_t, rate)
                rounds = pool.last_verify_rounds()
                res["calls"].append({"s": round(c["s"], 4), "gpu_s": round(c["gpu_s"], 4),
                                     "cpu_s": round(c["cpu_s"], 4), "boundary": c["boundary"], "ok": c["ok"],
                                     "decisions": decisions(pool),
                                     "rounds": [{"enq": round(x["enqueue_ms"], 2), "cs": round(x["copy_start_ms"], 2),
                                                 "ce": round(x["copy_end_ms"], 2), "ke": round(x["kernel_end_ms"], 2),
                                                 "mb": round(x["bytes"] / 1e6, 1), "lanes": x["lanes"]}
                                                for x in rounds]})
                summary_b.append(c["s"])
                k0 = n - plan["gpu_first"]
                fixed = {}
                for scale in sweep:  # fixed points: the planner's GPU share scaled
                    first = max(0, min(n, n - int(round(k0 * scale))))
                    evict()
                    f = bench.split_call(pool, [path], [total], n, pl, exp, first, io_t, pool_t)
                    fixed[first] = round(f["s"], 4)
                res["fixed"].append(fixed)
                alone = {}
                for name, first, io_c, pool_c in (("gpu", 0, threads, threads), ("pool", n, threads, threads)):
                    evict()
                    alone[name] = round(bench.split_call(pool, [path], [total], n, pl, exp, first, io_c, pool_c)["s"], 4)
                res["alone"].append(alone)
                print(f"rep {r}: balanced {c['s'] * 1e3:.1f} ms (gpu {c['gpu_s'] * 1e3:.1f}, pool "
                      f"{c['cpu_s'] * 1e3:.1f}, boundary {c['boundary']}); fixed "
                      + " ".join(f"@{k}:{v * 1e3:.1f}" for k, v in fixed.items())
                      + f"; alone gpu {alone['gpu'] * 1e3:.1f} pool {alone['pool'] * 1e3:.1f}", flush=True)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    res["balanced_median_s"] = med(summary_b)
    res["fixed_median_s"] = {k: med([f[k] for f in res["fixed"] if k in f]) for k in res["fixed"][0]}
    res["alone_median_s"] = {k: med([a[k] for a in res["alone"]]) for k in ("gpu", "pool")}
    print("median: balanced", res["balanced_median_s"], "fixed", res["fixed_median_s"], "alone",
          res["alone_median_s"], flush=True)
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main()
