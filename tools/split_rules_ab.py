#!/usr/bin/env python3
"""A/B of the split's rules for pieces of one chunk (GPU; test build).

vx_tuning_split_rules: `old` gives one-chunk pieces the multi-round rules (no
group until both sides have rates, the tenth rule), `new` lets them keep the
first group's rule while cold and skips the tenth rule, `capN` adds a cap of
N MiB (at least 1,024 lanes) on their rounds, `auto` is the default (cap64),
`perpiece` the default reading piece by piece instead of in runs, `nolag` the
default without the learned lag on the first group, `ewma` the default
learning by running mean instead of the median of the last five calls.
For each piece length this writes a ~2 GiB file of synthetic pieces, warms it, and alternates the variants' balanced splits
(bench.balanced_call) with the engine alone at the split's readers, every
verdict checked; prints the medians.

usage: python tools/split_rules_ab.py OUT.json [reps] [piece KiB list] [variants, e.g. old,new,cap64]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import oracle  # noqa: E402
from split_geom_probe import SEED, med, write  # noqa: E402
from vortex_amd.hash_pool import HashPool  # noqa: E402


def rules(name):
    if name == "old":
        return 0, 0, 1, 1
    if name == "new":
        return 1, 0, 1, 1
    if name == "auto":  # the default: 64 MiB, at least 1,024 lanes
        return 1, 64 << 20, 1, 1
    if name == "perpiece":  # the default, reading piece by piece
        return 2, 64 << 20, 1, 1
    if name == "nolag":  # the default, the first group without the learned lag
        return 1, 64 << 20, 0, 1
    if name == "ewma":  # the default, learning by running mean instead of the median of 5
        return 1, 64 << 20, 1, 0
    return 1, int(name[3:]) << 20, 1, 1


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    kibs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [16, 64, 256]
    variants = sys.argv[4].split(",") if len(sys.argv) > 4 else ["old", "new", "cap64", "cap128"]
    threads = bench.cpu_share()
    pool_t, io_t = max(1, threads * 3 // 4), max(2, threads // 2)
    res = {"threads": threads, "pool_threads": pool_t, "readers": io_t, "geoms": {}}
    for kib in kibs:
        pl = kib << 10
        total = (2 << 30) + pl // 3 + 4099
        path = os.path.join(bench.reverify_dir(), f"vx_rules_{os.getpid()}_{kib}.bin")
        try:
            n, last = write(path, pl, total)
            exp = oracle.pool_digest_synth(SEED, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
            for _ in range(2):
                oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
            t0 = time.perf_counter()
            oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
            rate = total / (time.perf_counter() - t0) / threads
            runs = {k: [] for k in ["engine"] + variants}
            bounds = {k: [] for k in variants}
            with HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=4096, hooks=True) as pool:
                pool.verify_files([path], [total], pl, exp, io_threads=io_t)
                for r in range(reps):
                    pool.lib.vx_tuning_split_rules(pool._h, 1, 64 << 20, 1, 1)
                    t0 = time.perf_counter()
                    _, bad = pool.verify_files([path], [total], pl, exp, io_threads=io_t)
                    runs["engine"].append(time.perf_counter() - t0)
                    assert bad == 0
                    for v in variants:
                        pool.lib.vx_tuning_split_rules(pool._h, *rules(v))
                        c = bench.balanced_call(pool, [path], [total], n, pl, exp, io_t, pool_t, rate)
                        assert c["ok"], f"{kib} KiB {v}: the split's verdicts differ"
                        runs[v].append(c["s"])
                        bounds[v].append(c["boundary"])
                pool.lib.vx_tuning_split_rules(pool._h, 1, 64 << 20, 1, 1)
            g = {k: round(total / med(v) / (1 << 30), 2) for k, v in runs.items()}
            res["geoms"][f"{kib}K"] = {"pieces": n, "GiBps": g, "boundaries": bounds,
                                      "s_runs": {k: [round(x, 4) for x in v] for k, v in runs.items()}}
            print(kib, "KiB:", g, flush=True)
        finally:
            if os.path.exists(path):
                os.unlink(path)
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
