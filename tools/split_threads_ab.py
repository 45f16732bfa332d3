#!/usr/bin/env python3
"""How many pool threads and engine readers the balanced split wants (GPU).

Alternates, call by call, the balanced split (bench.balanced_call) at several
(pool threads, engine readers) shapes on the warm linux-mint-geometry file,
every verdict checked, and prints each shape's median.  The round-5 shape
(3/4 of the threads for the pool, half for the readers) was chosen for the
planned split, where a pool too large for its fixed share ran bimodal; the
balanced split moves the boundary instead.

usage: python tools/split_threads_ab.py OUT.json [reps] [shapes, e.g. 12:8,16:8,14:6]
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
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 9
    threads = bench.cpu_share()
    shapes = [tuple(int(x) for x in s.split(":")) for s in sys.argv[3].split(",")] if len(sys.argv) > 3 else \
        [(threads * 3 // 4, threads // 2), (threads, threads // 2), (threads - 2, threads * 3 // 8)]
    pl = 2097152
    path = os.path.join(bench.reverify_dir(), f"vx_split_ab_{os.getpid()}.iso")
    runs = {f"{p}:{r}": [] for p, r in shapes}
    bounds = {k: [] for k in runs}
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
                for p, rd in shapes:
                    c = bench.balanced_call(pool, [path], [total], n, pl, exp, rd, p, rate)
                    assert c["ok"], "a verdict differs from the expected table"
                    runs[f"{p}:{rd}"].append(round(c["s"], 4))
                    bounds[f"{p}:{rd}"].append(c["boundary"])
                print(f"rep {r}: " + " ".join(f"{k} {v[-1] * 1e3:.1f}" for k, v in runs.items()), flush=True)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    med = {k: sorted(v)[len(v) // 2] for k, v in runs.items()}
    res = {"threads": threads, "rate_per_thread": rate, "runs_s": runs, "boundaries": bounds, "median_s": med,
           "median_GiBps": {k: round(total / v / (1 << 30), 2) for k, v in med.items()}}
    print("median GiB/s:", res["median_GiBps"], flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
