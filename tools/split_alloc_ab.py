#!/usr/bin/env python3
"""What the pool's per-segment buffers cost the balanced split (GPU, diagnostic).

vortex's re-verify reads every segment into a fresh zeroed Vec
(file_store.rs:272); the oracle's claim pool restates that.  Backend bit 0x100
makes it read into one buffer per thread instead.  This alternates, call by
call on the warm linux-mint-geometry file, the pool alone and the balanced
split (the engine through vx_verify_files_split) with both buffer policies,
every verdict checked, and prints the medians.

usage: python tools/split_alloc_ab.py OUT.json [reps]
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import oracle  # noqa: E402
from vortex_amd.hash_pool import HashPool, Split  # noqa: E402

REUSE = 0x100


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 9
    threads = bench.cpu_share()
    pool_t, io_t = max(1, threads * 3 // 4), max(2, threads // 2)
    pl = 2097152
    path = os.path.join(bench.reverify_dir(), f"vx_split_alloc_{os.getpid()}.iso")
    runs = {k: [] for k in ("alone_fresh", "alone_reuse", "split_fresh", "split_reuse")}
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
                for policy, backend in (("fresh", 0), ("reuse", REUSE)):
                    t0 = time.perf_counter()
                    ok = oracle.pool_verify_files([path], [total], pl, exp, threads=threads, backend=backend)
                    runs[f"alone_{policy}"].append(round(time.perf_counter() - t0, 4))
                    assert all(ok)
                    sp = Split(0, n, pool_t, rate)
                    res = {}

                    def engine():
                        res["bad"] = pool.verify_files_split([path], [total], pl, exp, sp, io_threads=io_t)

                    th = threading.Thread(target=engine)
                    t0 = time.perf_counter()
                    th.start()
                    oracle.pool_verify_files_claim([path], [total], pl, exp, pool_t, sp.claim_fn, sp.done_fn, sp.arg,
                                                   0, sp.matched, backend=backend)
                    th.join()
                    runs[f"split_{policy}"].append(round(time.perf_counter() - t0, 4))
                    assert all(sp.verdicts()) and res["bad"] == 0
                print(f"rep {r}: " + " ".join(f"{k} {v[-1] * 1e3:.1f}" for k, v in runs.items()), flush=True)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    med = {k: sorted(v)[len(v) // 2] for k, v in runs.items()}
    res = {"threads": threads, "pool_threads_split": pool_t, "readers": io_t, "runs_s": runs, "median_s": med,
           "median_GiBps": {k: round(total / v / (1 << 30), 2) for k, v in med.items()}}
    print("median GiB/s:", res["median_GiBps"], flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
