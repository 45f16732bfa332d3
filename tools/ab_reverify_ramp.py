#!/usr/bin/env python3
"""A/B of the re-verify head ramp on config 5's geometry:
rounds that double (default so far) against rounds that grow x5/4
(VX_VERIFY_RAMP_GROWTH=1), each with ramp depth 1 and 2.  One process, one
page-cache-warm file (synthetic data, linux-mint geometry), contexts created
per arm and call in rotating order; every call's verdicts are checked.
Prints one JSON line of per-arm GiB/s runs and medians.

usage: python tools/ab_reverify_ramp.py [--reps 6]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ARMS = {"double_d1": {"VX_VERIFY_RAMP_GROWTH": "0", "VX_VERIFY_RAMP": "1"},
        "gentle_d1": {"VX_VERIFY_RAMP_GROWTH": "1", "VX_VERIFY_RAMP": "1"},
        "double_d2": {"VX_VERIFY_RAMP_GROWTH": "0", "VX_VERIFY_RAMP": "2"},
        "gentle_d2": {"VX_VERIFY_RAMP_GROWTH": "1", "VX_VERIFY_RAMP": "2"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)

    import oracle
    from vortex_amd.hash_pool import HashPool

    pl, total = 2097152, 2907832320
    n = (total + pl - 1) // pl
    last = total - (n - 1) * pl
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"vx_ab_ramp_{os.getpid()}.iso")
    buf = ctypes.create_string_buffer(pl)
    try:
        with open(path, "wb") as f:
            for i in range(n):
                L = last if i == n - 1 else pl
                oracle.lib().vxo_gen_piece(0x5EED0005, i, L, 0, buf)
                f.write(memoryview(buf)[:L])
        exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
        runs = {k: [] for k in ARMS}
        for rep in range(a.reps + 1):
            order = list(ARMS)[rep % len(ARMS):] + list(ARMS)[:rep % len(ARMS)]
            for arm in order:
                os.environ.update(ARMS[arm])
                with HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=4096) as pool:
                    got, bad = pool.verify_files([path], [total], pl, exp, io_threads=threads)  # warm
                    assert all(got) and bad == 0
                    t0 = time.perf_counter()
                    got, bad = pool.verify_files([path], [total], pl, exp, io_threads=threads)
                    el = time.perf_counter() - t0
                    assert all(got) and bad == 0
                if rep:
                    runs[arm].append(round(total / el / (1 << 30), 2))
            print(f"rep {rep}: " + ", ".join(f"{k} {v[-1] if v else '-'}" for k, v in runs.items()), file=sys.stderr,
                  flush=True)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    print(json.dumps({"workload": "re-verify 1387 x 2 MiB (linux-mint geometry), warm file, 16 threads",
                      "runs_GiBps": runs, "median": {k: statistics.median(v) for k, v in runs.items()}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
