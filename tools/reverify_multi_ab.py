#!/usr/bin/env python3
"""A/B: config-5 re-verify through one context against two contexts on the
SAME GPU (vx_verify_files_multi: two independent read -> copy -> hash
pipelines, each on half the pieces and half the readers).  The question is
whether a second pipeline fills the first one's copy bubbles (the copy engine
idles 10-15 % of a warm call waiting for reads).  Same
pinned bytes on both sides (4 x 512 MiB against 2 x 4 x 256 MiB), warm and
evicted calls alternating per rep; every verdict checked.  One JSON line.

usage: python tools/reverify_multi_ab.py [--reps 8] [--cold-reps 3]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--cold-reps", type=int, default=3)
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)

    import bench
    import oracle
    from vortex_amd.hash_pool import HashPool, verify_files_multi

    pl, total = 2097152, 2907832320
    n = (total + pl - 1) // pl
    last = total - (n - 1) * pl
    threads = bench.cpu_share()
    path = os.path.join(bench.reverify_dir(), f"vx_multi_ab_{os.getpid()}.iso")
    buf = ctypes.create_string_buffer(pl)
    res = {"one": {"warm": [], "cold": []}, "two": {"warm": [], "cold": []}}
    try:
        with open(path, "wb") as f:
            for i in range(n):
                L = last if i == n - 1 else pl
                oracle.lib().vxo_gen_piece(0x5EED0005, i, L, 0, buf)
                f.write(memoryview(buf)[:L])
            f.flush()
            os.fsync(f.fileno())
        exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
        one = HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=4096)
        two = [HashPool(pl, slots=4, slot_bytes=256 << 20, batch_pieces=4096) for _ in range(2)]
        runs = {"one": lambda: one.verify_files([path], [total], pl, exp, io_threads=threads),
                "two": lambda: verify_files_multi(two, [path], [total], pl, exp, io_threads=threads)}
        for name in runs:  # warm-up, and the page cache filled
            got, bad = runs[name]()
            assert all(got) and bad == 0
        for leg, reps in (("warm", a.reps), ("cold", a.cold_reps)):
            for _ in range(reps):
                for name, run in runs.items():
                    if leg == "cold":
                        bench.drop_cache(path)
                    t0 = time.perf_counter()
                    got, bad = run()
                    el = time.perf_counter() - t0
                    assert all(got) and bad == 0 and len(got) == n
                    res[name][leg].append(round(total / el / (1 << 30), 2))
                    print(f"{leg} {name}: {res[name][leg][-1]} GiB/s", file=sys.stderr, flush=True)
        one.close()
        for p in two:
            p.close()
    finally:
        if os.path.exists(path):
            os.unlink(path)
    out = {"threads": threads, "dir": os.path.dirname(path)}
    for name, r in res.items():
        out[name] = {**r, "warm_median": statistics.median(r["warm"]) if r["warm"] else None,
                     "cold_median": statistics.median(r["cold"]) if r["cold"] else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
