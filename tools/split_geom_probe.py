#!/usr/bin/env python3
"""The balanced split across piece lengths (GPU, diagnostic).

The split's model was tuned on linux-mint's geometry (2 MiB pieces).  For each
piece length this writes a ~2 GiB file of synthetic pieces with a short last
piece, warms it, and alternates `reps` times: vortex's pool restated alone
(every thread, and the split's pool threads), the engine alone (vx_verify_files;
every thread reading, and the split's readers), and
the balanced split (bench.balanced_call, 3/4 of the threads in the pool, half
reading), every verdict checked.  Prints each geometry's medians and whether
the split beats both sides alone.

usage: python tools/split_geom_probe.py OUT.json [reps] [piece lengths in KiB, e.g. 16,256,4096]
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
from vortex_amd.hash_pool import HashPool  # noqa: E402

SEED = 0x5EED0007


def write(path, pl, total):
    n = (total + pl - 1) // pl
    last = total - (n - 1) * pl
    buf = ctypes.create_string_buffer(pl)
    with open(path, "wb") as f:
        for i in range(n):
            L = last if i == n - 1 else pl
            oracle.lib().vxo_gen_piece(SEED, i, L, 0, buf)
            f.write(memoryview(buf)[:L])
        f.flush()
        os.fsync(f.fileno())
    return n, last


def med(v):
    return sorted(v)[len(v) // 2]


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    kibs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [16, 64, 256, 1024, 2048, 4096, 16384]
    threads = bench.cpu_share()
    pool_t, io_t = max(1, threads * 3 // 4), max(2, threads // 2)
    res = {"threads": threads, "pool_threads_split": pool_t, "readers_split": io_t, "geoms": {}}
    for kib in kibs:
        pl = kib << 10
        total = (2 << 30) + pl // 3 + 4099
        path = os.path.join(bench.reverify_dir(), f"vx_geom_{os.getpid()}_{kib}.bin")
        try:
            n, last = write(path, pl, total)
            exp = oracle.pool_digest_synth(SEED, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
            for _ in range(2):
                oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
            t0 = time.perf_counter()
            oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
            rate = total / (time.perf_counter() - t0) / threads
            runs = {"pool": [], "pool_split_threads": [], "engine": [], "engine_split_readers": [],
                    "balanced": []}
            bounds, engine_s, pool_s = [], [], []
            with HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=4096) as pool:
                pool.verify_files([path], [total], pl, exp, io_threads=threads)
                for r in range(reps):
                    t0 = time.perf_counter()
                    ok = all(oracle.pool_verify_files([path], [total], pl, exp, threads=threads))
                    runs["pool"].append(time.perf_counter() - t0)
                    assert ok, f"{kib} KiB: the pool's verdicts differ"
                    t0 = time.perf_counter()
                    ok = all(oracle.pool_verify_files([path], [total], pl, exp, threads=pool_t))
                    runs["pool_split_threads"].append(time.perf_counter() - t0)
                    assert ok
                    t0 = time.perf_counter()
                    _, bad = pool.verify_files([path], [total], pl, exp, io_threads=threads)
                    runs["engine"].append(time.perf_counter() - t0)
                    assert bad == 0, f"{kib} KiB: the engine's verdicts differ"
                    t0 = time.perf_counter()
                    _, bad = pool.verify_files([path], [total], pl, exp, io_threads=io_t)
                    runs["engine_split_readers"].append(time.perf_counter() - t0)
                    assert bad == 0
                    c = bench.balanced_call(pool, [path], [total], n, pl, exp, io_t, pool_t, rate)
                    assert c["ok"], f"{kib} KiB: the split's verdicts differ"
                    runs["balanced"].append(c["s"])
                    bounds.append(c["boundary"])
                    engine_s.append(round(c["gpu_s"], 4))
                    pool_s.append(round(c["cpu_s"], 4))
            g = {k: round(total / med(v) / (1 << 30), 2) for k, v in runs.items()}
            rec = {"pieces": n, "last": last, "GiBps": g, "beats_both": g["balanced"] > max(g["pool"], g["engine"]),
                   "boundary_runs": bounds, "engine_s": engine_s, "pool_s": pool_s,
                   "s_runs": {k: [round(x, 4) for x in v] for k, v in runs.items()}}
            res["geoms"][f"{kib}K"] = rec
            print(kib, "KiB:", g, "boundaries", bounds, "engine_s", engine_s, "pool_s", pool_s, flush=True)
        finally:
            if os.path.exists(path):
                os.unlink(path)
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
