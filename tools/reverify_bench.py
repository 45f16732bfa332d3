#!/usr/bin/env python3
"""Config 5: full re-verify of a torrent's data from disk, end to end
(pread -> pinned host -> H2D -> kernel -> D2H verdicts), next to the CPU
restatement of vortex's own re-verify (par_iter over check_piece_hash_sync,
oracle/pool_oracle.cpp) on the same host cores and the same file.

The linux-mint ISO is not available offline, so a file with the exact
geometry of cli/linux-mint.torrent (2,907,832,320 B, 2 MiB pieces, last
1,179,648 B) is synthesised; verdicts are checked against digests of the
synthetic data (and every piece must match).

usage: python tools/reverify_bench.py [--dir /tmp] [--scale 1.0] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the linux-mint size")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--slot-mib", type=int, default=512)
    a = ap.parse_args()
    import ctypes

    import torch  # noqa: F401  (single HIP runtime)

    import oracle
    from vortex_amd.hash_pool import HashPool

    pl = 2097152
    total = 2907832320 if a.scale >= 1.0 else int(2907832320 * a.scale) // pl * pl + 1179648
    n = (total + pl - 1) // pl
    last = total - (n - 1) * pl
    threads = a.threads or max(1, min(16, len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16"))))
    path = os.path.join(a.dir, "vx_linuxmint_synth.iso")
    t0 = time.perf_counter()
    buf = ctypes.create_string_buffer(pl)
    with open(path, "wb") as f:
        for i in range(n):
            L = last if i == n - 1 else pl
            oracle.lib().vxo_gen_piece(0x5EED0005, i, L, 0, buf)
            f.write(buf.raw[:L])
    t_write = time.perf_counter() - t0
    exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
    res = {"workload": f"re-verify {n} x 2 MiB pieces ({total} B, linux-mint geometry) from a file",
           "file_bytes": total, "write_s": round(t_write, 2), "threads": threads, "runs": []}
    GiB = float(1 << 30)
    with HashPool(pl, slots=a.slots, slot_bytes=a.slot_mib << 20, batch_pieces=4096) as pool:
        for rep in range(a.reps):
            t0 = time.perf_counter()
            got, bad = pool.verify_files([path], [total], pl, exp, io_threads=threads)
            tg = time.perf_counter() - t0
            assert all(got) and bad == 0
            t0 = time.perf_counter()
            cpu = oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
            tc = time.perf_counter() - t0
            assert all(cpu)
            res["runs"].append({"gpu_e2e_GiBps": round(total / tg / GiB, 2), "gpu_s": round(tg, 3),
                                "cpu_pool_GiBps": round(total / tc / GiB, 2), "cpu_s": round(tc, 3)})
    best_g = max(r["gpu_e2e_GiBps"] for r in res["runs"])
    best_c = max(r["cpu_pool_GiBps"] for r in res["runs"])
    res["best"] = {"gpu_e2e_GiBps": best_g, "cpu_pool_GiBps": best_c}
    res["note"] = "file is page-cache resident after the write (warm); both legs read the same file"
    if not a.keep:
        os.unlink(path)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
