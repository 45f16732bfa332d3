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

Under torch.distributed.run (WORLD_SIZE > 1) every rank verifies its shard of
the pieces on its own GPU (shard.verify_files_sharded): the
time is the max over ranks, bracketed by barriers, and the CPU leg is skipped.
Rank 0 writes the file; ranks on one host read the same page cache.
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

    import torch  # (single HIP runtime)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        return dist_main(a, world)

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


def dist_main(a, world):
    import ctypes

    import torch
    import torch.distributed as dist

    import oracle
    from vortex_amd import shard
    from vortex_amd.hash_pool import HashPool

    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")  # verdict gather of a few KiB; the payload never crosses ranks
    rank = dist.get_rank()
    pl = 2097152
    total = 2907832320 if a.scale >= 1.0 else int(2907832320 * a.scale) // pl * pl + 1179648
    n = (total + pl - 1) // pl
    last = total - (n - 1) * pl
    threads = a.threads or max(1, min(16, len(os.sched_getaffinity(0))) // world)
    path = os.path.join(a.dir, "vx_linuxmint_synth.iso")
    if rank == 0:
        buf = ctypes.create_string_buffer(pl)
        with open(path, "wb") as f:
            for i in range(n):
                L = last if i == n - 1 else pl
                oracle.lib().vxo_gen_piece(0x5EED0005, i, L, 0, buf)
                f.write(buf.raw[:L])
    exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
    dist.barrier()
    runs = []
    with HashPool(pl, device=dev, slots=a.slots, slot_bytes=a.slot_mib << 20, batch_pieces=4096) as pool:
        for rep in range(a.reps):
            dist.barrier()
            t0 = time.perf_counter()
            got, bad = shard.verify_files_sharded(pool, [path], [total], pl, exp, io_threads=threads)
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            assert all(got) and bad == 0
            runs.append({"gpu_e2e_GiBps": round(total / t.item() / float(1 << 30), 2), "s": round(t.item(), 3)})
    dist.barrier()
    if rank == 0:
        print(json.dumps({"workload": f"sharded re-verify {n} x 2 MiB pieces ({total} B) over {world} ranks",
                          "ranks": world, "gpus": torch.cuda.device_count(), "threads_per_rank": threads,
                          "runs": runs, "best_GiBps": max(r["gpu_e2e_GiBps"] for r in runs)}))
        if not a.keep:
            os.unlink(path)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
