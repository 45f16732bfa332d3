#!/usr/bin/env python3
"""Where the warm config-5 re-verify's copy engine idles:
vx_verify_files over the linux-mint-geometry file for several context shapes,
alternating, each call's round timeline (vx_last_verify_rounds) reduced by
bench.copy_gaps to gaps by cause and by slot.  Prints one JSON line.

Shapes: "<slots>[s][h]"; "<slots>" (the engine's default: data copies on the context's copy
stream, lane tables on the slot streams) or "<slots>s" (each copy on its
slot's stream, round 4's form): vx_tuning_verify_copy_stream(ctx, 1 / 0),
test build; "h": pinned stages on huge pages (vx_tuning_stage_huge).  (Round 5 also measured the tables on the copy stream, and a
normal-priority copy stream: EXPERIMENTS.md §6.3.)

With --split "io:pool:gpu_frac,...": instead, the split of DESIGN.md §6.6
(bench.split_call: the engine on the tail with `io` readers while the CPU
pool restatement verifies the head on `pool` threads), gpu_frac of the pieces
on the GPU, configs alternating call by call.

usage: python tools/reverify_gaps.py [--reps 5] [--slots 4,4s,6,6s] [--scale 1.0]
       python tools/reverify_gaps.py --split 8:16:0.55,8:8:0.6,4:12:0.55 [--reps 9]
       python tools/reverify_gaps.py --cold 0,0h,1048576 [--reps 5]
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--slots", default="4,4s,6,6s")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--split", default="")
    ap.add_argument("--geometry", default="", help="N:MiB = N pieces of MiB each instead of linux-mint's")
    ap.add_argument("--cold", default="", help="cold A/B instead: verify_cold_chunk values, e.g. 0,1048576,0h (h: "
                                               "huge-page stages); each evicted call followed by the disk alone")
    a = ap.parse_args()
    import bench
    import oracle

    pl = 2097152
    if a.geometry:
        pl = int(a.geometry.split(":")[1]) << 20
    threads = bench.cpu_share()
    path = os.path.join(bench.reverify_dir(), f"vx_gaps_{os.getpid()}.iso")
    out = {"threads": threads, "shapes": {}}
    try:
        if a.geometry:
            n = int(a.geometry.split(":")[0])
            total, last = n * pl, pl
            import ctypes

            buf = ctypes.create_string_buffer(pl)
            with open(path, "wb") as f:
                for i in range(n):
                    oracle.lib().vxo_gen_piece(0x5EED0005, i, pl, 0, buf)
                    f.write(buf.raw)
                f.flush()
                os.fsync(f.fileno())
        else:
            total, n, last = bench.write_linuxmint_file(path, a.scale)
        exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
        if a.cold:
            out["cold"] = cold_ab(a, path, total, n, pl, exp, threads)
        elif a.split:
            out["split"] = split_sweep(a, path, total, n, pl, exp)
        else:
            slots_ab(a, out, path, total, n, pl, exp, threads)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    print(json.dumps(out))


def slots_ab(a, out, path, total, n, pl, exp, threads):
    import bench
    from vortex_amd.hash_pool import HashPool

    shapes = a.slots.split(",")
    pools = {}
    for s in shapes:  # "<slots>[s][h]": s = slot-stream copies, h = huge-page stages
        pools[s] = HashPool(pl, slots=int(s.rstrip("sh")), slot_bytes=512 << 20, batch_pieces=4096, hooks=True)
        pools[s].lib.vx_tuning_verify_copy_stream(pools[s]._h, 0 if s.rstrip("h").endswith("s") else 1)
        pools[s].lib.vx_tuning_stage_huge(pools[s]._h, int(s.endswith("h")))
    runs = {s: [] for s in shapes}
    for s, pool in pools.items():  # warm every context (stages, rows, page cache)
        got, bad = pool.verify_files([path], [total], pl, exp, io_threads=threads)
        assert all(got) and bad == 0
    for _ in range(a.reps):
        for s, pool in pools.items():
            t0 = time.perf_counter()
            got, bad = pool.verify_files([path], [total], pl, exp, io_threads=threads)
            el = time.perf_counter() - t0
            assert all(got) and bad == 0
            rounds = pool.last_verify_rounds()
            tr = pool.last_verify()
            g = bench.copy_gaps(rounds)
            by_slot = {}
            ns = int(s.rstrip("sh"))
            for k in range(1, len(rounds)):
                gap = rounds[k]["copy_start_ms"] - rounds[k - 1]["copy_end_ms"]
                by_slot[k % ns] = round(by_slot.get(k % ns, 0.0) + max(0.0, gap), 3)
            # copies that started within 0.1 ms of the previous round's kernel end
            after_kernel = sum(1 for k in range(1, len(rounds))
                               if 0 <= rounds[k]["copy_start_ms"] - rounds[k - 1]["kernel_end_ms"] < 0.1)
            runs[s].append({"GiBps": round(total / el / (1 << 30), 2), "copy_busy_frac": round(tr["copy_busy_frac"], 3),
                            "copy_GiBps": round(tr["copy_GiBps"], 2), "read_GiBps": round(tr["read_GiBps"], 2),
                            "wall_ms": round(tr["wall_ms"], 2), "copy_span_ms": round(tr["copy_span_ms"], 2),
                            "first_copy_ms": g["first_copy_start_ms"],
                            "gap_ms": g["gap_ms"], "by_cause": g["by_cause"], "gap_ms_by_slot": by_slot,
                            "copy_after_prev_kernel": after_kernel})
    for s in shapes:
        r = sorted(runs[s], key=lambda x: x["GiBps"])
        out["shapes"][f"slots{s}"] = {"median_GiBps": r[len(r) // 2]["GiBps"], "runs": runs[s]}
    for p in pools.values():
        p.close()


def cold_ab(a, path, total, n, pl, exp, threads):
    """Evicted re-verify calls per verify_cold_chunk value, alternating, each
    followed by the disk's own O_DIRECT rate over the same evicted file."""
    import bench
    from vortex_amd.hash_pool import HashPool

    # "<verify_cold_chunk>[h][w][@<slot MiB>][x<readers>]": h = huge-page stages (vx_tuning_stage_huge),
    # w = whole pieces (verify_chunk above half the piece: the whole-piece slots)
    chunks = a.cold.split(",")
    pools, readers = {}, {}
    for ch in chunks:
        spec, _, mib = ch.partition("x")[0].partition("@")
        readers[ch] = int(ch.partition("x")[2] or threads)
        extra = {"verify_chunk": 2 * pl} if "w" in spec else {}
        pools[ch] = HashPool(pl, slots=4, slot_bytes=int(mib or 512) << 20, batch_pieces=4096,
                             verify_cold_chunk=int(spec.rstrip("hw")), hooks=True, **extra)
        pools[ch].lib.vx_tuning_stage_huge(pools[ch]._h, int("h" in spec))
    res = {ch: [] for ch in chunks}
    for ch, pool in pools.items():
        pool.verify_files([path], [total], pl, exp, io_threads=threads)
    for _ in range(a.reps):
        for ch, pool in pools.items():
            bench.drop_cache(path)
            t0 = time.perf_counter()
            got, bad = pool.verify_files([path], [total], pl, exp, io_threads=readers[ch])
            el = time.perf_counter() - t0
            assert all(got) and bad == 0
            tr = pool.last_verify()
            bench.drop_cache(path)
            disk = bench.disk_direct_rate(path, total, threads)
            res[ch].append({"GiBps": round(total / el / (1 << 30), 2), "disk_GiBps": disk and round(disk, 2),
                            "chunk_bytes": tr["chunk_bytes"], "copy_busy_frac": tr["copy_busy_frac"] and round(tr["copy_busy_frac"], 3),
                            "read_GiBps": round(tr["read_GiBps"], 2)})
    for p in pools.values():
        p.close()
    out = {}
    for ch, runs in res.items():
        r = sorted(x["GiBps"] for x in runs)
        out[ch] = {"median_GiBps": r[len(r) // 2], "runs": runs}
    return out


def split_sweep(a, path, total, n, pl, exp):
    import bench
    from vortex_amd.hash_pool import HashPool

    cfgs = [tuple(x.split(":")) for x in a.split.split(",")]
    res = {c: [] for c in cfgs}
    with HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=4096) as pool:
        pool.verify_files([path], [total], pl, exp, io_threads=8)
        for _ in range(a.reps):
            for c in cfgs:
                io_t, pool_t, frac = int(c[0]), int(c[1]), float(c[2])
                first = n - int(round(n * frac))
                r = bench.split_call(pool, [path], [total], n, pl, exp, first, io_t, pool_t)
                assert r["ok"]
                res[c].append((round(r["s"] * 1e3, 2), round(r["gpu_s"] * 1e3, 2), round(r["cpu_s"] * 1e3, 2)))
    out = {}
    for c, v in res.items():
        med = sorted(v)[len(v) // 2]
        out[":".join(c)] = {"median_GiBps": round(total / (med[0] * 1e-3) / (1 << 30), 2),
                            "runs_ms_total_gpu_cpu": v}
    return out


if __name__ == "__main__":
    main()
