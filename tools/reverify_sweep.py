#!/usr/bin/env python3
"""Config 5 re-verify: A/B of round schedules.

Writes the linux-mint-geometry file once (as tools/reverify_bench.py does),
then for each rep runs every configuration once, interleaved, so page-cache
and clock drift hit all of them alike.  A configuration is a set of env
variables read at vx_create (VX_VERIFY_CHUNK, VX_VERIFY_RAMP, ...), so each
gets its own context.  Prints one JSON line: per config, every rep's GiB/s.

usage: python tools/reverify_sweep.py --configs 'VX_VERIFY_CHUNK=262144' \\
           'VX_VERIFY_CHUNK=65536,VX_VERIFY_RAMP=1' [--reps 5] [--scale 1.0]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", required=True)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--piece-len", type=int, default=2097152,
                    help="piece length over the same file size (<= 256 KiB takes the whole-piece path)")
    ap.add_argument("--cpu-between", action="store_true",
                    help="run the CPU pool restatement before every GPU run (as reverify_bench does)")
    a = ap.parse_args()
    import torch  # noqa: F401  (single HIP runtime)

    import oracle
    from vortex_amd.hash_pool import HashPool

    pl = a.piece_len
    total = 2907832320 if a.scale >= 1.0 else int(2907832320 * a.scale) // 2097152 * 2097152 + 1179648
    n = (total + pl - 1) // pl
    last = total - (n - 1) * pl
    path = os.path.join(a.dir, "vx_reverify_sweep.iso")
    buf = ctypes.create_string_buffer(pl)
    with open(path, "wb") as f:
        for i in range(n):
            L = last if i == n - 1 else pl
            oracle.lib().vxo_gen_piece(0x5EED0005, i, L, 0, buf)
            f.write(buf.raw[:L])
    exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=a.threads)
    envs = []
    for c in a.configs:
        env = dict(kv.split("=", 1) for kv in c.split(",") if kv and kv != "default")
        envs.append(env)
    pools = []
    for env in envs:
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        pools.append(HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=max(4096, (512 << 20) // pl)))
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    res = {c: [] for c in a.configs}
    GiB = float(1 << 30)
    try:
        for pool in pools:  # one untimed pass each (first-call allocations)
            got, bad = pool.verify_files([path], [total], pl, exp, io_threads=a.threads)
            assert all(got) and bad == 0
        for rep in range(a.reps):
            for c, pool in zip(a.configs, pools):
                if a.cpu_between:
                    assert all(oracle.pool_verify_files([path], [total], pl, exp, threads=a.threads))
                t0 = time.perf_counter()
                got, bad = pool.verify_files([path], [total], pl, exp, io_threads=a.threads)
                t = time.perf_counter() - t0
                assert all(got) and bad == 0
                res[c].append(round(total / t / GiB, 2))
            print(f"rep {rep} done", file=sys.stderr, flush=True)
    finally:
        for p in pools:
            p.close()
        os.unlink(path)
    out = {"workload": f"re-verify {n} x {pl} B pieces ({total} B) from a warm file, {a.threads} io threads",
           "GiBps": res, "median": {c: sorted(v)[len(v) // 2] for c, v in res.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
