#!/usr/bin/env python3
"""Soak the async download path (vx_submit / vx_flush / vx_poll) for a fixed
time: random piece lengths (empty to 3 MiB), pieces in registered pool
buffers (gather kernel) and in plain memory (staged), random mismatches,
random flush and poll cadence, pools of different piece lengths re-created
now and then.  Every completion is checked against hashlib; any mismatch,
loss or duplicate exits non-zero.  At the end of each pool the engine's
counters (vx_get_stats) must agree with the soak's own: pieces, planted
mismatches, bytes, staged bytes and batch-latency bookkeeping.  Prints one
JSON line.

usage: python tools/soak_async.py [--seconds 90] [--seed 1]
"""
import argparse
import hashlib
import json
import mmap
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=90)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    import oracle
    from vortex_amd.hash_pool import HashPool

    rng = random.Random(a.seed)
    t_end = time.time() + a.seconds
    stats = {"pools": 0, "pieces": 0, "bytes": 0, "mismatches_expected": 0}
    while time.time() < t_end:
        plen = rng.choice([16384, 65536, 262144, 1 << 20, 3 << 20])
        nbuf = rng.randint(8, 64)
        with HashPool(plen, slots=rng.choice([2, 3, 4]), batch_pieces=rng.choice([4, 16, 64])) as pool:
            stats["pools"] += 1
            bufs = [mmap.mmap(-1, plen) for _ in range(nbuf)]
            for b in bufs:
                pool.register_buffer(b)
            inflight = {}
            tag = 0
            own = {"pieces": 0, "bad": 0, "bytes": 0, "staged": 0}
            for _ in range(rng.randint(50, 400)):
                L = rng.choice([0, 1, 55, 56, 64, plen, plen, plen, rng.randint(1, plen)])
                body = oracle.gen_piece(a.seed, tag, L)
                if rng.random() < 0.7:
                    buf = bufs[tag % nbuf]
                    if any(v[2] is buf for v in inflight.values()):
                        buf = bytearray(body)  # that pool buffer is still in flight
                    else:
                        buf[:L] = body
                else:
                    buf = bytearray(body)
                good = hashlib.sha1(body).digest()
                exp = good if rng.random() > 0.05 else bytes(20)
                stats["mismatches_expected"] += exp != good
                pool.spawn(tag, 7, memoryview(buf)[:plen] if isinstance(buf, mmap.mmap) else buf, L, exp)
                own["pieces"] += 1
                own["bad"] += exp != good
                own["bytes"] += L
                own["staged"] += 0 if isinstance(buf, mmap.mmap) else L
                inflight[tag] = (good, exp == good, buf)
                tag += 1
                stats["pieces"] += 1
                stats["bytes"] += L
                if rng.random() < 0.2:
                    pool.flush()
                if rng.random() < 0.3:
                    for r in pool.try_iter():
                        good, ok, _ = inflight.pop(r.index)
                        if r.digest != good or r.hash_matched != ok:
                            print(json.dumps({"error": "wrong result", "index": r.index, "plen": plen}))
                            return 1
            pool.drain()
            for r in pool.try_iter():
                good, ok, _ = inflight.pop(r.index)
                if r.digest != good or r.hash_matched != ok:
                    print(json.dumps({"error": "wrong result", "index": r.index, "plen": plen}))
                    return 1
            if inflight:
                print(json.dumps({"error": "lost completions", "n": len(inflight), "plen": plen}))
                return 1
            st = pool.stats()
            got = {"pieces": st["pieces_completed"], "bad": st["pieces_mismatched"], "bytes": st["bytes_completed"],
                   "staged": st["staged_bytes"]}
            if got != own or sum(st["batch_latency_hist"]) != st["batch_latency_count"] or \
                    st["batch_latency_count"] != st["batches"]:
                print(json.dumps({"error": "stats disagree", "engine": st, "soak": own, "plen": plen}))
                return 1
            for b in bufs:
                pool.unregister_buffer(b)
        print(f"pools {stats['pools']} pieces {stats['pieces']}", file=sys.stderr, flush=True)
    stats["GiB"] = round(stats.pop("bytes") / (1 << 30), 2)
    print(json.dumps({"ok": True, "seconds": a.seconds, "seed": a.seed, **stats}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
