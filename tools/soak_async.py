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

With --faults, pools also get injected failures (vx_tuning.h): non-sticky
VX_ENOMEM submits now and then, and in some pools one launch that fails like
a device error (inside vx_submit, vx_flush or vx_poll's lazy launch,
whichever comes).  The ownership rule (include/vx_hash.h) is then checked:
every piece comes back exactly once — polled, refused by its spawn (the soak
hashes it itself), or handed back by take_unfinished() after the pool died —
and the counters of pools that stayed alive still agree.

usage: python tools/soak_async.py [--seconds 90] [--seed 1] [--faults]
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
    ap.add_argument("--faults", action="store_true", help="inject submit and launch failures")
    a = ap.parse_args()
    import oracle
    from vortex_amd._lib import VX_EDEVICE, VX_ENOMEM, VxError, lib
    from vortex_amd.hash_pool import HashPool

    rng = random.Random(a.seed)
    t_end = time.time() + a.seconds
    stats = {"pools": 0, "pieces": 0, "bytes": 0, "mismatches_expected": 0, "refused": 0, "dead_pools": 0,
             "unfinished": 0}

    def bad(what, **kw):
        print(json.dumps({"error": what, **kw}))
        return 1
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
            dead = False
            if a.faults and rng.random() < 0.3:
                lib().vx_tuning_fail_launch_after(pool._h, rng.randint(0, 12))
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
                if a.faults and rng.random() < 0.02:
                    lib().vx_tuning_fail_submit_after(pool._h, 0)
                try:
                    pool.spawn(tag, 7, memoryview(buf)[:plen] if isinstance(buf, mmap.mmap) else buf, L, exp)
                except VxError as e:
                    # not taken (the ownership rule): the caller hashes it itself
                    if e.refused is None or e.refused[0] != tag or e.code not in (VX_ENOMEM, VX_EDEVICE):
                        return bad("refused without the piece", code=e.code, index=tag)
                    stats["refused"] += 1
                    tag += 1
                    if e.code == VX_EDEVICE:
                        dead = True
                        break
                    continue
                own["pieces"] += 1
                own["bad"] += exp != good
                own["bytes"] += L
                own["staged"] += 0 if isinstance(buf, mmap.mmap) else L
                inflight[tag] = (good, exp == good, buf)
                tag += 1
                stats["pieces"] += 1
                stats["bytes"] += L
                try:
                    if rng.random() < 0.2:
                        pool.flush()
                    if rng.random() < 0.3:
                        for r in pool.try_iter():
                            if r.index not in inflight:
                                return bad("unknown or duplicate completion", index=r.index, plen=plen)
                            good, ok, _ = inflight.pop(r.index)
                            if r.digest != good or r.hash_matched != ok:
                                return bad("wrong result", index=r.index, plen=plen)
                except VxError as e:
                    if e.code != VX_EDEVICE:
                        return bad("unexpected error", code=e.code)
                    dead = True
                    break
            if not dead:
                try:
                    pool.drain()
                except VxError as e:
                    if e.code != VX_EDEVICE:
                        return bad("unexpected error", code=e.code)
                    dead = True
            while True:  # a dead pool hands out every finished result, then the error
                try:
                    got = pool.try_iter()
                except VxError as e:
                    if not dead or e.code != VX_EDEVICE:
                        return bad("unexpected error", code=e.code)
                    break
                for r in got:
                    if r.index not in inflight:
                        return bad("unknown or duplicate completion", index=r.index, plen=plen)
                    good, ok, _ = inflight.pop(r.index)
                    if r.digest != good or r.hash_matched != ok:
                        return bad("wrong result", index=r.index, plen=plen)
                if not dead:
                    break
            if dead:
                stats["dead_pools"] += 1
                pending = pool.pending
                lost = pool.take_unfinished()
                if len(lost) != pending or sorted(i for i, _, _ in lost) != sorted(inflight):
                    return bad("unfinished set differs", pending=pending, lost=len(lost), left=len(inflight))
                for i, _, b in lost:  # the caller's own pool takes these over
                    good, _, want_buf = inflight.pop(i)
                    if b is not want_buf and not (isinstance(want_buf, mmap.mmap)):
                        return bad("unfinished piece lost its buffer", index=i)
                stats["unfinished"] += len(lost)
                pool.close()  # waits for the device before the buffers are reused
                continue
            if inflight:
                return bad("lost completions", n=len(inflight), plen=plen)
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
