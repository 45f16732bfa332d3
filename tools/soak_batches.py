#!/usr/bin/env python3
"""Soak the synchronous host-batch path (vx_verify_batch / vx_sha1_batch) for a
fixed time: random ragged batches (empty to 5 MiB pieces, shuffled), held in
one registered mmap (strided or gather paths), in separately registered
buffers, at unaligned addresses, or in plain memory (parallel stage copies),
with random slot counts and sizes, chunk sizes (vx_config.batch_chunk, 0 =
whole-piece slots) and planted mismatches.  Every digest and
verdict is checked against the CPU pool restatement (oracle/, the checker).
Prints a progress line per pool and one JSON line at the end; exits non-zero
on any difference.

usage: python tools/soak_batches.py [--seconds 120] [--seed 1]
"""
import argparse
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
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (torch's HIP runtime first, as vortex_amd expects)

    import oracle
    from vortex_amd.hash_pool import HashPool

    rng = random.Random(a.seed)
    gen = np.random.default_rng(a.seed)
    t_end = time.time() + a.seconds
    st = {"pools": 0, "batches": 0, "pieces": 0, "GiB": 0.0, "mismatches_planted": 0}
    while time.time() < t_end:
        batch_chunk = rng.choice([65536, 65536, 32768, 131072, 0])
        max_len = rng.choice([1 << 16, 1 << 20, 3 << 20, 5 << 20])
        classes = [0, 1, 63, 64, 65, 16384, 65536, 65537, 200000, 262144, 1 << 20, (1 << 20) + 48, 3 << 20, 5 << 20]
        classes = [L for L in classes if L <= max_len]
        slots = rng.choice([2, 3, 4])
        slot_bytes = rng.choice([None, max(max_len, 4 << 20), max(max_len, 64 << 20)])
        with HashPool(max_len, slots=slots, slot_bytes=slot_bytes, batch_chunk=batch_chunk) as pool:
            st["pools"] += 1
            for _ in range(rng.randint(1, 4)):
                n = rng.randint(1, 600)
                lens = [rng.choice(classes) for _ in range(n)]
                mode = rng.choice(["one_mmap", "per_buffer", "unaligned", "plain"])
                bufs, pieces = [], []
                if mode in ("one_mmap", "unaligned"):
                    offs, o = [], 0
                    for L in lens:
                        o += 5 if mode == "unaligned" else 0
                        offs.append(o)
                        o = (o + L + 15) // 16 * 16
                    b = mmap.mmap(-1, max(o, 1))
                    np.frombuffer(b, dtype=np.uint8)[:] = gen.integers(0, 256, len(b), dtype=np.uint8)
                    bufs.append(b)
                    mv = memoryview(b)
                    pieces = [mv[x:x + L] for x, L in zip(offs, lens)]
                elif mode == "per_buffer":
                    for L in lens:
                        b = mmap.mmap(-1, max(L, 1))
                        np.frombuffer(b, dtype=np.uint8)[:] = gen.integers(0, 256, len(b), dtype=np.uint8)
                        bufs.append(b)
                        pieces.append(memoryview(b)[:L])
                else:
                    pieces = [gen.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
                for b in bufs:
                    pool.register_buffer(b)
                want, _ = oracle.pool_verify([bytes(p) for p in pieces], threads=8)
                want = [want[20 * i:20 * i + 20] for i in range(n)]
                bad = {i for i in range(n) if rng.random() < 0.05}
                exp = [bytes(20) if i in bad else w for i, w in enumerate(want)]
                if rng.random() < 0.5:
                    matched, dig = pool.verify_batch(pieces, exp)
                    ok = dig == want and matched == [i not in bad for i in range(n)]
                else:
                    ok = pool.sha1_batch(pieces) == want
                pieces = None  # release the memoryviews before the mmaps go
                for b in bufs:
                    pool.unregister_buffer(b)
                if not ok:
                    print(json.dumps({"ok": False, "seed": a.seed, "mode": mode, "lens": lens,
                                      "batch_chunk": batch_chunk}), flush=True)
                    return 1
                st["batches"] += 1
                st["pieces"] += n
                st["mismatches_planted"] += len(bad)
                st["GiB"] += sum(lens) / float(1 << 30)
        print(f"pools {st['pools']} batches {st['batches']} pieces {st['pieces']}", file=sys.stderr, flush=True)
    st["GiB"] = round(st["GiB"], 2)
    print(json.dumps({"ok": True, "seconds": a.seconds, "seed": a.seed, **st}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
