#!/usr/bin/env python3
"""A/B the uniform-batch kernel variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Checks every variant's digests are
identical, then prints per-variant median/min kernel ms and GB/s.

usage: python tools/ab_uniform.py [--pieces 65536] [--piece-len 262144] [--variants 1,2] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pieces", type=int, default=65536)
    ap.add_argument("--piece-len", type=int, default=262144)
    ap.add_argument("--variants", default="1,2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from vortex_amd import device as vdev

    n, plen = a.pieces, a.piece_len
    stride = (plen + 15) // 16 * 16
    variants = [int(v) for v in a.variants.split(",")]
    data = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    vdev.synth_fill(data, n, plen, stride=stride, seed=77)
    ref = None
    for v in variants:
        d, _ = vdev.sha1_uniform(data, n, plen, stride=stride, variant=v)
        torch.cuda.synchronize()
        if v == 6:  # diagnostic variant computes different digests on purpose
            continue
        if ref is None:
            ref = d.clone()
        assert torch.equal(ref, d), f"variant {v} digests differ"
    times = {v: [] for v in variants}
    scratch = torch.empty_like(ref)
    for _ in range(a.rounds):
        for v in variants:
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                vdev.sha1_uniform(data, n, plen, stride=stride, digests=scratch, variant=v)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1))
    out = {}
    for v in variants:
        med = statistics.median(times[v])
        out[v] = {"median_ms": round(med, 4), "min_ms": round(min(times[v]), 4),
                  "GBps_median": round(n * plen / med / 1e6, 1), "GiBps_median": round(n * plen / med / 1e3 / (1 << 30) * 1e6 / 1e3, 1)}
    print(json.dumps({"pieces": n, "piece_len": plen, "results": out}))


if __name__ == "__main__":
    main()
