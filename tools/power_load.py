#!/usr/bin/env python3
"""Sustained config-2 load for the power/clock probe (tools/gpu_power_probe.sh).

Runs the default uniform kernel over 65,536 x 256 KiB pieces back to back for
--seconds and prints one JSON line: per-launch kernel ms (HIP events on the
launch stream), median and first/last, so the clock the sampler sees can be
matched with the kernel time of the same period.

usage: python tools/power_load.py [--seconds 12] [--pieces 65536] [--piece-len 262144]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=12.0)
    ap.add_argument("--pieces", type=int, default=65536)
    ap.add_argument("--piece-len", type=int, default=262144)
    ap.add_argument("--variant", type=int, default=0)
    a = ap.parse_args()
    import torch

    from vortex_amd import device as vdev

    n, plen = a.pieces, a.piece_len
    stride = (plen + 15) // 16 * 16
    data = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    vdev.synth_fill(data, n, plen, stride=stride, seed=11)
    dig = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    times, stamps = [], []
    t0 = time.perf_counter()
    print(json.dumps({"event": "start", "t": time.time()}), flush=True)
    while time.perf_counter() - t0 < a.seconds:
        evs = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            vdev.sha1_uniform(data, n, plen, stride=stride, digests=dig, stream=s, variant=a.variant)
            e1.record(s)
            evs.append((e0, e1))
        torch.cuda.synchronize()
        times += [x.elapsed_time(y) for x, y in evs]
        stamps.append(round(time.perf_counter() - t0, 3))
    print(json.dumps({"event": "done", "t": time.time(), "launches": len(times),
                      "median_ms": round(statistics.median(times), 4), "min_ms": round(min(times), 4),
                      "first20_median_ms": round(statistics.median(times[:20]), 4),
                      "last20_median_ms": round(statistics.median(times[-20:]), 4),
                      "GBps_median": round(n * plen / statistics.median(times) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
