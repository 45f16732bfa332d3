#!/usr/bin/env python3
"""Device-resident ragged batches: BASELINE config 3 (16 KiB / 256 KiB / 1 MiB /
4 MiB, 4 GiB each, shuffled, longest-first lane order) and the config-5
geometry (1,387 x 2 MiB, last 1,179,648 B).  A/B of the ragged kernel
variants (1 = lane, 2 = split, 0 = the default kernel planned from the host
lengths, vx_sha1_device_ragged_hint) interleaved in one process; digests of
the variants must agree.

usage: python tools/ragged_bench.py [--scale 1.0] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(torch, vdev, classes, dev, seed_base):
    total = sum(L * n for L, n in classes)
    data = torch.empty(total, dtype=torch.uint8, device=dev)
    offs, lens, o = [], [], 0
    for k, (L, n) in enumerate(classes):
        vdev.synth_fill(data[o:o + L * n], n, L, seed=seed_base + k)
        offs.append(np.arange(n, dtype=np.int64) * L + o)
        lens.append(np.full(n, L, dtype=np.int32))
        o += L * n
    offs, lens = np.concatenate(offs), np.concatenate(lens)
    perm = np.random.default_rng(seed_base).permutation(len(offs))
    return data, offs[perm], lens[perm], total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="1,2,0", help="1 lane, 2 split, 0 default planned from host lengths")
    a = ap.parse_args()
    import torch

    from vortex_amd import device as vdev

    dev = torch.device("cuda:0")
    s = a.scale
    cfgs = {
        "config3_ragged_16GiB": [(16384, int(262144 * s)), (262144, int(16384 * s)), (1 << 20, int(4096 * s)),
                                 (4 << 20, max(1, int(1024 * s)))],
        "config5_geometry": None,
    }
    out = {}
    for name, classes in cfgs.items():
        if classes is None:
            n, pl, last = 1387, 2097152, 1179648
            data = torch.empty(n * pl, dtype=torch.uint8, device=dev)
            vdev.synth_fill(data, n - 1, pl, seed=0x5EED0005)
            vdev.synth_fill(data[(n - 1) * pl:], 1, last, first=n - 1, seed=0x5EED0005)
            offs = np.arange(n, dtype=np.int64) * pl
            lens = np.full(n, pl, dtype=np.int32)
            lens[-1] = last
            total = int(lens.sum())
        else:
            data, offs, lens, total = build(torch, vdev, classes, dev, 0x5EED0003)
        d_off = torch.from_numpy(offs).to(dev)
        d_len = torch.from_numpy(lens).to(dev)
        order = vdev.length_order(lens).to(dev)
        ref = None
        variants = [int(v) for v in a.variants.split(",")]
        names = {0: "default_planned", 1: "lane", 2: "split", 11: "split_opaque"}
        plan = vdev.ragged_plan(lens)
        times = {v: [] for v in variants}
        for r in range(a.rounds + 1):
            for v in variants:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                dig, _ = vdev.sha1_ragged(data, d_off, d_len, order=order, variant=v,
                                          plan=plan if v == 0 else None)
                e1.record()
                torch.cuda.synchronize()
                if ref is None:
                    ref = dig.clone()
                assert torch.equal(ref, dig), f"{name}: variant {v} differs"
                if r:
                    times[v].append(e0.elapsed_time(e1))
        res = {}
        for v in variants:
            med = statistics.median(times[v])
            res[names.get(v, str(v))] = {"median_ms": round(med, 3),
                                                  "GiBps": round(total / (med * 1e-3) / (1 << 30), 1)}
        out[name] = {"pieces": int(len(lens)), "bytes": int(total), "results": res}
        del data, d_off, d_len, ref
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
