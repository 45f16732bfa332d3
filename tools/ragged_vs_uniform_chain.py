#!/usr/bin/env python3
"""Per-block time of the split kernels on a chain-bound batch, alone on the
chip: the same N x L pieces through the uniform split kernel and the ragged
split kernel (offsets/lens of the same layout).  Tells whether config 3's
longest-chain time is the ragged kernel's own per-block cost
or the rest of the batch sharing the chip.  Prints one JSON line.

usage: python tools/ragged_vs_uniform_chain.py [--pieces 1024] [--piece-len 4194304] [--reps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pieces", type=int, default=1024)
    ap.add_argument("--piece-len", type=int, default=4 << 20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from vortex_amd import device as vdev

    n, L = a.pieces, a.piece_len
    stride = (L + 15) // 16 * 16
    dev = torch.device("cuda", 0)
    data = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    vdev.synth_fill(data, n, L, stride=stride, seed=7)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * stride
    lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    blocks = (L + 9 + 63) // 64

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = []
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            best.append(s.elapsed_time(e))
        return sorted(best)[len(best) // 2]

    du, _ = vdev.sha1_uniform(data, n, L, stride=stride, variant=2)
    dr, _ = vdev.sha1_ragged(data, offs, lens, variant=2)
    torch.cuda.synchronize()
    assert torch.equal(du, dr)
    tu = timed(lambda: vdev.sha1_uniform(data, n, L, stride=stride, variant=2))
    tr = timed(lambda: vdev.sha1_ragged(data, offs, lens, variant=2))
    print(json.dumps({"pieces": n, "piece_len": L, "blocks_per_piece": blocks,
                      "uniform_split_ms": round(tu, 3), "ragged_split_ms": round(tr, 3),
                      "uniform_us_per_block": round(tu * 1e3 / blocks, 4),
                      "ragged_us_per_block": round(tr * 1e3 / blocks, 4)}))


if __name__ == "__main__":
    main()
