#!/usr/bin/env python3
"""Same uniform batch through the uniform split kernel and the ragged split
kernel (offsets = i*len), interleaved in one process: isolates the ragged
kernel's structural overhead from batch raggedness."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pieces", type=int, default=8192)
    ap.add_argument("--piece-len", type=int, default=2097152)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    import torch

    from vortex_amd import device as vdev

    n, pl = a.pieces, a.piece_len
    data = torch.empty(n * pl, dtype=torch.uint8, device="cuda")
    vdev.synth_fill(data, n, pl, seed=3)
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * pl
    lens = torch.full((n,), pl, dtype=torch.int32, device="cuda")
    runs = {"uniform_split": lambda: vdev.sha1_uniform(data, n, pl, variant=2)[0],
            "ragged_split": lambda: vdev.sha1_ragged(data, offs, lens, variant=2)[0],
            "ragged_lane": lambda: vdev.sha1_ragged(data, offs, lens, variant=1)[0]}
    ref = None
    t = {k: [] for k in runs}
    for r in range(a.rounds + 1):
        for k, f in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            d = f()
            e1.record()
            torch.cuda.synchronize()
            if ref is None:
                ref = d.clone()
            assert torch.equal(ref, d), k
            if r:
                t[k].append(e0.elapsed_time(e1))
    print(json.dumps({k: round(statistics.median(v), 3) for k, v in t.items()}))


if __name__ == "__main__":
    main()
