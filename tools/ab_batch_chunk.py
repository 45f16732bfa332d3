#!/usr/bin/env python3
"""A/B the host-batch e2e path (bench.e2e_rate: registered mmap -> vx_verify_batch
-> verdicts + digests) over chunk sizes, in one process, interleaved rounds.
VX_BATCH_CHUNK=0 is the whole-piece slot path; other values are the strided
chunk path of DESIGN.md §6.4.  Prints one JSON line (GiB/s, best and median).

usage: python tools/ab_batch_chunk.py [--geoms 262144x8192,2097152x1024] [--chunks 0,32768,65536,131072] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--geoms", default="262144x8192,2097152x1024")
    ap.add_argument("--chunks", default="0,32768,65536,131072")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    geoms = [tuple(int(x) for x in g.split("x")) for g in a.geoms.split(",")]
    chunks = [int(c) for c in a.chunks.split(",")]
    res = {f"{pl}x{n}": {c: [] for c in chunks} for pl, n in geoms}
    h2d = {}
    for _ in range(a.rounds):
        for pl, n in geoms:
            for c in chunks:
                os.environ["VX_BATCH_CHUNK"] = str(c)
                r = bench.e2e_rate(pl, n)
                res[f"{pl}x{n}"][c].append(r["value"])
                h2d[f"{pl}x{n}"] = r["pinned_h2d_copy_GiBps"]
                print(f"{pl}x{n} chunk={c}: {r['value']} GiB/s", file=sys.stderr, flush=True)
    out = {g: {str(c): {"best": max(v), "median": round(statistics.median(v), 3)} for c, v in d.items()}
           for g, d in res.items()}
    print(json.dumps({"e2e_GiBps": out, "pinned_h2d_GiBps": h2d}))


if __name__ == "__main__":
    main()
