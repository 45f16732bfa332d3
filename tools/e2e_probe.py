#!/usr/bin/env python3
"""Host-resident e2e path only (bench.e2e_rate), for timeline profiling:
rocprofv3 --kernel-trace --memory-copy-trace -- python3 tools/e2e_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--pieces", type=int, default=8192)
    ap.add_argument("--piece-len", type=int, default=262144)
    a = ap.parse_args()
    print(json.dumps(bench.e2e_rate(a.piece_len, a.pieces)))
