#!/usr/bin/env python3
"""Print a merged copy/kernel (and optional HIP API) timeline from a
rocprofv3 --kernel-trace --memory-copy-trace [--hip-runtime-trace] CSV dir.

usage: python tools/timeline.py <dir> [prefix] [--api]"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    prefix = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    api = "--api" in sys.argv
    rows = []

    def one(pat):
        f = glob.glob(os.path.join(d, "**", f"{prefix}*{pat}"), recursive=True)
        return f[0] if f else None

    f = one("memory_copy_trace.csv")
    if f:
        for r in csv.DictReader(open(f)):
            rows.append(("copy", r["Direction"].replace("MEMORY_COPY_", ""), r.get("Stream_Id", ""),
                         int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    f = one("kernel_trace.csv")
    if f:
        for r in csv.DictReader(open(f)):
            rows.append(("kern", r["Kernel_Name"][:44], r.get("Stream_Id", ""), int(r["Start_Timestamp"]),
                         int(r["End_Timestamp"])))
    f = one("hip_api_trace.csv")
    if f and api:
        for r in csv.DictReader(open(f)):
            if r["Function"] in ("hipMemcpyAsync", "hipStreamWaitEvent", "hipEventRecord", "hipEventQuery",
                                 "hipEventSynchronize", "hipLaunchKernel", "hipExtLaunchKernel",
                                 "hipModuleLaunchKernel", "hipStreamSynchronize", "hipMemcpy"):
                rows.append(("api", r["Function"], r.get("Thread_Id", ""), int(r["Start_Timestamp"]),
                             int(r["End_Timestamp"])))
    rows.sort(key=lambda x: x[3])
    if not rows:
        print("no rows")
        return
    t0 = rows[0][3]
    for kind, name, st, a, b in rows:
        print(f"{kind} {name:46s} {st:>4} {(a - t0) / 1e6:10.3f} {(b - t0) / 1e6:10.3f}  dur {(b - a) / 1e6:8.3f}")


if __name__ == "__main__":
    main()
