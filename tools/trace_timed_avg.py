"""Per-dispatch durations of one kernel from a rocprofv3 kernel trace.

rocprofv3's --stats average covers every dispatch of the profiled command,
including bench.py's untimed warm-up dispatches, which run while the clock is
still ramping (the first one is ~25 % slower).  bench.py's `roofline.kernel_ms`
is the mean over the K timed steps only.  This prints both, so the profile and
the bench line can be compared like for like:

    python tools/trace_timed_avg.py <kernel_trace.csv> [--kernel sha1_uniform] [--timed K]
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="sha1_uniform_kernel")
    ap.add_argument("--timed", type=int, default=None,
                    help="number of trailing dispatches that are bench.py's timed steps")
    a = ap.parse_args()
    with open(a.trace) as f:
        rows = [r for r in csv.DictReader(f) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    out = {"kernel": a.kernel, "dispatches": len(ms),
           "all_avg_ms": round(sum(ms) / len(ms), 4) if ms else None,
           "min_ms": round(min(ms), 4) if ms else None,
           "per_dispatch_ms": [round(x, 3) for x in ms]}
    if a.timed:
        t = ms[-a.timed:]
        out["timed"] = len(t)
        out["timed_avg_ms"] = round(sum(t) / len(t), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
