#!/usr/bin/env python3
"""A/B two builds of libvortex_amd.so on ONE box: alternate child processes
(VX_LIB_OVERRIDE) running the same device-resident workloads, so clock and
box differences fall on both arms alike (cdna_hip_programming.md §5.4).
Prints one JSON line: per workload, each build's per-round median kernel ms.

usage: python tools/ab_builds.py --a tools/ab/libvortex_amd_base.so --b vortex_amd/libvortex_amd.so [--rounds 3]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOADS = {
    "config2_65536x256K_lane": ["tools/ab_uniform.py", "--variants", "0", "--rounds", "3"],
    "16384x256K_split": ["tools/ab_uniform.py", "--variants", "0", "--pieces", "16384", "--rounds", "3"],
    "8192x2MiB_split": ["tools/ab_uniform.py", "--variants", "0", "--pieces", "8192", "--piece-len", "2097152",
                        "--rounds", "2"],
    "ragged_config3_config5": ["tools/ragged_bench.py", "--variants", "0", "--rounds", "2"],
}


def run(lib, args):
    env = dict(os.environ, VX_LIB_OVERRIDE=os.path.abspath(lib))
    out = subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    if out.returncode:
        raise SystemExit(f"{args}: {out.stderr[-2000:]}")
    return json.loads(out.stdout.strip().splitlines()[-1])


def medians(res):
    if "results" in res:  # ab_uniform
        return {"ms": res["results"]["0"]["median_ms"]}
    return {k: v["results"]["default_planned"]["median_ms"] for k, v in res.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", required=True)
    ap.add_argument("--b", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    names = [n for n in WORKLOADS if not a.only or n in a.only.split(",")]
    res = {n: {"a": [], "b": []} for n in names}
    for r in range(a.rounds):
        for n in names:
            for arm in ("a", "b") if r % 2 == 0 else ("b", "a"):
                m = medians(run(getattr(a, arm), WORKLOADS[n]))
                res[n][arm].append(m)
                print(f"round {r} {n} {arm}: {m}", file=sys.stderr, flush=True)
    summary = {}
    for n, d in res.items():
        summary[n] = {}
        for key in d["a"][0]:
            ma = statistics.median(x[key] for x in d["a"])
            mb = statistics.median(x[key] for x in d["b"])
            summary[n][key] = {"a_ms": ma, "b_ms": mb, "b_vs_a": round(ma / mb, 4)}
    print(json.dumps({"a": a.a, "b": a.b, "rounds": a.rounds, "results": summary}))


if __name__ == "__main__":
    main()
