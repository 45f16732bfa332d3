#!/usr/bin/env python3
"""Are the balanced split's slow calls CPU-quota throttling? (GPU, diagnostic)

The split's calls are bimodal (EXPERIMENTS.md round 6: 36-42 ms or 55-101 ms a
call).  A container whose cgroup caps CPU time (cpu.max) throttles every thread
for the rest of a period once the quota is spent, which a call running more
busy threads than the quota allows would hit.  This prints the cgroup's quota
and, for each call (pool alone, engine alone, balanced split at several
pool:reader shapes, alternating), the wall time, the process's CPU time and the
cgroup's nr_throttled / throttled_usec deltas, every verdict checked.

usage: python tools/split_throttle_probe.py OUT.json [reps] [shapes, e.g. 12:8,8:8,4:12]
"""
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import oracle  # noqa: E402
from vortex_amd.hash_pool import HashPool  # noqa: E402


def cgroup_dir():
    try:
        with open("/proc/self/cgroup") as f:
            for line in f:
                hier, ctrl, path = line.rstrip("\n").split(":", 2)
                if hier == "0" or "cpu" in ctrl.split(","):
                    for base in ("/sys/fs/cgroup", "/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"):
                        d = base + path
                        if os.path.exists(os.path.join(d, "cpu.stat")):
                            return d
    except OSError:
        pass
    return "/sys/fs/cgroup"


def read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError as e:
        return f"<{e.strerror}>"


def stat(d):
    out = {}
    for line in read(os.path.join(d, "cpu.stat")).splitlines():
        k, _, v = line.partition(" ")
        if v.isdigit():
            out[k] = int(v)
    if "throttled_time" in out:  # cgroup v1: ns
        out["throttled_usec"] = out["throttled_time"] // 1000
    return out


def host_busy():
    """(busy, total) jiffies over every CPU of the host (/proc/stat's first line)."""
    v = [int(x) for x in read("/proc/stat").splitlines()[0].split()[1:]]
    idle = v[3] + (v[4] if len(v) > 4 else 0)
    return sum(v) - idle, sum(v)


def cpu_s():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    threads = bench.cpu_share()
    shapes = [tuple(int(x) for x in s.split(":")) for s in sys.argv[3].split(",")] if len(sys.argv) > 3 else \
        [(12, 8), (8, 8), (4, 12)]
    cg = cgroup_dir()
    info = {"cgroup": cg, "cpu.max": read(os.path.join(cg, "cpu.max")),
            "cfs_quota_us": read(os.path.join(cg, "cpu.cfs_quota_us")),
            "cfs_period_us": read(os.path.join(cg, "cpu.cfs_period_us")),
            "affinity": len(os.sched_getaffinity(0)), "cpu_share": threads, "os_cpu_count": os.cpu_count(),
            "loadavg": read("/proc/loadavg")}
    print(info, flush=True)
    pl = 2097152
    path = os.path.join(bench.reverify_dir(), f"vx_split_thr_{os.getpid()}.iso")
    calls = []
    try:
        total, n, last = bench.write_linuxmint_file(path)
        exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
        for _ in range(2):
            oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
        t0 = time.perf_counter()
        oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
        rate = total / (time.perf_counter() - t0) / threads
        with HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=4096) as pool:
            pool.verify_files([path], [total], pl, exp, io_threads=threads)
            kinds = [("pool", threads, 0), ("engine", 0, threads)] + [("split", p, r) for p, r in shapes]
            for rep in range(reps):
                for kind, p, r in kinds:
                    s0, h0, c0, t0 = stat(cg), host_busy(), cpu_s(), time.perf_counter()
                    if kind == "pool":
                        ok = all(oracle.pool_verify_files([path], [total], pl, exp, threads=p))
                        extra = {}
                    elif kind == "engine":
                        got, bad = pool.verify_files([path], [total], pl, exp, io_threads=r)
                        ok, extra = bad == 0, {}
                    else:
                        c = bench.balanced_call(pool, [path], [total], n, pl, exp, r, p, rate)
                        ok, extra = c["ok"], {"boundary": c["boundary"], "gpu_s": round(c["gpu_s"], 4),
                                              "cpu_s": round(c["cpu_s"], 4)}
                    wall, cpu = time.perf_counter() - t0, cpu_s() - c0
                    s1, h1 = stat(cg), host_busy()
                    assert ok, f"{kind} {p}:{r}: a verdict differs from the expected table"
                    rec = dict(kind=kind, shape=f"{p}:{r}", rep=rep, wall_ms=round(wall * 1e3, 2),
                               cpu_ms=round(cpu * 1e3, 1), cores=round(cpu / wall, 2),
                               throttled=s1.get("nr_throttled", 0) - s0.get("nr_throttled", 0),
                               throttled_ms=round((s1.get("throttled_usec", 0) - s0.get("throttled_usec", 0)) / 1e3, 2),
                               periods=s1.get("nr_periods", 0) - s0.get("nr_periods", 0),
                               host_busy=round((h1[0] - h0[0]) / max(1, h1[1] - h0[1]), 3), **extra)
                    calls.append(rec)
                    print(rec, flush=True)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    summary = {}
    for kind, p, r in kinds:
        rows = [c for c in calls if c["kind"] == kind and c["shape"] == f"{p}:{r}"]
        w = sorted(c["wall_ms"] for c in rows)
        summary[f"{kind} {p}:{r}"] = {"median_ms": w[len(w) // 2], "GiBps": round(total / (w[len(w) // 2] / 1e3) / (1 << 30), 2),
                                     "throttled_calls": sum(1 for c in rows if c["throttled"]),
                                     "median_cores": sorted(c["cores"] for c in rows)[len(rows) // 2]}
    print(json.dumps(summary, indent=1), flush=True)
    with open(out, "w") as f:
        json.dump({"info": info, "calls": calls, "summary": summary}, f, indent=1)


if __name__ == "__main__":
    main()
