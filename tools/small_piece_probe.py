#!/usr/bin/env python3
"""The engine alone on small warm pieces: where the time goes (GPU, diagnostic).

For each piece length, writes a ~2 GiB file of synthetic pieces, warms it, and
alternates vx_verify_files over it at several context shapes (slot bytes,
readers), every verdict checked.  Prints each shape's median rate with the
median call's vx_last_verify trace (read busy and span, H2D busy and span,
rounds / slots).

usage: python tools/small_piece_probe.py OUT.json [reps] [KiB list] [shapes "slotMiB:readers,..."]
  slotMiB 0 = vx_config_default's slot size
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import oracle  # noqa: E402
from split_geom_probe import SEED, write  # noqa: E402
from vortex_amd.hash_pool import HashPool  # noqa: E402


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    kibs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [16, 64]
    shapes = [tuple(int(v) for v in s.split(":")) for s in sys.argv[4].split(",")] if len(sys.argv) > 4 else \
        [(0, 16), (256, 16), (512, 16)]
    threads = bench.cpu_share()
    res = {"threads": threads, "geoms": {}}
    for kib in kibs:
        pl = kib << 10
        total = (2 << 30) + pl // 3 + 4099
        path = os.path.join(bench.reverify_dir(), f"vx_small_{os.getpid()}_{kib}.bin")
        try:
            n, last = write(path, pl, total)
            exp = oracle.pool_digest_synth(SEED, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
            oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
            pools = {}
            for mib, rd in shapes:
                if mib not in pools:
                    kw = {} if mib == 0 else {"slot_bytes": mib << 20, "batch_pieces": min(65536, (mib << 20) // pl)}
                    pools[mib] = HashPool(pl, **kw)
                    pools[mib].verify_files([path], [total], pl, exp, io_threads=threads)
            runs = {f"{m}:{r}": [] for m, r in shapes}
            for _ in range(reps):
                for mib, rd in shapes:
                    p = pools[mib]
                    t0 = time.perf_counter()
                    _, bad = p.verify_files([path], [total], pl, exp, io_threads=rd)
                    s = time.perf_counter() - t0
                    assert bad == 0, f"{kib} KiB {mib}:{rd}: a verdict differs"
                    runs[f"{mib}:{rd}"].append((s, p.last_verify()))
            g = {}
            for k, v in runs.items():
                v.sort(key=lambda x: x[0])
                s, tr = v[len(v) // 2]
                g[k] = {"GiBps": round(total / s / (1 << 30), 2), "ms": round(s * 1e3, 2),
                        "s_runs": [round(x[0] * 1e3, 1) for x in v],
                        "trace": {a: (round(b, 3) if isinstance(b, float) else b) for a, b in tr.items()}}
            for p in pools.values():
                p.close()
            res["geoms"][f"{kib}K"] = g
            print(kib, "KiB:", {k: (v["GiBps"], v["trace"].get("read_busy_ms"), v["trace"].get("copy_busy_ms"),
                                    v["trace"].get("rounds")) for k, v in g.items()}, flush=True)
        finally:
            if os.path.exists(path):
                os.unlink(path)
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
