#!/usr/bin/env python3
"""Summarise rocprofv3 PMC CSVs of the hot kernel into profiles/pmc_traffic.json
(read by bench.py as roofline.traffic) and print clock / issue statistics.

HBM bytes = FETCH_SIZE (KiB) * 1024 * 2: MI355X_MICROARCH.md §HBM — on gfx950
FETCH_SIZE reads exactly half of a 16-B/lane streaming read.
usage: python tools/pmc_summary.py <fetch_counter_collection.csv> <sq_counter_collection.csv> [pieces plen]
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path, kernel="sha1_uniform_kernel"):
    by = {}
    for r in csv.DictReader(open(path)):
        if kernel not in r["Kernel_Name"]:
            continue
        d = by.setdefault(r["Dispatch_Id"], {"t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(by.values())


def main():
    fetch_csv, sq_csv = sys.argv[1], sys.argv[2]
    pieces = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    plen = int(sys.argv[4]) if len(sys.argv) > 4 else 262144
    alg = pieces * plen
    f = rows(fetch_csv)
    hbm = [d["FETCH_SIZE"] * 1024 * 2 for d in f]
    med = statistics.median(hbm)
    sq = rows(sq_csv)
    stats = []
    for d in sq:
        clk = d["GRBM_GUI_ACTIVE"] / 8 / d["t"]
        stats.append({"kernel_ms": round(d["t"] * 1e3, 3), "clock_GHz": round(clk / 1e9, 3),
                      "cycles_per_valu": round(d["SQ_WAVE_CYCLES"] * 4 / d["SQ_INSTS_VALU"], 3),
                      "valu_active_frac": round(d["SQ_ACTIVE_INST_VALU"] / d["SQ_WAVE_CYCLES"], 4),
                      "wait_frac": round(d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"], 4),
                      "valu_per_block": round(d["SQ_INSTS_VALU"] / d["SQ_WAVES"] / ((plen + 9 + 63) // 64), 2)})
    out = {
        "_doc": ("HBM read bytes per sha1 uniform-kernel launch from rocprofv3 --pmc FETCH_SIZE, corrected per "
                 "MI355X_MICROARCH.md §HBM (KiB * 1024 * 2 on gfx950); median over the profiled dispatches. "
                 "Written by tools/pmc_summary.py; bench.py reads it as roofline.traffic."),
        f"{pieces}x{plen}": {"hbm_bytes_per_launch": int(med), "algorithmic_bytes_per_launch": alg,
                             "ratio": round(med / alg, 5), "dispatches": len(hbm),
                             "source": os.path.relpath(fetch_csv, ROOT), "sq": stats},
    }
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
