#!/usr/bin/env python3
"""Summarise one tools/gpu_dsp.sh output directory into profiles/ (committed evidence).

  python tools/prof_summary_dsp.py gpurun_out/<tag> <tag>

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_dispatches.csv     dsp_tiled_kernel durations split by grid size (tick vs large batch)
  profiles/<tag>_bench.json         the bench line of the same run
  profiles/traffic_dsp.json         HBM bytes per large-batch launch from FETCH_SIZE / WRITE_SIZE
                                    (bench.py --path dsp reads it)
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
KERNEL = "dsp_tiled_kernel"


def main():
    src, tag = sys.argv[1], sys.argv[2]
    os.makedirs(PROF, exist_ok=True)
    for pat, dst in (("*kernel_stats.csv", f"{tag}_kernel_stats.csv"),):
        f = glob.glob(os.path.join(src, "trace", "**", pat), recursive=True)
        if f:
            shutil.copy(f[0], os.path.join(PROF, dst))
    if os.path.exists(os.path.join(src, "bench.json")):
        shutil.copy(os.path.join(src, "bench.json"), os.path.join(PROF, f"{tag}_bench.json"))
    bench = json.load(open(os.path.join(src, "bench.json")))
    big_grid = (bench["roofline"]["batch_sources"] + 31) // 32 * 64

    dur = defaultdict(list)
    for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                dur[int(r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    rows = [{"kernel": KERNEL, "grid_size": g, "sources": g // 64 * 32, "dispatches": len(v),
             "mean_us": sum(v) / len(v), "min_us": min(v), "max_us": max(v)} for g, v in sorted(dur.items())]
    if rows:
        with open(os.path.join(PROF, f"{tag}_dispatches.csv"), "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
    for r in rows:
        print(r)

    cnt = defaultdict(lambda: defaultdict(float))  # (dispatch) -> counter -> sum over dimensions
    grid = {}
    for f in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            key = (f, r["Dispatch_Id"])
            cnt[key][r["Counter_Name"]] += float(r["Counter_Value"])
            grid[key] = int(r["Grid_Size"])
    per = defaultdict(list)
    for key, cs in cnt.items():
        if grid[key] == big_grid:
            for c, v in cs.items():
                per[c].append(v)
    if per:
        fetch_kb = sum(per["FETCH_SIZE"]) / max(1, len(per["FETCH_SIZE"]))
        write_kb = sum(per["WRITE_SIZE"]) / max(1, len(per["WRITE_SIZE"]))
        alg = bench["roofline"]["algorithmic_bytes"]
        rec = {
            "kernel": KERNEL, "batch_sources": bench["roofline"]["batch_sources"],
            "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
            "algorithmic_read_bytes": alg / 2, "algorithmic_write_bytes": alg / 2,
            "raw_fetch_over_algorithmic_read": fetch_kb * 1024 / (alg / 2),
            "dsp_bytes_per_launch_batch": (2.0 * fetch_kb + write_kb) * 1024.0,
            "correction": "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (MI355X_MICROARCH.md: gfx950 FETCH_SIZE tallies "
                          "half of a coalesced streaming read); raw_fetch_over_algorithmic_read calibrates it on this "
                          "kernel's 8-B-per-lane loads (0.5 = the halving holds)",
            "source": f"profiles/{tag}_* (separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --path dsp)",
        }
        json.dump(rec, open(os.path.join(PROF, "traffic_dsp.json"), "w"), indent=1)
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
