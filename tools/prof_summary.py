#!/usr/bin/env python3
"""Summarise one tools/gpu_round.sh output directory into profiles/ (committed evidence).

  python tools/prof_summary.py gpurun_out/<tag> <tag> [config]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.csv            per-kernel mean of every PMC counter collected (one pass each)
  profiles/<tag>_bench.json         the bench line of the same round
  profiles/traffic_config<k>.json   HBM bytes per raytrace launch from FETCH_SIZE / WRITE_SIZE,
                                    corrected as MI355X_MICROARCH.md prescribes, stamped with the
                                    sha256 of the libart.so the passes ran (bench.py uses it only
                                    for that same build)
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
HOT = ("nearest_first_kernel", "path_kernel", "vis_kernel", "muffle_kernel", "echo_muffle_kernel", "cells_collider_kernel",
       "raytrace_kernel", "permeate_kernel", "reduce_kernel")
# kernels of the timed raytrace stage (muffle_kernel runs once per frame; nearest, path and the echo
# vis_kernel once per bounce)
STAGE = ("nearest_first_kernel", "path_kernel", "vis_kernel", "muffle_kernel", "echo_muffle_kernel")


def short(name: str) -> str:
    base = name.split("(")[0].replace("void ", "").replace("art::", "")
    return base


def main():
    src, tag = sys.argv[1], sys.argv[2]
    cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    sha_f = os.path.join(src, "lib.sha256")
    lib_sha = open(sha_f).read().split()[0] if os.path.exists(sha_f) else None
    os.makedirs(PROF, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    bench = os.path.join(src, "bench.json")
    if os.path.exists(bench):
        shutil.copy(bench, os.path.join(PROF, f"{tag}_bench.json"))

    # counter_collection.csv: one row per (dispatch, counter)
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values per dispatch
    meta = {}
    for f in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        acc = defaultdict(float)  # (dispatch, kernel, counter) -> sum over dimensions
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not any(h in k for h in HOT):
                continue
            acc[(r["Dispatch_Id"], k, r["Counter_Name"])] += float(r["Counter_Value"])
            meta[k] = {x: r[x] for x in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
                                         "Accum_VGPR_Count", "SGPR_Count")}
        for (d, k, c), v in acc.items():
            per[k][c].append(v)
    rows = []
    for k, cs in sorted(per.items()):
        for c, vals in sorted(cs.items()):
            rows.append({"kernel": k, "counter": c, "dispatches": len(vals), "mean": sum(vals) / len(vals),
                         "min": min(vals), "max": max(vals), **meta.get(k, {})})
    if rows:
        with open(os.path.join(PROF, f"{tag}_pmc.csv"), "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)

    # HBM traffic of the timed raytrace stage per frame (sum over its kernels of the mean per launch)
    # (the <true> instantiations are the one test-counting launch of a run, not timed frames)
    stage = [k for k in per if k.startswith(STAGE) and "<true" not in k]
    if stage:
        def mean(k, c):
            v = per[k].get(c, [])
            return sum(v) / len(v) if v else 0.0
        # launches per frame from the frame's shape (config H): multi-hit frames run
        # nearest_first_kernel, path_kernel and the echo vis_kernel once per bounce, the muffle /
        # echo+muffle kernel once (round 4 scaled by the dispatch ratio to reduce_kernel, whose count
        # pass and executed-count pass made 4 of config 5's 5 bounces)
        sys.path.insert(0, os.path.join(ROOT, "audio-raytracer_amd"))
        import art  # noqa: E402
        H = art.CONFIGS[cfg].H
        per_bounce = ("nearest_first_kernel", "path_kernel", "vis_kernel")

        # round 6: bounce 0 of a frame may run the shared-origin instantiation of the nearest kernel
        # (nearest_first_kernel<EX, OBB, FOLD, true>, once per frame), the other bounces the plain one
        tab = any(k.startswith("nearest_first_kernel") and k.endswith(", true>") for k in stage)

        def launches(k):
            if k.startswith("nearest_first_kernel") and k.endswith(", true>"):
                return 1
            if k.startswith("nearest_first_kernel") and tab:
                return H - 1
            return H if k.startswith(per_bounce) else 1

        def per_frame(k, c):  # mean per dispatch x dispatches per frame
            v = per[k].get(c, [])
            return sum(v) / len(v) * launches(k) if v else 0.0
        fetch_kb = sum(per_frame(k, "FETCH_SIZE") for k in stage)
        write_kb = sum(per_frame(k, "WRITE_SIZE") for k in stage)
        per_kernel = {k: (2.0 * per_frame(k, "FETCH_SIZE") + per_frame(k, "WRITE_SIZE")) * 1024.0 for k in sorted(stage)}
        rec = {
            "kernels": sorted(stage),
            "fetch_size_kb_raw": fetch_kb,
            "write_size_kb": write_kb,
            # MI355X_MICROARCH.md (HBM / rocprofv3): on gfx950 FETCH_SIZE reports half the bytes of a
            # wide read (64 B tallied per 128-B request) -> double it; WRITE_SIZE is exact.
            "raytrace_bytes_per_launch": (2.0 * fetch_kb + write_kb) * 1024.0,
            "bytes_per_frame_by_kernel": per_kernel,
            "correction": "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024; FETCH_SIZE doubled per MI355X_MICROARCH.md gfx950 note",
            "launches_per_frame": {k: launches(k) for k in sorted(stage)},
            "source": f"profiles/{tag}_pmc.csv (separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --config {cfg})",
            "config": cfg,
            "lib_sha256": lib_sha,
        }
        json.dump(rec, open(os.path.join(PROF, f"traffic_config{cfg}.json"), "w"), indent=1)
        print(json.dumps(rec))
    for r in rows:
        print(f'{r["kernel"][:48]:48s} {r["counter"]:18s} {r["mean"]:.4g}')


if __name__ == "__main__":
    main()
