#!/bin/bash
# Kernel trace of config 2's rebuild frames (bench.py dynamic measurement: 25 host-API frames with
# every collider changed, after the resident-store dynamic steps) -> per-kernel means
set -uo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04_rebuild
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --config 2 --no-cpu-baseline --frames 5 --steps 50 > $out/bench.log 2>&1 || exit 1
grep '^{' $out/bench.log | tail -1 | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); d=r['dynamic']; print('dynamic %.4f rebuild p50 %.4f' % (d['ms_per_step_dynamic'], d['p50_frame_ms_rebuild']))"
python3 - $out/trace/run_kernel_stats.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows:
    if int(r["Calls"]) < 400:
        print("%-70s calls=%5d avg_us=%8.1f" % (r["Name"].split("(")[0].replace("void ", "").replace("art::", "")[:70], int(r["Calls"]), float(r["AverageNs"]) / 1e3))
PY
