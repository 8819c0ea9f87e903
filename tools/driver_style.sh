#!/bin/bash
# The driver's round-end commands on one GPU: smoke, `bench.py --steps 20 --warmup 5` (twice) and the
# default bench line, plus a kernel trace of the 20-step run (per-frame periods and gaps, so the
# first frames' clock ramp shows): gpurun_out/<tag>/
set -euo pipefail
tag=${1:-driver}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
tail -1 "$out/smoke.log"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dynamic > "$out/steps20_$i.log" 2>&1
  grep '^{' "$out/steps20_$i.log" | tail -1 | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('steps 20: ms_per_step %.4f' % r['ms_per_step'])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-dynamic > "$out/default.log" 2>&1
grep '^{' "$out/default.log" | tail -1 | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('default (%d steps): ms_per_step %.4f' % (r['steps'], r['ms_per_step']))"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out/trace20" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dynamic --frames 5 > "$out/trace20.log" 2>&1
python3 tools/trace_gaps.py "$out/trace20/run_kernel_trace.csv" nearest_first_kernel\<false 200 > "$out/trace20_gaps.txt"
