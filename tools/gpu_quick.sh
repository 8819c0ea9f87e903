#!/bin/bash
# Quick GPU iteration: parity tests (optional), a kernel trace of a short bench run, and the bench
# line without the CPU baseline.  bash tools/gpu_quick.sh <tag> [config] [tests]
set -euo pipefail
tag=${1:-quick}
cfg=${2:-2}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
if [ "${3:-}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$out/pytest_gpu.log" 2>&1 || { tail -40 "$out/pytest_gpu.log"; exit 1; }
  tail -1 "$out/pytest_gpu.log"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --no-dynamic --frames 5 --steps 50 > "$out/trace.log" 2>&1
python3 tools/kstats.py "$out/trace/run_kernel_stats.csv"
timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-dynamic > "$out/bench.log" 2>&1
tail -1 "$out/bench.log" | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('value', r['value'], 'ms_per_step', r['ms_per_step'], 'rt_ms', r['kernel_ms'], 'frac', r['roofline']['frac'])"
