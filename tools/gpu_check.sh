#!/bin/bash
# GPU check: parity tests (-m gpu), the smoke, and the default bench line (no CPU baseline).
#   bash tools/gpu_check.sh <tag> [pytest -k expr]
set -euo pipefail
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
kexpr=${2:-}
if [ -n "$kexpr" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$kexpr" --timeout 300 --timeout-method thread > "$out/pytest_gpu.log" 2>&1 || { tail -60 "$out/pytest_gpu.log"; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$out/pytest_gpu.log" 2>&1 || { tail -60 "$out/pytest_gpu.log"; exit 1; }
fi
tail -3 "$out/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -30 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-dynamic > "$out/bench.log" 2>&1 || { tail -30 "$out/bench.log"; exit 1; }
tail -1 "$out/bench.log" | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('value %.4g ms_per_step %.4f rt_ms %.4f frac %.4f p50 %s' % (r['value'], r['ms_per_step'], r['kernel_ms']['raytrace'], r['roofline']['frac'], r['p50_frame_ms']))"
