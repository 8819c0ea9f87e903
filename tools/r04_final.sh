#!/bin/bash
# Round-4 GPU pass over the committed build: parity suite + smoke, then tools/gpu_round.sh per config
# Usage (GPU box, repo root): bash tools/r04_final.sh "<configs>" [tests]
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04f
if [ "${2:-}" = "tests" ]; then
  echo "[r04_final] pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04f/pytest_gpu.log 2>&1
  tail -2 gpurun_out/r04f/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f/smoke.log 2>&1
  cat gpurun_out/r04f/smoke.log
fi
for c in $1; do
  bash tools/gpu_round.sh r04_c$c $c
done
