#!/bin/bash
# Round-4 GPU pass 10: GPU suite on the build with group-reduced kd surface-area bounds, the rebuild
# profile, the per-sample DSP row re-profiled (bench line, kernel trace, traffic passes).
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g10
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -1 $out/pytest_gpu.log
bash tools/r04_rebuild.sh
bash tools/gpu_dsp.sh r04_dsp
