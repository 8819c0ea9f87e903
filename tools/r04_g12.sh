#!/bin/bash
# Round-4 GPU pass 12: GPU suite on the two-pass kd split, its rebuild profile, then pass 11's A/B.
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g12
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -1 $out/pytest_gpu.log
bash tools/r04_rebuild.sh
bash tools/r04_g11.sh
