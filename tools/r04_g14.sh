#!/bin/bash
# Round-4 GPU pass 14: balanced per-face cell-list passes, batched kd prologue, wave-level kd pass
# (GPU suite, rebuild kernel trace with and without the wave pass, kd phase timings).
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g14
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_broadphase_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $out/pytest_bp.log 2>&1 || { tail -30 $out/pytest_bp.log; exit 1; }
tail -1 $out/pytest_bp.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
bash tools/r04_rebuild.sh
cp -r gpurun_out/r04_rebuild gpurun_out/r04_rebuild_wave
ART_KD_WAVE=0 bash tools/r04_rebuild.sh
bash tools/r04_kdprof.sh
