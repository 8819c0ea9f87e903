#!/bin/bash
# Experiment (not shipped): kd surface-area position loop unrolled (variant) vs the shipped build, rebuild frames
set -euo pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_broadphase_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k kd_wave > /dev/null 2>&1 || true
bash tools/r04_rebuild.sh | grep -E "rebuild|kd_"
cp -r gpurun_out/r04_rebuild gpurun_out/r04_rebuild_base
ART_LIB=variants/libart_sahunroll.so bash tools/r04_rebuild.sh | grep -E "rebuild|kd_"
