#!/bin/bash
# Per-ray traversal-step and per-wave cycle histograms (variants/libart_diag.so, -DART_DIAG) of 10
# device-loop frames per config:  bash tools/diag_steps.sh 2 3   -> gpurun_out/diag/steps_c<k>.txt
set -euo pipefail
mkdir -p gpurun_out/diag
for c in "$@"; do
  ART_LIB=$PWD/variants/libart_diag.so timeout -k 10 200 python3 tools/wt_run.py $c 10 > gpurun_out/diag/steps_c$c.log 2>&1
  grep "\[diag\]" gpurun_out/diag/steps_c$c.log > gpurun_out/diag/steps_c$c.txt
  cat gpurun_out/diag/steps_c$c.txt
done
