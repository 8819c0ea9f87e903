#!/bin/bash
# Wave timelines (variants/libart_wt.so, -DART_WAVE_TIMES) of the steady device loop per config:
#   bash tools/wt_all.sh 2 3    -> gpurun_out/wt/c<k>.txt
set -euo pipefail
mkdir -p gpurun_out/wt
for c in "$@"; do
  ART_LIB=$PWD/variants/libart_wt.so ART_WAVE_TIMES_OUT=gpurun_out/wt/c$c.bin timeout -k 10 200 python tools/wt_run.py $c 400 > gpurun_out/wt/c$c.log 2>&1
  python3 tools/wave_times.py gpurun_out/wt/c$c.bin > gpurun_out/wt/c$c.txt
done
