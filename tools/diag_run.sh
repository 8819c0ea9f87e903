#!/bin/bash
# Per-wave cycle and per-ray step histograms (variants/libart_diag.so, built with -DART_DIAG):
#   bash tools/diag_run.sh <config>...     -> gpurun_out/diag/c<k>.log
set -euo pipefail
mkdir -p gpurun_out/diag
for c in "$@"; do
  ART_LIB=$PWD/variants/libart_diag.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-dynamic \
    --frames 2 --steps 20 --warmup 1 > gpurun_out/diag/c$c.log 2>&1
  grep "\[diag\]" gpurun_out/diag/c$c.log
done
