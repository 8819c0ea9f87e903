#!/bin/bash
# Cell-list sizes and length histograms per config (ART_DEBUG_CELLS=1 prints them at each build).
#   bash tools/cell_lists.sh 2 3 4 5   -> gpurun_out/cells.txt
set -euo pipefail
mkdir -p gpurun_out
: > gpurun_out/cells.txt
for c in "$@"; do
  echo "config $c" >> gpurun_out/cells.txt
  ART_DEBUG_CELLS=1 timeout -k 10 120 python3 tools/rebuild_run.py $c 1 2>&1 | grep "^\[cells\]" | sort -u >> gpurun_out/cells.txt
done
cat gpurun_out/cells.txt
