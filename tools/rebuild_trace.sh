#!/bin/bash
# Rebuild-frame timeline: tools/rebuild_run.py alone, then under rocprofv3 --kernel-trace --memory-copy-trace.
#   bash tools/rebuild_trace.sh [config]   -> gpurun_out/rebuild/
set -euo pipefail
export TMPDIR=/tmp
c=${1:-2}
mode=${2:-}   # "static": the same scene every frame
mkdir -p gpurun_out/rebuild
timeout -k 10 120 python3 tools/rebuild_run.py $c 200 $mode > gpurun_out/rebuild/plain.log 2>&1
cat gpurun_out/rebuild/plain.log | tail -1
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/rebuild/trace -o run -- python3 tools/rebuild_run.py $c 40 $mode > gpurun_out/rebuild/trace.log 2>&1
tail -1 gpurun_out/rebuild/trace.log
