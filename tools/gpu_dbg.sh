#!/bin/bash
# Debug helper: run a pytest selection with and without graph replay, each under its own limit.
set -uo pipefail
out=gpurun_out/${1:-dbg}; sel=${2:-config_reduced}
mkdir -p "$out"
export TMPDIR=/tmp ART_SEGV_TRACE=1
ART_GRAPH=0 timeout -k 10 300 python -u -m pytest tests -x -v -m gpu -k "$sel" --timeout 200 --timeout-method thread > "$out/nograph.log" 2>&1
echo "nograph rc=$?"; tail -3 "$out/nograph.log"
rc=$(grep -c "Segmentation\|Aborted" "$out/nograph.log")
if [ "$rc" != "0" ]; then exit 1; fi
ART_GRAPH_KEEP=${KEEP:-} timeout -k 10 300 python -u -m pytest tests -x -v -s -p no:faulthandler -m gpu -k "$sel" --timeout 200 --timeout-method thread > "$out/graph.log" 2>&1
echo "graph rc=$?"; tail -3 "$out/graph.log"
