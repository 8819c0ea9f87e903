#!/bin/bash
# Per-sample DSP row: bench line, kernel trace and separate FETCH_SIZE / WRITE_SIZE passes.
# Run from the repo root on the GPU box:  bash tools/gpu_dsp.sh [tag]
set -euo pipefail
tag=${1:-r01_dsp}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
echo "[gpu_dsp] bench"
timeout -k 10 300 python bench.py --path dsp > "$out/bench.log" 2>&1
tail -1 "$out/bench.log" > "$out/bench.json"
cat "$out/bench.json"
echo "[gpu_dsp] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py --path dsp --no-cpu-baseline > "$out/trace.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  echo "[gpu_dsp] pmc $c"
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_$c" -o run -- python3 bench.py --path dsp --no-cpu-baseline --steps 5 --warmup 1 > "$out/pmc_$c.log" 2>&1
done
echo "[gpu_dsp] done"
