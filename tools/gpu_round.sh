#!/bin/bash
# One GPU pass: (optional) parity tests, the bench line, a kernel-trace profile and separate PMC passes.
# Run from the repo root on the GPU box:  bash tools/gpu_round.sh <tag> [config] [tests]
# Every GPU step has its own time limit; the first failure ends the script (set -e).
set -euo pipefail
tag=${1:-r02}
cfg=${2:-2}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
sha256sum audio-raytracer_amd/lib/libart.so | cut -d' ' -f1 > "$out/lib.sha256"
if [ "${3:-}" = "tests" ]; then
  echo "[gpu_round] pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
  tail -2 "$out/pytest_gpu.log"
fi
short="--config $cfg --no-cpu-baseline --no-dynamic"
echo "[gpu_round] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py $short --frames 5 --steps 50 > "$out/trace.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU"; do
  n=$(echo "$c" | cut -d' ' -f1)
  echo "[gpu_round] pmc $c"
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_$n" -o run -- python3 bench.py $short --steps 5 --warmup 1 --frames 1 > "$out/pmc_$n.log" 2>&1
done
# HBM traffic per raytrace launch from the two PMC passes, stamped with this build's sha256, so
# the bench line below reports it (bench.py reads profiles/traffic_config<k>.json)
python3 tools/prof_summary.py "$out" "$tag" "$cfg" > "$out/prof_summary.log" 2>&1
cp "profiles/traffic_config$cfg.json" "$out/"
echo "[gpu_round] bench"
timeout -k 10 400 python bench.py --config $cfg > "$out/bench.log" 2>&1
tail -1 "$out/bench.log" > "$out/bench.json"
cat "$out/bench.json"
echo "[gpu_round] done"
