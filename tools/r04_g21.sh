#!/bin/bash
# Driver-style bench runs of the final build (default command, and K=20 / W=5)
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g21
mkdir -p $out
timeout -k 10 600 python bench.py > $out/bench_default.log 2>&1
grep '^{' $out/bench_default.log | tail -1 | cut -c1-400
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench_20.log 2>&1
grep '^{' $out/bench_20.log | tail -1 | cut -c1-400
