#!/bin/bash
# kd split phase timings (diagnostic build -DART_KD_PROF: per-phase wall clock of workgroup 0, printf)
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04_kdprof
mkdir -p $out
ART_LIB=variants/libart_kdprof.so timeout -k 10 300 python3 bench.py --config 2 --no-cpu-baseline --frames 2 --steps 20 --warmup 2 > $out/bench.log 2>&1
grep '^\[kd\]' $out/bench.log | tail -14
