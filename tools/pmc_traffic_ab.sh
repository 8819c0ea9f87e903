#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separately) of a short bench run per library variant.
#   bash tools/pmc_traffic_ab.sh <config> <variant>...
set -euo pipefail
cfg=$1; shift
export TMPDIR=/tmp
for v in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    out=gpurun_out/pmcab/$v/$c
    mkdir -p "$out"
    ART_LIB=$PWD/variants/libart_$v.so timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d "$out" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --no-dynamic --steps 5 --warmup 1 --frames 1 > "$out.log" 2>&1
  done
done
