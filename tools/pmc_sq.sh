#!/bin/bash
# Two SQ counter passes (8 slots each) over a short bench run of each variant.
#   bash tools/pmc_sq.sh <variant>... [bench args in $PMC_ARGS]
set -euo pipefail
export TMPDIR=/tmp
for v in "$@"; do
  mkdir -p gpurun_out/pmc_$v
  i=0
  for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_WAVES SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    ART_LIB=$PWD/variants/libart_$v.so timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$v/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --frames 1 ${PMC_ARGS:-} > gpurun_out/pmc_$v/p$i.log 2>&1
  done
done
