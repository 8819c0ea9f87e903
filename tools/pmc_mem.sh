#!/bin/bash
# Memory-side counter passes (TCP/TA/TCC) over a short bench run of each variant.
#   bash tools/pmc_mem.sh <variant>... [bench args in $PMC_ARGS]
set -euo pipefail
export TMPDIR=/tmp
for v in "$@"; do
  lib=$PWD/variants/libart_$v.so
  mkdir -p gpurun_out/pmcm_$v
  i=0
  for c in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum" "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS"; do
    i=$((i+1))
    ART_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcm_$v/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --frames 1 ${PMC_ARGS:-} > gpurun_out/pmcm_$v/p$i.log 2>&1 || echo "pass $i failed"
  done
done
