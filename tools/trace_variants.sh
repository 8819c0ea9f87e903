#!/bin/bash
# Kernel-trace A/B: rocprofv3 --kernel-trace --stats of bench.py per variants/libart_<name>.so,
# then the per-kernel mean durations side by side.
#   bash tools/trace_variants.sh name1 name2 ...   [extra bench args in $AB_ARGS]
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
for v in "$@"; do
  lib=$PWD/variants/libart_$v.so
  [ "$v" = default ] && lib=$PWD/audio-raytracer_amd/lib/libart.so
  ART_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr/$v -o run -- \
    python3 bench.py --no-cpu-baseline --frames 3 --steps 20 --warmup 3 ${AB_ARGS:-} > gpurun_out/tr/$v.log 2>&1
done
python3 tools/trace_table.py "$@"
