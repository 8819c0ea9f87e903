#!/bin/bash
# A/B the variants/libart_<name>.so builds on the GPU box: one bench line each (no CPU baseline).
#   bash tools/ab.sh name1 name2 ...   [extra bench args in $AB_ARGS]
set -euo pipefail
mkdir -p gpurun_out/ab
for v in "$@"; do
  ART_LIB=$PWD/variants/libart_$v.so timeout -k 10 240 python bench.py --no-cpu-baseline --frames 3 ${AB_ARGS:-} > gpurun_out/ab/$v.log 2>&1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/$v.log').read().strip().splitlines()[-1]); print('$v', '%.1f Gt/s'%(d['value']/1e9), 'rt %.4f ms'%d['kernel_ms']['raytrace'], 'perm %.4f'%d['kernel_ms']['permeate'])"
done
