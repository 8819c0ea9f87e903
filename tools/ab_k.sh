#!/bin/bash
# A/B the variants/libart_<name>.so builds: per-kernel times (untimed HIP-event passes) and ms/step.
#   AB_CONFIGS="2 3" AB_REPS=2 bash tools/ab_k.sh name1 name2 ...
set -euo pipefail
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${AB_REPS:-1}); do
  for c in ${AB_CONFIGS:-2}; do
    for v in "$@"; do
      log=gpurun_out/ab/${v}_c$c.log
      ART_LIB=$PWD/variants/libart_$v.so timeout -k 10 240 python bench.py --config $c --no-cpu-baseline --no-dynamic --frames 3 > $log 2>&1
      python3 -c "
import json; d=json.loads([l for l in open('$log').read().splitlines() if l.startswith('{')][-1])
k={n: round(x * 1e3, 1) for n, x in d['kernel_ms'].items() if isinstance(x, float) and n not in ('raytrace', 'permeate', 'reduce')}
print('c$c $v', 'ms/step %.4f' % d['ms_per_step'], 'rt %.1f us' % (d['kernel_ms']['raytrace'] * 1e3), k)"
    done
  done
done
