#!/bin/bash
# Round-4 GPU pass 5: nearest-kernel A/B variants on configs 2 and 3 (ballot entered count, steal
# threshold 2, surface-area splits on 128 segments), each checked against the oracle at full size first.
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g5
mkdir -p $out
for v in nenb steal2 sah128; do
  ART_LIB=$PWD/variants/libart_$v.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "full_size or golden" --timeout 300 --timeout-method thread > $out/pytest_$v.log 2>&1
  echo "$v: $(tail -1 $out/pytest_$v.log)"
done
bash tools/ab_rt.sh 2 base nenb steal2 sah128 base
bash tools/ab_rt.sh 3 base nenb steal2 sah128
