#!/bin/bash
# Round-4 GPU pass 6: GPU suite on the committed build (kd split with LDS bounds, aggregated cell-row
# passes), its rebuild-frame profile, then combined nearest-kernel variants (parity at full size
# first, then A/B on configs 2, 3 and 5).
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g6
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_base.log 2>&1
tail -1 $out/pytest_base.log
bash tools/r04_rebuild.sh
for v in s2n s3n s4n s2ns s2nv2; do
  ART_LIB=$PWD/variants/libart_$v.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "full_size or golden" --timeout 300 --timeout-method thread > $out/pytest_$v.log 2>&1
  echo "$v: $(tail -1 $out/pytest_$v.log)"
done
bash tools/ab_rt.sh 2 base s2n s3n s4n s2ns s2nv2 base
bash tools/ab_rt.sh 3 base s2n s3n s4n s2ns s2nv2
bash tools/ab_rt.sh 5 base s2n s2ns s2nv2
