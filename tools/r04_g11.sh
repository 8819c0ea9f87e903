#!/bin/bash
# Round-4 GPU pass 11: echo-traversal knobs (wave priority, steal thresholds 3 / 4), nearest steal
# threshold 4, fan lanes 2 — parity at full size first, then A/B on configs 2 and 3.
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g11
mkdir -p $out
for v in vprio vst3 vst4 nst4; do
  ART_LIB=$PWD/variants/libart_$v.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "full_size or golden" --timeout 300 --timeout-method thread > $out/pytest_$v.log 2>&1
  echo "$v: $(tail -1 $out/pytest_$v.log)"
done
bash tools/ab_rt.sh 2 base vprio vst3 vst4 nst4 lanes2=ART_FAN_LANES=2 base
bash tools/ab_rt.sh 3 base vprio vst3 vst4 nst4
