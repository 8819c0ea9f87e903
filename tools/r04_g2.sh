#!/bin/bash
# Round-4 GPU pass 2: the fused nearest+echo variant at full size (parity + A/B), per-wave / per-ray
# step histograms of the diag build, the rebuild-frame profile, configs 4 and 5 profiles.
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g2
mkdir -p $out
ART_LIB=$PWD/variants/libart_fuse.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -v -m gpu -k "full_size_bench_path" --timeout 300 --timeout-method thread > $out/fuse_pytest.log 2>&1
tail -2 $out/fuse_pytest.log
bash tools/ab_rt.sh 2 base fuse
bash tools/diag_run.sh 2 3 5
bash tools/r04_rebuild.sh
for c in ${1:-4 5}; do bash tools/gpu_round.sh r04_c$c $c; done
