#!/bin/bash
# Round-4 GPU pass 3: GPU suite on the default plan and on the group plan (ART_GROUP_PLAN=1), then
# A/B of the plans (base / group / fused nearest+echo variant) on configs 2-4 and the diag histograms.
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g3
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_base.log 2>&1
tail -1 $out/pytest_base.log
ART_GROUP_PLAN=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_group.log 2>&1
tail -1 $out/pytest_group.log
ART_LIB=$PWD/variants/libart_fuse.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "full_size_bench_path" --timeout 300 --timeout-method thread > $out/fuse_pytest.log 2>&1
tail -1 $out/fuse_pytest.log
bash tools/ab_rt.sh 2 base group=ART_GROUP_PLAN=1 fuse
bash tools/ab_rt.sh 3 base group=ART_GROUP_PLAN=1
bash tools/ab_rt.sh 4 base group=ART_GROUP_PLAN=1
bash tools/diag_run.sh 2 3
