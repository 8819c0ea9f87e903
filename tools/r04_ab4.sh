#!/bin/bash
# Round-4 batch: parity suite, then A/B (prefold = before the folded path and the traversal
# changes; muf0 = before the 8-wave muffle kernel), the fused nearest+echo variant once at full size,
# the no-path echo+muffle launch on config 4, the rebuild profile, SQ counters
set -uo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04d
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $out/pytest.log | head -20; exit $rc; }
for c in 5 2 3; do bash tools/ab_rt.sh $c prefold muf0 base || exit 1; done
bash tools/ab_rt.sh 4 prefold base hm2any || exit 1
ART_LIB=$PWD/variants/libart_fuse.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "full_size_bench_path_sampled" --timeout 200 --timeout-method thread > $out/fuse_pytest.log 2>&1
rc=$?; echo "fused variant full-size parity rc=$rc"; tail -2 $out/fuse_pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3; do bash tools/ab_rt.sh $c fuse || exit 1; done
bash tools/r04_rebuild.sh || exit 1
PMC_ARGS="--config 2" bash tools/pmc_sq.sh prefold || exit 1
cp audio-raytracer_amd/lib/libart.so variants/libart_base.so && PMC_ARGS="--config 2" bash tools/pmc_sq.sh base || exit 1
