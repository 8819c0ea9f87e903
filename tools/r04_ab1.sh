#!/bin/bash
# Round-4 A/B batch 1: parity suite, traversal variants (timing + SQ counters), cell-list size,
# permeation bound, kd order on a 65,536-collider scene.
set -uo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04b
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_rt.sh 2 nospill base pcl || exit 1
bash tools/ab_rt.sh 3 nospill base pcl || exit 1
PMC_ARGS="--config 2" bash tools/pmc_sq.sh nospill base pcl || exit 1
ART_DEBUG_CELLS=1 timeout -k 10 120 python bench.py --config 2 --no-cpu-baseline --no-dynamic --steps 5 --frames 1 2>&1 | grep "\[cells\]" | head -3
for c in 3 4; do
  for v in base permempty; do
    lib=$PWD/variants/libart_$v.so
    ART_LIB=$lib timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-dynamic --frames 5 > $out/perm_${c}_$v.log 2>&1 || exit 1
    tail -1 $out/perm_${c}_$v.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg $c $v ms_per_step %.4f rt %.4f perm %.4f' % (r['ms_per_step'], r['kernel_ms']['raytrace'], r['kernel_ms']['permeate']))"
  done
done
for v in nospill base; do
  ART_LIB=$PWD/variants/libart_$v.so timeout -k 10 200 python bench.py --config 2 --collider-scale 16 --no-cpu-baseline --no-dynamic --frames 5 > $out/big_$v.log 2>&1 || exit 1
  tail -1 $out/big_$v.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('65536 colliders $v ms_per_step %.4f rt %.4f nearest %.4f' % (r['ms_per_step'], r['kernel_ms']['raytrace'], r['kernel_ms']['nearest']))"
done
ART_LIB=$PWD/variants/libart_diag.so timeout -k 10 200 python bench.py --config 2 --collider-scale 16 --no-cpu-baseline --no-dynamic --frames 2 --steps 20 --warmup 1 > $out/big_diag.log 2>&1 || exit 1
grep "\[diag\]" $out/big_diag.log
