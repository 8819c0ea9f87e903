#!/bin/bash
# Round-4 A/B batch 2: parity suite, configs 2-5 (nospill = this round's first build vs base), the
# permeation bound on the current build, config-2 traffic per kernel.
set -uo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04c
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $out/pytest.log | head -20; exit $rc; }
for c in 2 3 4 5; do bash tools/ab_rt.sh $c nospill base || exit 1; done
for c in 3 4; do
  ART_LIB=$PWD/variants/libart_permempty.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-dynamic --frames 5 > $out/perm_${c}.log 2>&1 || exit 1
  tail -1 $out/perm_${c}.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg $c permempty ms_per_step %.4f rt %.4f perm %.4f' % (r['ms_per_step'], r['kernel_ms']['raytrace'], r['kernel_ms']['permeate']))"
done
bash tools/pmc_traffic_ab.sh 2 base && python3 tools/pmc_traffic_print.py base | head -8
