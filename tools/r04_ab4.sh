#!/bin/bash
# Folded multi-bounce path + nearest leaf keys + stored-empty nodes: parity suite, then A/B
set -uo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04d
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $out/pytest.log | head -20; exit $rc; }
for c in 5 2 3; do bash tools/ab_rt.sh $c prefold fold base || exit 1; done
PMC_ARGS="--config 2" bash tools/pmc_sq.sh prefold || exit 1
cp audio-raytracer_amd/lib/libart.so variants/libart_base.so && PMC_ARGS="--config 2" bash tools/pmc_sq.sh base || exit 1
