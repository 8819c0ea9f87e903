#!/bin/bash
# Folded multi-bounce path: parity suite, then configs 5 and 2 against the build before it
set -uo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04d
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $out/pytest.log | head -20; exit $rc; }
for c in 5 4; do bash tools/ab_rt.sh $c prefold base || exit 1; done
