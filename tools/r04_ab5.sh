#!/bin/bash
# Round-4 batch 5: parity suite, the rebuild profile, config-5 per-bounce kernel times (prefold vs base)
set -uo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04e
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $out/pytest.log | head -20; exit $rc; }
bash tools/r04_rebuild.sh || exit 1
bash tools/ab_rt.sh 5 prefold || exit 1
python3 tools/bounce_table.py gpurun_out/ab/prefold/trace/run_kernel_trace.csv 5
bash tools/ab_rt.sh 5 base || exit 1
python3 tools/bounce_table.py gpurun_out/ab/base/trace/run_kernel_trace.csv 5
