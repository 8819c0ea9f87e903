#!/bin/bash
# Round-4 GPU pass 19 (final build): GPU suite + smoke, rebuild profile, profiles of configs 2-5.
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g19
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
bash tools/r04_rebuild.sh
for c in 2 3 4 5; do bash tools/gpu_round.sh r04e_c$c $c; done
