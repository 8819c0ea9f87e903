#!/bin/bash
# Round-4 GPU pass 9: echo verdicts from the nearest traversal (ART_ECHO_DECIDE=1): the GPU suite
# under it, then A/B on configs 2, 3 and 4.
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g9
mkdir -p $out
ART_ECHO_DECIDE=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_ed.log 2>&1
tail -1 $out/pytest_ed.log
bash tools/ab_rt.sh 2 base ed=ART_ECHO_DECIDE=1 base ed=ART_ECHO_DECIDE=1
bash tools/ab_rt.sh 3 base ed=ART_ECHO_DECIDE=1
bash tools/ab_rt.sh 4 base ed=ART_ECHO_DECIDE=1
# short-run gap: is it the warmup? (--steps 20 with 5 vs 200 warmup steps)
for w in 5 200; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup $w --no-cpu-baseline --no-dynamic > $out/drv20_w$w.log 2>&1
  tail -1 $out/drv20_w$w.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('steps 20 warmup $w: ms_per_step %.4f stage %.4f' % (r['ms_per_step'], r['kernel_ms']['raytrace']))"
done
