#!/bin/bash
# Round-4 GPU pass 8: per-bounce muffle launches on config 5 (A/B, parity first) and driver-style
# short bench runs of config 2 (--steps 20 --warmup 5, three processes) against a 2000-step run.
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g8
mkdir -p $out
ART_MUFFLE_PER_BOUNCE=1 timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_exec_counts_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_mpb.log 2>&1
echo "mpb: $(tail -1 $out/pytest_mpb.log)"
bash tools/ab_rt.sh 5 base mpb=ART_MUFFLE_PER_BOUNCE=1 base
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/drv20_$i.log 2>&1
  tail -1 $out/drv20_$i.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('steps 20: ms_per_step %.4f value %.4g' % (r['ms_per_step'], r['value']))"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 2000 --warmup 5 --no-cpu-baseline --no-dynamic > $out/drv2000.log 2>&1
tail -1 $out/drv2000.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('steps 2000: ms_per_step %.4f value %.4g' % (r['ms_per_step'], r['value']))"
