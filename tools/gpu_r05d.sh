set -euo pipefail
out=gpurun_out/r05d; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -60 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
ART_PATH_KERNEL=1 timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "bench_path or reduced or stage_subsets or many_targets" --timeout 300 --timeout-method thread > $out/pytest_path.log 2>&1 || { tail -40 $out/pytest_path.log; exit 1; }
tail -1 $out/pytest_path.log
show() { python3 -c "import json,sys; r=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(r['ms_per_step'],4), r['roofline']['kernel'], {k:round(v,4) for k,v in r['kernel_ms'].items() if isinstance(v,float)})"; }
for c in 2 3 5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-dynamic --frames 5 > $out/bench_c$c.log 2>&1 || { tail -20 $out/bench_c$c.log; exit 1; }
  show c$c < $out/bench_c$c.log
done
for c in 2 5; do
  ART_PATH_KERNEL=1 timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-dynamic --frames 5 > $out/bench_c${c}_path.log 2>&1
  show c${c}path < $out/bench_c${c}_path.log
done
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dynamic --frames 5 | show drv20
echo done
