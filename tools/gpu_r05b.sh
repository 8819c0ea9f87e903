set -euo pipefail
out=gpurun_out/r05b; mkdir -p $out; export TMPDIR=/tmp
for c in 5 2; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-dynamic --frames 5 > $out/bench_c$c.log 2>&1 || { tail -20 $out/bench_c$c.log; exit 1; }
  tail -1 $out/bench_c$c.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('c$c', r['ms_per_step'], r['roofline']['kernel'], {k:round(v,4) for k,v in r['kernel_ms'].items() if isinstance(v,float)})"
done
ART_PATH_ONE_HIT=1 timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --no-dynamic --frames 5 > $out/bench_c2_path.log 2>&1
tail -1 $out/bench_c2_path.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('c2 path', r['ms_per_step'], r['roofline']['kernel'], {k:round(v,4) for k,v in r['kernel_ms'].items() if isinstance(v,float)})"
ART_PATH_ONE_HIT=1 timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "bench_path or reduced or stage_subsets" --timeout 300 --timeout-method thread > $out/pytest_path1.log 2>&1 || { tail -40 $out/pytest_path1.log; exit 1; }
tail -1 $out/pytest_path1.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/drv -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dynamic --frames 5 > $out/drv.log 2>&1
echo done
