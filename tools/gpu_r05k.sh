set -euo pipefail
out=gpurun_out/r05k; mkdir -p $out; export TMPDIR=/tmp
show() { python3 -c "import json,sys; r=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]); print('$1', round(r['ms_per_step'],4), {k:round(v,4) for k,v in r['kernel_ms'].items() if isinstance(v,float)})"; }
for m in 0 2 0 2; do ART_MUFFLE_PER_BOUNCE=$m timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline --no-dynamic --frames 5 | show c5_m$m; done
ART_MUFFLE_PER_BOUNCE=2 timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "bench_path or reduced or stage_subsets" --timeout 300 --timeout-method thread > $out/pytest_m2.log 2>&1 || { tail -40 $out/pytest_m2.log; exit 1; }
tail -1 $out/pytest_m2.log
echo done
