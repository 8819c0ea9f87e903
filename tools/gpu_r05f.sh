set -euo pipefail
out=gpurun_out/r05f; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -60 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
show() { python3 -c "import json,sys; r=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]); print('$1', round(r['ms_per_step'],4), {k:round(v,4) for k,v in r['kernel_ms'].items() if isinstance(v,float)}, 'dyn', r['dynamic'] and (round(r['dynamic']['ms_per_step_dynamic'],4), round(r['dynamic']['p50_frame_ms_rebuild'],4)), 'p50', r['p50_frame_ms'])"; }
timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline > $out/bench_c2.log 2>&1; show c2 < $out/bench_c2.log
for m in 0 1 0 1; do ART_MUFFLE_PER_BOUNCE=$m timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline --no-dynamic --frames 5 | show c5_muffle_each_$m; done
ART_MUFFLE_PER_BOUNCE=1 timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "bench_path or reduced or stage_subsets or many_targets" --timeout 300 --timeout-method thread > $out/pytest_mpb.log 2>&1 || { tail -40 $out/pytest_mpb.log; exit 1; }
tail -1 $out/pytest_mpb.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rebuild -o run -- python3 bench.py --steps 200 --no-cpu-baseline --frames 5 > $out/rebuild.log 2>&1
python3 tools/kstats.py $out/rebuild/run_kernel_stats.csv
echo done
