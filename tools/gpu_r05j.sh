set -euo pipefail
out=gpurun_out/r05j; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_broadphase_gpu.py -x -q -m gpu -k "cell_lists_long or kd_wave or cells or overflow or capacity" --timeout 300 --timeout-method thread > $out/pytest_cells.log 2>&1 || { tail -60 $out/pytest_cells.log; exit 1; }
tail -1 $out/pytest_cells.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -60 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
show() { python3 -c "import json,sys; r=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]); print('$1', round(r['ms_per_step'],4), {k:round(v,4) for k,v in r['kernel_ms'].items() if isinstance(v,float)}, 'dyn', r['dynamic'] and (round(r['dynamic']['ms_per_step_dynamic'],4), round(r['dynamic']['p50_frame_ms_rebuild'],4)), 'p50', r['p50_frame_ms'])"; }
for c in 2 3 5; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $out/bench_c$c.log 2>&1; show c$c < $out/bench_c$c.log; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rebuild -o run -- python3 bench.py --steps 200 --no-cpu-baseline --frames 5 > $out/rebuild.log 2>&1
python3 tools/kstats.py $out/rebuild/run_kernel_stats.csv
echo done
