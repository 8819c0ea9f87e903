set -euo pipefail
out=gpurun_out/r05e; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -60 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
for c in 2 3 5 4; do
  ART_DEBUG_CELLS=1 timeout -k 10 100 python3 -c "
import sys; sys.path.insert(0,'audio-raytracer_amd'); import art
cfg=art.CONFIGS[$c]; scene, org, params = art.synth(cfg, S=4)
with art.Context(1) as c: c.bind(art.Frame(scene, params, org, art.FanOutputs(4, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)))
" 2>&1 | grep cells | sed "s/^/c$c /"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rebuild -o run -- python3 bench.py --steps 200 --no-cpu-baseline --frames 5 > $out/rebuild.log 2>&1
tail -1 $out/rebuild.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('c2', r['ms_per_step'], r['dynamic'])"
python3 tools/kstats.py $out/rebuild/run_kernel_stats.csv | head -40
echo done
show() { python3 -c "import json,sys; r=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(r['ms_per_step'],4), {k:round(v,4) for k,v in r['kernel_ms'].items() if isinstance(v,float)})"; }
for m in 0 1 0 1; do ART_MUFFLE_PER_BOUNCE=$m timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline --no-dynamic --frames 5 | show c5_muffle_each_$m; done
ART_MUFFLE_PER_BOUNCE=1 timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "bench_path or reduced or stage_subsets or many_targets" --timeout 300 --timeout-method thread > $out/pytest_mpb.log 2>&1 || { tail -40 $out/pytest_mpb.log; exit 1; }
tail -1 $out/pytest_mpb.log
