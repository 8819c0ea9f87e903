#!/bin/bash
# A/B of graph replay: bench configs 2 and 5 with ART_GRAPH=1 / 0, plus a kernel trace of config 2.
set -euo pipefail
out=gpurun_out/${1:-graph_ab}
mkdir -p "$out"
export TMPDIR=/tmp
for c in 2 5; do
  for g in 1 0; do
    ART_GRAPH=$g timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dynamic --frames 20 > "$out/bench_c${c}_g$g.log" 2>&1
    tail -1 "$out/bench_c${c}_g$g.log" | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg $c graph $g: ms_per_step %.4f rt_ms %.4f p50 %.4f' % (r['ms_per_step'], r['kernel_ms']['raytrace'], r['p50_frame_ms']))"
  done
done
