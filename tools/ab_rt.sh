#!/bin/bash
# A/B of library variants on one config: kernel-trace top kernels + bench ms/step + executed counts.
#   bash tools/ab_rt.sh <config> <variant|base|label=ENV=VALUE>...
# (label=ENV=VALUE runs the in-tree library with ENV=VALUE in the environment)
set -euo pipefail
cfg=$1; shift
export TMPDIR=/tmp
for spec in "$@"; do
  v=${spec%%=*}
  envset=()
  lib=$PWD/audio-raytracer_amd/lib/libart.so
  if [ "$spec" != "$v" ]; then envset=("${spec#*=}");
  elif [ "$v" != base ]; then lib=$PWD/variants/libart_$v.so; fi
  out=gpurun_out/ab/$v
  mkdir -p "$out"
  env "${envset[@]}" ART_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --no-dynamic --frames 5 --steps 50 > "$out/trace.log" 2>&1
  echo "== $v"
  python3 tools/kstats.py "$out/trace/run_kernel_stats.csv" > "$out/kstats.txt"; sed -n 1,6p "$out/kstats.txt"
  env "${envset[@]}" ART_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-dynamic --frames 5 > "$out/bench.log" 2>&1
  tail -1 "$out/bench.log" | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); c=r['roofline']['executed']['counts']; print('ms_per_step %.4f stage %.4f nearest %.4f echo_pairs %s cells %s fb %s' % (r['ms_per_step'], r['kernel_ms']['raytrace'], r['kernel_ms']['nearest'], c.get('echo_pairs'), c.get('cell_entries'), c.get('muffle_fallback')))"
done
