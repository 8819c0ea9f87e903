#!/bin/bash
# A/B of the dynamic-scene step (sync + refit + cell lists + frame) between library variants.
#   bash tools/ab_dyn.sh <config> <variant|base>...
set -euo pipefail
cfg=$1; shift
mkdir -p gpurun_out/ab
for v in "$@"; do
  lib=$PWD/audio-raytracer_amd/lib/libart.so
  [ "$v" != base ] && lib=$PWD/variants/libart_$v.so
  ART_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --frames 5 > gpurun_out/ab/dyn_$v.log 2>&1
  tail -1 gpurun_out/ab/dyn_$v.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); d=r['dynamic']; print('$v', 'ms_per_step %.4f dynamic %.4f rebuild_p50 %.4f' % (r['ms_per_step'], d['ms_per_step_dynamic'], d['p50_frame_ms_rebuild']))"
done
