#!/bin/bash
# Build libart.so with extra compile flags into variants/libart_<name>.so (A/B experiments;
# bench.py / tests pick it up through ART_LIB=variants/libart_<name>.so).
#   tools/build_variant.sh <name> [-DFLAG ...]
set -euo pipefail
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/audio-raytracer_amd
tmp=$(mktemp -d)
mkdir -p "$root/variants"
flags=(--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden "$@")
# the shipped build's scheduler (audio-raytracer_amd/Makefile SCHED; ART_SCHED= for the default one)
sched=(${ART_SCHED--mllvm -amdgpu-sched-strategy=max-ilp})
for f in art_kernels art_trace art_cells art_dsp; do
  hipcc "${flags[@]}" "${sched[@]}" -c "$pkg/csrc/$f.hip" -o "$tmp/$f.o" &
done
hipcc "${flags[@]}" -c "$pkg/csrc/art_bvh.hip" -o "$tmp/art_bvh.o" &
hipcc "${flags[@]}" "${sched[@]}" -x hip -c "$pkg/csrc/art_capi.cpp" -o "$tmp/art_capi.o" &
hipcc "${flags[@]}" "${sched[@]}" -x hip -c "$pkg/csrc/art_synth.cpp" -o "$tmp/art_synth.o" &
hipcc "${flags[@]}" "${sched[@]}" -x hip -c "$pkg/csrc/art_cpu.cpp" -o "$tmp/art_cpu.o" &
wait
hipcc --offload-arch=gfx950 -shared -fPIC -rdynamic -o "$root/variants/libart_$name.so" "$tmp"/*.o
rm -rf "$tmp"
echo "variants/libart_$name.so"
