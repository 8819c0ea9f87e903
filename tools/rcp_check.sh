#!/bin/bash
# Build and run tools/rcp_check.hip (the exhaustive recip_exact check) on the GPU box.
set -euo pipefail
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/rcp_check.hip -o gpurun_out/rcp_check
timeout -k 10 120 gpurun_out/rcp_check | tee gpurun_out/rcp_check.txt
