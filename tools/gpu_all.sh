#!/bin/bash
# Round profiles of every 1-GPU config: tools/gpu_round.sh for configs 2..5 (parity tests once, first).
#   bash tools/gpu_all.sh <round-tag>    -> gpurun_out/<round-tag>_c<k>/
set -euo pipefail
r=${1:-r02}
bash tools/gpu_round.sh "${r}_c2" 2 tests
for c in 3 4 5; do bash tools/gpu_round.sh "${r}_c$c" "$c"; done
