#!/bin/bash
# Round-4 GPU pass 4: configs 4 and 5 profiles (bench line, kernel trace, PMC) and the config-2
# rebuild-frame profile, on the committed build.
set -euo pipefail
export TMPDIR=/tmp
for c in ${1:-4 5}; do bash tools/gpu_round.sh r04_c$c $c; done
bash tools/r04_rebuild.sh
