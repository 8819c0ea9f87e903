#!/bin/bash
# kd phase timings of the final build (diagnostic variant) + bvh leaf/upper context
set -euo pipefail
export TMPDIR=/tmp
bash tools/r04_kdprof.sh
