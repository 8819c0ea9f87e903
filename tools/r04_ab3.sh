#!/bin/bash
# A/B of the muffle changes (XCD target order, 4-B cell entries) on configs 2 and 5
set -uo pipefail
export TMPDIR=/tmp
for c in 5 2; do bash tools/ab_rt.sh $c nospill base noxcd nocompact || exit 1; done
