#!/bin/bash
# Per-kernel VGPRs, spills, occupancy and LDS of one HIP source, as the compiler reports them.
#   tools/kres.sh [csrc/art_trace.hip] [-DFLAG ...]
set -euo pipefail
root=$(cd "$(dirname "$0")/.." && pwd)
src=${1:-$root/audio-raytracer_amd/csrc/art_trace.hip}; shift || true
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off "$@" -c "$src" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys, subprocess
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m: continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip().split("(")[0]}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    g = r.get
    print("%-60s vgpr=%s vspill=%s sspill=%s occ=%s lds=%s" % (g("name")[:60], g("VGPRs"), g("VGPRs Spill"), g("SGPRs Spill"), g("Occupancy [waves/SIMD]"), g("LDS Size [bytes/block]")))
'
