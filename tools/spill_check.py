#!/usr/bin/env python3
"""Static spill report of a HIP source's gfx950 kernels (the fused-variant hang).

  python3 tools/spill_check.py [csrc/art_trace.hip] [-DFLAG ...]

For every kernel: its VGPR count and scratch use, and for each spill slot the stores and reloads
with the loop they sit in (the compiler's "Loop Header" / "in Loop" block annotations). A spill
stored inside a divergent loop (a narrowed exec mask) and reloaded after it can hand the reloading
lanes values they never stored; spills outside every loop are read back by the lanes that stored them."""
import re
import subprocess
import sys
import tempfile

root = __file__.rsplit("/tools/", 1)[0]
src = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else f"{root}/audio-raytracer_amd/csrc/art_trace.hip"
flags = [a for a in sys.argv[1:] if a.startswith("-")]
import os
src = os.path.abspath(src)
with tempfile.TemporaryDirectory() as d:
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--save-temps", *flags, "-c",
                    src, "-o", f"{d}/o.o"], cwd=d, check=True, capture_output=True)
    import glob
    asm = open(glob.glob(f"{d}/*gfx950.s")[0]).read().splitlines()

kernels, cur = [], None
for i, line in enumerate(asm):
    m = re.match(r"^(_Z\S+):\s*;\s*@", line)
    if m:
        cur = {"name": m.group(1), "lines": []}
        kernels.append(cur)
        continue
    if cur is not None:
        if line.startswith(".Lfunc_end"):
            cur = None
        else:
            cur["lines"].append(line)

def demangle(n):
    return subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip().split("(")[0]

for k in kernels:
    loop = "not in a loop"
    sites = []
    for line in k["lines"]:
        if re.match(r"^(\.LBB\S+:|; %bb\.\d+:)", line):  # a block label: its loop annotation, if any
            loop = line.split(";", 1)[1].strip() if ("Loop" in line and ";" in line) else "not in a loop"
        elif "Loop Header" in line or "in Loop" in line or "Parent Loop" in line:
            loop = line.split(";", 1)[1].strip()
        m = re.search(r"scratch_(store|load)_dword\w*\s", line)
        if m:
            off = re.search(r"offset:(\d+)", line)
            sites.append((m.group(1), int(off.group(1)) if off else 0, loop))
    name = demangle(k["name"])
    if not sites:
        continue
    print(f"{name[:160]}: {len(sites)} scratch ops")
    for kind, off, lp in sites[:int(os.environ.get("SPILL_SITES", "1000"))]:
        print(f"   {kind:5s} slot {off:3d}  {lp}")
print("kernels with scratch:", sum(1 for k in kernels if any("scratch_" in l for l in k["lines"])), "of", len(kernels))
