"""The traversals' one-division sphere test (csrc/art_device_fns.hpp sphere_test_1div) against the
two-division RayIntersectsSphere (Jobs/AudioRaytracerJobBatched.cs:323-355, sphere_test): the same
verdict and distance bits on 2 x 10^6 random, scaled, degenerate and denormal cases, and on raw
bit patterns of the quotient selection (tools/check_sphere_1div.cpp, host-compiled; no GPU)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not found")
def test_sphere_one_division_equals_two(tmp_path):
    exe = tmp_path / "chk"
    subprocess.run(["hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-x", "hip",
                    "-I", os.path.join(ROOT, "audio-raytracer_amd", "csrc"),
                    os.path.join(ROOT, "tools", "check_sphere_1div.cpp"), "-o", str(exe)], check=True,
                   capture_output=True)
    r = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
