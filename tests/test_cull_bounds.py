"""CPU check of the OBB broad-phase bounds (prep_obb's rotated-box bounds).

tools/obb_cull_check.cpp builds the product's OBB records and cull bounds from random C# structs and
casts rays aimed at the boxes' faces, edges and corners through the product's exact OBB test (the
raytrace cast's stored rotation and the permeation first hit's inverse rotation): every reported
hit must pass the node test on the collider's bounds with a quarter of its margin, and the test must
catch a bound without margins (so it can fail)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which("hipcc") is None:
        pytest.skip("hipcc not available")
    exe = str(tmp_path_factory.mktemp("obb") / "obb_cull_check")
    subprocess.check_call(["hipcc", "-x", "hip", "-O2", "-std=c++17", "-ffp-contract=off", "-w",
                           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "audio-raytracer_amd", "csrc"),
                           os.path.join(ROOT, "tools", "obb_cull_check.cpp"), "-o", exe])
    return exe


def run(exe, cases, frac):
    p = subprocess.run([exe, str(cases), str(frac)], capture_output=True, text=True)
    line = p.stdout.strip().splitlines()[-1]
    fields = line.split(":")[1].split(",")
    hits, fails = int(fields[1].split()[0]), int(fields[2].split()[0])
    return p.returncode, hits, fails


def test_obb_bounds_hold_every_reported_hit(checker):
    rc, hits, fails = run(checker, 1_000_000, 0.25)
    assert hits > 900_000
    assert rc == 0 and fails == 0


def test_obb_bounds_check_is_sensitive(checker):
    rc, hits, fails = run(checker, 1_000_000, 0.0)  # no margin: grazing hits fall outside
    assert fails > 0 and rc != 0
