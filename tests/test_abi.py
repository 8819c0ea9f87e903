"""CPU tests of the C ABI library (no compute calls): it loads, exports every symbol the
headers declare, its struct layouts match the C# structs, and it fails loudly without a GPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import art
from art import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("art.h", "art_device.h", "art_synth.h", "art_dsp.h",
                                                                 "art_colliders.h")]


def declared_symbols():
    names = set()
    for h in HEADERS:
        for m in re.finditer(r"ART_API\s+[^;(]*?\b(art_\w+)\s*\(", open(h).read()):
            names.add(m.group(1))
    return names


def test_headers_declare_expected_surface():
    names = declared_symbols()
    for n in ("art_create", "art_schedule", "art_is_completed", "art_complete", "art_destroy", "art_last_error",
              "art_scene_bind", "art_launch_device", "art_synth_scene"):
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = art.load_library()
    missing = [n for n in sorted(declared_symbols()) if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding knows every one of them
    assert declared_symbols() == set(abi.SIGNATURES), declared_symbols() ^ set(abi.SIGNATURES)


def test_only_art_symbols_exported():
    import subprocess
    out = subprocess.check_output(["nm", "-D", "--defined-only", abi.LIB_PATH], text=True)
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert exported == declared_symbols(), exported ^ declared_symbols()


def test_struct_sizes_match_csharp_layouts():
    assert abi.AABB.itemsize == 20      # ColliderAABBStruct.cs:10-14
    assert abi.OBB.itemsize == 26       # ColliderOBBStruct.cs:10-24
    assert abi.SPHERE.itemsize == 16    # ColliderSphereStruct.cs:10-14
    assert abi.SETTINGS.itemsize == 24  # AudioTargetRTSettings.cs:11-16
    assert C.sizeof(abi.art_fan) == 12 + 4 + 8 * 8  # origin float[3] + pad + 8 pointers
    offs = {n: getattr(abi.art_fan, n).offset for n, _ in abi.art_fan._fields_}
    assert offs["ray_hit_counts"] == 64 and offs["ray_hit_ids"] == 72  # appended after the editor arrays
    assert C.sizeof(abi.art_fan_layout) == 9 * 4
    assert C.sizeof(abi.art_exec_counts) == 8 * 8 + 16 * 8 + 3 * 5 * 8  # 2.3: by_kernel appended
    assert C.sizeof(abi.art_kernel_times) == 3 * 8 + 2 * 4 + 4 * 8 + 4 * 4  # 3.0: per kernel family


def test_header_struct_sizes_match_bindings(tmp_path):
    """The C compiler's view of include/*.h (what a P/Invoke or cgo caller builds against) equals
    the ctypes mirror, struct by struct."""
    import subprocess
    structs = {"art_fan": abi.art_fan, "art_fan_layout": abi.art_fan_layout, "art_exec_counts": abi.art_exec_counts,
               "art_kernel_times": abi.art_kernel_times, "art_test_counts": abi.art_test_counts,
               "art_collider_sync_stats": abi.art_collider_sync_stats}
    src = tmp_path / "sizes.c"
    src.write_text('#include <stdio.h>\n#include "art_device.h"\n#include "art_colliders.h"\nint main(void) {\n' +
                   "".join(f'  printf("{n} %zu\\n", sizeof({n}));\n' for n in structs) + "  return 0;\n}\n")
    exe = tmp_path / "sizes"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict(l.split() for l in subprocess.check_output([str(exe)], text=True).splitlines())
    for n, t in structs.items():
        assert int(got[n]) == C.sizeof(t), (n, got[n], C.sizeof(t))


def test_version():
    v = art.load_library().art_version()
    # 3.0: art_kernel_times per kernel family (a grown struct: major bump); 3.1: ART_CTX_EVENT_EACH_LAUNCH,
    # art_recip_exact_device
    assert v >> 16 == 3 and v & 0xffff >= 1


def test_no_gpu_fails_loudly():
    lib = art.load_library()
    if lib.art_device_count() > 0:
        pytest.skip("a HIP device is present")
    p = C.c_void_p()
    assert lib.art_create(1, C.byref(p)) == abi.ART_E_DEVICE
    with pytest.raises(art.ArtError):
        art.Context(1)
    # device_mask 0 is the CPU backend: it needs no device; its device entry points refuse
    with art.Context(0) as cpu:
        assert cpu.lib.art_launch_device(cpu.ptr, None, 0, None, 0, None) == abi.ART_E_UNSUPPORTED


def _frame(ci=1, **over):
    scene, org, params = art.synth(art.CONFIGS[ci], S=2, R=64)
    for k, v in over.items():
        setattr(params, k, v)
    return art.Frame(scene, params, org, art.FanOutputs(2, 64, params.max_hits_per_ray, scene.T,
                                                         params.thread_count))


def test_layout_and_validation_without_device():
    fr = _frame()
    lay = art.fan_layout(fr)
    assert lay["stride"] % 16 == 0
    assert lay["echo_off"] >= lay["perm_off"] + 4 * 4
    lay_h = art.fan_layout(fr, abi.ART_OUT_HIT_RESULTS)
    assert lay_h["stride"] >= lay["stride"] + 64 * 5 * 6 + 64 + 64 * 5 * 4
    assert lay_h["hit_ids_off"] % 16 == 0 and lay_h["hit_ids_off"] >= lay_h["hit_counts_off"] + 64
    assert lay_h["hit_ids_off"] + 64 * 5 * 4 <= lay_h["stride"]
    with pytest.raises(art.ArtError) as e:
        art.fan_layout(_frame(max_hits_per_ray=33))
    assert e.value.code == abi.ART_E_UNSUPPORTED
    bad = _frame()
    bad.desc.audio_target_count = 0
    with pytest.raises(art.ArtError) as e:
        art.fan_layout(bad)
    assert e.value.code == abi.ART_E_INVALID


def test_synth_is_deterministic_and_matches_config():
    a = art.synth(art.CONFIGS[2], S=4, R=64)
    b = art.synth(art.CONFIGS[2], S=4, R=64)
    assert np.array_equal(a[0].aabbs.view(np.uint8), b[0].aabbs.view(np.uint8))
    assert np.array_equal(a[1], b[1])
    sc = a[0]
    assert sc.spheres.size == 2048 and sc.aabbs.size == 2048 and sc.obbs.size == 0 and sc.T == 4
    assert list(sc.spheres["audio_target_id"][:4]) == [0, 1, 2, 3]
    assert (sc.spheres["audio_target_id"][4:] == -1).all()


def test_fibonacci_directions_match_the_oracle():
    import oracle
    for R in (2, 64, 314, 512, 1000):
        d1 = np.zeros((R, 3), np.uint16)
        d2 = np.zeros((R, 3), np.uint16)
        art.load_library().art_fibonacci_directions(R, d1.ctypes.data)
        oracle.load().or_fibonacci_directions(R, d2.ctypes.data)
        assert np.array_equal(d1, d2)
        # Jobs/FibonacciDirectionsJobParallel.cs:27: first ray points straight up, last straight down
        assert d1[0].tolist() == [0, 0x3C00, 0] and d1[-1, 1] == 0xBC00


def test_batch_size_matches_reference_formula():
    p = art.FrameParams(thread_count=3)
    assert p.batch_size(314) == 105   # ceil(314 / 3) — AudioRayTracer.cs:161
    assert art.FrameParams(thread_count=1).batch_size(512) == 512


def test_hit_id_encoding():
    """ART_HIT_ID = ColliderType (Enums/ColliderType.cs: None, AABB, OBB, Sphere) << 30 | index."""
    hdr = open(os.path.join(ROOT, "include", "art.h")).read()
    for name, v in (("ART_COLLIDER_AABB", 1), ("ART_COLLIDER_OBB", 2), ("ART_COLLIDER_SPHERE", 3)):
        assert re.search(rf"#define {name}\s+{v}u", hdr)
        assert getattr(abi, name) == v
    assert "#define ART_HIT_NONE 0xFFFFFFFFu" in hdr and abi.ART_HIT_NONE == 0xFFFFFFFF
    assert abi.hit_id(abi.ART_COLLIDER_SPHERE, 5) == 0xC0000005
