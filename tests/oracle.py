"""TEST INFRASTRUCTURE: ctypes binding of the CPU oracle (oracle/libart_oracle.so).

The oracle is a plain-C restatement of the reference jobs (oracle/art_oracle.c). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and only as the checker /
CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-raytracer_amd"))

from art import abi  # noqa: E402
from art.frame import FanOutputs, Frame  # noqa: E402

ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "build", "libart_oracle.so")

_lib = None
_native = None


def load_native():
    """bench.py's CPU-baseline leg only: the oracle rebuilt with -march=native for the host it runs
    on (SURVEY.md 8(d)'s recipe), into a scratch directory, when gcc is present; otherwise the shipped
    x86-64-v3 library. Returns (library, label of the build that ran). The checker (load()) stays
    the portable build, so parity never depends on the host's instruction set."""
    global _native
    if _native is not None:
        return _native
    import shutil
    import tempfile
    label = "gcc -O3 -march=x86-64-v3 -ffp-contract=off (the shipped portable build: no compiler on this host)"
    path = None
    if shutil.which("gcc"):
        d = tempfile.mkdtemp(prefix="art_oracle_native_")
        path = os.path.join(d, "libart_oracle_native.so")
        cmd = ["gcc", "-O3", "-march=native", "-std=c11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-pthread",
               "-shared", "-o", path, os.path.join(ORACLE_DIR, "art_oracle.c"), "-lm"]
        try:
            subprocess.run(cmd, check=True, capture_output=True, timeout=120)
            label = "gcc -O3 -march=native -ffp-contract=off, built on this host at run time"
        except Exception as e:  # noqa: BLE001 - fall back to the portable build, and say so
            path = None
            label += f" (native build failed: {type(e).__name__})"
    lib = _bind(C.CDLL(path)) if path else load()
    _native = (lib, label)
    return _native


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_LIB):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    _lib = _bind(C.CDLL(ORACLE_LIB))
    return _lib


def _bind(lib):
    lib.or_f32tof16.restype = C.c_uint16
    lib.or_f32tof16.argtypes = [C.c_float]
    lib.or_f32tof16_range.argtypes = [C.c_uint32, C.c_uint32, C.c_void_p]
    lib.or_f16tof32.restype = C.c_float
    lib.or_f16tof32.argtypes = [C.c_uint16]
    lib.or_fibonacci_directions.argtypes = [C.c_int32, C.c_void_p]
    lib.or_run_frame.restype = C.c_int
    lib.or_run_frame.argtypes = [C.POINTER(abi.art_frame_desc), C.POINTER(abi.art_fan), C.c_int32, C.c_int32,
                                 C.POINTER(abi.art_test_counts)]
    f3 = C.c_float * 3
    f4 = C.c_float * 4
    for name in ("or_ray_intersects_aabb",):
        fn = getattr(lib, name); fn.restype = C.c_int; fn.argtypes = [f3, f3, f3, f3, C.POINTER(C.c_float)]
    lib.or_ray_intersects_sphere.restype = C.c_int
    lib.or_ray_intersects_sphere.argtypes = [f3, f3, f3, C.c_float, C.POINTER(C.c_float)]
    lib.or_ray_intersects_obb.restype = C.c_int
    lib.or_ray_intersects_obb.argtypes = [f3, f3, f3, f3, f4, C.POINTER(C.c_float)]
    lib.or_dsp_process.restype = C.c_int
    lib.or_dsp_process.argtypes = [C.POINTER(abi.art_spatializer_settings), C.POINTER(abi.art_audio_source), C.c_int32,
                                   C.c_int32]
    lib.or_half_quaternion_value.argtypes = [C.c_uint16, C.c_uint16, C.c_uint16, f4]
    lib.or_quat_inverse.argtypes = [f4, f4]
    lib.or_quat_mul_vec.argtypes = [f4, f3, f3]
    return lib


def run_frame(frame: Frame, threads: int = 1, lib=None):
    """Run the oracle on `frame` (writes into frame.out); returns the per-kind test counts."""
    lib = lib or load()
    cnt = abi.art_test_counts()
    rc = lib.or_run_frame(C.byref(frame.desc), frame.fans, frame.S, threads, C.byref(cnt))
    if rc:
        raise RuntimeError(f"or_run_frame failed: {rc}")
    return cnt.as_dict()


def run(scene, params, origins, out: FanOutputs, threads: int = 1, lib=None):
    fr = Frame(scene, params, origins, out)
    counts = run_frame(fr, threads, lib)
    return out, counts


def f32tof16(x: float) -> int:
    return int(load().or_f32tof16(x))


def f32tof16_range(first: int, count: int):
    import numpy as np
    out = np.empty(count, np.uint16)
    load().or_f32tof16_range(first, count, out.ctypes.data)
    return out


def f16tof32(h: int) -> float:
    return float(load().or_f16tof32(h))


def dsp_process(settings, sources, sample_rate: int = 48000):
    """Oracle AudioSpatializer.OnAudioFilterRead (art_oracle.c §8) over art.dsp.AudioSource objects."""
    from art import dsp
    lib = load()
    st = settings.to_c()
    arr = dsp.sources_to_c(sources)
    rc = lib.or_dsp_process(C.byref(st), arr, len(sources), sample_rate)
    assert rc == 0, rc
