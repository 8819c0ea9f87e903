"""f32tof16 over every one of the 2^32 float bit patterns (the conversion of
every echo, hit point and ray direction: Utility/HalfDataTypesUtility.cs:86-90 ->
Unity.Mathematics math.f32tof16 at AudioRaytracerJobBatched.cs:76,118,142).

The oracle (oracle/art_oracle.c or_f32tof16) restates the package's algorithm, including its
overflow "clamp" against the float literal 260042752.0f that never clamps: finite |x| >= 65520
give the bit patterns the package gives (e.g. 70000 -> 0x7C46), so the build matches Unity even
outside the half range and needs no |x| < 65504 guard at its conversion sites. Host product
(libart's unity_math.hpp through art_f32tof16_range) and device product (the kernels'
f32tof16 through art_f32tof16_device) must equal it on all 2^32 inputs.
"""
import numpy as np
import pytest

import art
from art import abi
import oracle

CHUNK = 1 << 27


def test_kat_outside_half_range():
    # the package's non-clamping literal: 70000 keeps its (rebased) bits instead of becoming inf
    from art.synth import f32tof16
    assert oracle.f32tof16(70000.0) == 0x7C46 == f32tof16(70000.0)
    assert oracle.f32tof16(65519.0) == 0x7BFF and oracle.f32tof16(-65520.0) == 0xFC00


def test_host_product_all_patterns():
    lib = art.load_library()
    got = np.empty(CHUNK, np.uint16)
    for first in range(0, 1 << 32, CHUNK):
        lib.art_f32tof16_range(first, CHUNK, got.ctypes.data)
        ref = oracle.f32tof16_range(first, CHUNK)
        bad = np.flatnonzero(got != ref)
        assert bad.size == 0, f"bits {first + int(bad[0]):#010x}: host {got[bad[0]]:#06x} oracle {ref[bad[0]]:#06x}"


@pytest.mark.gpu
def test_device_all_patterns(ctx):
    import torch
    d = torch.empty(CHUNK, dtype=torch.int16, device="cuda")
    host = torch.empty(CHUNK, dtype=torch.int16).pin_memory()
    st = torch.cuda.current_stream()
    for first in range(0, 1 << 32, CHUNK):
        rc = ctx.lib.art_f32tof16_device(ctx.ptr, first, CHUNK, d.data_ptr(), st.cuda_stream)
        assert rc == 0
        host.copy_(d)
        got = host.numpy().view(np.uint16)
        ref = oracle.f32tof16_range(first, CHUNK)
        bad = np.flatnonzero(got != ref)
        assert bad.size == 0, f"bits {first + int(bad[0]):#010x}: device {got[bad[0]]:#06x} oracle {ref[bad[0]]:#06x}"
