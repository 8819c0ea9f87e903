"""The OBB slab's reciprocal over every one of the 2^32 float bit patterns.

RayIntersectsOBB (Jobs/AudioRaytracerJobBatched.cs:314-320) runs RayIntersectsAABB's slab
(:284-308), whose `1.0f / rayDir` (:289) Burst evaluates as an IEEE division. The kernels compute
it with `recip_exact` (art_device_fns.hpp): v_rcp_f32 plus one Newton step where the exponent
field lies in [3, 251], the division elsewhere. The claim that this equals the IEEE quotient bit for
bit is checked here on the product function itself (art_recip_exact_device runs the kernels'
recip_exact), against numpy's float32 division (x86 divss, correctly rounded), for all 2^32 inputs.
NaN results compare as NaN (payloads free: a NaN operand never reaches a comparison that passes).
"""
import numpy as np
import pytest

CHUNK = 1 << 27


def _ieee_recip(first: int, count: int) -> np.ndarray:
    x = (np.arange(count, dtype=np.uint32) + np.uint32(first)).view(np.float32)  # (wraps past 0xFFFFFFFF)
    with np.errstate(divide="ignore", over="ignore", under="ignore", invalid="ignore"):
        return (np.float32(1.0) / x).view(np.uint32)


def test_ieee_reference_kats():
    # the host reference itself: 1/2 = 0.5, 1/-0 = -inf, 1/denormal_min = +inf (overflow), 1/3 rounded
    r = _ieee_recip(0x40000000, 1)[0]
    assert r == np.float32(0.5).view(np.uint32)
    assert _ieee_recip(0x80000000, 1)[0] == np.float32(-np.inf).view(np.uint32)
    assert _ieee_recip(0x00000001, 1)[0] == np.float32(np.inf).view(np.uint32)
    assert _ieee_recip(np.float32(3.0).view(np.uint32), 1)[0] == 0x3EAAAAAB


@pytest.mark.gpu
def test_device_recip_all_patterns(ctx):
    import torch
    d = torch.empty(CHUNK, dtype=torch.int32, device="cuda")
    host = torch.empty(CHUNK, dtype=torch.int32).pin_memory()
    st = torch.cuda.current_stream()
    for first in range(0, 1 << 32, CHUNK):
        rc = ctx.lib.art_recip_exact_device(ctx.ptr, first, CHUNK, d.data_ptr(), st.cuda_stream)
        assert rc == 0
        host.copy_(d)
        got = host.numpy().view(np.uint32)
        ref = _ieee_recip(first, CHUNK)
        nan_got = (got & 0x7F800000) == 0x7F800000
        nan_got &= (got & 0x007FFFFF) != 0
        nan_ref = ((ref & 0x7F800000) == 0x7F800000) & ((ref & 0x007FFFFF) != 0)
        bad = np.flatnonzero((got != ref) & ~(nan_got & nan_ref))
        assert bad.size == 0, f"x bits {first + int(bad[0]):#010x}: recip_exact {got[bad[0]]:#010x} IEEE {ref[bad[0]]:#010x}"
