"""Ray directions on the device (art_fibonacci_directions_device, SURVEY.md §8 f rank 3).

FibonacciDirectionsJobParallel.Execute (Jobs/FibonacciDirectionsJobParallel.cs:15-35) on the GPU
must equal, bit for bit, the host generator art_fibonacci_directions (the reference's float
sequence, cos/sin rounded correctly to float through double evaluation on both sides), and the
oracle's or_fibonacci_directions (the same sequence with glibc's cosf/sinf) up to 65536 rays;
past that glibc misses the correct rounding on a few arguments per million.
Burst's cos/sin (FloatPrecision.Standard) are not reproducible without the engine, so against
the reference itself this row is parity-unpinned; directions stay an input of the frame.
"""
import numpy as np
import pytest

import art
from art import abi
import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("count", [1, 2, 3, 64, 511, 512, 1000, 4096, 65536, 1 << 20])
def test_device_directions_equal_host_and_oracle(ctx, count):
    import torch
    d = torch.zeros(count * 3, dtype=torch.int16, device="cuda")
    rc = ctx.lib.art_fibonacci_directions_device(ctx.ptr, count, d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    dev = d.cpu().numpy().view(np.uint16).reshape(count, 3)
    host = np.zeros((count, 3), np.uint16)
    art.load_library().art_fibonacci_directions(count, host.ctypes.data)
    assert dev.tobytes() == host.tobytes(), f"{int((dev != host).any(axis=1).sum())} of {count} rays differ"
    ref = np.zeros((count, 3), np.uint16)
    oracle.load().or_fibonacci_directions(count, ref.ctypes.data)
    bad = (dev != ref).any(axis=1)
    if count <= 65536:
        assert not bad.any()
    else:
        # the product rounds cos/sin correctly (double evaluation); glibc's cosf/sinf (the oracle)
        # miss the correct rounding on a few arguments, and a half rounding flips with them: one
        # component, one half ulp apart
        assert bad.sum() <= 16, int(bad.sum())
        diff = np.abs(dev[bad].astype(np.int32) - ref[bad].astype(np.int32))
        assert (diff <= 1).all() and ((diff != 0).sum(axis=1) == 1).all()
    if count >= 2:  # :27 — the first ray is (0, 1, 0) up to the sign of zero, the last (0, -1, 0)
        assert dev[0, 1] == 0x3C00 and dev[-1, 1] == 0xBC00


def test_device_directions_invalid(ctx):
    with pytest.raises(Exception):
        rc = ctx.lib.art_fibonacci_directions_device(ctx.ptr, -1, None, None)
        if rc:
            ctx._raise(rc)
    assert ctx.lib.art_fibonacci_directions_device(ctx.ptr, 0, None, None) == abi.ART_OK
