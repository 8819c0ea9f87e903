"""Per-sample spatializer DSP (include/art_dsp.h, SURVEY.md §8 f rank 1).

CPU: the oracle's restatement of AudioSpatializer.OnAudioFilterRead against hand-derived answers
(impulse through the neutral chain, channel gate, state carry across buffers). GPU: libart.so
(art_dsp_process, art_dsp_process_device) against the oracle, bit for bit, over randomised
sources, settings and carried filter state. The per-buffer scalars use the host libm's atan2 /
sin / cos in both; Burst's are not reproducible here, so that part is parity-unpinned by the
reference (documented in DESIGN.md).
"""
import math

import numpy as np
import pytest

import art
from art import abi
from art.dsp import AudioSource, SpatializerSettings
import oracle

f32 = np.float32


def neutral_settings(**kw):
    s = SpatializerSettings(pan_strength=0.0, rear_attenuation_strength=0.2, distance_based_panning=False,
                            distance_based_rear_attenuation=False)
    for k, v in kw.items():
        setattr(s, k, v)
    return s


def test_oracle_impulse_neutral_chain():
    """Front source on the horizon (local_dir (0,0,1)): no muffle, dry boost 1 (curve(0) = 0),
    gains sqrt(0.5), rear attenuation 1, elevation 1, low pass at 5000 Hz * (1 - 0.5 * d/12)."""
    st = neutral_settings()
    x = np.zeros(2 * 8, np.float32)
    x[0] = 1.0
    x[1] = 1.0
    src = AudioSource(data=x.copy(), local_dir=(0.0, 0.0, 1.0), listener_distance=0.0)
    oracle.dsp_process(st, [src], 48000)
    g = np.sqrt(f32(0.5) * (f32(1) - f32(0)), dtype=np.float32)
    gain = f32(f32(g * f32(1)) * f32(1))
    cutoff = f32(f32(5000) * f32(f32(1) - f32(f32(0.5) * f32(0))))
    rc = f32(f32(1) / f32(cutoff * f32(f32(2) * f32(3.14159265))))
    dt = f32(f32(1) / f32(48000))
    alpha = f32(dt / f32(rc + dt))
    y = f32(0)
    expect = []
    for n in range(8):
        inp = f32(f32(x[2 * n] * f32(1)) * gain)
        y = f32(y + f32(alpha * f32(inp - y)))
        expect.append(y)
    assert np.array_equal(src.data[0::2], np.array(expect, np.float32))
    assert np.array_equal(src.data[1::2], np.array(expect, np.float32))
    assert src.state["previous_lp"][0][0] == expect[-1]


def test_oracle_mono_untouched_and_state_carry():
    rng = np.random.default_rng(5)
    st = SpatializerSettings()
    mono = AudioSource(data=rng.standard_normal(64).astype(np.float32), channels=1, muffle_strength=0.5)
    before = mono.data.copy()
    oracle.dsp_process(st, [mono], 48000)
    assert np.array_equal(mono.data, before)  # AudioSpatializer.cs:72
    # one 256-frame buffer == two 128-frame buffers with the state carried
    x = rng.standard_normal(512).astype(np.float32)
    kw = dict(muffle_strength=0.7, reverb_volume=0.4, local_dir=(0.3, 0.5, 0.81), listener_distance=3.0,
              volume_multiplier=1.3)
    whole = AudioSource(data=x.copy(), **kw)
    oracle.dsp_process(st, [whole], 44100)
    a = AudioSource(data=x[:256].copy(), **kw)
    oracle.dsp_process(st, [a], 44100)
    b = AudioSource(data=x[256:].copy(), state=a.state.copy(), **kw)
    oracle.dsp_process(st, [b], 44100)
    assert np.array_equal(whole.data, np.concatenate([a.data, b.data]))
    assert whole.state.tobytes() == b.state.tobytes()


def random_sources(rng, n, frames_choices=(1, 2, 3, 7, 64, 255, 256, 1024)):
    out = []
    for i in range(n):
        frames = int(rng.choice(frames_choices))
        d = rng.standard_normal(3)
        d /= np.linalg.norm(d)
        st = np.zeros(1, abi.DSP_STATE)
        st.view(np.float32)[:] = rng.standard_normal(8).astype(np.float32) * 0.1
        out.append(AudioSource(data=(rng.standard_normal(frames * 2) * 0.5).astype(np.float32),
                               channels=2 if i % 11 else 1,
                               muffle_strength=float(rng.choice([0.0, rng.random()])), reverb_volume=float(rng.random()),
                               local_dir=tuple(float(v) for v in d), listener_distance=float(rng.uniform(0, 30)),
                               volume_multiplier=float(rng.uniform(0, 2)), state=st))
    return out


def random_settings(rng):
    return SpatializerSettings(
        pan_strength=float(rng.random()), rear_attenuation_strength=float(rng.random()),
        distance_based_panning=bool(rng.random() < 0.5), max_pan_distance=float(rng.uniform(1, 10)),
        distance_based_rear_attenuation=bool(rng.random() < 0.5), max_rear_attenuation_distance=float(rng.uniform(1, 30)),
        max_elevation_effect_distance=float(rng.uniform(1, 20)),
        muffle_curve=rng.random(int(rng.integers(2, 60))).astype(np.float32),
        reverb_volume_curve=rng.random(int(rng.integers(2, 60))).astype(np.float32))


def _sat(x):
    return f32(max(f32(0), min(f32(1), f32(x))))


def _lerp(a, b, t):
    return f32(f32(a) + f32(f32(t) * f32(f32(b) - f32(a))))


def _curve(baked, length, time):
    n = baked.size
    cp = f32(max(f32(0), min(f32(n - 1), f32(f32(f32(time) / f32(length)) * f32(n - 1)))))
    fi, ci = int(np.floor(cp)), int(np.ceil(cp))
    return _lerp(baked[fi], baked[ci], f32(cp - f32(fi)))


def _alpha_lp(cutoff, sr):
    rc = f32(f32(1) / f32(f32(cutoff) * f32(f32(2) * f32(3.14159265))))
    dt = f32(f32(1) / f32(sr))
    return f32(dt / f32(rc + dt))


def _alpha_hp(cutoff, sr):
    rc = f32(f32(1) / f32(f32(cutoff) * f32(f32(2) * f32(3.14159265))))
    dt = f32(f32(1) / f32(sr))
    return f32(rc / f32(rc + dt))


def test_source_params_host_matches_definition():
    """art_dsp_source_params_get (host side of libart.so) against a numpy float32 restatement of
    MuffleDSP.cs:22-26/40-42, ReverbDSP.cs:12-13 and BinauralDSP.cs:17-50/65/73/89-101, bit for
    bit. BinauralDSP.Process is managed code (no [BurstCompile] under Audio/), so Unity.Mathematics'
    float atan2/sin/cos there are (float)System.Math.Atan2/Sin/Cos: evaluated in double, rounded
    once to float (Python's math module: the C double functions)."""
    rng = np.random.default_rng(9)
    st = random_settings(rng)
    sr = 48000
    for src in random_sources(rng, 400):
        if src.channels != 2:
            continue
        p = art.dsp.source_params(st, src, sr)[0]
        ld = [f32(v) for v in src.local_dir]
        dist = f32(src.listener_distance)
        muffle = src.muffle_strength > 0
        assert bool(p["flags"] & 1) == muffle
        if muffle:
            m = _curve(st.muffle_curve, st.muffle_curve_length, src.muffle_strength)
            cut = _lerp(st.muffle_cutoff[1], st.muffle_cutoff[0], m)
            assert p["muffle_alpha"] == _alpha_lp(cut, sr)
        t = _curve(st.reverb_volume_curve, st.reverb_volume_curve_length, src.reverb_volume)
        assert p["dry_boost"] == _lerp(st.reverb_dry_boost[0], st.reverb_dry_boost[1], t)
        assert bool(p["flags"] & 2) == bool(ld[1] <= 0)
        ef = _sat(f32(dist / f32(st.max_elevation_effect_distance)))
        if ld[1] <= 0:
            cut = f32(_lerp(st.low_pass_cutoff[0], st.low_pass_cutoff[1], _sat(-ld[1])) * f32(f32(1) - f32(f32(0.5) * ef)))
            assert p["filter_alpha"] == _alpha_lp(cut, sr)
        else:
            cut = f32(_lerp(st.high_pass_cutoff[0], st.high_pass_cutoff[1], _sat(ld[1])) * f32(f32(1) + f32(f32(0.5) * ef)))
            assert p["filter_alpha"] == _alpha_hp(cut, sr)
        az = f32(f32(math.atan2(float(ld[0]), float(ld[2]))) * f32(57.29578))
        eps = f32(st.pan_strength)
        if st.distance_based_panning:
            eps = f32(eps * _sat(f32(dist / f32(st.max_pan_distance))))
        pan = f32(f32(math.sin(float(f32(az * f32(0.0174532924))))) * eps)
        gl = np.sqrt(f32(f32(0.5) * f32(f32(1) - pan)), dtype=np.float32)
        gr = np.sqrt(f32(f32(0.5) * f32(f32(1) + pan)), dtype=np.float32)
        front = f32(max(f32(0), f32(math.cos(float(f32(az * f32(0.0174532924)))))))
        rear = _lerp(f32(1) - f32(st.rear_attenuation_strength), 1, front)
        if st.distance_based_rear_attenuation:
            df = _sat(f32(f32(1) - f32(dist / f32(st.max_rear_attenuation_distance))))
            lo = f32(f32(1) - f32(st.rear_attenuation_strength))
            rear = f32(max(lo, min(f32(1), f32(rear * df))))
        elev = _lerp(1, st.low_pass_volume, _sat(-ld[1])) if ld[1] <= 0 else _lerp(1, st.high_pass_volume, _sat(ld[1]))
        assert p["gain_left"] == f32(f32(gl * rear) * elev)
        assert p["gain_right"] == f32(f32(gr * rear) * elev)
        assert p["volume"] == f32(src.volume_multiplier)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_matches_oracle(ctx, seed):
    rng = np.random.default_rng(seed)
    st = random_settings(rng)
    srcs = random_sources(rng, 150)
    ref = [s.copy() for s in srcs]
    for call in range(3):  # state carried across calls
        for s, r in zip(srcs, ref):
            x = (rng.standard_normal(s.data.size) * 0.5).astype(np.float32)
            s.data[:] = x
            r.data[:] = x
        art.dsp.process(ctx, st, srcs, 48000)
        oracle.dsp_process(st, ref, 48000)
        for i, (s, r) in enumerate(zip(srcs, ref)):
            assert s.data.tobytes() == r.data.tobytes(), f"call {call} source {i}"
            assert s.state.tobytes() == r.state.tobytes(), f"call {call} source {i} state"


@pytest.mark.gpu
@pytest.mark.parametrize("count,frames", [(300, 512), (33, 37), (1, 1), (64, 1000)])
def test_gpu_device_batch_matches_oracle(ctx, count, frames):
    """Device-resident batch: the tiled kernel's full and partial tiles, partial waves, mixed
    filter classes (the per-lane select variant) and carried state."""
    import torch
    rng = np.random.default_rng(7 + count)
    st = random_settings(rng)
    srcs = random_sources(rng, count, frames_choices=(frames,))
    for s in srcs:
        s.channels = 2
    params = np.concatenate([art.dsp.source_params(st, s, 48000) for s in srcs])
    states = np.concatenate([s.state for s in srcs])
    data = np.stack([s.data for s in srcs])
    dev = torch.device("cuda", 0)
    d_data = torch.from_numpy(data.copy()).to(dev)
    d_params = torch.from_numpy(params.view(np.uint8).copy()).to(dev)
    d_state = torch.from_numpy(states.view(np.uint8).copy()).to(dev)
    rc = ctx.lib.art_dsp_process_device(ctx.ptr, d_data.data_ptr(), d_params.data_ptr(), d_state.data_ptr(), count,
                                        frames, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    oracle.dsp_process(st, srcs, 48000)
    assert d_data.cpu().numpy().tobytes() == np.stack([s.data for s in srcs]).tobytes()
    assert d_state.cpu().numpy().tobytes() == np.concatenate([s.state for s in srcs]).view(np.uint8).tobytes()
