"""Per-sample spatializer DSP (include/art_dsp.h; SURVEY.md §8 f rank 1).

Mirrors AudioSpatializer.OnAudioFilterRead (Audio/AudioTarget/AudioSpatializer.cs:70-87): each
AudioSource holds an interleaved stereo buffer processed in place and the filter state the C#
MuffleDSP / BinauralDSP structs keep between calls. The product path runs on the GPU through
libart.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import abi


def _linear_curve(n: int = 50) -> np.ndarray:
    # NativeSampledAnimationCurve.Default (NativeSampledAnimationCurve.cs:92-98) bakes Unity's
    # closed-source AnimationCurve.Evaluate: the baked table is an input; a ramp stands in for it.
    return (np.arange(n, dtype=np.float32) / np.float32(n - 1)).astype(np.float32)


@dataclass
class SpatializerSettings:
    """AudioSpatializerSettings (DataTypes/AudioSpatializerSettings.cs:4-45), Default at :47-73."""
    pan_strength: float = 0.8
    rear_attenuation_strength: float = 0.2
    distance_based_panning: bool = True
    max_pan_distance: float = 5.0
    distance_based_rear_attenuation: bool = True
    max_rear_attenuation_distance: float = 15.0
    max_elevation_effect_distance: float = 12.0
    low_pass_cutoff: tuple = (5000.0, 22000.0)
    low_pass_volume: float = 0.85
    high_pass_cutoff: tuple = (25.0, 150.0)
    high_pass_volume: float = 1.15
    muffle_curve: np.ndarray = field(default_factory=_linear_curve)
    muffle_curve_length: float = 1.0
    muffle_cutoff: tuple = (75.0, 8000.0)
    reverb_volume_curve: np.ndarray = field(default_factory=_linear_curve)
    reverb_volume_curve_length: float = 1.0
    reverb_dry_boost: tuple = (1.0, 3.0)

    def to_c(self) -> abi.art_spatializer_settings:
        self._mc = np.ascontiguousarray(self.muffle_curve, np.float32)
        self._rc = np.ascontiguousarray(self.reverb_volume_curve, np.float32)
        fp = C.POINTER(C.c_float)
        return abi.art_spatializer_settings(
            self.pan_strength, self.rear_attenuation_strength, int(self.distance_based_panning),
            self.max_pan_distance, int(self.distance_based_rear_attenuation), self.max_rear_attenuation_distance,
            self.max_elevation_effect_distance, self.low_pass_cutoff[0], self.low_pass_cutoff[1], self.low_pass_volume,
            self.high_pass_cutoff[0], self.high_pass_cutoff[1], self.high_pass_volume,
            abi.art_curve(self._mc.ctypes.data_as(fp), self._mc.size, self.muffle_curve_length),
            self.muffle_cutoff[0], self.muffle_cutoff[1],
            abi.art_curve(self._rc.ctypes.data_as(fp), self._rc.size, self.reverb_volume_curve_length),
            self.reverb_dry_boost[0], self.reverb_dry_boost[1])


@dataclass
class AudioSource:
    """One AudioSpatializer: its buffer for this OnAudioFilterRead call, the per-buffer inputs and
    the persistent filter state."""
    data: np.ndarray                     # float32 [frames * channels], processed in place
    channels: int = 2
    muffle_strength: float = 0.0         # audioTargetSettings.MuffleStrength
    reverb_volume: float = 0.0           # audioTargetSettings.ReverbVolume
    local_dir: tuple = (0.0, 0.0, 1.0)   # cachedLocalDir (AudioSpatializer.cs:64)
    listener_distance: float = 1.0       # cachedListenerDistance (:66)
    volume_multiplier: float = 1.0       # volumeMultiplier (:18)
    state: np.ndarray = field(default_factory=lambda: np.zeros(1, abi.DSP_STATE))

    def to_c(self) -> abi.art_audio_source:
        assert self.data.dtype == np.float32 and self.data.flags["C_CONTIGUOUS"]
        assert self.state.dtype == abi.DSP_STATE and self.state.flags["C_CONTIGUOUS"]
        return abi.art_audio_source(
            self.data.ctypes.data_as(C.POINTER(C.c_float)), self.data.size // self.channels, self.channels,
            self.muffle_strength, self.reverb_volume, (C.c_float * 3)(*self.local_dir), self.listener_distance,
            self.volume_multiplier, self.state.ctypes.data_as(C.POINTER(abi.art_dsp_state)))

    def copy(self) -> "AudioSource":
        return AudioSource(self.data.copy(), self.channels, self.muffle_strength, self.reverb_volume, self.local_dir,
                           self.listener_distance, self.volume_multiplier, self.state.copy())


def sources_to_c(sources: list[AudioSource]):
    arr = (abi.art_audio_source * max(1, len(sources)))()
    for i, s in enumerate(sources):
        arr[i] = s.to_c()
    return arr


def process(ctx, settings: SpatializerSettings, sources: list[AudioSource], sample_rate: int = 48000):
    """AudioSpatializer.OnAudioFilterRead for every source, on the GPU (art_dsp_process)."""
    st = settings.to_c()
    arr = sources_to_c(sources)
    rc = ctx.lib.art_dsp_process(ctx.ptr, C.byref(st), arr, len(sources), sample_rate)
    if rc:
        ctx._raise(rc)


def source_params(settings: SpatializerSettings, source: AudioSource, sample_rate: int = 48000) -> np.ndarray:
    """The per-buffer scalars art_dsp_process derives on the host (for the device-resident API)."""
    st = settings.to_c()
    src = source.to_c()
    out = np.zeros(1, abi.DSP_SOURCE_PARAMS)
    rc = abi.load_library().art_dsp_source_params_get(C.byref(st), C.byref(src), sample_rate,
                                                      out.ctypes.data_as(C.POINTER(abi.art_dsp_source_params)))
    if rc:
        raise ValueError(f"art_dsp_source_params_get: {rc}")
    return out
