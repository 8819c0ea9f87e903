"""art — MI355X-native audio ray tracer (Python binding over libart.so, include/art.h).

The hot path (AudioRaytracerJobBatched / AudioPermeationJobBatched / ProcessAudioDataJob of
FirePixel8422/Audio-Raytracer) runs as HIP kernels for gfx950 inside libart.so. This package is
a thin ctypes host: it never computes the hot path itself, and it raises when libart.so or a HIP
device is missing.
"""
from . import abi, colliders, dist, dsp
from .abi import load_library
from .frame import (ArtError, Context, DspSettings, FanOutputs, Frame, FrameParams, JobHandle, Scene, fan_layout,
                    pack_block, unpack_block)
from .synth import CONFIGS, Config, synth

__all__ = ["abi", "colliders", "dsp", "load_library", "ArtError", "Context", "DspSettings", "FanOutputs", "Frame", "FrameParams",
           "JobHandle", "Scene", "dist", "fan_layout", "pack_block", "unpack_block", "CONFIGS", "Config", "synth"]
