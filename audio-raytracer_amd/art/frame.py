"""Host-side mirror of the reference's per-frame job graph (Audio/AudioRayTracer.cs:161-237).

`Scene` holds the job inputs that AudioRayTracer.OnUpdate copies into the job structs
(RayDirections, AABB/OBB/SphereColliders, AudioTargetPositions), `FrameParams` the serialized
scalars (AudioRayTracer.cs:9-35, AudioRaytracingManager.cs:13-19), `FanOutputs` the per-fan
NativeArrays (EchoRayDistances, MuffleRayHits, PermeationPowerRemains, AudioTargetSettings,
RayHitResults, RayHitResultCounts, and the build's hit identities). `Context.schedule()` / `JobHandle.complete()` are the
Schedule / Complete surface over the C ABI (include/art.h).
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

import numpy as np

from . import abi


class ArtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{abi.ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


def _ptr(a: np.ndarray | None) -> int | None:
    if a is None or a.size == 0:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


@dataclass
class Scene:
    """Per-frame scene arrays (the job struct inputs)."""
    dirs: np.ndarray                                  # uint16 [R, 3] half3 bits
    targets: np.ndarray                               # float32 [T, 3]
    spheres: np.ndarray = field(default_factory=lambda: np.zeros(0, abi.SPHERE))
    aabbs: np.ndarray = field(default_factory=lambda: np.zeros(0, abi.AABB))
    obbs: np.ndarray = field(default_factory=lambda: np.zeros(0, abi.OBB))

    @property
    def R(self) -> int:
        return int(self.dirs.shape[0])

    @property
    def T(self) -> int:
        return int(self.targets.shape[0])

    @property
    def C(self) -> int:
        return int(self.spheres.size + self.aabbs.size + self.obbs.size)


@dataclass
class DspSettings:
    """AudioSpatializerSettings fields used by the DSP-parameter stage (baked curves are inputs)."""
    reverb_dry_level: tuple = (0.0, -2000.0)          # AudioSpatializerSettings.cs:69
    reverb_dry_boost: tuple = (1.0, 3.0)              # :71
    muffle_cutoff: tuple = (75.0, 8000.0)             # :67
    reverb_volume_curve: np.ndarray = None            # float32 [n]
    reverb_volume_length: float = 1.0
    muffle_curve: np.ndarray = None
    muffle_length: float = 1.0
    sample_rate: int = 48000

    @staticmethod
    def default(n: int = 50) -> "DspSettings":
        # NativeSampledAnimationCurve.Default: AnimationCurve.Linear(1, 1, 0, 0), 50 samples. The
        # bake itself calls Unity's closed-source AnimationCurve.Evaluate, so the baked table is an
        # input; this linear ramp stands in for it.
        ramp = (np.arange(n, dtype=np.float32) / np.float32(n - 1)).astype(np.float32)
        return DspSettings(reverb_volume_curve=ramp, muffle_curve=ramp.copy())


@dataclass
class FrameParams:
    max_ray_life: float = 125.0                  # Player.prefab:229
    max_hits_per_ray: int = 5                    # maxBounces + 1, Player.prefab:228
    max_muffle_hit_distance: float = 250.0       # Player.prefab:230
    muffle_effectiveness: float = 1.0            # Player.prefab:231
    permeation_strength_per_ray: float = 1.0     # Player.prefab:233
    permeation_effectiveness: float = 0.5        # AudioRayTracer.cs:29
    max_reverb_distance: float = 35.0            # Player.prefab:234
    thread_count: int = 1                        # TC = ToUseThreadCount (Sample Scene.unity:7398)
    stages: int = abi.ART_STAGE_RAYTRACE | abi.ART_STAGE_PERMEATE | abi.ART_STAGE_REDUCE
    dsp: DspSettings | None = None

    def batch_size(self, R: int) -> int:
        # AudioRayTracer.cs:161 — (int)max(1, ceil((float)rayCount / ToUseThreadCount))
        return int(max(1.0, math.ceil(np.float32(R) / np.float32(self.thread_count))))


class FanOutputs:
    """The per-fan in/out NativeArrays, batched over S fans."""

    def __init__(self, S: int, R: int, H: int, T: int, TC: int, hits: bool = False, dsp: bool = False):
        self.S, self.R, self.H, self.T, self.TC = S, R, H, T, TC
        self.echo = np.zeros((S, R * H), np.uint16)
        self.muffle = np.zeros((S, TC * T), np.uint16)
        self.perm = np.zeros((S, TC * T), np.float32)
        self.settings = np.zeros((S, T), abi.SETTINGS)
        self.dsp = np.zeros((S, T), abi.DSP_PARAMS) if dsp else None
        self.hit_points = np.zeros((S, R * H, 3), np.uint16) if hits else None
        self.hit_counts = np.zeros((S, R), np.uint8) if hits else None
        self.hit_ids = np.full((S, R * H), abi.ART_HIT_NONE, np.uint32) if hits else None

    def copy(self) -> "FanOutputs":
        o = FanOutputs.__new__(FanOutputs)
        o.__dict__.update({k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in self.__dict__.items()})
        return o

    def fill_random(self, seed: int = 1):
        """Random 'stale' contents (the reference's arrays persist between frames)."""
        rng = np.random.default_rng(seed)
        self.echo[:] = rng.integers(0, 0x7BFF, self.echo.shape, dtype=np.uint16)
        self.muffle[:] = rng.integers(0, 1000, self.muffle.shape, dtype=np.uint16)
        self.perm[:] = rng.standard_normal(self.perm.shape).astype(np.float32)
        if self.hit_points is not None:
            self.hit_points[:] = rng.integers(0, 0x7BFF, self.hit_points.shape, dtype=np.uint16)
            self.hit_counts[:] = rng.integers(0, 200, self.hit_counts.shape, dtype=np.uint8)
            self.hit_ids[:] = rng.integers(0, 2 ** 32, self.hit_ids.shape, dtype=np.uint32)
        return self

    def equal(self, other: "FanOutputs") -> dict:
        res = {
            "echo": np.array_equal(self.echo, other.echo),
            "muffle": np.array_equal(self.muffle, other.muffle),
            "perm": np.array_equal(self.perm.view(np.uint32), other.perm.view(np.uint32)),
            "settings": np.array_equal(self.settings.view(np.uint8), other.settings.view(np.uint8)),
        }
        if self.dsp is not None and other.dsp is not None:
            res["dsp"] = np.array_equal(self.dsp.view(np.uint8), other.dsp.view(np.uint8))
        if self.hit_points is not None and other.hit_points is not None:
            res["hit_points"] = np.array_equal(self.hit_points, other.hit_points)
            res["hit_counts"] = np.array_equal(self.hit_counts, other.hit_counts)
            res["hit_ids"] = np.array_equal(self.hit_ids, other.hit_ids)
        return res


class Frame:
    """A fully built frame: ctypes art_frame_desc + art_fan[S] pointing into numpy arrays."""

    def __init__(self, scene: Scene, params: FrameParams, origins: np.ndarray, out: FanOutputs):
        self.scene, self.params, self.out = scene, params, out
        self.origins = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
        R = scene.R
        d = abi.art_frame_desc()
        d.ray_directions = _ptr(scene.dirs); d.ray_count = R
        d.aabb_colliders = _ptr(scene.aabbs); d.aabb_count = scene.aabbs.size
        d.obb_colliders = _ptr(scene.obbs); d.obb_count = scene.obbs.size
        d.sphere_colliders = _ptr(scene.spheres); d.sphere_count = scene.spheres.size
        d.audio_target_positions = _ptr(scene.targets); d.audio_target_count = scene.T
        d.max_ray_life = params.max_ray_life; d.max_hits_per_ray = params.max_hits_per_ray
        d.max_muffle_hit_distance = params.max_muffle_hit_distance
        d.muffle_effectiveness = params.muffle_effectiveness
        d.permeation_strength_per_ray = params.permeation_strength_per_ray
        d.permeation_effectiveness = params.permeation_effectiveness
        d.max_reverb_distance = params.max_reverb_distance
        d.batch_size = params.batch_size(R)
        d.batch_slots = params.thread_count
        d.stages = params.stages
        self._keep = []
        if params.dsp is not None:
            p = params.dsp
            vc = np.ascontiguousarray(p.reverb_volume_curve, np.float32)
            mc = np.ascontiguousarray(p.muffle_curve, np.float32)
            self._keep += [vc, mc]
            dd = abi.art_dsp_desc()
            dd.reverb_dry_level_min, dd.reverb_dry_level_max = p.reverb_dry_level
            dd.reverb_dry_boost_min, dd.reverb_dry_boost_max = p.reverb_dry_boost
            dd.muffle_cutoff_min, dd.muffle_cutoff_max = p.muffle_cutoff
            dd.reverb_volume_curve = abi.art_curve(vc.ctypes.data_as(C.POINTER(C.c_float)), vc.size, p.reverb_volume_length)
            dd.muffle_curve = abi.art_curve(mc.ctypes.data_as(C.POINTER(C.c_float)), mc.size, p.muffle_length)
            dd.sample_rate = p.sample_rate
            self._dsp = dd
            d.dsp = C.pointer(dd)
        self.desc = d
        S = self.origins.shape[0]
        fans = (abi.art_fan * max(S, 1))()
        for i in range(S):
            f = fans[i]
            f.origin[:] = [float(x) for x in self.origins[i]]
            f.echo_ray_distances = out.echo[i].ctypes.data
            f.muffle_ray_hits = out.muffle[i].ctypes.data
            f.permeation_power_remains = out.perm[i].ctypes.data
            f.settings = out.settings[i].ctypes.data
            f.dsp_params = out.dsp[i].ctypes.data if out.dsp is not None else None
            f.ray_hit_points = out.hit_points[i].ctypes.data if out.hit_points is not None else None
            f.ray_hit_counts = out.hit_counts[i].ctypes.data if out.hit_counts is not None else None
            f.ray_hit_ids = out.hit_ids[i].ctypes.data if out.hit_ids is not None else None
        self.fans = fans
        self.S = S


class JobHandle:
    """JobHandle mirror: IsCompleted / Complete (AudioRayTracer.cs:95,97)."""

    def __init__(self, ctx: "Context", h: int):
        self.ctx, self.h = ctx, h

    @property
    def is_completed(self) -> bool:
        rc = self.ctx.lib.art_is_completed(self.ctx.ptr, self.h)
        if rc < 0:
            self.ctx._raise(rc)
        return rc == 1

    def complete(self):
        rc = self.ctx.lib.art_complete(self.ctx.ptr, self.h)
        if rc:
            self.ctx._raise(rc)


class Context:
    """An art_ctx. device_mask bit i selects HIP device i (one stream each; ArtError(ART_E_DEVICE)
    without a GPU); device_mask 0 is the CPU backend (worker threads, host entry points only)."""

    def __init__(self, device_mask: int = 1, flags: int = 0, devices: list[int] | None = None):
        """device_mask: bit i selects HIP device i, 0 the CPU backend (art_create); devices: an
        explicit device list, ids may repeat (art_create_on: shards on separate streams of one
        device)."""
        self.lib = abi.load_library()
        p = C.c_void_p()
        if devices is not None:
            ids = (C.c_int32 * len(devices))(*devices)
            rc = self.lib.art_create_on(ids, len(devices), C.byref(p))
        else:
            rc = self.lib.art_create(device_mask, C.byref(p))
        if rc:
            raise ArtError(rc, "art_create failed (no HIP device?) — GPU contexts have no CPU fallback; "
                               "device_mask 0 selects the CPU backend explicitly")
        self.ptr = p
        if flags:
            self.lib.art_set_flags(self.ptr, flags)

    def _raise(self, rc: int):
        raise ArtError(rc, self.lib.art_last_error(self.ptr).decode())

    def set_flags(self, flags: int):
        self.lib.art_set_flags(self.ptr, flags)

    def schedule(self, frame: Frame) -> JobHandle:
        h = C.c_uint64()
        rc = self.lib.art_schedule(self.ptr, C.byref(frame.desc), frame.fans, frame.S, C.byref(h))
        if rc:
            self._raise(rc)
        return JobHandle(self, h.value)

    def run(self, frame: Frame) -> FanOutputs:
        self.schedule(frame).complete()
        return frame.out

    def last_test_counts(self) -> dict:
        c = abi.art_test_counts()
        rc = self.lib.art_last_test_counts(self.ptr, C.byref(c))
        if rc:
            self._raise(rc)
        return c.as_dict()

    # --- device-resident path (include/art_device.h) ---
    def bind(self, frame: Frame):
        rc = self.lib.art_scene_bind(self.ptr, C.byref(frame.desc))
        if rc:
            self._raise(rc)

    def debug_leaf_order(self, cap: int = 1 << 24) -> np.ndarray:
        """The bound scene's BVH leaf order (art_debug_leaf_order; diagnostics)."""
        buf = np.zeros(cap, dtype=np.uint32)
        rc = self.lib.art_debug_leaf_order(self.ptr, buf.ctypes.data_as(C.POINTER(C.c_uint32)), cap)
        if rc < 0:
            self._raise(rc)
        return buf[:rc].copy()

    def launch_device(self, d_origins: int, fan_count: int, d_block: int, out_flags: int = 0, stream: int | None = None):
        rc = self.lib.art_launch_device(self.ptr, d_origins, fan_count, d_block, out_flags, stream)
        if rc:
            self._raise(rc)

    def count_device(self, d_origins: int, fan_count: int, d_block: int, out_flags: int = 0,
                     stream: int | None = None) -> dict:
        c = abi.art_test_counts()
        rc = self.lib.art_count_device(self.ptr, d_origins, fan_count, d_block, out_flags, stream, C.byref(c))
        if rc:
            self._raise(rc)
        return c.as_dict()

    def kernel_timing(self) -> dict:
        t = abi.art_kernel_times()
        rc = self.lib.art_kernel_timing(self.ptr, C.byref(t))
        if rc:
            self._raise(rc)
        return {"raytrace_ms": t.raytrace_ms, "permeate_ms": t.permeate_ms, "reduce_ms": t.reduce_ms,
                "launches": t.launches, "kernel_marks_dropped": t.kernel_marks_dropped,
                "kernel_ms": {k: t.kernel_ms[i] for i, k in enumerate(abi.KERNEL_FAMILIES)},
                "kernel_launches": {k: t.kernel_launches[i] for i, k in enumerate(abi.KERNEL_FAMILIES)}}

    def executed_counts(self) -> dict:
        """Work the throughput kernel executed since the last call (needs ART_CTX_COUNT_EXECUTED)."""
        t = abi.art_exec_counts()
        rc = self.lib.art_executed_counts(self.ptr, C.byref(t))
        if rc:
            self._raise(rc)
        out = {k: int(getattr(t, k)) for k, ty in abi.art_exec_counts._fields_ if k not in ("bounce_rays", "by_kernel")}
        out["bounce_rays"] = [int(v) for v in t.bounce_rays]
        out["by_kernel"] = {name: {f: int(getattr(t.by_kernel[i], f)) for f, _ in abi.art_exec_kernel._fields_}
                            for i, name in enumerate(abi.EXEC_KERNELS)}
        return out

    def close(self):
        if getattr(self, "ptr", None):
            self.lib.art_destroy(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fan_layout(frame: Frame, out_flags: int = 0) -> dict:
    lib = abi.load_library()
    L = abi.art_fan_layout()
    rc = lib.art_fan_layout_get(C.byref(frame.desc), out_flags, C.byref(L))
    if rc:
        raise ArtError(rc, "art_fan_layout_get")
    return {n: int(getattr(L, n)) for n, _ in L._fields_}


def unpack_block(block: np.ndarray, layout: dict, S: int, R: int, H: int, T: int, TC: int,
                 hits: bool = False, dsp: bool = False) -> FanOutputs:
    """Split packed per-fan records (uint8 [S * stride]) into FanOutputs arrays."""
    st = layout["stride"]
    b = np.ascontiguousarray(block, np.uint8).reshape(S, st)
    out = FanOutputs(S, R, H, T, TC, hits=hits, dsp=dsp)

    def sec(off, nbytes, dtype):
        return np.ascontiguousarray(b[:, off:off + nbytes]).view(dtype)

    out.settings[:] = sec(layout["settings_off"], T * 24, abi.SETTINGS).reshape(S, T)
    if dsp:
        out.dsp[:] = sec(layout["dsp_off"], T * 24, abi.DSP_PARAMS).reshape(S, T)
    out.muffle[:] = sec(layout["muffle_off"], TC * T * 2, np.uint16)
    out.perm[:] = sec(layout["perm_off"], TC * T * 4, np.float32)
    out.echo[:] = sec(layout["echo_off"], R * H * 2, np.uint16)
    if hits:
        out.hit_points[:] = sec(layout["hit_points_off"], R * H * 6, np.uint16).reshape(S, R * H, 3)
        out.hit_counts[:] = sec(layout["hit_counts_off"], R, np.uint8)
        out.hit_ids[:] = sec(layout["hit_ids_off"], R * H * 4, np.uint32)
    return out


def pack_block(out: FanOutputs, layout: dict) -> np.ndarray:
    """Inverse of unpack_block: FanOutputs -> packed per-fan records (uint8 [S * stride])."""
    S, R, H, T, TC = out.S, out.R, out.H, out.T, out.TC
    st = layout["stride"]
    b = np.zeros((S, st), np.uint8)

    def put(off, arr):
        v = np.ascontiguousarray(arr).reshape(S, -1).view(np.uint8)
        b[:, off:off + v.shape[1]] = v

    put(layout["settings_off"], out.settings)
    if out.dsp is not None:
        put(layout["dsp_off"], out.dsp)
    put(layout["muffle_off"], out.muffle)
    put(layout["perm_off"], out.perm)
    put(layout["echo_off"], out.echo)
    if out.hit_points is not None:
        put(layout["hit_points_off"], out.hit_points)
        put(layout["hit_counts_off"], out.hit_counts)
        put(layout["hit_ids_off"], out.hit_ids)
    return b.reshape(-1)
