"""Device-resident collider store (include/art_colliders.h; SURVEY.md §8 f rank 2).

Mirrors the reference's collider lists: AudioColliderManager (Audio/AudioColliderManager.cs:42-122)
over three NativeJobBatch<T> (DataTypes/NativeJobBatch.cs:8-56). `add` / `set` /
`remove_swapback` edit the NextBatch mirror; `sync` is UpdateJobBatch and publishes the mirror to
the device, uploading only the records that changed. Frames then read the colliders from HBM
(`resident_frame`, ART_CTX_RESIDENT_COLLIDERS).
"""
from __future__ import annotations

import ctypes as C
import copy

import numpy as np

from . import abi
from .frame import Context, Frame

KINDS = {abi.ART_KIND_SPHERE: abi.SPHERE, abi.ART_KIND_AABB: abi.AABB, abi.ART_KIND_OBB: abi.OBB}


class ColliderStore:
    """The resident collider lists of one Context."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def _check(self, rc: int):
        if rc < 0:
            self.ctx._raise(rc)
        return rc

    def add(self, kind: int, rec: np.ndarray) -> int:
        """NativeJobBatch.Add (:27-30); returns the new record's index (AudioColliderId)."""
        r = np.ascontiguousarray(rec, KINDS[kind]).reshape(1)
        out = C.c_int32()
        self._check(self.ctx.lib.art_collider_add(self.ctx.ptr, kind, r.ctypes.data, C.byref(out)))
        return out.value

    def add_many(self, kind: int, recs: np.ndarray) -> list[int]:
        return [self.add(kind, recs[i]) for i in range(recs.size)]

    def set(self, kind: int, idx: int, rec: np.ndarray):
        """NativeJobBatch[idx] = rec (UpdateColiderInSystem, AudioColliderManager.cs:107-110)."""
        r = np.ascontiguousarray(rec, KINDS[kind]).reshape(1)
        self._check(self.ctx.lib.art_collider_set(self.ctx.ptr, kind, idx, r.ctypes.data))

    def set_many(self, kind: int, ids, recs: np.ndarray):
        """Batched set: recs[j] -> ids[j] (one call)."""
        i = np.ascontiguousarray(ids, np.int32)
        r = np.ascontiguousarray(recs, KINDS[kind])
        assert i.size == r.size
        self._check(self.ctx.lib.art_collider_set_many(self.ctx.ptr, kind, i.ctypes.data, r.ctypes.data, i.size))

    def remove_swapback(self, kind: int, idx: int):
        """RemoveAtSwapBack (:31-34); out-of-range ids are skipped (AudioColliderManager.cs:92-93)."""
        self._check(self.ctx.lib.art_collider_remove_swapback(self.ctx.ptr, kind, idx))

    def get(self, kind: int, idx: int) -> np.ndarray:
        r = np.zeros(1, KINDS[kind])
        self._check(self.ctx.lib.art_collider_get(self.ctx.ptr, kind, idx, r.ctypes.data))
        return r[0]

    def count(self, kind: int) -> int:
        return self._check(self.ctx.lib.art_collider_count(self.ctx.ptr, kind))

    def array(self, kind: int) -> np.ndarray:
        """The whole NextBatch mirror of a kind (read back record by record)."""
        out = np.zeros(self.count(kind), KINDS[kind])
        for i in range(out.size):
            out[i] = self.get(kind, i)
        return out

    def clear(self):
        self._check(self.ctx.lib.art_colliders_clear(self.ctx.ptr))

    def sync(self) -> dict:
        """UpdateJobBatch (AudioColliderManager.cs:115-122); returns what the sync moved."""
        self._check(self.ctx.lib.art_colliders_sync(self.ctx.ptr))
        st = abi.art_collider_sync_stats()
        self._check(self.ctx.lib.art_colliders_last_sync(self.ctx.ptr, C.byref(st)))
        return {k: int(getattr(st, k)) for k, _ in abi.art_collider_sync_stats._fields_}


def resident_frame(frame: Frame) -> Frame:
    """A shallow copy of `frame` whose desc carries no colliders (for ART_CTX_RESIDENT_COLLIDERS)."""
    f = copy.copy(frame)
    d = abi.art_frame_desc()
    C.pointer(d)[0] = frame.desc
    d.aabb_colliders = None; d.aabb_count = 0
    d.obb_colliders = None; d.obb_count = 0
    d.sphere_colliders = None; d.sphere_count = 0
    f.desc = d
    return f
