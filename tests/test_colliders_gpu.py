"""Resident collider store (include/art_colliders.h, SURVEY.md §8 f rank 2) on the GPU.

A pure-Python model of the reference's collider lists (NativeJobBatch<T>.Add / this[i] set /
RemoveAtSwapBack, DataTypes/NativeJobBatch.cs:14-34, and AudioColliderManager.SwapRemove's skip of
invalid ids, Audio/AudioColliderManager.cs:92-93) is the checker for the store's mirror. Frames
that read the resident store (ART_CTX_RESIDENT_COLLIDERS) must equal, byte for byte, frames that
upload the model's arrays the reference way (every collider, every frame), and those equal the
oracle (one round per test checks the oracle directly).
"""
import numpy as np
import pytest

import art
from art import abi
from art.colliders import KINDS, ColliderStore, resident_frame
import oracle

pytestmark = pytest.mark.gpu

KIND_FIELDS = {abi.ART_KIND_SPHERE: "spheres", abi.ART_KIND_AABB: "aabbs", abi.ART_KIND_OBB: "obbs"}


class ListsModel:
    """NativeJobBatch semantics for the three kinds, plus the indices touched since the last sync."""

    def __init__(self):
        self.lists = {k: [] for k in KINDS}
        self.touched = {k: set() for k in KINDS}

    def add(self, k, rec):
        self.lists[k].append(rec.copy())
        self.touched[k].add(len(self.lists[k]) - 1)
        return len(self.lists[k]) - 1

    def set(self, k, i, rec):
        self.lists[k][i] = rec.copy()
        self.touched[k].add(i)

    def remove_swapback(self, k, i):
        L = self.lists[k]
        if i < 0 or i >= len(L):
            return
        if i != len(L) - 1:
            L[i] = L[-1]
            self.touched[k].add(i)
        L.pop()

    def array(self, k):
        return np.array(self.lists[k], dtype=KINDS[k]) if self.lists[k] else np.zeros(0, KINDS[k])

    def expected_dirty(self):
        return sum(len([i for i in self.touched[k] if i < len(self.lists[k])]) for k in KINDS)

    def synced(self):
        self.touched = {k: set() for k in KINDS}


def scene_with(scene, model):
    return art.Scene(dirs=scene.dirs, targets=scene.targets, spheres=model.array(abi.ART_KIND_SPHERE),
                     aabbs=model.array(abi.ART_KIND_AABB), obbs=model.array(abi.ART_KIND_OBB))


def run_both(ctx, scene, params, org, model, check_oracle=False):
    """Resident-store frame vs the reference-style upload frame of the model's arrays."""
    sc = scene_with(scene, model)
    o_up = art.FanOutputs(org.shape[0], sc.R, params.max_hits_per_ray, sc.T, params.thread_count)
    o_res = o_up.copy()
    ctx.set_flags(0)
    ctx.run(art.Frame(sc, params, org, o_up))
    ctx.set_flags(abi.ART_CTX_RESIDENT_COLLIDERS)
    ctx.run(resident_frame(art.Frame(sc, params, org, o_res)))
    ctx.set_flags(0)
    eq = o_res.equal(o_up)
    assert all(eq.values()), eq
    if check_oracle:
        o_ref = art.FanOutputs(org.shape[0], sc.R, params.max_hits_per_ray, sc.T, params.thread_count)
        oracle.run_frame(art.Frame(sc, params, org, o_ref), threads=16)
        eq = o_res.equal(o_ref)
        assert all(eq.values()), f"oracle: {eq}"
    return o_res


@pytest.fixture
def fresh_ctx():
    c = art.Context(1)
    yield c
    c.close()


def load(store, model, scene):
    for k, name in KIND_FIELDS.items():
        arr = getattr(scene, name)
        for i in range(arr.size):
            assert store.add(k, arr[i]) == model.add(k, arr[i])


@pytest.mark.parametrize("ci", [2, 3, 5])
def test_resident_frame_equals_upload_frame(fresh_ctx, ci):
    scene, org, params = art.synth(art.CONFIGS[ci], S=8, R=128, C_scale=0.25)
    store, model = ColliderStore(fresh_ctx), ListsModel()
    load(store, model, scene)
    st = store.sync()
    assert st["reallocated"] == 1 and st["full_prep"] == 1
    assert st["dirty_records"] == scene.spheres.size + scene.aabbs.size + scene.obbs.size
    model.synced()
    out = run_both(fresh_ctx, scene, params, org, model, check_oracle=True)
    assert (out.echo != 0).any()


def test_edit_sequence_uploads_only_changes(fresh_ctx):
    """Random moves (set), swap-back removes (including invalid ids) and adds between syncs."""
    rng = np.random.default_rng(3)
    cfg = art.CONFIGS[5]
    scene, org, params = art.synth(cfg, S=8, R=128, C_scale=0.25)
    pool, _, _ = art.synth(cfg, S=8, R=128, C_scale=0.25, seed=99)  # replacement records
    store, model = ColliderStore(fresh_ctx), ListsModel()
    load(store, model, scene)
    store.sync()
    model.synced()
    for rnd in range(6):
        for k, name in KIND_FIELDS.items():
            src = getattr(pool, name)
            n = len(model.lists[k])
            if src.size == 0:
                continue
            if n and rnd % 2 == 0:  # moved colliders, batched
                ids = rng.integers(0, n, int(rng.integers(1, 8))).astype(np.int32)
                recs = src[rng.integers(0, src.size, ids.size)]
                store.set_many(k, ids, recs)
                for i, rec in zip(ids, recs):
                    model.set(k, int(i), rec)
            for _ in range(int(rng.integers(0, 6))):  # moved colliders, one by one
                if n:
                    i = int(rng.integers(0, n))
                    rec = src[int(rng.integers(0, src.size))]
                    store.set(k, i, rec)
                    model.set(k, i, rec)
            if rnd % 2 == 1:
                for _ in range(int(rng.integers(1, 4))):  # removes, some invalid
                    i = int(rng.integers(-2, len(model.lists[k]) + 3))
                    store.remove_swapback(k, i)
                    model.remove_swapback(k, i)
            if rnd % 3 == 2:
                for _ in range(int(rng.integers(1, 4))):
                    rec = src[int(rng.integers(0, src.size))]
                    assert store.add(k, rec) == model.add(k, rec)
        for k in KINDS:
            assert store.count(k) == len(model.lists[k])
            assert store.array(k).tobytes() == model.array(k).tobytes()
        st = store.sync()
        if not st["reallocated"]:
            assert st["dirty_records"] == model.expected_dirty(), (rnd, st)
        model.synced()
        run_both(fresh_ctx, scene, params, org, model, check_oracle=(rnd == 5))
    # nothing changed: an empty sync
    st = store.sync()
    assert st["dirty_records"] == 0 and st["bytes_uploaded"] == 0 and st["full_prep"] == 0


def test_resident_test_counts(fresh_ctx):
    """Counting frames on the resident store: the permeation loss counts use the store's
    audio_target_id histogram, kept incrementally across edits; they must equal the oracle's."""
    cfg = art.CONFIGS[3]
    scene, org, params = art.synth(cfg, S=4, R=64, C_scale=0.05)
    pool, _, _ = art.synth(cfg, S=4, R=64, C_scale=0.05, seed=11)
    store, model = ColliderStore(fresh_ctx), ListsModel()
    load(store, model, scene)
    for rnd in range(3):
        st = store.sync()
        model.synced()
        sc = scene_with(scene, model)
        o_res = art.FanOutputs(4, sc.R, params.max_hits_per_ray, sc.T, params.thread_count)
        o_ref = o_res.copy()
        cref = oracle.run_frame(art.Frame(sc, params, org, o_ref), threads=16)
        fresh_ctx.set_flags(abi.ART_CTX_RESIDENT_COLLIDERS | abi.ART_CTX_COUNT_TESTS)
        fresh_ctx.run(resident_frame(art.Frame(sc, params, org, o_res)))
        fresh_ctx.set_flags(0)
        assert all(o_res.equal(o_ref).values())
        assert fresh_ctx.last_test_counts() == cref, (rnd, st)
        for k, name in KIND_FIELDS.items():  # retarget / move / remove some colliders
            src = getattr(pool, name)
            if src.size and model.lists[k]:
                store.set(k, 0, src[-1])
                model.set(k, 0, src[-1])
                store.remove_swapback(k, len(model.lists[k]) // 2)
                model.remove_swapback(k, len(model.lists[k]) // 2)


def test_growth_from_empty(fresh_ctx):
    scene, org, params = art.synth(art.CONFIGS[2], S=4, R=64, C_scale=0.25)
    store, model = ColliderStore(fresh_ctx), ListsModel()
    store.sync()  # empty lists: a frame with no colliders
    run_both(fresh_ctx, scene, params, org, model)
    grew = 0
    for step in range(3):  # 64 -> beyond the initial capacity
        for k, name in KIND_FIELDS.items():
            arr = getattr(scene, name)
            for i in range(min(arr.size, 40 * (step + 1))):
                assert store.add(k, arr[i]) == model.add(k, arr[i])
        grew += store.sync()["reallocated"]
        model.synced()
        run_both(fresh_ctx, scene, params, org, model)
    assert grew >= 1


def test_device_resident_path_follows_syncs(fresh_ctx):
    """art_scene_bind in resident mode, then edits + sync without binding again."""
    import torch
    scene, org, params = art.synth(art.CONFIGS[2], S=8, R=128, C_scale=0.25)
    pool, _, _ = art.synth(art.CONFIGS[2], S=8, R=128, C_scale=0.25, seed=7)
    store, model = ColliderStore(fresh_ctx), ListsModel()
    load(store, model, scene)
    store.sync()
    model.synced()
    dev = torch.device("cuda", 0)
    ref_ctx = art.Context(1)
    try:
        fr = art.Frame(scene, params, org, art.FanOutputs(8, scene.R, params.max_hits_per_ray, scene.T, params.thread_count))
        lay = art.fan_layout(fr)
        fresh_ctx.set_flags(abi.ART_CTX_RESIDENT_COLLIDERS)
        fresh_ctx.bind(resident_frame(fr))
        d_org = torch.from_numpy(np.ascontiguousarray(org)).to(dev)
        for rnd in range(2):
            blk = torch.zeros(8 * lay["stride"], dtype=torch.uint8, device=dev)
            fresh_ctx.launch_device(d_org.data_ptr(), 8, blk.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            ref_ctx.bind(art.Frame(scene_with(scene, model), params, org, fr.out))
            rblk = torch.zeros_like(blk)
            ref_ctx.launch_device(d_org.data_ptr(), 8, rblk.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert torch.equal(blk, rblk), rnd
            for k, name in KIND_FIELDS.items():  # move a few colliders, then sync (no rebind)
                src = getattr(pool, name)
                for i in range(min(5, len(model.lists[k]))):
                    store.set(k, i, src[i])
                    model.set(k, i, src[i])
            store.sync()
            model.synced()
    finally:
        fresh_ctx.set_flags(0)
        ref_ctx.close()


def test_pipelined_device_frames_and_syncs(fresh_ctx):
    """Device frames on the caller's stream and collider syncs issued back to back with no host
    wait: each sync (record rewrite + in-place BVH refit on the context stream) must wait for the
    frame before it, and each frame for the sync before it. Every frame's block must equal a frame
    computed from its own collider snapshot."""
    import torch
    S, R = 64, 512
    scene, org, params = art.synth(art.CONFIGS[2], S=S, R=R, C_scale=0.5)
    store, model = ColliderStore(fresh_ctx), ListsModel()
    load(store, model, scene)
    store.sync()
    model.synced()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    fr = art.Frame(scene, params, org, art.FanOutputs(S, R, params.max_hits_per_ray, scene.T, params.thread_count))
    lay = art.fan_layout(fr)
    fresh_ctx.set_flags(abi.ART_CTX_RESIDENT_COLLIDERS)
    snapshots, blocks = [], []
    try:
        fresh_ctx.bind(resident_frame(fr))
        d_org = torch.from_numpy(np.ascontiguousarray(org)).to(dev)
        st = torch.cuda.current_stream().cuda_stream
        for rnd in range(6):
            snapshots.append(scene_with(scene, model))
            blk = torch.zeros(S * lay["stride"], dtype=torch.uint8, device=dev)
            fresh_ctx.launch_device(d_org.data_ptr(), S, blk.data_ptr(), 0, st)
            blocks.append(blk)
            for k in KINDS:  # move a third of the colliders far (the refit changes many bounds)
                arr = model.array(k)
                if not arr.size:
                    continue
                ids = rng.choice(arr.size, max(1, arr.size // 3), replace=False)
                recs = arr[ids].copy()
                c = recs["center"].view(np.float16).astype(np.float32)
                c += rng.uniform(-8, 8, c.shape).astype(np.float32)
                recs["center"] = c.astype(np.float16).view(np.uint16).reshape(recs["center"].shape)
                store.set_many(k, ids.astype(np.int32), recs)
                for j, i in enumerate(ids):
                    model.set(k, int(i), recs[j])
            store.sync()
            model.synced()
        torch.cuda.synchronize()
    finally:
        fresh_ctx.set_flags(0)
    ref_ctx = art.Context(1)
    try:
        for rnd, (snap, blk) in enumerate(zip(snapshots, blocks)):
            out = art.FanOutputs(S, R, params.max_hits_per_ray, scene.T, params.thread_count)
            ref_ctx.run(art.Frame(snap, params, org, out))
            got = art.unpack_block(blk.cpu().numpy(), lay, S, R, params.max_hits_per_ray, scene.T, 1)
            assert all(got.equal(out).values()), (rnd, got.equal(out))
    finally:
        ref_ctx.close()


def test_errors_and_state(fresh_ctx):
    scene, org, params = art.synth(art.CONFIGS[2], S=2, R=64, C_scale=0.05)
    store = ColliderStore(fresh_ctx)
    out = art.FanOutputs(2, scene.R, params.max_hits_per_ray, scene.T, params.thread_count)
    fr = art.Frame(scene, params, org, out)
    fresh_ctx.set_flags(abi.ART_CTX_RESIDENT_COLLIDERS)
    with pytest.raises(art.ArtError) as e:  # no sync yet
        fresh_ctx.run(resident_frame(fr))
    assert e.value.code == abi.ART_E_STATE
    store.sync()
    with pytest.raises(art.ArtError) as e:  # desc still carries colliders
        fresh_ctx.run(fr)
    assert e.value.code == abi.ART_E_INVALID
    h = fresh_ctx.schedule(resident_frame(fr))
    with pytest.raises(art.ArtError) as e:  # sync while a frame is in flight
        store.sync()
    assert e.value.code == abi.ART_E_STATE
    h.complete()
    fresh_ctx.set_flags(0)
    rec = scene.aabbs[0]
    with pytest.raises(art.ArtError) as e:
        store.set(abi.ART_KIND_AABB, 0, rec)  # empty list
    assert e.value.code == abi.ART_E_INVALID
    store.remove_swapback(abi.ART_KIND_AABB, 0)  # skipped like SwapRemove (:92-93)
    assert store.count(abi.ART_KIND_AABB) == 0
    with pytest.raises(art.ArtError):
        store.count(7)
    i = store.add(abi.ART_KIND_AABB, rec)
    assert i == 0 and store.get(abi.ART_KIND_AABB, 0).tobytes() == np.asarray(rec).tobytes()
    with pytest.raises(art.ArtError) as e:  # one bad id: nothing is written
        store.set_many(abi.ART_KIND_AABB, [0, 5], scene.aabbs[1:3])
    assert e.value.code == abi.ART_E_INVALID
    assert store.get(abi.ART_KIND_AABB, 0).tobytes() == np.asarray(rec).tobytes()
    store.clear()
    assert [store.count(k) for k in KINDS] == [0, 0, 0]


def _jitter(recs, rng, scale):
    out = recs.copy()
    c = out["center"].view(np.float16).astype(np.float32)
    c += rng.uniform(-scale, scale, c.shape).astype(np.float32)
    out["center"] = c.astype(np.float16).view(np.uint16).reshape(out["center"].shape)
    return out


@pytest.mark.parametrize("ci", [2, 5])
def test_small_moves_keep_cell_lists(fresh_ctx, ci):
    """Syncs whose moved colliders stay within the cell lists' motion slack (cell_slack) refit the
    BVH but keep the muffle cell lists; larger moves and size changes rebuild them. Every round's
    device frame must equal a fresh bind of the same colliders byte for byte, and the last round
    the oracle too."""
    import torch
    cfg = art.CONFIGS[ci]
    scene, org, params = art.synth(cfg, S=8, R=128, C_scale=0.25)
    store, model = ColliderStore(fresh_ctx), ListsModel()
    load(store, model, scene)
    store.sync()
    model.synced()
    dev = torch.device("cuda", 0)
    ref_ctx = art.Context(1)
    rng = np.random.default_rng(11)
    try:
        fr = art.Frame(scene, params, org, art.FanOutputs(8, scene.R, cfg.H, scene.T, params.thread_count,
                                                          dsp=params.dsp is not None))
        lay = art.fan_layout(fr)
        fresh_ctx.set_flags(abi.ART_CTX_RESIDENT_COLLIDERS)
        fresh_ctx.bind(resident_frame(fr))
        d_org = torch.from_numpy(np.ascontiguousarray(org)).to(dev)
        st = torch.cuda.current_stream().cuda_stream
        # small jitters from the original positions (lists kept), then a large move and a resize
        for rnd, scale in enumerate((0.05, 0.05, 0.1, 0.05, 2.0, 0.05, "resize", 0.05)):
            for k, name in KIND_FIELDS.items():
                src = getattr(scene, name)
                if src.size == 0:
                    continue
                ids = rng.choice(src.size, max(1, src.size // 10), replace=False)
                if scale == "resize":
                    recs = src[ids].copy()
                    if name == "spheres":
                        recs["radius"] = (recs["radius"].view(np.float16) * np.float16(1.5)).view(np.uint16)
                    else:
                        recs["size"] = (recs["size"].view(np.float16) * np.float16(1.5)).view(np.uint16).reshape(
                            recs["size"].shape)
                else:
                    recs = _jitter(src[ids], rng, scale)
                for j, i in enumerate(ids):
                    store.set(k, int(i), recs[j])
                    model.set(k, int(i), recs[j])
            stats = store.sync()
            model.synced()
            # the lists are kept while the moves stay in the slack (the first rounds: every record
            # within 0.05 per axis of the records the lists were built from), rebuilt after the large
            # move and the resize (art_collider_sync_stats.cells_rebuilt)
            if rnd in (0, 1):
                assert stats["cells_rebuilt"] == 0, (rnd, stats)
            if scale in (2.0, "resize"):
                assert stats["cells_rebuilt"] == 1, (rnd, stats)
            blk = torch.zeros(8 * lay["stride"], dtype=torch.uint8, device=dev)
            fresh_ctx.launch_device(d_org.data_ptr(), 8, blk.data_ptr(), 0, st)
            torch.cuda.synchronize()
            ref_ctx.bind(art.Frame(scene_with(scene, model), params, org, fr.out))
            rblk = torch.zeros_like(blk)
            ref_ctx.launch_device(d_org.data_ptr(), 8, rblk.data_ptr(), 0, st)
            torch.cuda.synchronize()
            assert torch.equal(blk, rblk), (rnd, scale)
        got = art.unpack_block(blk.cpu().numpy(), lay, 8, scene.R, cfg.H, scene.T, params.thread_count,
                               dsp=params.dsp is not None)
        ref = art.FanOutputs(8, scene.R, cfg.H, scene.T, params.thread_count, dsp=params.dsp is not None)
        oracle.run_frame(art.Frame(scene_with(scene, model), params, org, ref), threads=8)
        assert all(got.equal(ref).values())
    finally:
        fresh_ctx.set_flags(0)
        ref_ctx.close()
