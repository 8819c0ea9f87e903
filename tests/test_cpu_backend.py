"""The CPU backend (art_create with device_mask 0) against the oracle, bit for bit.

The backend is libart's own host code (art_cpu.cpp: worker threads over fans, batches in order,
the kernels' host+device arithmetic); the oracle (oracle/art_oracle.c) is the independent literal
restatement of the Burst jobs. Every output array and the per-kind test counts must be identical.
These tests need no GPU.
"""
import numpy as np
import pytest

import art
from art import abi
import golden_util as G
import kat_scenes as K
import oracle


@pytest.fixture(scope="module")
def cpu():
    c = art.Context(0)
    yield c
    c.close()


def cpu_vs_oracle(cpu, scene, params, org, hits=False, stale=None, prime=None):
    S = org.shape[0]
    o_cpu = art.FanOutputs(S, scene.R, params.max_hits_per_ray, scene.T, params.thread_count, hits=hits,
                           dsp=params.dsp is not None)
    if stale is not None:
        o_cpu.fill_random(stale)
    if prime is not None:
        prime(o_cpu)
    o_ref = o_cpu.copy()
    cref = oracle.run_frame(art.Frame(scene, params, org, o_ref), threads=8)
    cpu.set_flags(abi.ART_CTX_COUNT_TESTS)
    cpu.run(art.Frame(scene, params, org, o_cpu))
    cpu.set_flags(0)
    eq = o_cpu.equal(o_ref)
    assert all(eq.values()), eq
    assert cpu.last_test_counts() == cref
    return o_cpu, cref


REDUCED = {1: (8, 64, None), 2: (6, 64, 0.05), 3: (4, 64, 0.03), 4: (3, 64, 1 / 64), 5: (4, 64, 0.05)}


@pytest.mark.parametrize("ci", [1, 2, 3, 4, 5])
def test_configs_reduced(cpu, ci):
    S, R, cs = REDUCED[ci]
    scene, org, params = art.synth(art.CONFIGS[ci], S=S, R=R, C_scale=cs)
    out, counts = cpu_vs_oracle(cpu, scene, params, org, hits=True)
    assert (out.echo != 0).any()


@pytest.mark.parametrize("tc,R", [(3, 64), (4, 9), (2, 31), (5, 64)])
def test_thread_count_batches(cpu, tc, R):
    """TC > 1: sequential batches, Q1 echo reset index, Q7 slot collapse, Q18 stale slots."""
    scene, org, params = art.synth(art.CONFIGS[1], S=4, R=R)
    params.thread_count = tc
    cpu_vs_oracle(cpu, scene, params, org, hits=True, stale=7)


def test_stage_subsets_and_many_targets(cpu):
    scene, org, params = art.synth(art.CONFIGS[5], S=3, R=64, C_scale=0.05)
    for stages in (abi.ART_STAGE_RAYTRACE, abi.ART_STAGE_PERMEATE, abi.ART_STAGE_REDUCE,
                   abi.ART_STAGE_RAYTRACE | abi.ART_STAGE_REDUCE):
        params.stages = stages
        params.dsp = None
        cpu_vs_oracle(cpu, scene, params, org, stale=11)
    rng = np.random.default_rng(0)
    many = art.Scene(dirs=scene.dirs, targets=rng.uniform(-10, 10, (37, 3)).astype(np.float32), spheres=scene.spheres,
                     aabbs=scene.aabbs, obbs=scene.obbs)
    params.stages = abi.ART_STAGE_ALL
    params.dsp = art.DspSettings.default()
    cpu_vs_oracle(cpu, many, params, org, hits=True)


@pytest.mark.parametrize("name", sorted(K.KATS))
def test_kats(cpu, name):
    sc, p, org, expect, *prime = K.KATS[name]()
    out, _ = cpu_vs_oracle(cpu, sc, p, org, hits=True, prime=prime[0] if prime else None)
    expect(out)


@pytest.mark.parametrize("name", G.names())
def test_golden(cpu, name):
    scene, org, params, fresh, expected, counts = G.load(name)
    cpu.set_flags(abi.ART_CTX_COUNT_TESTS)
    cpu.run(art.Frame(scene, params, org, fresh))
    cpu.set_flags(0)
    assert all(fresh.equal(expected).values())
    assert cpu.last_test_counts() == counts


def test_schedule_semantics_and_threads(cpu):
    scene, org, params = art.synth(art.CONFIGS[1])
    out = art.FanOutputs(8, 64, 5, 4, 1)
    h = cpu.schedule(art.Frame(scene, params, org, out))
    with pytest.raises(art.ArtError) as e:  # one frame in flight per context
        cpu.schedule(art.Frame(scene, params, org, art.FanOutputs(8, 64, 5, 4, 1)))
    assert e.value.code == abi.ART_E_STATE
    while not h.is_completed:
        pass
    h.complete()
    h.complete()
    ref = art.FanOutputs(8, 64, 5, 4, 1)
    oracle.run(scene, params, org, ref)
    assert all(out.equal(ref).values())


def test_one_worker_equals_many(monkeypatch):
    """ART_CPU_THREADS=1: the same bytes from one worker thread."""
    scene, org, params = art.synth(art.CONFIGS[5], S=5, R=64, C_scale=0.05)
    a = art.FanOutputs(5, 64, params.max_hits_per_ray, scene.T, 1, dsp=True, hits=True)
    b = a.copy()
    with art.Context(0) as many:
        many.run(art.Frame(scene, params, org, a))
    monkeypatch.setenv("ART_CPU_THREADS", "1")
    with art.Context(0) as one:
        one.run(art.Frame(scene, params, org, b))
    assert all(a.equal(b).values())


def test_resident_colliders(cpu):
    """The collider store (art_colliders.h) feeds the CPU backend from the last sync's snapshot."""
    from art.colliders import ColliderStore, resident_frame
    scene, org, params = art.synth(art.CONFIGS[5], S=3, R=64, C_scale=0.05)
    with art.Context(0) as c:
        store = ColliderStore(c)
        for k, arr in ((abi.ART_KIND_SPHERE, scene.spheres), (abi.ART_KIND_AABB, scene.aabbs), (abi.ART_KIND_OBB, scene.obbs)):
            for i in range(arr.size):
                store.add(k, arr[i])
        store.sync()
        store.set(abi.ART_KIND_SPHERE, 0, scene.spheres[1])  # after the sync: not in this frame
        c.set_flags(abi.ART_CTX_RESIDENT_COLLIDERS)
        out = art.FanOutputs(3, 64, params.max_hits_per_ray, scene.T, 1, dsp=True)
        c.run(resident_frame(art.Frame(scene, params, org, out)))
    ref = art.FanOutputs(3, 64, params.max_hits_per_ray, scene.T, 1, dsp=True)
    oracle.run(scene, params, org, ref)
    assert all(out.equal(ref).values())


def test_device_entry_points_refused(cpu):
    scene, org, params = art.synth(art.CONFIGS[1], S=2)
    fr = art.Frame(scene, params, org, art.FanOutputs(2, 64, 5, 4, 1))
    with pytest.raises(art.ArtError) as e:
        cpu.bind(fr)
    assert e.value.code == abi.ART_E_UNSUPPORTED
