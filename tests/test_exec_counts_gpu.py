"""Executed-work counters (art_executed_counts, ART_CTX_COUNT_EXECUTED) of the throughput stage.

The counters are measurement support (bench.py's roofline and per-bounce breakdown), so they are
checked against what the frame's outputs imply rather than against the oracle's own counts:
  * bounce_rays[k] (rays the nearest traversal traced at bounce k, AudioRaytracerJobBatched.cs
    :104-208): every ray is traced at bounce 0; a ray with more than k recorded hits was alive
    entering bounce k, and a ray traced at bounce k has at least k hits, so
    #(hits > k) <= bounce_rays[k] <= #(hits >= k), with the hit counts taken from the oracle;
  * counting leaves the outputs unchanged (the counting instantiations run the same traversals);
  * a second call returns zeros (the counters reset on read).
"""
import numpy as np
import pytest

import art
from art import abi
import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg_index,S,R,scale", [(5, 8, 128, 0.25), (2, 16, 128, 0.25), (3, 8, 96, 0.125)])
def test_bounce_rays_bounded_by_hit_counts(cfg_index, S, R, scale):
    cfg = art.CONFIGS[cfg_index]
    scene, org, params = art.synth(cfg, S=S, R=R, C_scale=scale)
    H = params.max_hits_per_ray
    out = art.FanOutputs(S, scene.R, H, scene.T, params.thread_count, hits=True, dsp=params.dsp is not None)
    ref = out.copy()
    oracle.run(scene, params, org, ref)
    with art.Context(1) as ctx:
        ctx.set_flags(abi.ART_CTX_COUNT_EXECUTED)
        ctx.executed_counts()  # reset
        ctx.run(art.Frame(scene, params, org, out))
        ex = ctx.executed_counts()
        again = ctx.executed_counts()
        ctx.set_flags(0)
    eq = out.equal(ref)
    assert all(eq.values()), eq
    assert ex["launches"] == 1
    hc = ref.hit_counts.astype(np.int64).ravel()
    br = ex["bounce_rays"]
    assert br[0] == S * scene.R
    for k in range(H):
        assert int((hc > k).sum()) <= br[k] <= int((hc >= k).sum()), (k, br[:H])
    assert all(v == 0 for v in br[H:])
    assert ex["sphere"] + ex["aabb"] + ex["obb"] > 0 and ex["cull_box"] > 0
    # the per-kernel split sums to the totals; box culls come from the two traversals only,
    # list entries from the muffle rays only
    bk = ex["by_kernel"]
    for f in ("sphere", "aabb", "obb", "cull_box", "cell_entries"):
        assert sum(bk[k][f] for k in abi.EXEC_KERNELS) == ex[f], f
    assert bk["nearest"]["cull_box"] > 0 and bk["echo"]["cull_box"] > 0 and bk["muffle"]["cull_box"] == 0
    assert bk["nearest"]["cell_entries"] == 0 and bk["echo"]["cell_entries"] == 0
    assert again["launches"] == 0 and all(v == 0 for v in again["bounce_rays"])
