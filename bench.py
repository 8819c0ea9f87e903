#!/usr/bin/env python3
"""Benchmark: ray-collider tests/s + p50 per-frame batch ms (BASELINE.json "metric").

Workload (N=1): BASELINE config 2 — 256 sources (fans) x 512 rays x 4096 colliders
(2048 AABB + 2048 Sphere), T = 4 audio targets, maxBounces 0, stages raytrace + reduce.
A "step" = one frame of the hot path over every fan of this rank, inputs resident in HBM,
launched through the C ABI (art_launch_device) on torch's current HIP stream.
Multi-GPU (one process per GPU, RCCL): config 2 runs weak (256 fans per rank); config 4 runs as
BASELINE.json names it, strong: 1024 fans split contiguously over the G ranks (SURVEY.md §8 e);
each step all-gathers the per-fan result blocks (art.dist.all_gather_fan_blocks).

value = (tests the reference algorithm executes on all ranks' fans per frame) * K / max over ranks
of the timed region: "equivalent ray-collider tests/s" — the kernels use an exact broad phase
(BVH, culls) and execute far fewer tests (roofline.executed says how many). Test counts come from
the counting kernel (art_count_device), which tests/test_parity_gpu.py checks against the oracle.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 the driver uses
torch.distributed.run (one process per GPU, MASTER_ADDR=127.0.0.1).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "audio-raytracer_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import art  # noqa: E402
from art import abi  # noqa: E402

# Broad-phase work, same counting rule: BVH node box vs segment (margin 2, 6 widened bounds, 6
# compares) and muffle cell-list entries scanned (a load and a distance compare: 2).
CULL_OPS = {"cull_box": 14, "cell_entries": 2}
# Algorithmic FP32 ops per test (SURVEY.md §8 d; miss path, IEEE add/sub/mul/div/sqrt/min/max/cmp = 1).
OPS = {"rt_sphere": 26, "rt_aabb": 34, "rt_obb": 118, "perm_hit_sphere": 26, "perm_hit_aabb": 34, "perm_hit_obb": 134,
       "perm_loss_sphere": 18, "perm_loss_aabb": 33, "perm_loss_obb": 117}
FP32_VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md "Peak FP32 (vector)"
# one non-FMA wave64 VALU op issues over 2 cycles per SIMD-32 (MI355X_MICROARCH.md:54, :473):
# 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T lane-op/s (SURVEY.md 8(d)'s 64 lanes/CU/clk undercounts 2x)
SINGLE_ISSUE_TLOPS = 78.6
SINGLE_ISSUE_TLOPS_64 = 39.3   # 256 CU x 64 lanes/clk x 2.4 GHz (SURVEY.md 8(d)'s figure), reported beside it
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md "HBM3E peak BW" (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=0, help="timed steps (0 = enough for about 1.5 s)")
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--prewarm-s", type=float, default=0.3,
                   help="untimed frames (launches only, no collective) for this many seconds before the W warmup "
                        "steps: the GPU clock of a fresh process ramps over its first few hundred frames, which a "
                        "game's continuous frame loop never sees (0 = off)")
    p.add_argument("--config", type=int, default=None, help="BASELINE config (default: 2; 1 for --path cpu)")
    p.add_argument("--frames", type=int, default=50, help="host-API frames for the p50 frame latency")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-fans", type=int, default=0, help="fans in the CPU-baseline sample (0 = auto)")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--collider-scale", type=float, default=None,
                   help="scale the config's collider count (experiments only; the metric is quoted at 1)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="minimum wall time of each CPU-baseline leg")
    p.add_argument("--scaling", choices=("auto", "weak", "strong"), default="auto",
                   help="N > 1: weak = cfg.S fans per rank; strong = cfg.S fans split over the ranks "
                        "(auto: strong for config 4, as BASELINE.json names it, weak otherwise)")
    p.add_argument("--no-dynamic", action="store_true", help="skip the dynamic-scene and rebuild measurements")
    p.add_argument("--no-overlap", action="store_true",
                   help="N > 1 over RCCL: run each frame's all-gather after it on the launch stream instead of "
                        "beside the next frame's kernels")
    p.add_argument("--overlap", choices=("auto", "on"), default="auto",
                   help="N > 1 over RCCL with even shards: auto = time the overlapped and the serial all-gather "
                        "before the timed region and run the faster; on = always overlap (--no-overlap: never)")
    p.add_argument("--nccl-priority", choices=("normal", "high"), default="normal",
                   help="N > 1 over RCCL: priority of the collective's stream")
    p.add_argument("--force-dist", action="store_true",
                   help="run the N > 1 code path (process group, all-gathers, overlap, self-check) even with one "
                        "rank: a one-GPU rehearsal of the RCCL branch; launch under torch.distributed.run")
    p.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                   help="N > 1: torch.distributed backend (nccl = RCCL over xGMI; gloo: host-side all-gather, "
                        "e.g. ranks sharing one GPU in tests)")
    p.add_argument("--targets", type=int, default=None,
                   help="audio targets T (experiments; BASELINE's configs use 4): the same scene generator with T targets")
    p.add_argument("--path", choices=("raytrace", "dsp", "dirs", "cpu"), default="raytrace",
                   help="raytrace: the headline metric; dsp: the per-sample spatializer DSP (SURVEY.md 8 f rank 1); "
                        "dirs: Fibonacci ray directions on the device (rank 3); cpu: config 1 through the C ABI's "
                        "CPU backend (device_mask 0) on N threads and 1 thread")
    p.add_argument("--dirs-count", type=int, default=1 << 24, help="directions per launch (dirs path)")
    p.add_argument("--dsp-frames", type=int, default=1024, help="frames per OnAudioFilterRead buffer (dsp path)")
    p.add_argument("--dsp-batch", type=int, default=65536, help="sources of the large-batch roofline run (dsp path)")
    p.add_argument("--dsp-sort", action="store_true",
                   help="group the device batch by filter class, as art_dsp_process does (dsp path)")
    return p.parse_args()


def host_cpu_info():
    """The host cores this job may use: the affinity set, capped by the cgroup CPU quota (a GPU
    box's share of a large machine: nproc shows the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except Exception:
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    threads = min(aff, max(1, int(quota + 0.5))) if quota else aff
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota, "model": model,
            "threads_used": threads}


def cpu_leg(cfg, scene, params, org, threads, min_seconds):
    """The oracle (C restatement of the reference jobs, oracle/art_oracle.c) timed on `threads`
    host threads, one fan per task (TC = 1, as the shipped scene): batches of whole fans of this
    config until at least `min_seconds` of wall time (a bounded sample; fans wrap around). The
    oracle is rebuilt -march=native for this host when gcc is present (oracle.load_native)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle  # CPU baseline leg only

    lib, label = oracle.load_native()
    S = org.shape[0]
    tests, fans, dt, nxt, batch = 0, 0, 0.0, 0, max(1, min(threads, S))
    while dt < min_seconds:
        idx = (nxt + np.arange(batch)) % S
        nxt = (nxt + batch) % S
        out = art.FanOutputs(batch, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)
        t0 = time.perf_counter()
        _, counts = oracle.run(scene, params, np.ascontiguousarray(org[idx]), out, threads=threads, lib=lib)
        dt += time.perf_counter() - t0
        tests += sum(counts.values())
        fans += batch
        per_fan = dt / fans
        want = int((min_seconds - dt) / per_fan) + 1
        batch = max(1, min(S, -(-want // threads) * threads))
    return {"value": tests / dt, "seconds": dt, "tests": tests, "fans": fans, "build": label}


def cpu_baseline(cfg, scene, params, org, min_seconds):
    host = host_cpu_info()
    n = host["threads_used"]
    many = cpu_leg(cfg, scene, params, org, n, min_seconds)
    one = cpu_leg(cfg, scene, params, org, 1, max(3.0, min_seconds / 2))
    return {"value": many["value"], "unit": "ray-collider tests/s", "cores": n, "kind": "port",
            "label": "reference algorithm (C restatement of the Burst jobs, oracle/art_oracle.c; Burst cannot run here)",
            "sample": f"{many['fans']} fans of config {cfg.index} ({many['tests']} reference tests, {many['seconds']:.1f} s) "
                      f"on {n} threads, one fan per task; oracle built with {many['build']}",
            "build": many["build"],
            "one_thread": {"value": one["value"], "unit": "ray-collider tests/s",
                           "sample": f"{one['fans']} fans ({one['tests']} tests, {one['seconds']:.1f} s) on 1 thread"},
            "host": host}


DSP_BYTES_PER_FRAME = 16     # one stereo frame read + written (8 B each way)
DSP_BYTES_PER_SOURCE = 32 + 64  # art_dsp_source_params read + art_dsp_state read and written


def dsp_sources(rng, n, frames):
    from art.dsp import AudioSource, SpatializerSettings
    st = SpatializerSettings(muffle_curve=rng.random(50).astype(np.float32),
                             reverb_volume_curve=rng.random(50).astype(np.float32))
    srcs = []
    for i in range(n):
        d = rng.standard_normal(3)
        d /= np.linalg.norm(d)
        srcs.append(AudioSource(data=(rng.standard_normal(frames * 2) * 0.3).astype(np.float32),
                                muffle_strength=float(rng.random()) if i % 3 else 0.0, reverb_volume=float(rng.random()),
                                local_dir=tuple(float(v) for v in d), listener_distance=float(rng.uniform(0, 30))))
    return st, srcs


def dsp_device_run(ctx, d_data, d_params, d_state, count, frames, steps, warmup):
    """Time `steps` launches of art_dsp_process_device on torch's current stream (HIP events on
    that stream); returns ms per launch."""
    sp = torch.cuda.current_stream().cuda_stream
    for _ in range(warmup):
        assert ctx.lib.art_dsp_process_device(ctx.ptr, d_data.data_ptr(), d_params.data_ptr(), d_state.data_ptr(),
                                              count, frames, sp) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        ctx.lib.art_dsp_process_device(ctx.ptr, d_data.data_ptr(), d_params.data_ptr(), d_state.data_ptr(), count,
                                       frames, sp)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main_dsp(a):
    """Per-sample spatializer DSP (include/art_dsp.h): one step = one audio tick, every source's
    OnAudioFilterRead buffer (AudioSpatializer.cs:70-87) processed on the device. Sources are
    independent: N ranks run N shards of sources (weak scaling, no collective)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    cfg = art.CONFIGS[a.config]
    S, F, sr = cfg.S, a.dsp_frames, 48000
    rng = np.random.default_rng(1234 + rank)
    st, srcs = dsp_sources(rng, S, F)
    params = np.concatenate([art.dsp.source_params(st, x, sr) for x in srcs])
    if a.dsp_sort:
        order = np.argsort(params["flags"] & 3, kind="stable")
        srcs = [srcs[i] for i in order]
        params = params[order]
    ctx = art.Context(1 << torch.cuda.current_device())
    d_data = torch.from_numpy(np.stack([x.data for x in srcs])).to(dev)
    d_params = torch.from_numpy(params.view(np.uint8).copy()).to(dev)
    d_state = torch.zeros(S * abi.DSP_STATE.itemsize, dtype=torch.uint8, device=dev)

    sp = torch.cuda.current_stream().cuda_stream
    for _ in range(a.warmup):
        ctx.lib.art_dsp_process_device(ctx.ptr, d_data.data_ptr(), d_params.data_ptr(), d_state.data_ptr(), S, F, sp)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.steps):
        ctx.lib.art_dsp_process_device(ctx.ptr, d_data.data_ptr(), d_params.data_ptr(), d_state.data_ptr(), S, F, sp)
    e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / a.steps
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    frames_all = S * F * world * a.steps

    if rank != 0:
        dist.destroy_process_group()
        return
    # host API (art_dsp_process): host buffers, H2D + kernel + D2H, per tick
    import ctypes as C
    c_st = st.to_c()
    c_srcs = art.dsp.sources_to_c(srcs)  # the C# caller's struct array: built once, reused per tick
    host_ms = []
    for i in range(25):
        t1 = time.perf_counter()
        rc = ctx.lib.art_dsp_process(ctx.ptr, C.byref(c_st), c_srcs, S, sr)
        if i >= 5:
            host_ms.append((time.perf_counter() - t1) * 1e3)
        assert rc == 0, rc
    # large batch: the same sources repeated; HBM roofline of the kernel
    B = a.dsp_batch
    reps = (B + S - 1) // S
    b_data = d_data.repeat(reps, 1)[:B].contiguous()
    b_params = d_params.view(S, -1).repeat(reps, 1)[:B].contiguous()
    b_state = torch.zeros(B * abi.DSP_STATE.itemsize, dtype=torch.uint8, device=dev)
    big_ms = dsp_device_run(ctx, b_data, b_params, b_state, B, F, max(3, a.steps // 10), 2)
    big_bytes = B * F * DSP_BYTES_PER_FRAME + B * DSP_BYTES_PER_SOURCE
    big_gbs = big_bytes / (big_ms * 1e-3) / 1e9
    tick_bytes = S * F * DSP_BYTES_PER_FRAME + S * DSP_BYTES_PER_SOURCE
    tick_gbs = tick_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    prof = os.path.join(ROOT, "profiles", "traffic_dsp.json")
    if os.path.exists(prof):
        try:
            traffic = json.load(open(prof)).get("dsp_bytes_per_launch_batch")
        except Exception:
            traffic = None

    cpu = None
    if world == 1 and not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle  # CPU baseline leg only
        oracle.load()
        n, t1 = 0, time.perf_counter()
        while True:
            oracle.dsp_process(st, srcs, sr)
            n += 1
            cdt = time.perf_counter() - t1
            if cdt >= a.cpu_seconds or n >= 20000:
                break
        cpu = {"value": n * S * F / cdt, "unit": "stereo frames/s", "cores": 1, "kind": "port",
               "sample": f"{n} ticks x {S} sources x {F} frames ({cdt:.1f} s) through or_dsp_process "
                         f"(oracle/art_oracle.c, gcc -O3 -ffp-contract=off), one thread"}
    value = frames_all / dt
    res = {
        "metric": "spatializer DSP stereo frames/s (per-sample OnAudioFilterRead chain)",
        "value": value,
        "unit": "stereo frames/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "realtime_sources_at_48k": value / sr,
        "p50_host_tick_ms": statistics.median(host_ms),
        "p50_host_tick_ms_note": "art_dsp_process on host buffers: pack, H2D, kernel, D2H, unpack (PCIe-inclusive)",
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": f"dsp tick: {S} spatializers (config{cfg.index} sources) x {F} stereo frames @ 48 kHz",
                   "sources_per_gpu": S, "frames": F, "grouped_by_filter_class": bool(a.dsp_sort), "parallelism": f"source-sharded x{world} (replicas, no collective)"},
        "roofline": {"bound": "hbm", "achieved": big_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": big_gbs / HBM_PEAK_GBS, "traffic": traffic, "kernel": "dsp_tiled_kernel",
                     "kernel_ms": big_ms, "batch_sources": B, "algorithmic_bytes": big_bytes,
                     "note": f"large batch ({B} sources x {F} frames, {DSP_BYTES_PER_FRAME} B/frame + "
                             f"{DSP_BYTES_PER_SOURCE} B/source); the {S}-source tick is bound by the serial "
                             "per-channel recurrence (one lane per chain), not HBM",
                     "tick": {"kernel_ms": kern_ms, "achieved": tick_gbs, "frac": tick_gbs / HBM_PEAK_GBS,
                              "algorithmic_bytes": tick_bytes}},
        "cpu_baseline": cpu,
    }
    print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


def main_dirs(a):
    """FibonacciDirectionsJobParallel on the device (art_fibonacci_directions_device): one step =
    one launch generating --dirs-count half3 directions in HBM. Single GPU (an init-time step)."""
    torch.cuda.set_device(0)
    n = a.dirs_count
    ctx = art.Context(1)
    d = torch.empty(n * 3, dtype=torch.int16, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    for _ in range(a.warmup):
        assert ctx.lib.art_fibonacci_directions_device(ctx.ptr, n, d.data_ptr(), sp) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.steps):
        ctx.lib.art_fibonacci_directions_device(ctx.ptr, n, d.data_ptr(), sp)
    e1.record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    k_ms = e0.elapsed_time(e1) / a.steps
    gbs = n * 6 / (k_ms * 1e-3) / 1e9  # 6 B (half3) written per direction, nothing read
    cpu = None
    if not a.no_cpu_baseline:
        m = min(n, 1 << 20)
        host = np.zeros((m, 3), np.uint16)
        reps, t1 = 0, time.perf_counter()
        while True:
            art.load_library().art_fibonacci_directions(m, host.ctypes.data)
            reps += 1
            cdt = time.perf_counter() - t1
            if cdt >= min(a.cpu_seconds, 5.0):
                break
        cpu = {"value": reps * m / cdt, "unit": "directions/s", "cores": 1, "kind": "port",
               "sample": f"{reps} x {m} directions ({cdt:.1f} s) through art_fibonacci_directions (host C++, one thread)"}
    print(json.dumps({
        "metric": "Fibonacci ray directions/s (FibonacciDirectionsJobParallel)", "value": n * a.steps / dt,
        "unit": "directions/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"{n} directions per launch", "parallelism": "single GPU"},
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                     "traffic": None, "kernel": "fibonacci_kernel", "kernel_ms": k_ms,
                     "note": "6 B written per direction; double-precision cos/sin make it FP64-VALU-heavy"},
        "cpu_baseline": cpu}))


def lib_sha256():
    import hashlib
    return hashlib.sha256(open(abi.LIB_PATH, "rb").read()).hexdigest()


def read_traffic(cfg_index):
    """HBM bytes per raytrace frame from the PMC passes (tools/gpu_round.sh -> tools/prof_summary.py,
    FETCH_SIZE and WRITE_SIZE in separate passes), total and per kernel — used only when they were
    measured on this exact libart.so."""
    prof = os.path.join(ROOT, "profiles", f"traffic_config{cfg_index}.json")
    if not os.path.exists(prof):
        return None, {}, "no PMC traffic file for this config"
    try:
        t = json.load(open(prof))
    except Exception as e:  # noqa: BLE001
        return None, {}, f"unreadable traffic file: {e}"
    if t.get("lib_sha256") != lib_sha256():
        return None, {}, f"traffic file measured on another build ({str(t.get('lib_sha256'))[:12]}); not used"
    return (t.get("raytrace_bytes_per_launch"), t.get("bytes_per_frame_by_kernel", {}),
            f"PMC pass on this build (lib sha256 {t['lib_sha256'][:12]})")


def stage_kernels(cfg, thread_count, has_obb):
    """The kernels of the timed raytrace stage as launch_raytrace_fast (csrc/art_trace.hip) picks
    them for this frame shape (no hit outputs, as the bench launches it)."""
    obb = "true" if has_obb else "false"
    if cfg.H > 1 and thread_count == 1:  # one batch slot, no hit outputs: the path kernel's work folds into the nearest kernel
        return (f"per bounce: nearest_first_kernel<false, {obb}, true> (path epilogue folded in), that bounce's echo "
                f"vis_kernel<false, {obb}, false> on the side stream; then muffle_kernel<false, {obb}, false>")
    if cfg.H > 1:
        return (f"per bounce: nearest_first_kernel<false, {obb}, false> -> path_kernel<false, true>, that bounce's echo "
                f"vis_kernel<false, {obb}, false> on the side stream; then muffle_kernel<false, {obb}, false>")
    if thread_count == 1:  # one-hit frames, one batch slot, no hit outputs (any size): echo + muffle from the nearest hits
        return f"nearest_first_kernel<false, {obb}, false> -> echo_muffle_kernel<false, {obb}> (one stream, no path kernel)"
    return (f"nearest_first_kernel<false, {obb}, false> -> path_kernel<false, false> -> echo vis_kernel<false, {obb}, false>, "
            f"muffle_kernel<false, {obb}, false> on the side stream")


def jitter_records(rng, recs, scale):
    """Moved copies of collider records: centres shifted by up to `scale` (half bits via float16)."""
    out = recs.copy()
    c = out["center"].view(np.float16).astype(np.float32)
    c += rng.uniform(-scale, scale, c.shape).astype(np.float32)
    out["center"] = c.astype(np.float16).view(np.uint16).reshape(out["center"].shape)
    return out


def dynamic_step(cfg, scene, params, org, S, steps, warmup, sp):
    """Device step with a moving scene: per step 1 % of the colliders move (art_collider_set_many),
    art_colliders_sync uploads only those, decodes them and refits the BVH / sorted copies in place,
    then the frame runs on the resident scene (AudioColliderManager.UpdateJobBatch
    Audio/AudioColliderManager.cs:115-122 -> NativeJobBatch.UpdateJobBatch NativeJobBatch.cs:36-50,
    then the jobs). Also: a frame whose colliders all change (full upload, decode, BVH rebuild)."""
    from art.colliders import ColliderStore, resident_frame
    dev = torch.device("cuda", torch.cuda.current_device())
    rctx = art.Context(1 << torch.cuda.current_device())
    store = ColliderStore(rctx)
    fields = {abi.ART_KIND_SPHERE: scene.spheres, abi.ART_KIND_AABB: scene.aabbs, abi.ART_KIND_OBB: scene.obbs}
    for k, arr in fields.items():
        for i in range(arr.size):
            store.add(k, arr[i])
    store.sync()
    rctx.set_flags(abi.ART_CTX_RESIDENT_COLLIDERS)
    out = art.FanOutputs(S, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)
    rframe = resident_frame(art.Frame(scene, params, org, out))
    lay = art.fan_layout(rframe)
    rctx.bind(rframe)
    d_org = torch.from_numpy(np.ascontiguousarray(org)).to(dev)
    d_blk = torch.zeros(S * lay["stride"], dtype=torch.uint8, device=dev)
    rng = np.random.default_rng(7)
    n_all = sum(x.size for x in fields.values())
    variants = []
    for v in range(8):  # pre-baked moved records (the caller's bake is not part of the step)
        moves = {}
        for k, arr in fields.items():
            if arr.size:
                ids = rng.choice(arr.size, max(1, arr.size // 100), replace=False).astype(np.int32)
                moves[k] = (ids, jitter_records(rng, arr[ids], 0.05))
        variants.append(moves)

    def one(i):
        for k, (ids, recs) in variants[i % len(variants)].items():
            store.set_many(k, ids, recs)
        store.sync()
        rctx.launch_device(d_org.data_ptr(), S, d_blk.data_ptr(), 0, sp)

    for i in range(warmup):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        one(i)
    torch.cuda.synchronize()
    dyn_ms = (time.perf_counter() - t0) / steps * 1e3
    moved = int(sum(ids.size for ids, _ in variants[0].values()))
    rctx.close()

    # full rebuild: every collider changed each frame through the Unity-facing API (upload, decode,
    # Morton sort, BVH build, frame, D2H)
    ctx = art.Context(1 << torch.cuda.current_device())
    scenes = []
    for v in range(2):
        sc = art.Scene(dirs=scene.dirs, targets=scene.targets, spheres=jitter_records(rng, scene.spheres, 0.05) if scene.spheres.size else scene.spheres,
                       aabbs=jitter_records(rng, scene.aabbs, 0.05) if scene.aabbs.size else scene.aabbs,
                       obbs=jitter_records(rng, scene.obbs, 0.05) if scene.obbs.size else scene.obbs)
        scenes.append(art.Frame(sc, params, org, art.FanOutputs(S, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)))
    ms = []
    for i in range(25):
        t1 = time.perf_counter()
        ctx.run(scenes[i % 2])
        if i >= 5:
            ms.append((time.perf_counter() - t1) * 1e3)
    ctx.close()
    return {"ms_per_step_dynamic": dyn_ms, "moved_per_step": moved, "colliders": n_all,
            "note": "device step incl. art_collider_set_many + art_colliders_sync (H2D of the moved records, decode, "
                    "in-place BVH/sorted-copy refit) + art_launch_device, timed over the same K steps",
            "p50_frame_ms_rebuild": statistics.median(ms),
            "p50_frame_ms_rebuild_note": "art_schedule..art_complete with every collider changed each frame: full "
                                         "H2D, record decode, Morton sort and BVH build, kernels, D2H"}


def cpu_frames(ctx, frame, min_seconds, max_frames=2000):
    """p50 and mean art_schedule..art_complete time (ms) of repeated frames on a CPU-backend context."""
    for _ in range(3):
        ctx.run(frame)
    ms, t0 = [], time.perf_counter()
    while len(ms) < max_frames and (time.perf_counter() - t0 < min_seconds or len(ms) < 5):
        t1 = time.perf_counter()
        ctx.run(frame)
        ms.append((time.perf_counter() - t1) * 1e3)
    return statistics.median(ms), sum(ms) / len(ms), len(ms)


def main_cpu(a):
    """BASELINE config 1 (8 sources x 64 rays x 256 AABB colliders, the reference's CPU-runnable
    case): frames through the C ABI's CPU backend (art_create(0): worker threads over fans, the
    jobs' loop order) on the host's cores and on one thread."""
    cfg = art.CONFIGS[a.config]
    scene, org, params = art.synth(cfg, C_scale=a.collider_scale)
    host = host_cpu_info()
    res = {}
    for label, threads in (("n", host["threads_used"]), ("one", 1)):
        os.environ["ART_CPU_THREADS"] = str(threads)
        with art.Context(0) as ctx:
            out = art.FanOutputs(cfg.S, cfg.R, cfg.H, cfg.T, 1, hits=True, dsp=params.dsp is not None)
            frame = art.Frame(scene, params, org, out)
            ctx.set_flags(abi.ART_CTX_COUNT_TESTS)
            ctx.run(frame)
            tests = sum(ctx.last_test_counts().values())
            ctx.set_flags(0)
            p50, mean, n = cpu_frames(ctx, frame, a.cpu_seconds / 2)
        res[label] = {"threads": threads, "p50_frame_ms": p50, "mean_frame_ms": mean, "frames": n,
                      "tests_per_frame": tests, "tests_per_s": tests / (mean * 1e-3)}
    os.environ.pop("ART_CPU_THREADS", None)
    print(json.dumps({
        "metric": f"config{cfg.index} CPU-backend ray-collider tests/s + p50 frame ms (plumbing through the C ABI)",
        "value": res["n"]["tests_per_s"], "unit": "ray-collider tests/s", "n_gpus": 0, "steps": res["n"]["frames"],
        "warmup": 3, "ms_per_step": res["n"]["mean_frame_ms"], "p50_frame_ms": res["n"]["p50_frame_ms"],
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"config{cfg.index}: {cfg.description}", "backend": "art_create(device_mask = 0)",
                   "fans": cfg.S, "rays": cfg.R, "colliders": cfg.C, "targets": cfg.T, "max_hits_per_ray": cfg.H},
        "threads_n": res["n"], "threads_1": res["one"], "host": host}))


def verify_allgather(ctx, dist, backend, world, rank, org_all, S_total, d_org, S, d_blk, stride, dev, sp, timed_full=None):
    """N > 1, outside the timed region: the process group has the expected size, every rank sits on
    its own device under RCCL (ranks may share one only over gloo, the CPU tests' setup), and the
    all-gathered result blocks equal, byte for byte, rank 0's own launch of a sample of every rank's
    fans (first, middle and last of each shard; fans are independent, Audio/AudioRayTracer.cs:161-237).
    Raises on any failure, so a scaling run never reports a number without its correctness check."""
    import torch.distributed as tdist
    if tdist.get_world_size() != world:
        raise RuntimeError(f"process group size {tdist.get_world_size()} != WORLD_SIZE {world}")
    props = torch.cuda.get_device_properties(dev)
    ident = (socket_host(), str(getattr(props, "uuid", "")), int(getattr(props, "pci_bus_id", -1)),
             int(getattr(props, "pci_domain_id", -1)), dev.index)
    idents = [None] * world
    tdist.all_gather_object(idents, ident)
    distinct = len({i[:4] if i[1] or i[2] >= 0 else i for i in idents}) == world
    if backend == "nccl" and not distinct:
        raise RuntimeError(f"RCCL ranks share a device: {idents}")
    ctx.launch_device(d_org.data_ptr(), S, d_blk.data_ptr(), 0, sp)
    full = art.dist.all_gather_fan_blocks(d_blk[: S * stride], S_total, stride, world)
    torch.cuda.synchronize()
    sample = []
    for r in range(world):
        b, e = art.dist.shard_range(S_total, world, r)
        if e > b:
            sample += sorted({b, (b + e) // 2, e - 1})
    ok = True
    if rank == 0:
        d_s = torch.from_numpy(np.ascontiguousarray(org_all[sample])).to(dev)
        d_ref = torch.zeros(len(sample) * stride, dtype=torch.uint8, device=dev)
        ctx.launch_device(d_s.data_ptr(), len(sample), d_ref.data_ptr(), 0, sp)
        torch.cuda.synchronize()
        got = torch.stack([full[i * stride:(i + 1) * stride] for i in sample])
        ok = bool(torch.equal(got.reshape(-1), d_ref))
        if timed_full is not None:  # the last timed frame's gather (overlapped with the next frame's kernels)
            got_t = torch.stack([timed_full[i * stride:(i + 1) * stride] for i in sample])
            ok = ok and bool(torch.equal(got_t.reshape(-1), d_ref))
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev if backend == "nccl" else "cpu")
    tdist.broadcast(flag, 0)
    if not flag.item():
        raise RuntimeError("all-gathered fan blocks differ from rank 0's own launch of the sampled fans")
    return {"verified": True, "world_size": tdist.get_world_size(), "backend": backend, "distinct_devices": distinct,
            "devices": [{"host": i[0], "uuid": i[1], "pci_bus_id": i[2], "local_index": i[4]} for i in idents],
            "sampled_fans": sample, "bytes_compared": len(sample) * stride,
            "note": "untimed, after the timed region: the all-gather's output for the sampled fans equals rank 0's own "
                    "art_launch_device of the same fans byte for byte"}


def socket_host():
    import socket
    return socket.gethostname()


def main():
    a = parse()
    if a.config is None:
        a.config = 1 if a.path == "cpu" else 2
    if a.path != "raytrace" and a.steps <= 0:
        a.steps = 50
    if a.path == "cpu":
        return main_cpu(a)
    if a.path == "dsp":
        return main_dsp(a)
    if a.path == "dirs":
        return main_dirs(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --force-dist: the N > 1 code path (process group, all-gathers, overlap, self-check) at any N,
    # so a one-GPU box can run the RCCL branch with one rank (a rehearsal of the driver's N > 1 runs)
    dist_on = world > 1 or a.force_dist
    if dist_on:
        import torch.distributed as dist
        gpu = local % max(1, torch.cuda.device_count())  # ranks may share a GPU (gloo tests)
        torch.cuda.set_device(gpu)
        if a.dist_backend == "nccl":
            # --nccl-priority high puts the collective's stream at high priority (measured with one rank:
            # the overlapped form 0.1106 -> 0.1124 ms per step, so the default stays normal)
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = a.nccl_priority == "high"
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu), pg_options=opts)
        else:
            dist.init_process_group("gloo")
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    # scalar reductions over ranks (timing, counts): device tensors over RCCL, host tensors over gloo
    red_dev = dev if a.dist_backend == "nccl" else torch.device("cpu")

    def allreduce(v, dtype, op=None):
        t = torch.tensor([v], dtype=dtype, device=red_dev)
        dist.all_reduce(t, op=op if op is not None else dist.ReduceOp.SUM)
        return t.item()

    cfg = art.CONFIGS[a.config]
    if a.targets:
        import dataclasses
        cfg = dataclasses.replace(cfg, T=a.targets, description=f"{cfg.description}, T = {a.targets} audio targets")
    scaling = a.scaling if a.scaling != "auto" else ("strong" if cfg.index == 4 else "weak")
    S_total = cfg.S if scaling == "strong" else cfg.S * world
    scene, org_all, params = art.synth(cfg, S=S_total, C_scale=a.collider_scale)
    b0, b1 = art.dist.shard_range(S_total, world, rank)
    org = np.ascontiguousarray(org_all[b0:b1])
    S = b1 - b0
    ctx = art.Context(1 << torch.cuda.current_device())
    out0 = art.FanOutputs(S, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)
    frame = art.Frame(scene, params, org, out0)
    lay = art.fan_layout(frame)
    ctx.bind(frame)
    d_org = torch.from_numpy(org).to(dev)
    d_blk = torch.zeros(max(S, 1) * lay["stride"], dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream

    counts = ctx.count_device(d_org.data_ptr(), S, d_blk.data_ptr(), 0, sp)
    tests_rank = sum(counts.values())
    bf_ops = sum(counts[k] * OPS[k] for k in ("rt_sphere", "rt_aabb", "rt_obb"))

    # N > 1 over RCCL with even shards: frame i's all-gather runs on the collective's stream beside
    # frame i + 1's kernels. Two result blocks alternate; before frame i + 2 rewrites block i % 2 the
    # launch stream waits for gather i (Work.wait: a stream wait, the host does not block).
    overlap = dist_on and a.dist_backend == "nccl" and not a.no_overlap and S * world == S_total
    stride = lay["stride"]
    og = None
    if overlap:  # (--overlap auto: kept only if it measures faster than the serial form, below)
        og = art.dist.OverlappedGather(
            [d_blk, torch.zeros_like(d_blk)], [torch.empty(S_total * stride, dtype=torch.uint8, device=dev) for _ in range(2)],
            lambda b: ctx.launch_device(d_org.data_ptr(), S, b.data_ptr(), 0, sp),
            lambda out, b: dist.all_gather_into_tensor(out, b[: S * stride], async_op=True))

    mode = {"og": og is not None}

    def step():
        if mode["og"]:
            og.step()
            return
        ctx.launch_device(d_org.data_ptr(), S, d_blk.data_ptr(), 0, sp)
        if dist_on:
            art.dist.all_gather_fan_blocks(d_blk[: S * stride], S_total, stride, world)

    def drain():  # the pending all-gathers (their output is then ready on the launch stream)
        if og is not None:
            og.drain()

    torch.cuda.synchronize()
    prewarm_frames, tp = 0, time.perf_counter()
    while time.perf_counter() - tp < a.prewarm_s:  # (untimed: the clock ramp of a fresh process)
        for _ in range(32):
            ctx.launch_device(d_org.data_ptr(), S, d_blk.data_ptr(), 0, sp)
        prewarm_frames += 32
        torch.cuda.synchronize()
    for _ in range(a.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    # --overlap auto (RCCL, even shards): the overlapped and the serial all-gather are each timed over
    # untimed frames (twice, alternating; max over ranks) and the faster form runs the timed region.
    # Measured on one GPU with one rank (--force-dist), the overlap's cross-stream waits cost ~13 us per
    # frame against ~0.4 us for a serial one-rank gather; across GPUs the serial gather carries the
    # xGMI transfer, so which form wins depends on N and is measured, not assumed.
    overlap_tune = None
    if og is not None and a.overlap == "auto":
        def trial(use):
            mode["og"] = use
            dist.barrier()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(48):
                step()
            drain()
            torch.cuda.synchronize()
            return float(allreduce(time.perf_counter() - t, torch.float64, dist.ReduceOp.MAX)) / 48 * 1e3
        ser = [trial(False), None]
        ovl = [trial(True), None]
        ser[1], ovl[1] = trial(False), trial(True)
        mode["og"] = min(ovl) < min(ser)
        overlap_tune = {"serial_ms_per_step": min(ser), "overlapped_ms_per_step": min(ovl),
                        "chosen": "overlapped" if mode["og"] else "serial",
                        "note": "untimed trials of 48 frames each (twice, alternating, max over ranks) before the "
                                "timed region; the faster all-gather form runs the timed steps"}
    overlap = mode["og"]
    steps = a.steps
    if steps <= 0:  # about 1.5 s of timed work, so the driver's sampler sees the GPU busy
        tp = time.perf_counter()  # per-step time from 10 steps after the warmup (first-call costs excluded)
        for _ in range(10):
            step()
        drain()
        torch.cuda.synchronize()
        per = (time.perf_counter() - tp) / 10
        steps = int(min(5000, max(20, 1.5 / max(per, 1e-6))))
        if dist_on:
            steps = int(allreduce(steps, torch.int64, dist.ReduceOp.MAX))
    # The timed region: K frames and nothing else between them (no event records, each of which
    # costs a few us of GPU idle: kernel durations are measured in the passes after it).
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    drain()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    dt = time.perf_counter() - t0
    # (overlapped gathers: the timed region's last gathered blocks are checked too)
    last_full = og.last() if mode["og"] else None
    verify = verify_allgather(ctx, dist, a.dist_backend, world, rank, org_all, S_total, d_org, S, d_blk, stride, dev,
                              sp, last_full) if dist_on else None
    if verify is not None:
        verify["overlapped_allgather"] = overlap
        if overlap_tune is not None:
            verify["overlap_tune"] = overlap_tune

    # Kernel durations: untimed passes of the same launches after the timed region, HIP events on
    # the streams the kernels run on. Pass 1: the frame's stages only (raytrace stage, permeation
    # job, reduce: 6 events per frame). Pass 2: also every kernel of the raytrace stage
    # (ART_CTX_TIME_EACH_KERNEL: two more events per launch, so pass 2's stage times are not used).
    n_pass = 64
    ctx.set_flags(abi.ART_CTX_TIME_KERNELS)
    ctx.kernel_timing()  # reset
    for _ in range(n_pass):
        ctx.launch_device(d_org.data_ptr(), S, d_blk.data_ptr(), 0, sp)
    ktimes = ctx.kernel_timing()
    ctx.set_flags(abi.ART_CTX_TIME_KERNELS | abi.ART_CTX_TIME_EACH_KERNEL)
    for _ in range(n_pass):
        ctx.launch_device(d_org.data_ptr(), S, d_blk.data_ptr(), 0, sp)
    keach = ctx.kernel_timing()
    ctx.set_flags(0)
    if keach["kernel_marks_dropped"]:  # a family's time would be missing launches: never report it silently
        raise RuntimeError(f"per-kernel timing dropped {keach['kernel_marks_dropped']} launch marks")
    # the all-gather alone: HIP events on the launch stream around the collective of n_pass frames
    allgather_ms = None
    if dist_on:
        evs = []
        for _ in range(n_pass):
            ctx.launch_device(d_org.data_ptr(), S, d_blk.data_ptr(), 0, sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            art.dist.all_gather_fan_blocks(d_blk[: S * lay["stride"]], S_total, lay["stride"], world)
            e1.record(stream)
            evs.append((e0, e1))
        torch.cuda.synchronize()
        allgather_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / len(evs)
        allgather_ms = allreduce(allgather_ms, torch.float64, dist.ReduceOp.MAX)
    # work the kernels actually executed in one frame (broad phase: far fewer exact tests)
    ctx.set_flags(abi.ART_CTX_COUNT_EXECUTED)
    ctx.executed_counts()  # reset
    ctx.launch_device(d_org.data_ptr(), S, d_blk.data_ptr(), 0, sp)
    torch.cuda.synchronize()
    executed = ctx.executed_counts()
    ctx.set_flags(0)
    if dist_on:
        dt = float(allreduce(dt, torch.float64, dist.ReduceOp.MAX))
        tests_all = float(allreduce(tests_rank, torch.float64))
    else:
        tests_all = float(tests_rank)

    # p50 per-frame latency through the Unity-facing API (host arrays, H2D + kernels + D2H)
    frame_ms = []
    if rank == 0:
        for i in range(a.frames + 5):
            t1 = time.perf_counter()
            ctx.run(frame)
            if i >= 5:
                frame_ms.append((time.perf_counter() - t1) * 1e3)
    # release this context (its streams) before the dynamic measurement opens its own: HIP maps a
    # process's streams onto GPU_MAX_HW_QUEUES (4) hardware queues, and a second live context's
    # side streams would share a queue with its main stream (streams)
    ctx.close()

    dyn = None
    if rank == 0 and world == 1 and not a.no_dynamic:
        dyn = dynamic_step(cfg, scene, params, org, S, steps, a.warmup, sp)

    if rank != 0:
        if dist_on:
            dist.destroy_process_group()
        return

    n_rt = max(1, ktimes["launches"])
    rt_ms = ktimes["raytrace_ms"] / n_rt
    bf_tflops = bf_ops / (rt_ms * 1e-3) / 1e12
    ex_launches = max(1, executed["launches"])
    ex_ops = (executed["sphere"] * OPS["rt_sphere"] + executed["aabb"] * OPS["rt_aabb"] + executed["obb"] * OPS["rt_obb"] +
              executed["cull_box"] * CULL_OPS["cull_box"] + executed["cell_entries"] * CULL_OPS["cell_entries"]) / ex_launches
    ex_tests = (executed["sphere"] + executed["aabb"] + executed["obb"]) / ex_launches
    ex_tflops = ex_ops / (rt_ms * 1e-3) / 1e12

    def kernel_ops(k):  # executed ops of one kernel family per frame (art_exec_counts.by_kernel)
        b = executed["by_kernel"][k]
        return (b["sphere"] * OPS["rt_sphere"] + b["aabb"] * OPS["rt_aabb"] + b["obb"] * OPS["rt_obb"] +
                b["cull_box"] * CULL_OPS["cull_box"] + b["cell_entries"] * CULL_OPS["cell_entries"]) / ex_launches
    by_kernel_ops = {k: kernel_ops(k) for k in abi.EXEC_KERNELS}
    # Every kernel family of the raytrace stage: its duration per frame (pass 2's HIP events around
    # each launch, on the stream it runs on) and the ops it executed per frame; the roofline line is
    # the family with the longest measured time per frame (the dominant kernel), the others beside it.
    fam_ops = {"nearest_first_kernel": by_kernel_ops["nearest"],
               "echo_muffle_kernel": by_kernel_ops["echo"] + by_kernel_ops["muffle"],
               "vis_kernel": by_kernel_ops["echo"], "muffle_kernel": by_kernel_ops["muffle"]}
    obb_s = "true" if scene.obbs.size > 0 else "false"
    fam_inst = {"nearest_first_kernel": f"nearest_first_kernel<false, {obb_s}, {'true' if cfg.H > 1 else 'false'}>",
                "echo_muffle_kernel": f"echo_muffle_kernel<false, {obb_s}>",
                "vis_kernel": f"vis_kernel<false, {obb_s}, false>", "muffle_kernel": f"muffle_kernel<false, {obb_s}, false>"}
    traffic, traffic_by_kernel, traffic_note = read_traffic(cfg.index)
    n_each = max(1, keach["launches"])
    kernels = {}
    for fam in abi.KERNEL_FAMILIES:
        n_l = keach["kernel_launches"][fam]
        if n_l == 0:
            continue
        k_ms = keach["kernel_ms"][fam] / n_each  # per frame (all its launches)
        tf = fam_ops[fam] / (k_ms * 1e-3) / 1e12 if k_ms > 0 else 0.0
        kernels[fam] = {"instantiation": fam_inst[fam], "ms_per_frame": k_ms, "launches_per_frame": n_l / n_each,
                        "ms_per_launch": keach["kernel_ms"][fam] / n_l, "ops_per_frame": fam_ops[fam],
                        "achieved": tf, "frac": tf / FP32_VALU_PEAK_TFLOPS,
                        "traffic": sum(v for k, v in traffic_by_kernel.items() if k.startswith(fam)) or None}
    dom = max(kernels, key=lambda k: kernels[k]["ms_per_frame"]) if kernels else "nearest_first_kernel"
    dk = kernels.get(dom, {"ms_per_frame": 0.0, "achieved": 0.0, "frac": 0.0, "traffic": None, "ops_per_frame": 0.0,
                           "launches_per_frame": 0.0, "instantiation": fam_inst[dom]})
    # algorithmic HBM bytes of one raytrace launch: the decoded collider records, directions,
    # origins and the fans' result blocks (everything else is L2-resident scratch)
    rec_bytes = scene.spheres.size * 32 + scene.aabbs.size * 32 + scene.obbs.size * 64  # hot records
    alg_bytes = rec_bytes + cfg.R * 6 + S * 12 + S * lay["stride"]
    hbm_gbs = alg_bytes / (rt_ms * 1e-3) / 1e9

    cpu = None
    if world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(cfg, scene, params, org, a.cpu_seconds)

    value = tests_all * steps / dt
    res = {
        "metric": "ray-collider tests/sec + p50 per-frame batch ms, 256src\u00d7512ray\u00d74096col",  # BASELINE.json "metric"
        "value": value,
        "unit": "equivalent ray-collider tests/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": a.warmup,
        "prewarm": {"seconds": a.prewarm_s, "frames": prewarm_frames,
                    "note": "untimed frames before the warmup steps (GPU clock ramp of a fresh process); the timed "
                            "region holds exactly `steps` frames"},
        "ms_per_step": dt / steps * 1e3,
        "p50_frame_ms": statistics.median(frame_ms) if frame_ms else None,
        "p50_frame_ms_note": "art_schedule..art_complete on rank 0, host arrays, H2D + kernels + D2H (PCIe-inclusive)",
        "dynamic": dyn,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": f"config{cfg.index}: {cfg.description}", "fans_total": S_total, "fans_rank0": S,
                   "rays": cfg.R, "colliders": cfg.C, "targets": cfg.T, "max_hits_per_ray": cfg.H,
                   "reference_tests_per_frame_rank0": tests_rank, "reference_tests_per_frame_all": tests_all,
                   "parallelism": f"fan-sharded x{world}" + (f" + all-gather ({'RCCL' if a.dist_backend == 'nccl' else 'gloo'})"
                                                              if dist_on else "")},
        "allgather_ms": allgather_ms,
        "allgather_verified": verify["verified"] if verify else None,
        "allgather_verify": verify,
        "allgather_bytes": (S_total * lay["stride"]) if dist_on else None,
        "allgather_note": (f"HIP events on the launch stream around the all-gather of {n_pass} untimed frames after the "
                           "timed region, max over ranks; " + ("in the timed steps each frame's all-gather runs beside the "
                           "next frame's kernels (RCCL stream, two result blocks alternating); every gather is inside "
                           "the timed region" if overlap else "the step time includes it")) if dist_on else None,
        "roofline": {"bound": "valu", "kernel": dk["instantiation"],
                     "achieved": dk["achieved"], "peak": FP32_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": dk["frac"], "traffic": dk["traffic"],
                     "kernel_ms": dk["ms_per_frame"], "launches_per_frame": dk["launches_per_frame"],
                     "ops_per_frame": dk["ops_per_frame"],
                     "note": "the dominant kernel: the stage's kernel family with the longest measured time per frame "
                             "(FP32 VALU roof: branchy intersection math, no MFMA-shaped work). achieved = ops it executed "
                             "per frame (exact lane-tests x SURVEY.md 8(d) ops per test + BVH box tests x 14 + cell entries "
                             "x 2, art_exec_counts.by_kernel) / its duration per frame (HIP events around each of its "
                             f"launches on the stream it runs on, {n_pass} untimed frames after the timed region, "
                             "ART_CTX_TIME_EACH_KERNEL); traffic = its HBM bytes per frame from same-build FETCH_SIZE / "
                             "WRITE_SIZE passes (" + traffic_note + ")",
                     "kernels": kernels,
                     "single_issue": {"achieved": dk["achieved"], "peak": SINGLE_ISSUE_TLOPS, "unit": "T lane-op/s",
                                      "frac": dk["achieved"] / SINGLE_ISSUE_TLOPS,
                                      "frac_at_64_lanes_per_clk": dk["achieved"] / SINGLE_ISSUE_TLOPS_64,
                                      "note": "one non-FMA lane-op per lane per issue. peak assumes a wave64 VALU op issues "
                                              "over 2 cycles per SIMD (32 lanes/clk/SIMD, MI355X_MICROARCH.md line 54): "
                                              "256 CU x 128 lanes/clk x 2.4 GHz = 78.6 T; frac_at_64_lanes_per_clk is the "
                                              "fraction of 39.3 T (64 lanes/clk/CU, SURVEY.md 8(d)) if that issue rate is "
                                              "not reached without packed math"},
                     "stage": {"kernels": stage_kernels(cfg, params.thread_count, scene.obbs.size > 0), "kernel_ms": rt_ms, "achieved": ex_tflops,
                               "frac": ex_tflops / FP32_VALU_PEAK_TFLOPS,
                               "single_issue_frac": ex_ops / (rt_ms * 1e-3) / 1e12 / SINGLE_ISSUE_TLOPS,
                               "traffic": traffic, "traffic_by_kernel": traffic_by_kernel, "traffic_note": traffic_note,
                               "note": "the whole raytrace stage (HIP events on the launch stream): executed ops of "
                                       "every kernel / stage time"},
                     "executed": {"ops_per_launch": ex_ops, "exact_lane_tests_per_launch": ex_tests,
                                  "ops_per_frame_by_kernel": by_kernel_ops,
                                  "counts": {k: v // ex_launches for k, v in executed.items()
                                             if k not in ("launches", "bounce_rays", "by_kernel")},
                                  "counts_by_kernel": {k: {f: v // ex_launches for f, v in d.items()}
                                                       for k, d in executed["by_kernel"].items()},
                                  "bounce_rays": [v // ex_launches for v in executed["bounce_rays"][:cfg.H]]},
                     "equivalent": {"achieved": bf_tflops, "frac": bf_tflops / FP32_VALU_PEAK_TFLOPS,
                                    "reference_tests_per_launch": tests_rank,
                                    "note": "brute-force-equivalent: the reference algorithm's tests x ops per test / "
                                            "stage time; the broad phase skips most of them, so this is not a roofline"},
                     "hbm": {"achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_gbs / HBM_PEAK_GBS,
                             "algorithmic_bytes": alg_bytes,
                             "counter_gbs": traffic / (rt_ms * 1e-3) / 1e9 if traffic else None,
                             "counter_frac": traffic / (rt_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None,
                             "note": "achieved = algorithmic bytes / stage time; counter_gbs = the stage's PMC HBM bytes "
                                     "(2 x FETCH_SIZE + WRITE_SIZE, same build) / stage time"}},
        "kernel_ms": {"raytrace": rt_ms, "permeate": ktimes["permeate_ms"] / n_rt, "reduce": ktimes["reduce_ms"] / n_rt,
                      **{k: v["ms_per_frame"] for k, v in kernels.items()},
                      "frames_timed": n_rt, "kernel_marks_dropped": keach["kernel_marks_dropped"],
                      "note": f"pass 1 (stage events only, {n_pass} untimed frames after the timed "
                                                    "region); per kernel family: pass 2 (ART_CTX_TIME_EACH_KERNEL)"},
        "lib_sha256": lib_sha256(),
        "cpu_baseline": cpu,
    }
    print(json.dumps(res))
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
