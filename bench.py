#!/usr/bin/env python3
"""Benchmark of the two hot paths on MI355X (contract: one JSON line on rank 0).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Primary metric (BASELINE.json): Mrays/s of the path tracer on C3 — the 250k-triangle Sponza-like
atrium at 1920x1080, 64 samples per pixel per GPU (one step = one 64-spp frame = one launch of
pt_camera_kernel). Rays = extension + shadow segments, counted exactly by the kernel.
Multi-GPU: sample-index shard (rank g renders frame counts g, g+N, ...; weak scaling: 64 spp per
GPU) + one RCCL reduce (sum) of the radiance buffer to rank 0 inside the timed region.
Secondary (same JSON line, "gs"): 3DGS forward on C2 — 100k Gaussians at 1920x1080, Gsplats/s.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/s (path trace) + Gsplats/s (3DGS) at 1920×1080, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md §L2: ~34.5 TB/s aggregate


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--triangles", type=int, default=250_000)
    ap.add_argument("--gaussians", type=int, default=100_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gs", action="store_true")
    ap.add_argument("--no-pt", action="store_true")
    ap.add_argument("--no-hybrid", action="store_true")
    ap.add_argument("--no-gpu-bvh", action="store_true")
    ap.add_argument("--no-wavefront", action="store_true")
    ap.add_argument("--headline-only", action="store_true",
                    help="only the timed C3 launch and C2 loop among the PT / 3DGS legs (no viewer, unsorted, "
                         "views4, orbit legs): profiles/profile.sh, so that per-kernel averages are per-launch figures")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 Cornell-box leg")
    ap.add_argument("--no-torus", action="store_true", help="skip the torus data-collection leg (SURVEY 8f #1)")
    ap.add_argument("--no-capture", action="store_true", help="skip the dataset capture / export leg (SURVEY 8f #4)")
    ap.add_argument("--no-gs-1m", action="store_true", help="skip the 1M-Gaussian splat and the point-cloud init legs")
    ap.add_argument("--no-splat-overlap", action="store_true",
                    help="time the C2 splat one frame at a time (default: frames in flight, PTGS_FLAG_SPLAT_OVERLAP)")
    ap.add_argument("--no-gs-10m", action="store_true", help="skip the 10M-Gaussian 3840x2160 splat leg (C5's splat)")
    ap.add_argument("--hybrid-gaussians", type=int, default=1_000_000)
    ap.add_argument("--hybrid-spp", type=int, default=16)
    ap.add_argument("--count-spp", type=int, default=4, help="spp of the instrumented counting pass")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip BASELINE config 5 (10M Gaussians + 1M-tri mesh, 3840x2160, 256 spp in total: "
                         "sample shard + RCCL all-reduce, splat-over composite by tile-row shard + reduce; "
                         "~20 s of scene generation and two ~4 s frames on one GPU)")
    ap.add_argument("--c5", action="store_true", help="(default; kept for old command lines)")
    return ap.parse_args()


def _profiled(kernel: str, need_traffic: bool = True):
    """rocprof figures of `kernel` from profiles/traffic_latest.json, only if they were collected on this
    exact libptgs.so (sha256) — otherwise None (the numbers would describe another build). need_traffic:
    only an entry the counter passes saw (HBM bytes per launch); else the kernel trace's duration suffices."""
    import hashlib
    tpath = os.path.join(ROOT, "profiles", "traffic_latest.json")
    try:
        tj = json.load(open(tpath))
        lib_sha = hashlib.sha256(open(os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs.so"),
                                      "rb").read()).hexdigest()
        if tj.get("lib_sha256") != lib_sha:
            return None
        e = tj.get("kernels", {}).get(kernel)
        return e if e and (e.get("hbm_bytes_per_launch") or (not need_traffic and e.get("avg_ms"))) else None
    except (OSError, ValueError):
        return None


def _roofline(kernel: str, traffic, kernel_ms: float, prof, cache_inclusive: dict) -> dict:
    """HBM roofline of one kernel: achieved = counter-measured HBM bytes per launch (rocprof PMC,
    2*FETCH_SIZE+WRITE_SIZE) / the launch duration measured live here with HIP events."""
    ach = traffic / (kernel_ms * 1e-3) / 1e9 if traffic else None
    r = {"bound": "hbm", "kernel": kernel, "achieved": None if ach is None else round(ach, 2),
         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None if ach is None else round(ach / HBM_PEAK_GBS, 5),
         "traffic": traffic, "kernel_ms": round(kernel_ms, 4),
         "basis": "HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, "
                  "profiles/traffic_latest.json, same libptgs.so sha256) / HIP-event launch time"}
    if prof:
        r["profile"] = {k: prof.get(k) for k in ("avg_ms", "l2_hit", "valu_lane_util", "valu_issue_share",
                                                  "wave_wait_share")}
    r["cache_inclusive"] = cache_inclusive
    return r


def band_split_leg(r, Renderer, g, ubo, W, H, img, full_ms, stream, ranks=8, frames=10):
    """The 8-GPU tile-row split of a large splat frame, rehearsed on this GPU: the
    Gaussians' Morton copy with chunk bounds (what each rank renders from), rows balanced by a full frame's
    per-row pair counts (dist.balanced_tile_rows), then re-split once from the measured band times
    (dist.rebalance_tile_rows, two feedback steps, the better kept); each band on a context of its own (a rank renders its band every frame),
    timed one after another. The 8-GPU frame is bounded below by the slowest band (plus the row gather,
    ~16.6 MB per rank at 4K, overlapped by RowGatherPipeline). Unmeasured on 8 GPUs: no such node here."""
    import torch
    from pathtracer_gaussiansplatting_amd import dist as D
    dg = r.sort_gaussians_spatial(g, stream=stream)
    dg = dict(dg, chunk_bounds=r.gaussians_chunk_bounds(dg, stream=stream))
    rp = Renderer(r.device, publish_splat_buffers=True)
    st = rp.splat_gaussians(dg, ubo, W, H, img, want_stats=True, stream=stream)
    b = rp.splat_buffers()
    rng = np.zeros(2 * b.num_tiles, np.uint32)
    rp.copy_d2h(rng, b.tile_ranges, rng.nbytes)
    rp.close()
    row_pairs = D.row_pairs_from_ranges(rng, st.tiles_x)
    split = D.balanced_tile_rows(row_pairs, ranks, st.tiles_x)

    def time_split(sp):
        ms = []
        for rows in sp:
            rk = Renderer(r.device)
            rk.splat_reserve(int(st.num_rendered))
            for _ in range(6):
                rk.splat_gaussians(dg, ubo, W, H, img, tile_rows=tuple(rows), stream=stream)
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(frames):
                rk.splat_gaussians(dg, ubo, W, H, img, tile_rows=tuple(rows), stream=stream)
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) / frames * 1e3)
            rk.close()
        return ms

    ms0 = time_split(split)
    split1 = D.rebalance_tile_rows(split, ms0, row_pairs, st.tiles_x)
    ms1 = time_split(split1)
    split2 = D.rebalance_tile_rows(split1, ms1, row_pairs, st.tiles_x)  # (a second feedback step)
    ms2 = time_split(split2)
    if max(ms2) < max(ms1):
        split1, ms1 = split2, ms2
    del dg
    return {"ranks": ranks, "rows_by_pairs": split, "band_ms_by_pairs": [round(x, 4) for x in ms0],
            "rows_rebalanced": split1, "band_ms_rebalanced": [round(x, 4) for x in ms1],
            "slowest_band_ms": round(max(ms1), 4), "full_frame_ms": round(full_ms, 4),
            "full_over_slowest": round(full_ms / max(ms1), 3),
            "note": "one GPU, bands one after another (Morton copy + chunk bounds); the 8-GPU frame itself is "
                    "unmeasured (no 8-GPU node in this pool)"}


def log2ceil(n):
    return max(0, math.ceil(math.log2(max(n, 1))))


def gs_orbit_ubos(Camera, make_ubo, scene, W, H, frames):
    """The viewer-protocol camera path of the gs_orbit leg: orbit the C2 cloud's centre (0, 0, -8) at
    1.5 degrees per frame while dollying from 8 units (the C2 camera) to 5 and back."""
    c = np.array([0.0, 0.0, -8.0])
    out = []
    for k in range(frames):
        rr = 8.0 - 3.0 * math.sin(math.pi * k / max(1, frames - 1))
        th = math.radians(1.5 * k)
        eye = c + np.array([rr * math.sin(th), 0.1 * rr * math.sin(0.5 * th), rr * math.cos(th)])
        out.append(make_ubo(Camera(aspect=W / H).look_at(eye.tolist(), c.tolist()), scene, 0))
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    # (local % device count: lets a 1-GPU box rehearse several ranks with BENCH_DIST_BACKEND=gloo;
    # one rank per GPU otherwise)
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            dist.barrier()

    def reduce_to_root(t):
        # RCCL reduce(SUM) to rank 0 through the library's communicator (ptgs_reduce_radiance); the gloo
        # rehearsal (several ranks on one GPU) has no CUDA reduce: torch all-reduce instead
        if world > 1:
            if native_comm:
                r.reduce_radiance(t, root=0, stream=stream)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.SUM)

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def assert_complete(rr, where: str, strm=None) -> int:
        # every timed splat frame must have been rendered completely: tiles that outgrow the buffers
        # sized from earlier frames are completed through the spill pool on the device (counted); a
        # frame whose spilled tiles exceed the pool would be incomplete (ptgs_splat_status_read counts
        # those) and cheaper than real work, so the bench refuses to report it. Returns the spilled tiles.
        st = rr.splat_status(stream if strm is None else strm)
        if int(st.frames) or int(st.incomplete_tiles):
            raise SystemExit(f"bench: {int(st.frames)} splat frame(s) incomplete in {where} (spill pool exhausted)")
        return int(st.spilled_tiles)

    def sum_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    from pathtracer_gaussiansplatting_amd import (ACCUM_RUNNING_MEAN, ACCUM_SUM, FLAG_COUNT_TRAVERSAL, FLAG_GPU_BVH, FLAG_GPU_LBVH,
                                                  FLAG_TIME_STAGES, Camera, Renderer, make_ubo)
    from pathtracer_gaussiansplatting_amd import synthetic as Y

    W, H, SPP = args.width, args.height, args.spp
    r = Renderer(dev)
    stream = torch.cuda.current_stream()
    from pathtracer_gaussiansplatting_amd import dist as D
    # the library's own RCCL communicator (one rank per GPU): frame reduce and row gather through the C-ABI
    native_comm = world > 1 and dist.get_backend() == "nccl"
    if native_comm:
        D.init_native_comm(r)
    out = {"metric": METRIC, "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32"}

    # ------------------------------------------------------------------ path tracer (C3)
    if not args.no_pt:
        scene = Y.atrium_scene(target_tris=args.triangles, seed=2)
        scene.blue_noise = Y.blue_noise(1024)
        info = r.upload_scene(scene)
        pose = Camera(aspect=W / H).look_at([-15.0, 4.0, 5.0], [10.0, 3.0, -3.0])
        accum = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        mode = ACCUM_RUNNING_MEAN if world == 1 else ACCUM_SUM
        frame_base = 0

        def pt_step(ev0=None, ev1=None):
            nonlocal frame_base
            # sample shard: global sample index s*world + rank (frame_stride = world)
            ubo = make_ubo(pose, scene, frame_base * world + rank, ambient=(0.3, 0.4, 0.5, 1.0), height=H)
            if mode == ACCUM_SUM:
                accum.zero_()
            if ev0 is not None:
                ev0.record(stream)
            r.trace_camera(ubo, W, H, accum, spp=SPP, frame_stride=world, mode=mode, stream=stream)
            if ev1 is not None:
                ev1.record(stream)
            reduce_to_root(accum)
            frame_base += SPP

        for _ in range(args.warmup):
            pt_step()
        torch.cuda.synchronize()
        r.stats_reset(stream)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            pt_step(*evs[k])
        torch.cuda.synchronize()
        barrier()
        dt = time.perf_counter() - t0
        kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        st = r.stats()
        rays_local = float(st.extension_rays + st.shadow_rays)
        dt_max = max_over_ranks(dt)
        rays_total = sum_over_ranks(rays_local)
        mrays = rays_total / dt_max / 1e6
        # instrumented counting pass (same scene / camera, count_spp samples) -> bytes per ray
        r.set_flags(FLAG_COUNT_TRAVERSAL)
        r.stats_reset(stream)
        tmp = torch.zeros_like(accum)
        cnt_ubo = make_ubo(pose, scene, 0, ambient=(0.3, 0.4, 0.5, 1.0), height=H)
        r.trace_camera(cnt_ubo, W, H, tmp, spp=args.count_spp, mode=ACCUM_RUNNING_MEAN, stream=stream)
        torch.cuda.synchronize()
        cs = r.stats()
        r.set_flags(0)
        del tmp
        n_l = len(scene.light_cdf)
        rays_c = cs.extension_rays + cs.shadow_rays
        bytes_c = (cs.node_visits * 32 + cs.tri_tests * 36 + cs.closest_hits * 576
                   + cs.shadow_rays * (16 * log2ceil(n_l) + 16 + 3 * 80 + 308)
                   + cs.samples * (16 + 16 + 16))
        bytes_per_ray = bytes_c / max(rays_c, 1)
        rays_per_launch = rays_local / args.steps
        alg_bytes = bytes_per_ray * rays_per_launch
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
        # HBM bytes per launch from the rocprof PMC passes of THIS library build (profiles/profile.sh +
        # parse_rocprof.py record the sha256 of libptgs.so); null when the profile is stale or absent
        prof = _profiled("pt_camera_kernel")
        traffic = prof["hbm_bytes_per_launch"] if prof else None
        out.update({
            "value": round(mrays, 3), "unit": "Mrays/s", "ms_per_step": round(dt_max / args.steps * 1e3, 3),
            "data": "synthetic: seeded procedural 250k-triangle atrium (no dataset/network)",
            "config": {"workload": f"C3 path trace: {args.triangles}-tri Sponza-like atrium, {W}x{H}, {SPP} spp per GPU",
                       "width": W, "height": H, "spp_per_gpu": SPP, "triangles": int(info.num_triangles),
                       "bvh_nodes": int(info.num_bvh_nodes), "bvh_depth": int(info.bvh_depth),
                       "bvh_build": f"host binned SAH, {info.build_ms:.1f} ms",
                       "parallelism": "single GPU" if world == 1 else f"sample-shard x{world} + RCCL reduce"},
            "rays_per_step": rays_total / args.steps,
            "samples_per_s": st.samples * world / dt_max,
            "kernel_ms": round(kernel_ms, 3),
            "roofline": _roofline("pt_camera_kernel", traffic, kernel_ms, prof, {
                "bound": "l2", "achieved": round(achieved, 2), "peak": L2_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / L2_PEAK_GBS, 5), "alg_bytes_per_launch": alg_bytes,
                "bytes_per_ray": round(bytes_per_ray, 2),
                "counts_per_ray": {"node_visits": cs.node_visits / max(rays_c, 1),
                                   "tri_tests": cs.tri_tests / max(rays_c, 1)},
                "note": "cache-inclusive: B_pt (SURVEY 8d) prices every BVH node / triangle / shading fetch the "
                        "kernel issues; the C3 scene is L2/MALL-resident, so it is priced against the L2 peak"}),
        })
        # the wavefront path tracer (PTGS_FLAG_PT_WAVEFRONT) on the same frames: raygen / extend / shade /
        # shadow / accumulate stages over compacted ray queues
        if not args.no_wavefront:
            r.set_wavefront(True)
            for _ in range(max(args.warmup, 1)):
                pt_step()
            torch.cuda.synchronize()
            r.stats_reset(stream)
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(args.steps):
                pt_step()
            torch.cuda.synchronize()
            barrier()
            wdt = max_over_ranks(time.perf_counter() - t0)
            wst = r.stats()
            r.set_wavefront(False)
            out["pt_wavefront"] = {"value": round(sum_over_ranks(float(wst.extension_rays + wst.shadow_rays)) / wdt / 1e6,
                                                  3), "unit": "Mrays/s", "ms_per_step": round(wdt / args.steps * 1e3, 3),
                                   "note": "same C3 frames through the wavefront stages (PTGS_FLAG_PT_WAVEFRONT)"}
        # the viewer's protocol (recordCommandBuffer, engine.cpp:1971-1976): one sample per call at the
        # swapchain size, running mean of raygen_camera.rgen:80-87 into the accumulator, frame_count
        # advancing per call - SPP consecutive 1-spp calls against the one SPP-sample launch above
        if world == 1 and not args.headline_only:
            vacc = torch.zeros_like(accum)
            for k in range(4):
                r.trace_camera(make_ubo(pose, scene, k, ambient=(0.3, 0.4, 0.5, 1.0), height=H), W, H, vacc, spp=1,
                               stream=stream)
            vubos = [make_ubo(pose, scene, k, ambient=(0.3, 0.4, 0.5, 1.0), height=H) for k in range(SPP)]
            torch.cuda.synchronize()
            r.stats_reset(stream)
            t0 = time.perf_counter()
            for u in vubos:
                r.trace_camera(u, W, H, vacc, spp=1, stream=stream)
            torch.cuda.synchronize()
            vdt = time.perf_counter() - t0
            vst = r.stats()
            vm = (vst.extension_rays + vst.shadow_rays) / vdt / 1e6
            out["viewer_1spp"] = {"value": round(vm, 3), "unit": "Mrays/s", "ms_per_call": round(vdt / SPP * 1e3, 4),
                                  "calls": SPP, "vs_launch": round(vm / mrays, 4),
                                  "workload": f"C3, {SPP} consecutive ptgs_trace_camera(spp=1) calls at {W}x{H} "
                                              "(the viewer's per-frame call; running mean)"}
            del vacc
        # the GPU BVH builders on the same scene: build time and one traced frame each. PTGS_FLAG_GPU_BVH
        # is the host's binned SAH run on the GPU (the same tree: the same traversal cost);
        # PTGS_FLAG_GPU_LBVH the linear BVH (fastest rebuilds, weaker tree)
        if world == 1 and not args.no_gpu_bvh:
            out["bvh_gpu"] = {}
            for key, flags, note in (("sah", FLAG_GPU_BVH, "host binned-SAH algorithm on the GPU: the host tree"),
                                     ("lbvh", FLAG_GPU_BVH | FLAG_GPU_LBVH, "linear BVH (Morton order)")):
                r.set_flags(flags)
                r.upload_scene(scene)  # first build pays module first-use costs
                ginfo = r.upload_scene(scene)
                r.set_flags(0)
                pt_step()
                torch.cuda.synchronize()
                r.stats_reset(stream)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pt_step()
                torch.cuda.synchronize()
                gdt_pt = time.perf_counter() - t0
                gst = r.stats()
                out["bvh_gpu"][key] = {"build_ms": round(float(ginfo.build_ms), 3), "nodes": int(ginfo.num_bvh_nodes),
                                       "depth": int(ginfo.bvh_depth),
                                       "mrays_per_s": round((gst.extension_rays + gst.shadow_rays) / gdt_pt / 1e6, 2),
                                       "note": note}
            out["bvh_gpu"]["host_sah_build_ms"] = round(float(info.build_ms), 3)
            r.upload_scene(scene)  # back to the SAH tree for the legs below
        del accum

    # ------------------------------------------------------------------ 3DGS (C2)
    if not args.no_gs:
        g = Y.gaussians_c2(args.gaussians, seed=1)  # one scene: every rank holds all Gaussians
        dg0 = {k: torch.from_numpy(v).cuda() for k, v in g.items()}  # the generator's (random) order
        # scene preparation (untimed, like the BVH build): a copy in 3D Morton order of the means with
        # the original indices (ptgs_gaussians_sort_spatial); it renders exactly like dg0 (checked below)
        torch.cuda.synchronize()
        tprep = time.perf_counter()
        dg = r.sort_gaussians_spatial(dg0, stream=stream)
        prep_ms = (time.perf_counter() - tprep) * 1e3
        gpose = Camera(aspect=W / H).look_at([0.0, 0.0, 0.0], [0.0, 0.0, -1.0])
        from pathtracer_gaussiansplatting_amd import cornell_box_scene
        gubo = make_ubo(gpose, cornell_box_scene(), 0)
        img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        # frames in flight (the viewer's loop; reference MAX_FRAMES_IN_FLIGHT = 2, engine.h:33): each call's
        # front end runs on the context's second stream beside the previous calls' blends, which stay ordered
        # on `stream` (PTGS_FLAG_SPLAT_OVERLAP; same images bit for bit, tests/test_splat_moving_gpu.py).
        # Every frame still runs its own preprocess, binning, sort and blend.
        gs_overlap = not args.no_splat_overlap
        r.set_splat_overlap(gs_overlap)
        for _ in range(max(args.warmup, 1)):
            r.splat_gaussians(dg, gubo, W, H, img, stream=stream)
        torch.cuda.synchronize()
        # ~0.05 ms per frame: 500 consecutive frames (~25 ms) for a stable mean, the frames-in-flight pipeline's
        # fill (the first front end alone) and drain amortised as in a viewer's continuous loop (100 frames had
        # read 0.0501-0.0506 ms where 400 read 0.0497, same box)
        gsteps = max(args.steps, 500)
        gs_rows = None
        gs_policy = "single"
        gubo_rank = gubo
        if world > 1:
            # how the ranks split C2 frames (dist.splat_policy): tile rows only when a rank's band
            # outlasts rank 0's intake of the rows over xGMI; at C2 a band is ~7 us against ~83 us of gather,
            # so each rank renders whole frames of its own view (replicas, the capture loop's many views)
            for _ in range(20):
                r.splat_gaussians(dg, gubo, W, H, img, stream=stream)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(50):
                r.splat_gaussians(dg, gubo, W, H, img, stream=stream)
            torch.cuda.synchronize()
            full_ms = max_over_ranks((time.perf_counter() - t1) / 50 * 1e3)
            gs_policy = D.splat_policy(full_ms, W, H, world)
            # (replicas: rank r's view turns the C2 camera by 360 r / world degrees about the cloud's centre)
            th = 2.0 * math.pi * rank / world
            gubo_rank = make_ubo(Camera(aspect=W / H).look_at([8.0 * math.sin(th), 0.0, -8.0 + 8.0 * math.cos(th)],
                                                              [0.0, 0.0, -8.0]), cornell_box_scene(), 0)
            # SURVEY 8e tile-row shard: rows balanced by a full frame's per-row pair counts (the same
            # split on every rank), each rank renders its rows, rank 0 gathers them (W*H*16/G B each)
            st0 = r.splat_gaussians(dg, gubo, W, H, img, want_stats=True, stream=stream)
            b0 = r.splat_buffers()
            rng = np.zeros(2 * b0.num_tiles, np.uint32)
            r.copy_d2h(rng, b0.tile_ranges, rng.nbytes)
            gs_rows = D.balanced_tile_rows(D.row_pairs_from_ranges(rng, st0.tiles_x), world, st0.tiles_x)
            gs_px = [D.pixel_rows(t, H) for t in gs_rows]
            hostimg = None if native_comm else torch.zeros((H, W, 4), dtype=torch.float32)
            # frame f's row gather (RCCL, second stream) overlaps frame f + 1's band (two alternating images)
            gs_pipe = D.RowGatherPipeline(r, W, H, gs_rows, rank, world, stream=stream) if native_comm else None

        def gs_step():
            if world == 1 or gs_policy == "replicas":
                r.splat_gaussians(dg, gubo_rank, W, H, img, stream=stream)
            else:
                gs_step_tiles()

        def gs_step_tiles():
            if native_comm:
                gs_pipe.submit(dg, gubo)
            else:  # gloo rehearsal: the rows through host memory
                if gs_rows[rank][1] > gs_rows[rank][0]:
                    r.splat_gaussians(dg, gubo, W, H, img, tile_rows=gs_rows[rank], stream=stream)
                p0, p1 = gs_px[rank]
                hostimg[p0:p1].copy_(img[p0:p1])
                D.gather_rows(hostimg, gs_px, dst=0)

        for _ in range(max(args.warmup, 1)):
            gs_step()
        # untimed warm-up until the GPU has run ~0.3 s of these frames (the frames are ~0.1 ms: a few
        # warm-up frames leave the clocks of the preceding leg / idle state; measured 0.081 vs 0.076 ms)
        tw = time.perf_counter()
        while time.perf_counter() - tw < 0.3:
            for _ in range(20):
                gs_step()
            torch.cuda.synchronize()
        r.splat_status(stream)  # (clears: warm-up frames may have grown the buffers)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(gsteps):  # timed: no per-stage events, no stats read-back
            gs_step()
        if gs_policy == "tile_rows" and native_comm:
            gs_pipe.wait()  # (the last frames' gathers are inside the timed region)
        torch.cuda.synchronize()
        barrier()
        gdt = max_over_ranks(time.perf_counter() - t0)
        c2_spilled = assert_complete(r, "C2 timed loop")

        def frame_latency_ms():  # one frame from its call to its image, alone (median of 21)
            lat = []
            for _ in range(21):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                gs_step()
                torch.cuda.synchronize()
                lat.append((time.perf_counter() - t1) * 1e3)
            return float(np.median(lat))

        gs_lat = frame_latency_ms()
        gs_serial = None
        if gs_overlap and not args.headline_only:  # the same loop one frame at a time (secondary figure)
            r.set_splat_overlap(False)
            tw = time.perf_counter()
            while time.perf_counter() - tw < 0.2:
                for _ in range(20):
                    gs_step()
                torch.cuda.synchronize()
            r.splat_status(stream)
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(gsteps):
                gs_step()
            if gs_policy == "tile_rows" and native_comm:
                gs_pipe.wait()
            torch.cuda.synchronize()
            barrier()
            sdt = max_over_ranks(time.perf_counter() - t0)
            assert_complete(r, "C2 serial loop")
            gs_serial = {"value": round(args.gaussians * (world if gs_policy == "replicas" else 1) / (sdt / gsteps) / 1e9, 4),
                         "unit": "Gsplats/s", "ms_per_step": round(sdt / gsteps * 1e3, 4),
                         "frame_latency_ms": round(frame_latency_ms(), 4),
                         "note": "one frame at a time on the caller's stream (front end, then blend)"}
        gs_tiles = None
        if gs_policy == "replicas":  # the tile-row shard of the same frame (secondary: the north_star's split)
            r.set_splat_overlap(gs_overlap)
            for _ in range(20):
                gs_step_tiles()
            if native_comm:
                gs_pipe.wait()
            torch.cuda.synchronize()
            r.splat_status(stream)
            barrier()
            t0 = time.perf_counter()
            for _ in range(gsteps):
                gs_step_tiles()
            if native_comm:
                gs_pipe.wait()
            torch.cuda.synchronize()
            barrier()
            tdt = max_over_ranks(time.perf_counter() - t0)
            assert_complete(r, "C2 tile-row shard")
            gs_tiles = {"value": round(args.gaussians / (tdt / gsteps) / 1e9, 4), "unit": "Gsplats/s",
                        "ms_per_step": round(tdt / gsteps * 1e3, 4), "scaling": "strong", "rows": gs_rows,
                        "note": "one C2 frame split by tile rows balanced by pair counts + row gather to rank 0"}
        r.set_splat_overlap(False)
        # the same frames from the Gaussians in their generated (random) order: the same image bit for
        # bit, timed alone (secondary figure)
        udt = None
        img0 = torch.zeros_like(img)
        r.splat_gaussians(dg0, gubo, W, H, img0, stream=stream)
        r.splat_gaussians(dg, gubo, W, H, img, stream=stream)
        torch.cuda.synchronize()
        same_image = bool(torch.equal(img0, img))
        if not same_image:
            raise SystemExit("bench: the spatially ordered Gaussians render a different C2 frame")
        if not args.headline_only:
            for _ in range(3):
                r.splat_gaussians(dg0, gubo, W, H, img0, stream=stream)
            r.splat_status(stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(gsteps):
                r.splat_gaussians(dg0, gubo, W, H, img0, stream=stream)
            torch.cuda.synchronize()
            udt = time.perf_counter() - t0
            assert_complete(r, "C2 unsorted loop")
        del img0
        # the reference's pair count (3-sigma rectangles: a frame with stats) beside the timed frames' own
        # (alpha-box binning, published by every frame: ptgs_splat_status last_pairs)
        st = r.splat_gaussians(dg, gubo, W, H, img, want_stats=True, stream=stream)
        K_exact = int(st.num_rendered)
        # per-stage split of the timed mode (separate, untimed pass: the stage events themselves cost ~40 us
        # per frame; no stats, so the same frames as the timed loop)
        r.set_flags(FLAG_TIME_STAGES)
        stages = np.zeros(6)
        for _ in range(3):
            r.splat_gaussians(dg, gubo, W, H, img, stream=stream)
        for _ in range(gsteps):
            r.splat_gaussians(dg, gubo, W, H, img, stream=stream)
            stages += r.splat_stage_ms()
        r.set_flags(0)
        stages /= gsteps
        gstat = r.splat_status(stream)
        N = args.gaussians
        K = int(gstat.last_pairs)  # the timed frames' pairs
        P = math.ceil((32 + log2ceil(st.tiles_x * st.tiles_y)) / 8)
        b_gs = N * (56 + 48) + N * 48 + K * 12 + P * K * 24 + K * (4 + 48) + W * H * 16
        gms = gdt / gsteps * 1e3
        out["gs"] = {
            "value": round(N * (world if gs_policy == "replicas" else 1) / (gdt / gsteps) / 1e9, 4), "unit": "Gsplats/s",
            "ms_per_step": round(gms, 4),
            "frames_in_flight": ("on: each call's front end on the context's second stream beside the previous calls' "
                                 "blends (PTGS_FLAG_SPLAT_OVERLAP, 3 workspaces), every frame fully rendered")
            if gs_overlap else "off",
            "frame_latency_ms": round(gs_lat, 4),
            "serial": gs_serial,
            "workload": f"C2 3DGS forward: {N} synthetic Gaussians, {W}x{H}", "pairs_K": int(K),
            "pairs_K_3sigma": K_exact,
            "skipped_frames": 0,  # incomplete frames: checked after every timed splat loop (ptgs_splat_status_read)
            "spilled_tiles": c2_spilled,
            "scaling": "weak" if gs_policy == "replicas" else "strong",
            "policy": gs_policy,
            "parallelism": "single GPU" if world == 1 else
            (f"replicas x{world}: each rank renders whole frames of its own view (dist.splat_policy: a C2 band "
             "would be shorter than rank 0's row intake over xGMI); nothing crosses the links"
             if gs_policy == "replicas" else
             f"tile-row shard x{world} (rows balanced by pair counts: {gs_rows}) + row gather to rank 0"
             + (" (ptgs_gather_rows, RCCL, on a second stream: frame f's gather overlaps frame f + 1's band)"
                if native_comm else " (gloo rehearsal, host copies)")),
            "tile_shard": gs_tiles,
            "front_end": "fused single launch" if gstat.fused else "count + colscan + scatter",
            # per-stage split: kernel-trace averages of this libptgs.so when profiled (profiles/traffic_latest.json),
            # else per-stage HIP events of an untimed serial pass (each event pair adds its launch gap: the stages
            # sum past ms_per_step, which is the timed frame)
            "stages_us_kernel_trace": {k: round(float(e["avg_ms"]) * 1e3, 2) for k, e in
                                       (("front_end_overlapped", _profiled("gs_bin_fused_kernel_ov", False)),
                                        ("front_end_serial", _profiled("gs_bin_fused_kernel", False)),
                                        ("sort_blend", _profiled("gs_sort_blend_kernel", False))) if e} or None,
            "stages_ms_event_timed": {k: round(float(v), 4) for k, v in
                          zip(["front_end" if gstat.fused else "preprocess+count", "colscan", "scatter", "sort_large",
                               "-", "sort_blend"], stages) if k != "-" and not (gstat.fused and k in ("colscan", "scatter"))},
            "gaussian_order": f"3D Morton order of the means (ptgs_gaussians_sort_spatial, {prep_ms:.2f} ms once, "
                              "untimed scene preparation; identical image to the generated order, checked)",
            "unsorted_order": None if udt is None else {
                "value": round(N / (udt / gsteps) / 1e9, 4), "unit": "Gsplats/s", "ms_per_step": round(udt / gsteps * 1e3, 4),
                "note": "the same frames from the Gaussians in their generated (random) order"},
            "roofline": {"bound": "hbm", "kernel": "whole pipeline", "achieved": round(b_gs / (gms * 1e-3) / 1e9, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(b_gs / (gms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5), "alg_bytes": b_gs},
        }
        # per-kernel roofline of the blend (the dominant 3DGS kernel): counter-measured HBM bytes per launch
        # over its kernel-trace duration (rocprofv3 of this libptgs.so, profiles/traffic_latest.json; the
        # per-stage HIP events of the untimed serial pass when no matching profile exists: they inflate each
        # stage by its event gaps); algorithmic bytes = 8-B key + 48-B record per pair read, 16 B per pixel
        # written (no publish in production frames)
        bprof = _profiled("gs_sort_blend_kernel")
        blend_ms = float(bprof["avg_ms"]) if bprof and bprof.get("avg_ms") else float(stages[5])
        b_alg = K * (8 + 48) + W * H * 16
        out["gs"]["roofline_blend"] = _roofline("gs_sort_blend_kernel", bprof["hbm_bytes_per_launch"] if bprof else None,
                                                blend_ms, bprof, {
            "bound": "hbm", "achieved": round(b_alg / (blend_ms * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(b_alg / (blend_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "alg_bytes_per_launch": b_alg,
            "time_basis": "rocprofv3 kernel-trace average of this libptgs.so (profiles/traffic_latest.json)" if bprof
                          else "per-stage HIP events (untimed serial pass)",
            "note": "algorithmic: 8-B key + 48-B blend record per (Gaussian, tile) pair + 16 B per pixel"})
        out["gs"]["splat_pairs_per_s"] = round(K * (world if gs_policy == "replicas" else 1) / (gdt / gsteps) / 1e9, 4)
        if world == 1 and not args.headline_only:
            # four views of the C2 Gaussians per call (ptgs_splat_gaussians_views: forked streams, one
            # workspace per view), the capture-loop use: aggregate Gaussians x views per second
            vubos = [make_ubo(Camera(aspect=W / H).look_at([0.25 * k, 0.0, 0.0], [0.25 * k, 0.0, -1.0]),
                              cornell_box_scene(), 0) for k in range(4)]
            vouts = [torch.zeros_like(img) for _ in vubos]
            for _ in range(3):
                r.splat_gaussians_views(dg, vubos, W, H, vouts, stream=stream)
            torch.cuda.synchronize()
            r.splat_status(stream)
            vsteps = max(gsteps // 4, 25)
            t0 = time.perf_counter()
            for _ in range(vsteps):
                r.splat_gaussians_views(dg, vubos, W, H, vouts, stream=stream)
            torch.cuda.synchronize()
            vdt = (time.perf_counter() - t0) / vsteps
            assert_complete(r, "views4")
            out["gs"]["views4"] = {"value": round(N * len(vubos) / vdt / 1e9, 4), "unit": "Gsplats/s",
                                   "ms_per_call": round(vdt * 1e3, 4),
                                   "note": "4 camera views of the C2 Gaussians per ptgs_splat_gaussians_views call"}
            del vouts
            # the viewer's protocol (engine.cpp:2070-2072, camera.cpp:11): a new view every frame. The C2
            # Gaussians under a camera orbiting the cloud's centre and dollying in and out; every frame
            # stream-ordered (rows, pair buffer and tile order from the previous frame), timed in one run;
            # tiles that outgrow the buffers are completed through the spill pool (counted)
            orbit = gs_orbit_ubos(Camera, make_ubo, cornell_box_scene(), W, H, 120)  # (the path: 120 frames)

            host_ms = {}

            def orbit_pass(mode):
                # one untimed pass of the whole path first: buffers grown to the path's largest frame in every
                # workspace the mode uses (frames in flight: a ring of three; growth frees and reallocates,
                # which waits for the device), as in a viewer's steady orbit
                for u in orbit:
                    r.splat_gaussians(dg, u, W, H, img, stream=stream)
                torch.cuda.synchronize()
                r.splat_status(stream)
                t1 = time.perf_counter()
                for u in orbit:
                    r.splat_gaussians(dg, u, W, H, img, stream=stream)
                host_ms[mode] = round((time.perf_counter() - t1) / len(orbit) * 1e3, 4)  # (enqueue only)
                torch.cuda.synchronize()
                return (time.perf_counter() - t1) / len(orbit)

            r.set_splat_overlap(gs_overlap)  # (frames in flight, as the C2 loop)
            odt = orbit_pass("overlap")
            o_spilled = assert_complete(r, "gs_orbit")
            r.set_splat_overlap(False)
            odt_serial = orbit_pass("serial") if gs_overlap else odt
            assert_complete(r, "gs_orbit serial")
            # the timed frames' own pairs (alpha-box binning, what the blend processed): the same stream-ordered
            # frames replayed untimed, each one's count read after it (ptgs_splat_status last_pairs; the pairs
            # depend only on the camera), and the front end each frame took
            opairs, ofused = [], 0
            for u in orbit:
                r.splat_gaussians(dg, u, W, H, img, stream=stream)
                ost = r.splat_status(stream)
                opairs.append(int(ost.last_pairs))
                ofused += int(ost.fused)
            ks = []
            for u in orbit[:: max(1, len(orbit) // 12)]:  # (untimed: the 3-sigma pair counts along the path)
                ks.append(int(r.splat_gaussians(dg, u, W, H, img, want_stats=True, stream=stream).num_rendered))
            out["gs"]["gs_orbit"] = {"value": round(N / odt / 1e9, 4), "unit": "Gsplats/s", "ms_per_step": round(odt * 1e3, 4),
                                     "frames": len(orbit), "skipped_frames": 0, "spilled_tiles": o_spilled,
                                     "pairs_timed_mean": round(float(np.mean(opairs)), 1),
                                     "pairs_timed_range": [min(opairs), max(opairs)],
                                     "splat_pairs_per_s": round(sum(opairs) / (odt * len(orbit)) / 1e9, 4),
                                     "static_splat_pairs_per_s": out["gs"]["splat_pairs_per_s"],
                                     "fused_frames": ofused,
                                     "serial": {"value": round(N / odt_serial / 1e9, 4), "unit": "Gsplats/s",
                                                "ms_per_step": round(odt_serial * 1e3, 4)},
                                     "pairs_K_range": [min(ks), max(ks)],
                                     "host_enqueue_ms_per_frame": host_ms,
                                     "workload": f"C2 Gaussians, {len(orbit)} frames orbiting the cloud (1.5 deg per frame) "
                                                 "while dollying from 8 to 5 units and back, stream-ordered"}
        del dg
        # the same forward at the C4 hybrid's Gaussian count (1M), splat only
        if world == 1 and not args.no_gs_1m:
            g1 = {k: torch.from_numpy(v).cuda() for k, v in Y.gaussians_c2(args.hybrid_gaussians, seed=3).items()}
            r.splat_gaussians(g1, gubo, W, H, img, want_stats=True, stream=stream)  # sizes the pair buffer
            for _ in range(2):
                r.splat_gaussians(g1, gubo, W, H, img, stream=stream)
            torch.cuda.synchronize()
            r.splat_status(stream)
            t0 = time.perf_counter()
            for _ in range(gsteps):
                r.splat_gaussians(g1, gubo, W, H, img, stream=stream)
            torch.cuda.synchronize()
            d1 = (time.perf_counter() - t0) / gsteps
            assert_complete(r, "gs_1m")
            st1 = r.splat_gaussians(g1, gubo, W, H, img, want_stats=True, stream=stream)
            out["gs_1m"] = {"workload": f"3DGS forward only: {args.hybrid_gaussians} C2-distributed Gaussians, {W}x{H}",
                            "value": round(args.hybrid_gaussians / d1 / 1e9, 4), "unit": "Gsplats/s",
                            "ms_per_step": round(d1 * 1e3, 4), "pairs_K": int(st1.num_rendered)}
            # 3DGS initialisation from a point cloud of that size (exact 3-NN scales, ptgs_gaussians_from_points)
            pts = g1["means"]
            rgbp = torch.randint(0, 256, (pts.shape[0], 3), dtype=torch.uint8, device="cuda")
            r.gaussians_from_points(pts, rgbp, stream=stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                r.gaussians_from_points(pts, rgbp, stream=stream)
            torch.cuda.synchronize()
            di = (time.perf_counter() - t0) / 3
            out["gs_init"] = {"workload": f"3DGS init from a {pts.shape[0]}-point cloud (exact 3-NN scales)",
                              "ms": round(di * 1e3, 3), "mpoints_per_s": round(pts.shape[0] / di / 1e6, 1)}
            del g1, pts, rgbp
        # C5's splat on one GPU: 10M C2-distributed Gaussians at 3840x2160 (tiles up to ~28k pairs: the
        # global-scratch radix path); the 8-GPU C5 shards these tile rows across ranks (dist.tile_row_shard)
        if world == 1 and not args.no_gs_10m:
            W5, H5, N5 = 3840, 2160, 10_000_000
            g5 = {k: torch.from_numpy(v).cuda() for k, v in Y.gaussians_c2(N5, seed=5).items()}
            img5 = torch.zeros((H5, W5, 4), dtype=torch.float32, device="cuda")
            g5pose = Camera(aspect=W5 / H5).look_at([0.0, 0.0, 0.0], [0.0, 0.0, -1.0])
            g5ubo = make_ubo(g5pose, cornell_box_scene(), 0)
            # untimed: one frame with stats sizes the pair buffer for this frame's K (160M pairs; without
            # stats an over-capacity frame is skipped and the buffer grows on the next call), then the
            # sort sizes follow the previous frames' tiles
            r.splat_gaussians(g5, g5ubo, W5, H5, img5, want_stats=True, stream=stream)
            for _ in range(3):
                r.splat_gaussians(g5, g5ubo, W5, H5, img5, stream=stream)
            torch.cuda.synchronize()
            r.splat_status(stream)
            n5 = 5
            t0 = time.perf_counter()
            for _ in range(n5):
                r.splat_gaussians(g5, g5ubo, W5, H5, img5, stream=stream)
            torch.cuda.synchronize()
            d5 = (time.perf_counter() - t0) / n5
            assert_complete(r, "gs_10m_4k")
            st5 = r.splat_gaussians(g5, g5ubo, W5, H5, img5, want_stats=True, stream=stream)
            out["gs_10m_4k"] = {"workload": f"C5 splat on one GPU: {N5} C2-distributed Gaussians, {W5}x{H5}",
                                "value": round(N5 / d5 / 1e9, 4), "unit": "Gsplats/s", "ms_per_step": round(d5 * 1e3, 3),
                                "pairs_K": int(st5.num_rendered)}
            if not args.headline_only:
                out["gs_10m_4k"]["bands8"] = band_split_leg(r, Renderer, g5, g5ubo, W5, H5, img5, d5 * 1e3, stream)
            del g5, img5
        if args.no_pt:
            out.update({"value": out["gs"]["value"], "unit": "Gsplats/s", "ms_per_step": out["gs"]["ms_per_step"],
                        "config": {"workload": out["gs"]["workload"]}, "data": "synthetic Gaussians (seeded)"})

    # ------------------------------------------------------------------ hybrid (C4), one GPU
    # C2-distributed Gaussians (seed 3) placed in the C3 camera's frame + the C3 mesh: path trace
    # (hybrid_spp), primary-hit depth, splat over the traced frame (build-defined).
    if not args.no_pt and not args.no_hybrid and world == 1:
        hg = Y.gaussians_in_view(args.hybrid_gaussians, 3, make_ubo(pose, scene, 0, height=H))
        hdg = {k: torch.from_numpy(v).cuda() for k, v in hg.items()}
        haccum = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        hdepth = torch.zeros((H, W), dtype=torch.float32, device="cuda")
        hframe = 0

        def hybrid_step(want_stats=False):
            nonlocal hframe
            hubo = make_ubo(pose, scene, hframe, ambient=(0.3, 0.4, 0.5, 1.0), height=H)
            r.trace_camera(hubo, W, H, haccum, spp=args.hybrid_spp, stream=stream)
            r.trace_depth(hubo, W, H, hdepth, stream=stream)
            r.splat_gaussians(hdg, hubo, W, H, haccum, over=(hdepth, haccum), want_stats=want_stats, stream=stream)
            hframe += args.hybrid_spp

        for k in range(max(args.warmup, 1)):
            hybrid_step(want_stats=k == 0)  # the first sizes the pair buffer
        torch.cuda.synchronize()
        r.splat_status(stream)
        r.stats_reset(stream)
        hsteps = max(args.steps, 3)
        t0 = time.perf_counter()
        for _ in range(hsteps):
            hybrid_step()
        torch.cuda.synchronize()
        hdt = (time.perf_counter() - t0) / hsteps
        assert_complete(r, "hybrid")
        hst = r.stats()
        out["hybrid"] = {
            "workload": f"C4 hybrid: {args.hybrid_gaussians} C2-distributed Gaussians + the C3 mesh, {W}x{H}, "
                        f"{args.hybrid_spp} spp path trace + primary-hit depth + splat-over composite",
            "frames_per_s": round(1.0 / hdt, 3), "ms_per_frame": round(hdt * 1e3, 3),
            "mrays_per_s": round((hst.extension_rays + hst.shadow_rays) / hsteps / hdt / 1e6, 2),
            "gsplats_per_s": round(args.hybrid_gaussians / hdt / 1e9, 4),
        }
        del haccum, hdepth, hdg

    # ------------------------------------------------------------------ C1: Cornell box, 256x256, 1 spp
    # (BASELINE config 1, the reference's CPU-runnable case: here on the GPU, one launch per frame)
    if not args.no_pt and not args.no_c1 and world == 1:
        from pathtracer_gaussiansplatting_amd import cornell_box_scene
        c1 = cornell_box_scene()
        c1.blue_noise = Y.blue_noise(1024)
        r.upload_scene(c1)
        c1pose = Camera(aspect=1.0).toroidal(218.6429, 21.5660, 3.5, 3.0)
        c1acc = torch.zeros((256, 256, 4), dtype=torch.float32, device="cuda")
        c1n = 50
        for k in range(3):
            r.trace_camera(make_ubo(c1pose, c1, k), 256, 256, c1acc, spp=1, stream=stream)
        torch.cuda.synchronize()
        r.stats_reset(stream)
        t0 = time.perf_counter()
        for k in range(c1n):
            r.trace_camera(make_ubo(c1pose, c1, k), 256, 256, c1acc, spp=1, stream=stream)
        torch.cuda.synchronize()
        c1dt = (time.perf_counter() - t0) / c1n
        c1st = r.stats()
        out["c1"] = {"workload": "C1 Cornell box (rt-box of bunny_box.json), 256x256, 1 spp per frame",
                     "ms_per_frame": round(c1dt * 1e3, 4),
                     "mrays_per_s": round((c1st.extension_rays + c1st.shadow_rays) / c1n / c1dt / 1e6, 2),
                     "note": "launch-bound: 65k pixels per frame"}
        del c1acc

    # ------------------------------------------------------------------ torus data collection
    # rt_datacollect: 1M RaySamples (the reference's RANDOM generator, Morton-sorted) shot from the
    # torus around the C1 Cornell box, 16 accumulation frames into the HitData running mean
    if not args.no_pt and not args.no_torus and world == 1:
        from pathtracer_gaussiansplatting_amd import HITDATA_DTYPE, cornell_box_scene, torus_push
        tsc = cornell_box_scene()
        tsc.blue_noise = Y.blue_noise(1024)
        r.upload_scene(tsc)
        tn = 1 << 20
        tsamp = torch.from_numpy(np.ascontiguousarray(Y.torus_samples(tn)).view(np.float32)).cuda()
        thits = torch.zeros(tn * (HITDATA_DTYPE.itemsize // 4), dtype=torch.float32, device="cuda")
        tpush = torus_push(major_radius=3.5, minor_radius=1.0, height=3.0)
        tpose = Camera(aspect=1.0).toroidal(218.6429, 21.5660, 3.5, 3.0)
        tframes = 16
        for k in range(2):
            r.trace_torus(make_ubo(tpose, tsc, k), tpush, tsamp, tn, thits, stream=stream)
        torch.cuda.synchronize()
        r.stats_reset(stream)
        t0 = time.perf_counter()
        for k in range(tframes):
            r.trace_torus(make_ubo(tpose, tsc, k), tpush, tsamp, tn, thits, stream=stream)
        torch.cuda.synchronize()
        tdt = time.perf_counter() - t0
        tst = r.stats()
        out["torus"] = {"workload": f"torus data collection: {tn} RaySamples (RANDOM, Morton-sorted) x {tframes} "
                                    "accumulation frames, C1 Cornell box", "ms_per_frame": round(tdt / tframes * 1e3, 4),
                        "mrays_per_s": round((tst.extension_rays + tst.shadow_rays) / tdt / 1e6, 1),
                        "msamples_per_s": round(tn * tframes / tdt / 1e6, 1)}
        del tsamp, thits

    # ------------------------------------------------------------------ capture / export
    # Engine::captureSceneData: views on the toroidal pose sequence, each accumulated on the GPU, sRGB8,
    # every-2nd-pixel downscale, JPEG q90, transforms_{train,test}.json, then the torus point cloud
    # (1M RaySamples) -> points3d.ply; 8 of the reference's 336 positions, 128 of its 512 steps
    if not args.no_pt and not args.no_capture and world == 1:
        import shutil
        import tempfile
        from pathtracer_gaussiansplatting_amd import HITDATA_DTYPE, capture, cornell_box_scene, torus_push
        csc = cornell_box_scene()
        csc.blue_noise = Y.blue_noise(1024)
        r.upload_scene(csc)
        cubo_c = make_ubo(Camera(aspect=W / H).toroidal(218.6429, 21.5660, 3.5, 3.0), csc, 0, height=H)
        cn = 1 << 20
        csamp = torch.from_numpy(np.ascontiguousarray(Y.torus_samples(cn)).view(np.float32)).cuda()
        cviews, csteps = 8, 128
        cdir = tempfile.mkdtemp(prefix="ptgs_capture_")
        try:
            r.stats_reset(stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            capture.capture_dataset(r, cubo_c, cdir, W, H, samples=csamp, num_samples=cn,
                                    torus_push=torus_push(major_radius=3.5, minor_radius=1.0, height=3.0),
                                    total_positions=cviews, accumulation_steps=csteps, stream=stream)
            torch.cuda.synchronize()
            cdt = time.perf_counter() - t0
            cst = r.stats()
            out["capture"] = {"workload": f"dataset capture: C1 Cornell box, {cviews} views at {W}x{H} x {csteps} "
                                          f"accumulation steps (JPEG q90 at half size, transforms json) + "
                                          f"{cn}-sample torus point cloud x {csteps} steps -> PLY",
                              "s_total": round(cdt, 3), "views_per_s": round(cviews / cdt, 2),
                              "mrays_per_s": round((cst.extension_rays + cst.shadow_rays) / cdt / 1e6, 1)}
        finally:
            shutil.rmtree(cdir, ignore_errors=True)
        del csamp

    # ------------------------------------------------------------------ C5: the 8-GPU config
    # 1M-tri atrium + 10M C2-distributed Gaussians in its camera frame, 3840x2160, 256 spp in total.
    # Rank g traces samples g, g+N, ... (256/N each, SUM), a reduce-scatter of the radiance by the
    # ranks' tile rows (each receives the sums under its own splat rows), mean + primary-hit depth,
    # splat-over of its tile rows, row gather to rank 0 (dist.render_hybrid_frame; SURVEY 8e: strong
    # scaling).
    if not args.no_c5 and not args.no_pt:
        from pathtracer_gaussiansplatting_amd import ACCUM_SUM as _SUM
        from pathtracer_gaussiansplatting_amd import dist as D
        W5, H5, T5, G5, SPP5 = 3840, 2160, 1_000_000, 10_000_000, 256
        if SPP5 % world:
            raise SystemExit("--c5 needs a world size dividing 256")
        sc5 = Y.atrium_scene(target_tris=T5, seed=2)
        sc5.blue_noise = Y.blue_noise(1024)
        info5 = r.upload_scene(sc5)
        pose5 = Camera(aspect=W5 / H5).look_at([-15.0, 4.0, 5.0], [10.0, 3.0, -3.0])
        g5 = Y.gaussians_in_view(G5, 5, make_ubo(pose5, sc5, 0, height=H5))
        dg5 = {k: torch.from_numpy(v).cuda() for k, v in g5.items()}
        del g5
        acc5 = torch.zeros((H5, W5, 4), dtype=torch.float32, device="cuda")
        dep5 = torch.zeros((H5, W5), dtype=torch.float32, device="cuda")
        comp5 = torch.zeros((H5, W5, 4), dtype=torch.float32, device="cuda")
        rows5 = D.tile_row_shard(rank, world, H5)
        rows5_all = [D.tile_row_shard(k, world, H5) for k in range(world)]

        def c5_frame(want_stats=False):
            if world == 1 or native_comm:
                # dist.render_hybrid_frame: sample shard, reduce-scatter of the radiance by tile rows (each
                # rank receives only its rows' sums), mean + depth, splat-over of its rows, row gather
                u5 = make_ubo(pose5, sc5, 0, ambient=(0.3, 0.4, 0.5, 1.0), height=H5)
                D.render_hybrid_frame(r, dg5, u5, W5, H5, acc5, dep5, comp5, SPP5, rank, world, tile_rows=rows5_all,
                                      stream=stream, want_stats=want_stats)
                return
            # gloo rehearsal (ranks sharing one GPU: no CUDA reduce / send in gloo): full-frame all-reduces
            u5 = make_ubo(pose5, sc5, rank, ambient=(0.3, 0.4, 0.5, 1.0), height=H5)
            acc5.zero_()
            r.trace_camera(u5, W5, H5, acc5, spp=SPP5 // world, frame_stride=world, mode=_SUM, stream=stream)
            D.all_reduce_sum(acc5)
            mean5 = D.resolve_mean(acc5)
            r.trace_depth(u5, W5, H5, dep5, stream=stream)
            comp5.zero_()
            if rows5[1] > rows5[0]:
                r.splat_gaussians(dg5, u5, W5, H5, comp5, tile_rows=rows5, over=(dep5, mean5), want_stats=want_stats,
                                  stream=stream)
            reduce_to_root(comp5)

        c5_frame(want_stats=True)  # warm-up: sizes the pair buffer (sort sizes follow the previous frame's tiles)
        torch.cuda.synchronize()
        r.splat_status(stream)
        r.stats_reset(stream)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c5_frame()
        torch.cuda.synchronize()
        barrier()
        d5 = max_over_ranks(time.perf_counter() - t0)
        assert_complete(r, "c5")
        s5 = r.stats()
        rays5 = sum_over_ranks(float(s5.extension_rays + s5.shadow_rays))
        out["c5"] = {"workload": f"C5: {G5} Gaussians + {int(info5.num_triangles)}-tri mesh, {W5}x{H5}, {SPP5} spp "
                                 f"in total ({SPP5 // world} per GPU), sample shard + tile-row shard x{world}",
                     "ms_per_frame": round(d5 * 1e3, 2), "mrays_per_s": round(rays5 / d5 / 1e6, 1),
                     "gsplats_per_s": round(G5 / d5 / 1e9, 4), "scaling": "strong",
                     "collectives": ("reduce-scatter of the radiance by tile rows + row gather (RCCL, "
                                     "dist.render_hybrid_frame)") if (world == 1 or native_comm) else
                                    "gloo rehearsal: full-frame all-reduces",
                     "bvh_nodes": int(info5.num_bvh_nodes), "bvh_depth": int(info5.bvh_depth)}
        del dg5, acc5, dep5, comp5

    # ------------------------------------------------------------------ CPU baseline (rank 0, N=1)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.no_pt:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        oracle.build()
        threads = min(16, os.cpu_count() or 1)
        row_stride, spp_cpu = 1, 64  # the whole C3 frame (every row, 64 spp): ~20 s of CPU work on the box
        acc = np.zeros((H, W, 4), np.float32)
        desc = scene.desc()
        cubo = make_ubo(pose, scene, 0, ambient=(0.3, 0.4, 0.5, 1.0), height=H)
        t0 = time.perf_counter()
        cst = oracle.trace_camera(desc, cubo, W, H, acc, spp=spp_cpu, row_stride=row_stride, threads=threads)
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {
            "value": round((cst.extension_rays + cst.shadow_rays) / cdt / 1e6, 4), "unit": "Mrays/s",
            "cores": threads, "kind": "port",
            "sample": f"C3 scene at {W}x{H}, every {row_stride}th row, {spp_cpu} spp "
                      f"({cst.samples} samples, {cst.extension_rays + cst.shadow_rays} rays, {cdt:.1f} s, "
                      f"incl. oracle BVH build)",
        }
        if "c1" in out:
            # C1 (timed in full on the CPU): the Cornell frames of the GPU leg
            from pathtracer_gaussiansplatting_amd import cornell_box_scene
            c1 = cornell_box_scene()
            c1.blue_noise = Y.blue_noise(1024)
            c1pose = Camera(aspect=1.0).toroidal(218.6429, 21.5660, 3.5, 3.0)
            c1acc = np.zeros((256, 256, 4), np.float32)
            c1desc = c1.desc()
            nfr, rays, t0 = 0, 0, time.perf_counter()
            while nfr == 0 or time.perf_counter() - t0 < 2.0:
                c1st = oracle.trace_camera(c1desc, make_ubo(c1pose, c1, nfr), 256, 256, c1acc, spp=1, threads=threads)
                rays += c1st.extension_rays + c1st.shadow_rays
                nfr += 1
            c1dt = time.perf_counter() - t0
            out["cpu_baseline"]["c1"] = {"value": round(rays / c1dt / 1e6, 4), "unit": "Mrays/s", "cores": threads,
                                         "kind": "port", "sample": f"{nfr} full C1 frames (256x256, 1 spp), "
                                                                   f"{c1dt / nfr * 1e3:.2f} ms each"}
        if not args.no_gs:
            # the oracle's 3DGS forward is OpenMP-threaded (preprocess, duplicate-with-keys, blend; the
            # pair sort is serial): OMP_NUM_THREADS threads, whole C2 frames for >= 3 s
            omp = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
            nfr, t0 = 0, time.perf_counter()
            while nfr == 0 or time.perf_counter() - t0 < 3.0:
                oracle.splat_gaussians(g, gubo, W, H)
                nfr += 1
            gcdt = (time.perf_counter() - t0) / nfr
            out["cpu_baseline"]["gs"] = {"value": round(args.gaussians / gcdt / 1e9, 6), "unit": "Gsplats/s",
                                         "cores": omp, "kind": "port",
                                         "sample": f"{nfr} full C2 frames, {gcdt * 1e3:.1f} ms each"}

    if rank == 0:
        print(json.dumps(out), flush=True)
    r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
