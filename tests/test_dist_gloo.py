"""Multi-process sharding logic on CPU: world_size 2 (and 3) with the gloo backend.

Each rank computes its shard with the CPU oracle (standing in for its GPU), the shards are combined
with the same torch.distributed reduce the GPU path uses (RCCL there), and rank 0 checks the result
against a single-process render.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        import scenes_util as U
        from pathtracer_gaussiansplatting_amd import ACCUM_SUM, Camera, make_ubo
        from pathtracer_gaussiansplatting_amd import dist as D
        from pathtracer_gaussiansplatting_amd import synthetic as Y

        # --- path tracer: sample shard + SUM reduce
        sc = U.cornell()
        W, H, spp = 24, 20, 2
        f, stride = D.sample_shard(rank, world, frame0=0)
        ubo = make_ubo(U.cornell_pose(W / H), sc, f)
        acc = np.zeros((H, W, 4), np.float32)
        oracle.trace_camera(sc.desc(), ubo, W, H, acc, spp=spp, frame_stride=stride, mode=ACCUM_SUM)
        t = torch.from_numpy(acc)
        D.reduce_sum(t, dst=0)
        # --- 3DGS: tile-row shard
        g = Y.gaussians_c2(1500, seed=5)
        gu = make_ubo(Camera(aspect=96 / 70).look_at([0, 0, 0], [0, 0, -1]), sc, 0)
        rows = D.tile_row_shard(rank, world, 70)
        part = oracle.splat_gaussians(g, gu, 96, 70, tile_rows=rows)["image"]
        gt = torch.from_numpy(part)
        D.reduce_sum(gt, dst=0)
        if rank == 0:
            ref = np.zeros((H, W, 4), np.float32)
            oracle.trace_camera(sc.desc(), make_ubo(U.cornell_pose(W / H), sc, 0), W, H, ref, spp=spp * world)
            mean = D.resolve_mean(t).numpy()
            err = U.rel_l2(mean[..., :3], ref[..., :3])
            full = oracle.splat_gaussians(g, gu, 96, 70)["image"]
            q.put(("ok", err, float(t[..., 3].min()), float(t[..., 3].max()), bool(np.array_equal(gt.numpy(), full))))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_frames_gloo(world, oracle_lib, native_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
    assert res[0] == "ok", res[1]
    _, err, cmin, cmax, gs_equal = res
    assert err < 1e-5, err
    assert cmin == cmax == 2 * world
    assert gs_equal


def test_shard_helpers():
    from pathtracer_gaussiansplatting_amd import dist as D
    assert D.sample_shard(2, 8, 100) == (102, 8)
    rows = [D.tile_row_shard(r, 8, 1080) for r in range(8)]
    assert rows[0][0] == 0 and rows[-1][1] == 68
    assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))
    assert max(e - b for b, e in rows) - min(e - b for b, e in rows) <= 1
    assert D.tile_row_shard(9, 10, 64) == (4, 4)  # more ranks than rows: empty shard
    with pytest.raises(ValueError):
        D.sample_shard(3, 3)


class _OracleRenderer:
    """Test stand-in for one rank's GPU renderer (the trace_camera / splat_gaussians interface of
    pathtracer_gaussiansplatting_amd.Renderer), backed by the CPU oracle: the product's sharding
    helpers (dist.render_path_traced_frame / render_gaussian_frame) run unchanged on top of it."""

    def __init__(self, scene):
        import oracle
        self.oracle = oracle
        self.scene = scene
        self.comm_world = 0  # no native communicator: the torch.distributed (gloo) collectives

    def trace_camera(self, ubo, width, height, accum, spp=1, frame_stride=1, mode=0, rows=None, stream=None):
        acc = accum.numpy()
        self.oracle.trace_camera(self.scene.desc(), ubo, width, height, acc, spp=spp, frame_stride=frame_stride,
                                 mode=mode, rows=rows)

    def trace_depth(self, ubo, width, height, depth, stream=None, rows=None):
        d = torch.from_numpy(self.oracle.trace_depth(self.scene.desc(), ubo, width, height))
        r0, r1 = (0, height) if rows is None else rows
        depth[r0:r1] = d[r0:r1]  # (rows outside are left untouched, as ptgs_trace_depth_rows)

    def splat_gaussians(self, g, ubo, width, height, out, bg=(0.0, 0.0, 0.0), tile_rows=None, stream=None,
                        want_stats=False, over=None):
        ov = None if over is None else (over[0].numpy().copy(), over[1].numpy().copy())
        ref = self.oracle.splat_gaussians({k: v.numpy() for k, v in g.items()}, ubo, width, height, bg=bg,
                                          tile_rows=tile_rows, over=ov)
        r0, r1 = (0, height) if tile_rows is None else (min(tile_rows[0] * 16, height), min(tile_rows[1] * 16, height))
        out[r0:r1] = torch.from_numpy(ref["image"][r0:r1])
        return ref


def _frame_worker(rank, world, port, q):
    """dist.render_path_traced_frame + dist.render_gaussian_frame (balanced tile rows, row gather)."""
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        import scenes_util as U
        from pathtracer_gaussiansplatting_amd import Camera, make_ubo
        from pathtracer_gaussiansplatting_amd import dist as D
        from pathtracer_gaussiansplatting_amd import synthetic as Y

        sc = U.cornell()
        r = _OracleRenderer(sc)
        W, H, spp = 24, 20, 2
        acc = torch.zeros((H, W, 4), dtype=torch.float32)
        D.render_path_traced_frame(r, make_ubo(U.cornell_pose(W / H), sc, 0), W, H, acc, spp, rank, world)
        # 3DGS: rows balanced by the pair counts of a full-frame pass (every rank computes the same split)
        GW, GH = 96, 70
        g = {k: torch.from_numpy(v) for k, v in Y.gaussians_c2(1500, seed=5).items()}
        gu = make_ubo(Camera(aspect=GW / GH).look_at([0, 0, 0], [0, 0, -1]), sc, 0)
        full = oracle.splat_gaussians({k: v.numpy() for k, v in g.items()}, gu, GW, GH)
        tiles_x = (GW + 15) // 16
        rows = D.balanced_tile_rows(D.row_pairs_from_ranges(full["ranges"], tiles_x), world, tiles_x)
        out = torch.full((GH, GW, 4), -1.0, dtype=torch.float32)  # rows not rendered here stay -1 unless gathered
        D.render_gaussian_frame(r, g, gu, GW, GH, out, rank, world, tile_rows=rows)
        if rank == 0:
            ref = np.zeros((H, W, 4), np.float32)
            oracle.trace_camera(sc.desc(), make_ubo(U.cornell_pose(W / H), sc, 0), W, H, ref, spp=spp * world)
            err = U.rel_l2(D.resolve_mean(acc).numpy()[..., :3], ref[..., :3])
            q.put(("ok", err, float(acc[..., 3].min()), float(acc[..., 3].max()),
                   bool(np.array_equal(out.numpy(), full["image"])), rows))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc()))


def test_dist_render_frames_gloo():
    """world 2: the product's frame helpers (sample shard + reduce; balanced tile rows + row gather)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_frame_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
    assert res[0] == "ok", res[1]
    _, err, cmin, cmax, gs_equal, rows = res
    assert err < 1e-5, err
    assert cmin == cmax == 2 * world
    assert gs_equal, rows
    assert rows[0][0] == 0 and rows[-1][1] == 5 and rows[0][1] == rows[1][0]


def test_balanced_tile_rows():
    from pathtracer_gaussiansplatting_amd import dist as D
    rows = D.balanced_tile_rows([0, 0, 100, 500, 500, 100, 0, 0], 3, 10)
    assert rows == [(0, 3), (3, 5), (5, 8)]
    even = D.balanced_tile_rows([5] * 68, 8, 120)
    assert [e - b for b, e in even] == [9, 8, 9, 8, 9, 8, 9, 8]
    assert D.balanced_tile_rows([1, 2], 4, 1) == [(0, 1), (1, 1), (1, 2), (2, 2)]
    assert list(D.row_pairs_from_ranges(np.array([[0, 3], [3, 3], [3, 10], [10, 12]], np.uint32), 2)) == [3, 9]


def _hybrid_worker(rank, world, port, q):
    """dist.render_hybrid_frame (C5's split): sample shard, reduce-scatter by tile rows, mean + depth,
    splat-over of the rank's rows, row gather; rank 0 compares with the single-process hybrid frame."""
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        import scenes_util as U
        from pathtracer_gaussiansplatting_amd import ACCUM_SUM, make_ubo
        from pathtracer_gaussiansplatting_amd import dist as D
        from pathtracer_gaussiansplatting_amd import synthetic as Y

        sc = U.cornell()
        W, H, spp = 40, 36, 2 * world
        ubo = make_ubo(U.cornell_pose(W / H), sc, 0, ambient=(0.3, 0.4, 0.5, 1.0))
        g = {k: torch.from_numpy(v) for k, v in Y.gaussians_in_view(600, 3, ubo).items()}
        r = _OracleRenderer(sc)
        acc = torch.zeros((H, W, 4), dtype=torch.float32)
        dep = torch.zeros((H, W), dtype=torch.float32)
        out = torch.full((H, W, 4), -1.0, dtype=torch.float32)
        rows = [D.tile_row_shard(k, world, H) for k in range(world)]
        D.render_hybrid_frame(r, g, ubo, W, H, acc, dep, out, spp, rank, world, tile_rows=rows)
        if rank == 0:
            ref_acc = np.zeros((H, W, 4), np.float32)
            u0 = make_ubo(U.cornell_pose(W / H), sc, 0, ambient=(0.3, 0.4, 0.5, 1.0))
            oracle.trace_camera(sc.desc(), u0, W, H, ref_acc, spp=spp, mode=ACCUM_SUM)
            mean = D.resolve_mean(torch.from_numpy(ref_acc)).numpy()
            depth = oracle.trace_depth(sc.desc(), u0, W, H)
            ref = oracle.splat_gaussians({k: v.numpy() for k, v in g.items()}, u0, W, H, over=(depth, mean))
            hits = int(np.count_nonzero(ref["image"] != mean))
            q.put(("ok", U.rel_l2(out.numpy(), ref["image"]), hits, bool((out.numpy() != -1.0).all())))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_dist_render_hybrid_frame_gloo(world, oracle_lib, native_lib):
    """the C5 split moves only what each rank's rows need (reduce-scatter of the
    radiance by tile rows, then the row gather) and composes the single-process hybrid frame."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hybrid_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
    assert res[0] == "ok", res[1]
    _, err, hits, covered = res
    assert covered, "every row of rank 0's frame is rendered or gathered"
    assert hits > 50, hits  # the Gaussians change the frame
    assert err < 1e-5, err



class _ReportingRenderer(_OracleRenderer):
    """A rank whose splat call renders its rows and then reports an EARLIER incomplete frame, as
    ptgs_splat_gaussians does with PTGS_EINCOMPLETE (ptgs.h): the frame is rendered, the code is news."""

    def splat_gaussians(self, *a, **kw):
        from pathtracer_gaussiansplatting_amd._abi import PTGS_EINCOMPLETE, PtgsError
        super().splat_gaussians(*a, **kw)
        raise PtgsError("ptgs_splat_gaussians failed: PTGS_EINCOMPLETE an earlier splat frame left tiles "
                        "incomplete (spill pool exhausted; grown)", PTGS_EINCOMPLETE)


def _report_worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        import scenes_util as U
        from pathtracer_gaussiansplatting_amd import Camera, make_ubo
        from pathtracer_gaussiansplatting_amd import dist as D
        from pathtracer_gaussiansplatting_amd import synthetic as Y
        from pathtracer_gaussiansplatting_amd._abi import PTGS_EINCOMPLETE, PtgsError
        sc = U.cornell()
        r = _ReportingRenderer(sc) if rank == 1 else _OracleRenderer(sc)
        GW, GH = 64, 48
        g = {k: torch.from_numpy(v) for k, v in Y.gaussians_c2(800, seed=9).items()}
        gu = make_ubo(Camera(aspect=GW / GH).look_at([0, 0, 0], [0, 0, -1]), sc, 0)
        out = torch.full((GH, GW, 4), -1.0, dtype=torch.float32)
        code = 0
        try:
            D.render_gaussian_frame(r, g, gu, GW, GH, out, rank, world)
        except PtgsError as e:
            code = e.code
        if rank == 0:
            full = oracle.splat_gaussians({k: v.numpy() for k, v in g.items()}, gu, GW, GH)
            q.put(("ok", code, bool(np.array_equal(out.numpy(), full["image"]))))
        else:
            q.put(("rank1", code == PTGS_EINCOMPLETE))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc()))


def test_dist_splat_report_does_not_hang_gloo():
    """a rank whose splat call reports an earlier incomplete frame (PTGS_EINCOMPLETE) still
    joins the row gather (the report is raised after it), so rank 0 gets the whole frame and nothing hangs."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_report_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict()
    for _ in range(world):
        m = q.get(timeout=180)
        assert m[0] != "err", m[1]
        res[m[0]] = m[1:]
    for p in procs:
        p.join(timeout=60)
    assert res["ok"] == (0, True), res
    assert res["rank1"] == (True,), res


def _pipeline_worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import oracle
        import scenes_util as U
        from pathtracer_gaussiansplatting_amd import Camera, make_ubo
        from pathtracer_gaussiansplatting_amd import dist as D
        from pathtracer_gaussiansplatting_amd import synthetic as Y
        sc = U.cornell()
        r = _OracleRenderer(sc)
        GW, GH = 80, 60
        g = {k: torch.from_numpy(v) for k, v in Y.gaussians_c2(1200, seed=13).items()}
        ubos = [make_ubo(Camera(aspect=GW / GH).look_at([0.3 * f, 0.1 * f, 0.0], [0.2 * f, 0.0, -1.0]), sc, 0)
                for f in range(4)]
        full0 = oracle.splat_gaussians({k: v.numpy() for k, v in g.items()}, ubos[0], GW, GH)
        tiles_x = (GW + 15) // 16
        rows = D.balanced_tile_rows(D.row_pairs_from_ranges(full0["ranges"], tiles_x), world, tiles_x)
        pipe = D.RowGatherPipeline(r, GW, GH, rows, rank, world, device="cpu", bg=(0.1, 0.2, 0.3))
        got = []
        for u in ubos:
            img = pipe.submit(g, u)
            pipe.wait(img)
            got.append(img.clone())
        if rank == 0:
            same = []
            for u, im in zip(ubos, got):
                ref = oracle.splat_gaussians({k: v.numpy() for k, v in g.items()}, u, GW, GH, bg=(0.1, 0.2, 0.3))
                same.append(bool(np.array_equal(im.numpy(), ref["image"])))
            q.put(("ok", same, rows))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc()))


def test_row_gather_pipeline_gloo():
    """VERDICT r4 next #3c: the pipelined tile-row frames (dist.RowGatherPipeline: frame f's row gather
    overlapped with frame f + 1's band, two alternating images) compose, on rank 0, the single-process
    frames of a moving camera bit for bit (world 2, gloo, the oracle as each rank's renderer)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
    assert res[0] == "ok", res[1]
    assert res[1] == [True] * 4, res


def test_splat_policy():
    """DESIGN §6, VERDICT r5 next #3: how several GPUs split 3DGS frames. C2 (100k Gaussians, 1080p, one
    frame ~0.053 ms on one GPU): a rank's band (~7 us at 8 ranks) is far shorter than rank 0's intake of a
    peer's rows over one xGMI link (1920*1080*16/8 B at 50 GB/s ~ 83 us) -> replicas; C5's splat (10M
    Gaussians, 3840x2160, ~8.5 ms) -> tile rows from 2 ranks on; one GPU -> single."""
    from pathtracer_gaussiansplatting_amd import dist as D
    assert D.splat_policy(0.053, 1920, 1080, 1) == "single"
    for world in (2, 4, 8):
        assert D.splat_policy(0.053, 1920, 1080, world) == "replicas"
        assert D.splat_policy(8.5, 3840, 2160, world) == "tile_rows"
    # the crossover: a band of frame_ms / world against W*H*16/world B at 50 GB/s
    gather_ms = 1920 * 1080 * 16 / 50e9 * 1e3  # (x world / world)
    assert D.splat_policy(gather_ms * 1.01, 1920, 1080, 8) == "tile_rows"
    assert D.splat_policy(gather_ms * 0.99, 1920, 1080, 8) == "replicas"


def _replica_worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import math
        import oracle
        import scenes_util as U
        from pathtracer_gaussiansplatting_amd import Camera, make_ubo
        from pathtracer_gaussiansplatting_amd import dist as D
        from pathtracer_gaussiansplatting_amd import synthetic as Y
        g = Y.gaussians_c2(1500, seed=5)
        W, H = 96, 70
        # the policy from the slowest rank's frame time (bench.py: max over ranks), the same on every rank
        t = torch.tensor([0.053 if rank == 0 else 0.051], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        policy = D.splat_policy(float(t.item()), 1920, 1080, world)
        # replicas: rank r renders whole frames of its own view (bench.py's C2 leg at world > 1)
        th = 2.0 * math.pi * rank / world
        ubo = make_ubo(Camera(aspect=W / H).look_at([8.0 * math.sin(th), 0.0, -8.0 + 8.0 * math.cos(th)],
                                                    [0.0, 0.0, -8.0]), U.cornell(), 0)
        img = torch.from_numpy(oracle.splat_gaussians(g, ubo, W, H)["image"])
        frames = torch.tensor([1.0])
        dist.all_reduce(frames)  # (the whole job's frames: one per rank per step)
        outs = [torch.zeros_like(img) for _ in range(world)] if rank == 0 else None
        dist.gather(img, outs, dst=0)  # (test only: each rank's frame checked on rank 0)
        if rank == 0:
            ok = []
            for rr in range(world):
                th2 = 2.0 * math.pi * rr / world
                u2 = make_ubo(Camera(aspect=W / H).look_at([8.0 * math.sin(th2), 0.0, -8.0 + 8.0 * math.cos(th2)],
                                                           [0.0, 0.0, -8.0]), U.cornell(), 0)
                ok.append(bool(np.array_equal(outs[rr].numpy(), oracle.splat_gaussians(g, u2, W, H)["image"])))
            distinct = not np.array_equal(outs[0].numpy(), outs[1].numpy())
            q.put(("ok", policy, float(frames.item()), ok, distinct))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc()))


def test_splat_replicas_gloo(oracle_lib, native_lib):
    """The C2 policy at small N (world 2, gloo, the oracle as each rank's renderer): every rank picks
    "replicas" from the same (max-over-ranks) frame time and renders whole frames of its own view; the views
    differ, each frame equals the single-process render of that view, and the job renders world frames per
    step with no image crossing between ranks in the timed path."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replica_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == "ok", res[1]
    _, policy, frames, ok, distinct = res
    assert policy == "replicas" and frames == world and all(ok) and distinct, res


def test_rebalance_tile_rows():
    """dist.rebalance_tile_rows: bands whose measured time exceeds the others' give rows away; a split whose
    band times are equal is kept; the result covers every row once, in order."""
    import numpy as np
    from pathtracer_gaussiansplatting_amd import dist as D
    row_pairs = np.full(40, 1000.0)
    split = D.balanced_tile_rows(row_pairs, 4, 10)
    assert split == [(0, 10), (10, 20), (20, 30), (30, 40)]
    assert D.rebalance_tile_rows(split, [1.0, 1.0, 1.0, 1.0], row_pairs, 10) == split
    # band 0 measured twice as slow: it shrinks, the others grow
    new = D.rebalance_tile_rows(split, [2.0, 1.0, 1.0, 1.0], row_pairs, 10)
    assert new[0][0] == 0 and new[-1][1] == 40 and all(a[1] == b[0] for a, b in zip(new, new[1:]))
    assert new[0][1] - new[0][0] < 10 and new[-1][1] - new[-1][0] > 10, new
    # the re-split's predicted band costs are about equal (rows of band 0 cost 0.2, the rest 0.1)
    cost = np.where(np.arange(40) < 10, 0.2, 0.1)
    per = [cost[a:b].sum() for a, b in new]
    assert max(per) - min(per) <= 0.2 + 1e-9, per


def test_refine_split_lowers_the_costliest_band():
    """dist._refine_split (the feedback re-split's last step): the result still covers every row once, in
    order, with the same number of bands, and its costliest band is never above the equal-share cut's; on
    a split that left a band one heavy row above its neighbour it moves that row over."""
    from pathtracer_gaussiansplatting_amd import dist as D
    rng = np.random.default_rng(3)
    for _ in range(200):
        n, world = int(rng.integers(4, 40)), int(rng.integers(2, 6))
        cost = rng.uniform(0.05, 1.0, n) ** 3
        base = D._split_rows(cost, world)
        ref = D._refine_split(base, cost)
        assert len(ref) == world and ref[0][0] == 0 and ref[-1][1] == n
        assert all(a[1] == b[0] and a[0] <= a[1] for a, b in zip(ref, ref[1:]))
        band_max = lambda sp: max(cost[a:b].sum() for a, b in sp)
        assert band_max(ref) <= band_max(base) + 1e-12
    cost = np.array([1.0, 1.0, 1.0, 1.0, 3.0, 3.0, 1.0, 1.0])
    split = [(0, 5), (5, 8)]  # 7 vs 5: moving the heavy row over would give 4 vs 8, so it stays
    assert D._refine_split(split, cost) == [(0, 5), (5, 8)]
    split = [(0, 6), (6, 8)]  # 10 vs 2: the heavy row moves -> 7 vs 5
    assert D._refine_split(split, cost) == [(0, 5), (5, 8)]
