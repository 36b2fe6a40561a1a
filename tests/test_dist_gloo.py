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
