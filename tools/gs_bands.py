#!/usr/bin/env python3
"""Tile-row bands of the 3DGS forward (the 8-GPU split of bench.py's gs leg): frame time of band k of
GS_BANDS (default 8) equal tile-row bands, with and without ptgs_gaussians.chunk_bounds (per-rank chunk
culling before the preprocess), against the full frame. One configuration per process so that a
kernel trace (rocprofv3 --kernel-trace) separates the front end's kernels per configuration:
   GS_CFG=c2|10m GS_BAND=full|<k>|balanced GS_BOUNDS=0|1 [GS_LIB=libptgs_<variant>.so] tools/gs_bands.py
(balanced: every band of the pair-balanced split, see balanced())
Prints ms per frame (stream-ordered, steady state) and the frame's pairs."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {"c2": (100_000, 1920, 1080, 200), "10m": (10_000_000, 3840, 2160, 10)}


def main():
    import torch
    from pathtracer_gaussiansplatting_amd import Camera, Renderer, cornell_box_scene, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    cfg = os.environ.get("GS_CFG", "c2")
    band = os.environ.get("GS_BAND", "full")
    bounds = os.environ.get("GS_BOUNDS", "1") == "1"
    nb = int(os.environ.get("GS_BANDS", "8"))
    n, W, H, iters = CONFIGS[cfg]
    lib = os.environ.get("GS_LIB", "libptgs.so")
    r = Renderer(0, lib_path=lib if os.path.isabs(lib) else os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", lib))
    g = {k: torch.from_numpy(v).cuda() for k, v in Y.gaussians_c2(n, seed=1).items()}
    dg = r.sort_gaussians_spatial(g)
    del g
    if bounds:
        dg = dict(dg, chunk_bounds=r.gaussians_chunk_bounds(dg))
    ubo = make_ubo(Camera(aspect=W / H).look_at([0, 0, 0], [0, 0, -1]), cornell_box_scene(), 0)
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    gy = (H + 15) // 16
    if band.startswith("balanced"):  # the pair-balanced split (dist.balanced_tile_rows): every band, or band k
        balanced(r, dg, ubo, W, H, nb, iters, img, int(band.split(":")[1]) if ":" in band else None)
        r.close()
        return
    rows = None if band == "full" else (gy * int(band) // nb, gy * (int(band) + 1) // nb)
    for _ in range(3):
        r.splat_gaussians(dg, ubo, W, H, img, tile_rows=rows)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        r.splat_gaussians(dg, ubo, W, H, img, tile_rows=rows)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / iters
    st = r.splat_status()
    print(f"{os.path.basename(lib)} {cfg} band {band}/{nb} rows {rows} bounds {int(bounds)}: {dt * 1e3:.4f} ms/frame, pairs {st.last_pairs}, "
          f"fused {st.fused}", flush=True)
    r.close()


def balanced(r, dg, ubo, W, H, nb, iters, img, only=None):
    """The rank split bench.py's multi-GPU gs leg uses: tile rows balanced by a full frame's per-row pair
    counts (3-sigma pairs of a frame with stats; dist.balanced_tile_rows), each band on a context of its own
    (a rank renders its band every frame: its own hints), timed one after the other on this GPU. Prints
    every band's ms per frame and pairs, the slowest band and the full frame."""
    import numpy as np
    import torch
    from pathtracer_gaussiansplatting_amd import Renderer
    from pathtracer_gaussiansplatting_amd import dist as D
    st = r.splat_gaussians(dg, ubo, W, H, img, want_stats=True)
    b = r.splat_buffers()
    rng = np.zeros(2 * b.num_tiles, np.uint32)
    r.copy_d2h(rng, b.tile_ranges, rng.nbytes)
    split = D.balanced_tile_rows(D.row_pairs_from_ranges(rng, st.tiles_x), nb, st.tiles_x)

    def timed(rr, rows):
        rr.splat_reserve(int(st.num_rendered))  # (a rank renders its band for many frames: its buffers sized)
        for _ in range(8):
            rr.splat_gaussians(dg, ubo, W, H, img, tile_rows=rows)
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(iters):
            rr.splat_gaussians(dg, ubo, W, H, img, tile_rows=rows)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / iters * 1e3, int(rr.splat_status().last_pairs)

    if only is not None:  # (one band per process: kernel traces per band)
        ms, kp = timed(r, tuple(split[only]))
        print(f"band {only}/{nb} rows {tuple(split[only])}: {ms:.4f} ms/frame, pairs {kp}", flush=True)
        return
    full_ms, full_k = timed(r, None)
    res = []
    for k, rows in enumerate(split):
        rk = Renderer(0)
        ms, kp = timed(rk, tuple(rows))
        res.append((ms, kp))
        print(f"band {k}/{nb} rows {tuple(rows)}: {ms:.4f} ms/frame, pairs {kp}", flush=True)
        rk.close()
    worst = max(m for m, _ in res)
    print(f"balanced split {split}: slowest band {worst:.4f} ms ({full_ms / worst:.2f}x of the full frame "
          f"{full_ms:.4f} ms, pairs {full_k}); band pairs {[k for _, k in res]}", flush=True)
    # feedback: re-split from the measured band times (dist.rebalance_tile_rows), twice
    row_pairs = D.row_pairs_from_ranges(rng, st.tiles_x)
    for it in range(int(os.environ.get("GS_REBALANCE", "2"))):
        split = D.rebalance_tile_rows(split, [m for m, _ in res], row_pairs, st.tiles_x)
        res = []
        for k, rows in enumerate(split):
            rk = Renderer(0)
            res.append(timed(rk, tuple(rows)))
            rk.close()
        worst = max(m for m, _ in res)
        print(f"rebalanced {it + 1}: {split}: bands {' '.join(f'{m:.4f}' for m, _ in res)} ms; slowest {worst:.4f} ms "
              f"({full_ms / worst:.2f}x of the full frame)", flush=True)


if __name__ == "__main__":
    main()
