#!/usr/bin/env python3
"""Tile-row bands of the 3DGS forward (the 8-GPU split of bench.py's gs leg): frame time of band k of
GS_BANDS (default 8) equal tile-row bands, with and without ptgs_gaussians.chunk_bounds (per-rank chunk
culling before the preprocess), against the full frame. One configuration per process so that a
kernel trace (rocprofv3 --kernel-trace) separates the front end's kernels per configuration:
   GS_CFG=c2|10m GS_BAND=full|<k> GS_BOUNDS=0|1 [GS_LIB=libptgs_<variant>.so] tools/gs_bands.py
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


if __name__ == "__main__":
    main()
