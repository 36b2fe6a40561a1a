#!/usr/bin/env python3
"""Interleaved A/B of the bench's gs_orbit leg (C2 Gaussians, Morton copy with ids, 120 stream-ordered
frames orbiting + dollying) over library variants in one process:
   tools/gs_orbit_ab.py base pr0 ...     (variant "base" = libptgs.so)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from pathtracer_gaussiansplatting_amd import Camera, Renderer, cornell_box_scene, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    variants = sys.argv[1:] or ["base"]
    W, H, n = 1920, 1080, 100_000
    frames = int(os.environ.get("GS_FRAMES", "120"))
    rounds = int(os.environ.get("AB_ROUNDS", "4"))
    g = Y.gaussians_c2(n, seed=1)
    ubos = bench.gs_orbit_ubos(Camera, make_ubo, cornell_box_scene(), W, H, frames)
    rs, dgs = {}, {}
    for v in variants:
        lib = os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs.so" if v == "base" else f"libptgs_{v}.so")
        rs[v] = Renderer(0, lib_path=lib)
        dgs[v] = rs[v].sort_gaussians_spatial({k: torch.from_numpy(a).cuda() for k, a in g.items()})
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    res = {v: [] for v in variants}
    for rd in range(rounds + 1):
        for v in variants:
            r, dg = rs[v], dgs[v]
            for u in ubos[:3]:
                r.splat_gaussians(dg, u, W, H, img)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for u in ubos:
                r.splat_gaussians(dg, u, W, H, img)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / frames
            if rd:
                res[v].append(dt)
    for v in variants:
        m = np.median(res[v])
        print(f"{v:8s} orbit {m * 1e3:.4f} ms/frame ({n / m / 1e9:.3f} Gsplats/s)  rounds "
              + " ".join(f"{x * 1e3:.4f}" for x in res[v]), flush=True)


if __name__ == "__main__":
    main()
