#!/usr/bin/env python3
"""Run the C2 3DGS workload (100k Gaussians, 1920x1080; GS_N / GS_W / GS_H override) a few times (for rocprofv3 /
A-B timing)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from pathtracer_gaussiansplatting_amd import FLAG_TIME_STAGES, Camera, Renderer, cornell_box_scene, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    variants = sys.argv[1:] or ["base"]
    iters = int(os.environ.get("GS_ITERS", "20"))
    n = int(os.environ.get("GS_N", "100000"))
    W, H = int(os.environ.get("GS_W", "1920")), int(os.environ.get("GS_H", "1080"))
    g = Y.gaussians_c2(n, seed=1)
    if os.environ.get("GS_SORTED", "0") == "1":  # experiment: Gaussians in 3D Morton order of their means
        m = g["means"]
        q = ((m - m.min(0)) / np.maximum(m.max(0) - m.min(0), 1e-30) * 1023).astype(np.uint64)
        code = np.zeros(len(m), np.uint64)
        for b in range(10):
            for a in range(3):
                code |= ((q[:, a] >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + a)
        order = np.argsort(code, kind="stable")
        g = {k: np.ascontiguousarray(v[order]) for k, v in g.items()}
    dg = {k: torch.from_numpy(v).cuda() for k, v in g.items()}
    if os.environ.get("GS_SORTED", "0") == "2":  # device Morton sort with ids (renders like the generated order)
        dg = Renderer(0).sort_gaussians_spatial(dg)
    ubo = make_ubo(Camera(aspect=W / H).look_at([0, 0, 0], [0, 0, -1]), cornell_box_scene(), 0)
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    # rotate the order per call (GS_ROUND): the second library loaded in one process measured ~3% faster
    rot = int(os.environ.get("GS_ROUND", "0")) % max(1, len(variants))
    for v in variants[rot:] + variants[:rot]:
        path = os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs.so" if v == "base" else f"libptgs_{v}.so")
        r = Renderer(0, lib_path=path)
        if os.environ.get("GS_STAGES", "1") == "1":
            r.set_flags(FLAG_TIME_STAGES)
        st = np.zeros(6)
        r.splat_gaussians(dg, ubo, W, H, img)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(iters):
            r.splat_gaussians(dg, ubo, W, H, img)
            st += r.splat_stage_ms()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / iters
        print(f"{v:10s} {dt * 1e3:.4f} ms/frame  {n / dt / 1e9:.4f} Gsplats/s  stages(ms) "
              + " ".join(f"{x / iters:.4f}" for x in st), flush=True)
        r.close()


if __name__ == "__main__":
    main()
