#!/usr/bin/env python3
"""The gs_orbit leg in the order bench.py runs it (after the static C2 loop, the views4 leg and the generated-
order frames, the stats frame and the per-stage event pass: GS_STATS / GS_STAGES=0 leave them out) against
right after the static loop, frames in flight and serial, GS_REPS times each, one process: does what ran
before change the overlapped orbit?   tools/gs_orbit_seq.py"""
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
    W, H, n = 1920, 1080, 100_000
    reps = int(os.environ.get("GS_REPS", "3"))
    g = Y.gaussians_c2(n, seed=1)
    r = Renderer(0)
    dg0 = {k: torch.from_numpy(v).cuda() for k, v in g.items()}
    dg = r.sort_gaussians_spatial(dg0)
    ubo = make_ubo(Camera(aspect=W / H).look_at([0.0, 0.0, 0.0], [0.0, 0.0, -1.0]), cornell_box_scene(), 0)
    orbit = bench.gs_orbit_ubos(Camera, make_ubo, cornell_box_scene(), W, H, 120)
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")

    def orbit_pass():
        for u in orbit[:6]:
            r.splat_gaussians(dg, u, W, H, img)
        torch.cuda.synchronize()
        r.splat_status()
        t1 = time.perf_counter()
        for u in orbit:
            r.splat_gaussians(dg, u, W, H, img)
        torch.cuda.synchronize()
        return (time.perf_counter() - t1) / len(orbit) * 1e3

    def static(frames=500):
        r.set_splat_overlap(True)
        for _ in range(frames):
            r.splat_gaussians(dg, ubo, W, H, img)
        torch.cuda.synchronize()

    def other_legs():
        from pathtracer_gaussiansplatting_amd import FLAG_TIME_STAGES
        r.set_splat_overlap(False)
        if os.environ.get("GS_STATS", "1") == "1":  # the bench's stats frame (3-sigma rectangles, K read back)
            r.splat_gaussians(dg, ubo, W, H, img, want_stats=True)
        if os.environ.get("GS_STAGES", "1") == "1":  # the bench's per-stage event pass
            r.set_flags(FLAG_TIME_STAGES)
            for _ in range(100):
                r.splat_gaussians(dg, ubo, W, H, img)
                r.splat_stage_ms()
            r.set_flags(0)
        vubos = [make_ubo(Camera(aspect=W / H).look_at([0.25 * k, 0.0, 0.0], [0.25 * k, 0.0, -1.0]),
                          cornell_box_scene(), 0) for k in range(4)]
        vouts = [torch.zeros_like(img) for _ in vubos]
        for _ in range(30):
            r.splat_gaussians_views(dg, vubos, W, H, vouts)
        r.set_splat_overlap(False)
        for _ in range(100):
            r.splat_gaussians(dg0, ubo, W, H, img)
        torch.cuda.synchronize()

    for order in ("after the static loop", "after the other legs"):
        for _ in range(reps):
            static()
            if order.startswith("after the other"):
                other_legs()
            r.set_splat_overlap(True)
            ov = orbit_pass()
            r.set_splat_overlap(False)
            se = orbit_pass()
            print(f"{order:32s} orbit overlapped {ov:.4f} ms  serial {se:.4f} ms  ({se / ov:.3f}x)", flush=True)
    r.close()


if __name__ == "__main__":
    main()
