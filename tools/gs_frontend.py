#!/usr/bin/env python3
"""Front-end A/B: frame time of the 3DGS forward per Gaussian order (generated / 3D Morton) at C2 (100k,
1080p), C4's count (1M, 1080p) and C5's splat (10M, 4K), with the front end PTGS_GS_FRONTEND selects
(run once per setting: the library reads it once). Prints the touched (workgroup, tile) runs too.
   PTGS_GS_FRONTEND=fused tools/gs_frontend.py [configs: c2,1m,10m]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {"c2": (100_000, 1920, 1080, 200), "1m": (1_000_000, 1920, 1080, 40), "10m": (10_000_000, 3840, 2160, 5)}


def main():
    import torch
    from pathtracer_gaussiansplatting_amd import Camera, Renderer, cornell_box_scene, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    which = (sys.argv[1] if len(sys.argv) > 1 else "c2,1m,10m").split(",")
    fe = os.environ.get("PTGS_GS_FRONTEND", "auto")
    r = Renderer(0)
    for name in which:
        n, W, H, iters = CONFIGS[name]
        g = {k: torch.from_numpy(v).cuda() for k, v in Y.gaussians_c2(n, seed=1).items()}
        sg = r.sort_gaussians_spatial(g)
        ubo = make_ubo(Camera(aspect=W / H).look_at([0, 0, 0], [0, 0, -1]), cornell_box_scene(), 0)
        img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        for order, gg in (("generated", g), ("morton", sg)):
            r.splat_gaussians(gg, ubo, W, H, img, want_stats=True)
            t = time.perf_counter()
            while time.perf_counter() - t < 0.5:  # clocks up, buffers sized
                r.splat_gaussians(gg, ubo, W, H, img)
                torch.cuda.synchronize()
            st = r.splat_status()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(iters):
                r.splat_gaussians(gg, ubo, W, H, img)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / iters
            st = r.splat_status()
            print(f"{name:4s} {order:9s} frontend={fe:5s} fused={st.fused} {dt * 1e3:8.4f} ms  {n / dt / 1e9:6.3f} Gsplats/s  "
                  f"runs {st.touched_runs} ({st.touched_runs / ((W + 15) // 16 * ((H + 15) // 16)):.1f} per tile)  "
                  f"skipped {st.frames}", flush=True)
        del g, sg, img
    r.close()


if __name__ == "__main__":
    main()
