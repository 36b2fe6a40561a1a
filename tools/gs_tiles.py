#!/usr/bin/env python3
"""Distribution of (Gaussian, tile) pairs per tile for the C2 distribution at GS_N Gaussians."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from pathtracer_gaussiansplatting_amd import Camera, Renderer, cornell_box_scene, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    W, H = 1920, 1080
    for n in [int(x) for x in os.environ.get("GS_N", "100000,1000000").split(",")]:
        g = {k: torch.from_numpy(v).cuda() for k, v in Y.gaussians_c2(n, seed=3).items()}
        ubo = make_ubo(Camera(aspect=W / H).look_at([0, 0, 0], [0, 0, -1]), cornell_box_scene(), 0)
        img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        r = Renderer(0)
        r.splat_gaussians(g, ubo, W, H, img)
        torch.cuda.synchronize()
        b = r.splat_buffers()
        rng = np.zeros(b.num_tiles * 2, np.uint32)
        r.copy_d2h(rng, b.tile_ranges, rng.nbytes)
        rng = rng.reshape(-1, 2).astype(np.int64)
        cnt = rng[:, 1] - rng[:, 0]
        q = np.percentile(cnt, [50, 90, 99, 99.9, 100])
        print(f"N={n}: tiles {len(cnt)}  K={cnt.sum()}  p50/p90/p99/p99.9/max = {q}  "
              f">256: {(cnt > 256).sum()}  >2048: {(cnt > 2048).sum()}  >8192: {(cnt > 8192).sum()}", flush=True)
        r.close()


if __name__ == "__main__":
    main()
