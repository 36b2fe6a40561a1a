#!/usr/bin/env python3
"""The bench's C2 timed loop alone (100k Gaussians, Morton copy with ids, 1920x1080, stream-ordered, no
stats; ~0.3 s warm-up, then GS_FRAMES frames between two synchronisations) for A/B runs of library
variants or environment switches, one process per arm:
   tools/gs_c2.py [libptgs_<variant>.so]   (or GS_LIB=libptgs_<variant>.so)      -> "C2 <lib> <ms> ms/frame <Gsplats/s>" (GS_REPS timed loops)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pathtracer_gaussiansplatting_amd import Camera, Renderer, cornell_box_scene, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    lib = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("GS_LIB", "libptgs.so")
    if not os.path.isabs(lib):
        lib = os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", lib)
    n = int(os.environ.get("GS_N", "100000"))
    frames = int(os.environ.get("GS_FRAMES", "400"))
    W, H = 1920, 1080
    r = Renderer(0, lib_path=lib)
    dg0 = {k: torch.from_numpy(v).cuda() for k, v in Y.gaussians_c2(n, seed=1).items()}
    dg = r.sort_gaussians_spatial(dg0)
    ubo = make_ubo(Camera(aspect=W / H).look_at([0.0, 0.0, 0.0], [0.0, 0.0, -1.0]), cornell_box_scene(), 0)
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    tw = time.perf_counter()
    while time.perf_counter() - tw < 0.3:
        for _ in range(20):
            r.splat_gaussians(dg, ubo, W, H, img)
        torch.cuda.synchronize()
    res = []
    for _ in range(int(os.environ.get("GS_REPS", "3"))):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            r.splat_gaussians(dg, ubo, W, H, img)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) / frames * 1e3)
    st = r.splat_status()
    ms = min(res)
    tag = os.environ.get("GS_TAG", os.path.basename(lib))
    print(f"C2 {tag} {ms:.4f} ms/frame {n / ms / 1e6:.4f} Gsplats/s (loops {' '.join(f'{x:.4f}' for x in res)}; "
          f"fused {st.fused})", flush=True)
    r.close()


if __name__ == "__main__":
    main()
