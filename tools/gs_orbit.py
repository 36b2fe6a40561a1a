#!/usr/bin/env python3
"""The bench's gs_orbit camera path (C2 Gaussians, Morton copy with ids) frame by frame: pair count K,
largest tile, front end, per-frame wall time of a stream-ordered run. GS_FRAMES (default 120); GS_OVERLAP=1:
frames in flight (PTGS_FLAG_SPLAT_OVERLAP). Run under rocprofv3 --kernel-trace to see the kernels per frame
(tools/kt_overlap.py <dir> 6 240: the timed orbit's dispatches).
   tools/gs_orbit.py [libptgs variant]"""
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
    v = sys.argv[1] if len(sys.argv) > 1 else "base"
    lib = os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs.so" if v == "base" else f"libptgs_{v}.so")
    W, H, n = 1920, 1080, 100_000
    frames = int(os.environ.get("GS_FRAMES", "120"))
    r = Renderer(0, lib_path=lib)
    r.set_splat_overlap(os.environ.get("GS_OVERLAP", "0") == "1")
    dg = r.sort_gaussians_spatial({k: torch.from_numpy(a).cuda() for k, a in Y.gaussians_c2(n, seed=1).items()})
    ubos = bench.gs_orbit_ubos(Camera, make_ubo, cornell_box_scene(), W, H, frames)
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    for u in ubos[:3]:
        r.splat_gaussians(dg, u, W, H, img)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for u in ubos:
        r.splat_gaussians(dg, u, W, H, img)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / frames
    st = r.splat_status()
    print(f"orbit: {frames} frames, {dt * 1e3:.4f} ms/frame, {n / dt / 1e9:.3f} Gsplats/s, spilled tiles "
          f"{st.spilled_tiles}, incomplete frames {st.frames}")
    # per frame, one at a time (synchronised): front end of the stream-ordered frame, K, largest tile
    ref = Renderer(0, lib_path=lib, publish_splat_buffers=True)
    for k in range(0, frames, max(1, frames // 20)):
        u = ubos[k]
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            r.splat_gaussians(dg, u, W, H, img)
        torch.cuda.synchronize()
        ft = (time.perf_counter() - t) / 5
        s = r.splat_status()
        sts = ref.splat_gaussians(dg, u, W, H, img, want_stats=True)
        b = ref.splat_buffers()
        rng = np.zeros(2 * b.num_tiles, np.uint32)
        ref.copy_d2h(rng, b.tile_ranges, rng.nbytes)
        per = np.diff(rng.reshape(-1, 2), axis=1).ravel()
        print(f"frame {k:4d}: K {sts.num_rendered:8d}  largest tile {int(per.max()):5d}  tiles>512 {int((per > 512).sum()):4d}"
              f"  fused {s.fused}  touched runs/tile {s.touched_runs / per.size:6.2f}  {ft * 1e3:.4f} ms (same view x5)")
    ref.close()
    r.close()


if __name__ == "__main__":
    main()
