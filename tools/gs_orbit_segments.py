#!/usr/bin/env python3
"""Where along the bench's gs_orbit path frames in flight gain or lose: the 120 views in segments of
GS_SEG (10) consecutive frames; each segment rendered GS_REPS (5) times in a row per mode (frames in
flight / one at a time, interleaved per segment, each mode on its own warmed renderer), ms per frame
per segment, beside the segment's mean pair count K and the front end's touched runs per tile (from the
serial renderer's status after its run).
   tools/gs_orbit_segments.py"""
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
    seg = int(os.environ.get("GS_SEG", "10"))
    reps = int(os.environ.get("GS_REPS", "5"))
    g = Y.gaussians_c2(n, seed=1)
    ubos = bench.gs_orbit_ubos(Camera, make_ubo, cornell_box_scene(), W, H, 120)
    rs, dgs = {}, {}
    for mode in ("overlap", "serial"):
        r = Renderer(0)
        dgs[mode] = r.sort_gaussians_spatial({k: torch.from_numpy(a).cuda() for k, a in g.items()})
        r.splat_reserve(int(40 * n))
        rs[mode] = r
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    for mode, r in rs.items():  # warm: the whole path once per mode (buffers grown), then the mode's flag
        r.set_splat_overlap(False)
        for u in ubos:
            r.splat_gaussians(dgs[mode], u, W, H, img)
        r.set_splat_overlap(mode == "overlap")
        for u in ubos:
            r.splat_gaussians(dgs[mode], u, W, H, img)
    torch.cuda.synchronize()
    ref = Renderer(0, publish_splat_buffers=True)
    dref = ref.sort_gaussians_spatial({k: torch.from_numpy(a).cuda() for k, a in g.items()})
    tot = {"overlap": 0.0, "serial": 0.0, "best": 0.0}
    for s0 in range(0, len(ubos), seg):
        views = ubos[s0:s0 + seg]
        ms = {}
        for rd in range(2):
            for mode, r in rs.items():
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(reps):
                    for u in views:
                        r.splat_gaussians(dgs[mode], u, W, H, img)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t) / (reps * len(views)) * 1e3
                ms[mode] = min(ms.get(mode, 1e9), dt)
        for mode in ms:
            tot[mode] += ms[mode] * len(views)
        tot["best"] += min(ms.values()) * len(views)
        ks = [ref.splat_gaussians(dref, u, W, H, img, want_stats=True).num_rendered for u in views]
        st = rs["serial"].splat_status()
        print(f"frames {s0:3d}-{s0 + len(views) - 1:3d}: overlap {ms['overlap']:.4f}  serial {ms['serial']:.4f} ms/frame "
              f"({ms['serial'] / ms['overlap']:.3f}x)  mean K {np.mean(ks) / 1e3:7.1f}k  touched runs/tile "
              f"{st.touched_runs / (120 * 68):6.2f}", flush=True)
    print(f"path: overlap {tot['overlap'] / len(ubos):.4f}  serial {tot['serial'] / len(ubos):.4f}  best of the two per "
          f"segment {tot['best'] / len(ubos):.4f} ms/frame")
    for r in list(rs.values()) + [ref]:
        r.close()


if __name__ == "__main__":
    main()
