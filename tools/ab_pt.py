#!/usr/bin/env python3
"""A/B timing of path-tracer library variants (libptgs_<variant>.so built with extra -D flags) on the
C3 workload, interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24).

  python tools/ab_pt.py base w4 ...     (variant "base" = libptgs.so)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from pathtracer_gaussiansplatting_amd import Camera, Renderer, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    variants = sys.argv[1:] or ["base"]
    spp = int(os.environ.get("AB_SPP", "16"))
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    calls = int(os.environ.get("AB_CALLS", "1"))  # consecutive calls per measurement (the viewer: AB_SPP=1 AB_CALLS=64)
    W, H = 1920, 1080
    scene = Y.atrium_scene(250_000, seed=2)
    scene.blue_noise = Y.blue_noise(1024)
    pose = Camera(aspect=W / H).look_at([-15.0, 4.0, 5.0], [10.0, 3.0, -3.0])
    rs = {}
    for v in variants:
        path = os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs.so" if v == "base" else f"libptgs_{v}.so")
        r = Renderer(0, lib_path=path)
        r.upload_scene(scene)
        if os.environ.get("AB_WF", "0") == "1":  # the wavefront tracer (PTGS_FLAG_PT_WAVEFRONT)
            r.set_wavefront(True)
        rs[v] = r
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    res = {v: [] for v in variants}
    ref = None
    for rd in range(rounds + 1):
        for v in variants:
            r = rs[v]
            ubos = [make_ubo(pose, scene, k * spp, ambient=(0.3, 0.4, 0.5, 1.0), height=H) for k in range(calls)]
            r.stats_reset()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for ubo in ubos:
                r.trace_camera(ubo, W, H, acc, spp=spp)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            st = r.stats()
            img = acc.cpu().numpy()
            if ref is None:
                ref = img.copy()
            same = bool(np.array_equal(img, ref))
            if rd > 0:
                res[v].append(((st.extension_rays + st.shadow_rays) / dt / 1e6, dt * 1e3, same))
    for v in variants:
        m = [x[0] for x in res[v]]
        print(f"{v:12s} Mrays/s median {np.median(m):9.1f} min {min(m):9.1f} max {max(m):9.1f} "
              f"ms {np.median([x[1] for x in res[v]]):8.2f} identical_to_first={all(x[2] for x in res[v])}", flush=True)


if __name__ == "__main__":
    main()
