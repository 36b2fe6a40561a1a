#!/usr/bin/env python3
"""A/B of BVH shapes (leaf size : fan-out : SAH depth budget, api.cpp PTGS_BVH_TRIES) on C5's mesh and
camera: each arm uploads the same scene under its own tree list, then interleaved rounds trace the 4K
frame at AB_SPP samples in ONE process (cdna_hip_programming.md §5.4 rule 24).

  PTGS_BVH_LOG=1 python tools/ab_tree.py default 4:4:38 3:4:34 ...
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from pathtracer_gaussiansplatting_amd import ACCUM_SUM, FLAG_COUNT_TRAVERSAL, Camera, Renderer, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    arms = sys.argv[1:] or ["default"]
    spp = int(os.environ.get("AB_SPP", "16"))
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    W, H = int(os.environ.get("AB_W", "3840")), int(os.environ.get("AB_H", "2160"))  # (C3: 1920 x 1080, AB_TRIS=250000)
    scene = Y.atrium_scene(target_tris=int(os.environ.get("AB_TRIS", "1000000")), seed=2)
    scene.blue_noise = Y.blue_noise(1024)
    pose = Camera(aspect=W / H).look_at([-15.0, 4.0, 5.0], [10.0, 3.0, -3.0])
    rs = {}
    for a in arms:
        env = {}
        if a.startswith("env:"):  # env:KEY=VAL+KEY=VAL (e.g. the collapse: env:PTGS_BVH_COLLAPSE=sah+PTGS_BVH_CTRI=0.4)
            env = dict(kv.split("=", 1) for kv in a[4:].split("+"))
        elif a != "default":
            env = {"PTGS_BVH_TRIES": a}
        for k in ("PTGS_BVH_TRIES", "PTGS_BVH_COLLAPSE", "PTGS_BVH_CNODE", "PTGS_BVH_CTRI"):
            os.environ.pop(k, None)
        os.environ.update(env)
        r = Renderer(0)
        info = r.upload_scene(scene)
        for k in env:
            os.environ.pop(k, None)
        print(f"{a:12s} nodes {info.num_bvh_nodes} depth {info.bvh_depth} leaf {info.max_leaf_size} "
              f"build {info.build_ms:.0f} ms", flush=True)
        rs[a] = r
    os.environ.pop("PTGS_BVH_TRIES", None)
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    res = {a: [] for a in arms}
    ref = None
    for rd in range(rounds + 1):
        for a in arms:
            r = rs[a]
            ubo = make_ubo(pose, scene, 0, ambient=(0.3, 0.4, 0.5, 1.0), height=H)
            r.stats_reset()
            acc.zero_()
            torch.cuda.synchronize()
            t = time.perf_counter()
            r.trace_camera(ubo, W, H, acc, spp=spp, mode=ACCUM_SUM)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            st = r.stats()
            img = acc.cpu().numpy()
            if ref is None:
                ref = img.copy()
            err = float(np.linalg.norm(img - ref) / max(np.linalg.norm(ref), 1e-30))
            if rd > 0:
                res[a].append(((st.extension_rays + st.shadow_rays) / dt / 1e6, dt * 1e3, err))
    cnt = {}
    for a in arms:  # traversal work per ray (an untimed pass with the counting kernels)
        r = rs[a]
        r.set_flags(FLAG_COUNT_TRAVERSAL)
        r.stats_reset()
        r.trace_camera(make_ubo(pose, scene, 0, ambient=(0.3, 0.4, 0.5, 1.0), height=H), W, H, acc, spp=spp, mode=ACCUM_SUM)
        torch.cuda.synchronize()
        st = r.stats()
        r.set_flags(0)
        nr = max(st.extension_rays + st.shadow_rays, 1)
        cnt[a] = (st.node_visits / nr, st.tri_tests / nr)
    for a in arms:
        m = [x[0] for x in res[a]]
        ms = np.median([x[1] for x in res[a]])
        print(f"{a:12s} Mrays/s median {np.median(m):9.1f} min {min(m):9.1f} max {max(m):9.1f} ms {ms:8.2f} "
              f"(x{256 // spp} = {ms * 256 / spp:8.1f} ms for 256 spp) rel L2 vs first {max(x[2] for x in res[a]):.1e} "
              f"child-box tests/ray {cnt[a][0]:.2f} tri tests/ray {cnt[a][1]:.2f}",
              flush=True)


if __name__ == "__main__":
    main()
