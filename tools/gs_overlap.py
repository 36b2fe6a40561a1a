#!/usr/bin/env python3
"""Frames in flight (PTGS_FLAG_SPLAT_OVERLAP) against serial frames, one process, interleaved:
the bench's static C2 loop and its gs_orbit leg (100k Gaussians, Morton copy with ids, 1920x1080,
stream-ordered, no stats), each frame of the orbit rendered into its own image by both arms and compared
bit for bit, plus the single-frame latency (enqueue -> synchronised) of each arm.
   tools/gs_overlap.py            (env: GS_LIB, GS_FRAMES, GS_REPS, GS_ARMS="serial,overlap")"""
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
    lib = os.environ.get("GS_LIB", "libptgs.so")
    if not os.path.isabs(lib):
        lib = os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", lib)
    W, H, n = 1920, 1080, int(os.environ.get("GS_N", "100000"))
    frames = int(os.environ.get("GS_FRAMES", "400"))
    reps = int(os.environ.get("GS_REPS", "4"))
    arms = os.environ.get("GS_ARMS", "serial,overlap").split(",")
    g = Y.gaussians_c2(n, seed=1)
    ubo = make_ubo(Camera(aspect=W / H).look_at([0.0, 0.0, 0.0], [0.0, 0.0, -1.0]), cornell_box_scene(), 0)
    orbit = bench.gs_orbit_ubos(Camera, make_ubo, cornell_box_scene(), W, H, 120)
    rs, dgs = {}, {}
    for a in arms:
        rs[a] = Renderer(0, lib_path=lib)
        rs[a].set_splat_overlap(a == "overlap")
        dgs[a] = rs[a].sort_gaussians_spatial({k: torch.from_numpy(v).cuda() for k, v in g.items()})
    torch.cuda.synchronize()
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")

    # parity: every orbit frame of each arm into its own image (after a warm-up pass that sizes the rows)
    imgs = {}
    for a in arms:
        r, dg = rs[a], dgs[a]
        for u in orbit[:8]:
            r.splat_gaussians(dg, u, W, H, img)
        torch.cuda.synchronize()
        out = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in orbit]
        for u, o in zip(orbit, out):
            r.splat_gaussians(dg, u, W, H, o)
        torch.cuda.synchronize()
        st = r.splat_status()
        imgs[a] = out
        print(f"{a:8s} orbit pass: incomplete frames {st.frames}, spilled tiles {st.spilled_tiles}, fused {st.fused}",
              flush=True)
    if len(arms) > 1:
        a0 = arms[0]
        for a in arms[1:]:
            diff = [i for i in range(len(orbit)) if not torch.equal(imgs[a0][i], imgs[a][i])]
            print(f"orbit images {a} vs {a0}: {len(orbit) - len(diff)} / {len(orbit)} bit-identical"
                  + (f" (differ: {diff[:10]})" if diff else ""), flush=True)
    del imgs

    # warm clocks
    for a in arms:
        tw = time.perf_counter()
        while time.perf_counter() - tw < 0.3:
            for _ in range(20):
                rs[a].splat_gaussians(dgs[a], ubo, W, H, img)
            torch.cuda.synchronize()
    res = {a: {"static": [], "orbit": [], "latency": []} for a in arms}
    for rep in range(reps):
        for a in arms:
            r, dg = rs[a], dgs[a]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(frames):
                r.splat_gaussians(dg, ubo, W, H, img)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            res[a]["static"].append((time.perf_counter() - t0) / frames * 1e3)
            res[a].setdefault("host", []).append((t1 - t0) / frames * 1e3)
            for u in orbit[:3]:
                r.splat_gaussians(dg, u, W, H, img)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for u in orbit:
                r.splat_gaussians(dg, u, W, H, img)
            torch.cuda.synchronize()
            res[a]["orbit"].append((time.perf_counter() - t0) / len(orbit) * 1e3)
            lat = []
            for _ in range(20):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r.splat_gaussians(dg, ubo, W, H, img)
                torch.cuda.synchronize()
                lat.append((time.perf_counter() - t0) * 1e3)
            res[a]["latency"].append(float(np.median(lat)))
    for a in arms:
        st = rs[a].splat_status()
        s, o, l = (float(np.median(res[a][k])) for k in ("static", "orbit", "latency"))
        print(f"{a:8s} static {s:.4f} ms ({n / s / 1e6:.4f} Gsplats/s)  orbit {o:.4f} ms ({n / o / 1e6:.4f})  "
              f"latency {l:.4f} ms  host enqueue {float(np.median(res[a]['host'])):.4f} ms/call  | static {' '.join(f'{x:.4f}' for x in res[a]['static'])} | orbit "
              f"{' '.join(f'{x:.4f}' for x in res[a]['orbit'])} | incomplete {st.frames}", flush=True)
    for r in rs.values():
        r.close()


if __name__ == "__main__":
    main()
