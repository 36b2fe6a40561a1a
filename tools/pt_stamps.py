#!/usr/bin/env python3
"""Workgroup timeline of one C3 path-traced frame from a PT_STAMP build (libptgs_ptstamp.so: per-
workgroup s_memrealtime at start and end of pt_camera_kernel, 100 MHz): workgroup durations, resident
workgroups over time and the schedule's tail.
   tools/pt_stamps.py [libptgs_ptstamp.so]     (AB_SPP: samples per pixel, default 64)"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from pathtracer_gaussiansplatting_amd import Camera, Renderer, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs_ptstamp.so")
    spp = int(os.environ.get("AB_SPP", "64"))
    W, H = 1920, 1080
    scene = Y.atrium_scene(250_000, seed=2)
    scene.blue_noise = Y.blue_noise(1024)
    pose = Camera(aspect=W / H).look_at([-15.0, 4.0, 5.0], [10.0, 3.0, -3.0])
    r = Renderer(0, lib_path=lib)
    r.upload_scene(scene)
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    ubo = make_ubo(pose, scene, 0, ambient=(0.3, 0.4, 0.5, 1.0), height=H)
    for _ in range(2):
        r.trace_camera(ubo, W, H, acc, spp=spp)
        torch.cuda.synchronize()
    dll = C.CDLL(lib)
    dll.ptgs_debug_pt_stamps.argtypes = [C.c_void_p, C.c_uint]
    T = int(os.environ.get("PT_TILE", "8"))  # the workgroup tile edge (PTGS_PT_WG 64: 8, 256: 16)
    TY = int(os.environ.get("PT_TILE_Y", "4" if T == 8 else str(T)))  # (8x4 tiles: two lanes per pixel)
    nwg = ((W + T - 1) // T) * ((H + TY - 1) // TY)
    st = np.zeros(2 * nwg, np.uint64)
    assert dll.ptgs_debug_pt_stamps(st.ctypes.data, 2 * nwg) == 0
    st = st.reshape(-1, 2).astype(np.int64)
    t0 = st[:, 0].min()
    s0 = (st[:, 0] - t0) * 0.01e-3  # ms
    s1 = (st[:, 1] - t0) * 0.01e-3
    d = s1 - s0
    span = s1.max()
    print(f"{nwg} workgroups, span {span:.2f} ms, last start {s0.max():.2f} ms")
    print(f"workgroup ms: mean {d.mean():.3f} p10 {np.percentile(d, 10):.3f} p50 {np.median(d):.3f} "
          f"p90 {np.percentile(d, 90):.3f} max {d.max():.3f}")
    ts = np.linspace(0, span, 60)
    conc = [int(np.count_nonzero((s0 <= t) & (s1 > t))) for t in ts]
    print("resident workgroups at 60 points: " + " ".join(str(c) for c in conc))
    cap = max(conc)
    work = float(d.sum())
    print(f"ideal span at {cap} resident: {work / cap:.2f} ms ({100 * (1 - work / cap / span):.1f}% of the span idle)")
    # heaviest workgroups' start times
    idx = np.argsort(-d)[:10]
    print("10 longest: " + ", ".join(f"{d[i]:.2f}ms@{s0[i]:.2f}" for i in idx))
    r.close()


if __name__ == "__main__":
    main()
