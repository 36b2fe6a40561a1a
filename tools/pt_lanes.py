#!/usr/bin/env python3
"""Lane utilisation of the path tracer by loop, from a PT_LANES build
(libptgs_ptlanes.so: `python -c "from pathtracer_gaussiansplatting_amd import build as B;
B.build(defines=('PT_LANES',), variant='ptlanes')"`): for each loop of pt_camera_kernel (pt_device.h
PtLoop) the wave iterations and the active lanes summed over them, on one C3 frame (250k-tri atrium,
1920x1080, AB_SPP samples, default 64). utilisation = lanes / (64 x wave iterations).
   tools/pt_lanes.py [libptgs_ptlanes.so]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LOOPS = ["closest-hit node step", "closest-hit leaf phase", "closest-hit triangle", "shadow node step",
         "shadow triangle", "bounce (shade + NEE)", "sample (primary ray setup)"]


def main():
    import numpy as np
    import torch
    from pathtracer_gaussiansplatting_amd import Camera, Renderer, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs_ptlanes.so")
    spp = int(os.environ.get("AB_SPP", "64"))
    W, H = 1920, 1080
    scene = Y.atrium_scene(250_000, seed=2)
    scene.blue_noise = Y.blue_noise(1024)
    pose = Camera(aspect=W / H).look_at([-15.0, 4.0, 5.0], [10.0, 3.0, -3.0])
    r = Renderer(0, lib_path=lib)
    r.upload_scene(scene)
    fn = r.lib.ptgs_debug_pt_lanes
    fn.argtypes = [C.c_void_p, C.c_uint]
    fn.restype = C.c_int
    n = 2 * len(LOOPS)
    buf = np.zeros(n, np.uint64)
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    ubo = make_ubo(pose, scene, 0, ambient=(0.3, 0.4, 0.5, 1.0), height=H)
    r.trace_camera(ubo, W, H, acc, spp=spp)  # (warm-up: the tile schedule's first launch)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, n) == 0
    r.stats_reset()
    r.trace_camera(ubo, W, H, acc, spp=spp)
    torch.cuda.synchronize()
    st = r.stats()
    assert fn(buf.ctypes.data, n) == 0
    rays = st.extension_rays + st.shadow_rays
    print(f"C3 frame, {spp} spp: {st.extension_rays / 1e6:.1f} M extension + {st.shadow_rays / 1e6:.1f} M shadow rays")
    print(f"{'loop':28s} {'wave iters (M)':>15s} {'lane iters (M)':>15s} {'per ray':>8s} {'utilisation':>12s}")
    for i, name in enumerate(LOOPS):
        w, l = int(buf[2 * i]), int(buf[2 * i + 1])
        print(f"{name:28s} {w / 1e6:15.2f} {l / 1e6:15.2f} {l / max(rays, 1):8.2f} {l / max(64 * w, 1):12.3f}")
    r.close()


if __name__ == "__main__":
    main()
