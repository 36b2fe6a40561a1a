"""One C3 frame (1920x1080, 64 spp, 250k tris) through the wavefront path tracer, for rocprofv3."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from pathtracer_gaussiansplatting_amd import Camera, Renderer, make_ubo
from pathtracer_gaussiansplatting_amd import synthetic as Y

W, H = 1920, 1080
SPP = int(os.environ.get("SPP", "64"))
WF = os.environ.get("WF", "1") == "1"
sc = Y.atrium_scene(target_tris=250_000, seed=2)
sc.blue_noise = Y.blue_noise(1024)
r = Renderer(0, lib_path=os.environ.get("PTGS_LIB"), wavefront=WF)
r.upload_scene(sc)
pose = Camera(aspect=W / H).look_at([-15.0, 4.0, 5.0], [10.0, 3.0, -3.0])
acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
for it in range(2):
    ubo = make_ubo(pose, sc, it * SPP, ambient=(0.3, 0.4, 0.5, 1.0), height=H)
    r.stats_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.trace_camera(ubo, W, H, acc, spp=SPP)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = r.stats()
    print(f"{'wavefront' if WF else 'megakernel'} frame {it}: {dt * 1e3:.1f} ms, "
          f"{(st.extension_rays + st.shadow_rays) / dt / 1e6:.0f} Mrays/s (ext {st.extension_rays}, shadow {st.shadow_rays})")
r.close()
