"""Wavefront vs megakernel on the ingested scene-JSON fixture (GPU): differing pixels and ray counts
per spp, to bisect a wavefront-only difference. Usage: python tools/wf_ingest_debug.py [lib-variant]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np
import torch

import scenes_util as U
from pathtracer_gaussiansplatting_amd import Camera, Renderer, make_ubo
from pathtracer_gaussiansplatting_amd.scene import SceneBuilder

lib = None
if len(sys.argv) > 1:
    lib = os.path.join(os.path.dirname(__file__), "..", "pathtracer_gaussiansplatting_amd", f"libptgs_{sys.argv[1]}.so")
r = Renderer(0, lib_path=lib)
fix = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "ingest")
b = SceneBuilder()
st = b.load_scene_json("main_scene.json", root_dir=fix)
sc = b.finalize()
sc.blue_noise = U.blue_noise()
W, H = 160, 120
pose = Camera(aspect=W / H).look_at([0.0, 0.2, 4.3], [0.2, -1.2, 0.0])
ubo = make_ubo(pose, sc, 0, ambient=tuple(st.ambient_light), height=H, use_lod=st.use_lod, lod_factor=st.lod_factor)
r.upload_scene(sc)
print("env", {k: v for k, v in os.environ.items() if k.startswith("PTGS_")}, "lib", sys.argv[1:] or "default")
for spp in (1, 4):
    res = []
    for wf in (False, True):
        r.set_wavefront(wf)
        acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        r.stats_reset()
        r.trace_camera(ubo, W, H, acc, spp=spp)
        torch.cuda.synchronize()
        s = r.stats()
        res.append((acc.cpu().numpy(), s.extension_rays, s.shadow_rays))
    a, bb = res
    d = np.any(a[0] != bb[0], -1)
    ys, xs = np.nonzero(d)
    print(f"spp {spp}: differ {int(d.sum())} px; ext {a[1]} vs {bb[1]}, shadow {a[2]} vs {bb[2]}; "
          f"first {list(zip(ys[:8].tolist(), xs[:8].tolist()))}")
    # per-row-range bisection at spp 1: which 8-row bands carry the differences
    if spp == 1 and d.any():
        for y0 in sorted(set((ys // 8 * 8).tolist()))[:6]:
            out = []
            for wf in (False, True):
                r.set_wavefront(wf)
                acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
                r.stats_reset()
                r.trace_camera(ubo, W, H, acc, spp=1, rows=(y0, y0 + 8))
                torch.cuda.synchronize()
                s = r.stats()
                out.append((s.extension_rays, s.shadow_rays))
            print(f"   rows {y0}-{y0 + 8}: mega {out[0]} wf {out[1]}")
r.close()
