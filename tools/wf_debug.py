"""Bisect wavefront vs megakernel differences on the feature scene variants (GPU)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np, torch
import scenes_util as U
from pathtracer_gaussiansplatting_amd import Renderer, make_ubo

r = Renderer(0, lib_path=(os.path.join(os.path.dirname(__file__), "..", "pathtracer_gaussiansplatting_amd", f"libptgs_{sys.argv[1]}.so") if len(sys.argv) > 1 else None))
for variant in ("mask_only",):
    sc = U.features(with_punctual=False, transparent=True)
    m = sc.materials
    blend = (m["pad"] > 0.5) & (m["alpha_cutoff"] == 0)
    mask = (m["pad"] > 0.5) & (m["alpha_cutoff"] > 0)
    if variant == "blend_only":
        m["pad"][mask] = 0.0
        m["alpha_cutoff"][mask] = 0.0
    elif variant == "mask_only":
        m["pad"][blend] = 0.0
    r.upload_scene(sc)
    W, H = 160, 120
    ubo = make_ubo(U.cornell_pose(W / H), sc, 0, ambient=(0.05, 0.05, 0.08, 1.0))
    for spp in (1,):
        res = []
        for wf in (False, True):
            r.set_wavefront(wf)
            acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
            r.stats_reset()
            r.trace_camera(ubo, W, H, acc, spp=spp)
            torch.cuda.synchronize()
            st = r.stats()
            res.append((acc.cpu().numpy(), st.extension_rays, st.shadow_rays))
        a, b = res
        d = np.any(a[0] != b[0], -1)
        ys, xs = np.nonzero(d)
        print(f"{variant} blend={blend.sum()} mask={mask.sum()}: differ {d.sum()} px; ext {a[1]} vs {b[1]}, shadow {a[2]} vs {b[2]}")
        big = np.abs(a[0] - b[0]).max(-1) > 1e-3
        print("   big diffs", big.sum(), "rows with diffs", np.unique(ys)[:20])
r.close()
