#!/usr/bin/env python3
"""Reproducer for the round-2 "-O3 miscompile" note (pt_device.h anyhit_accept_call): the textured
feature scene through the wavefront tracer, per library variant, against the CPU oracle (pixels that
differ, ray counts). Variants: libptgs_<name>.so next to libptgs.so ("base" = libptgs.so), e.g. built
with -DPTGS_WF_AH_CALL=false (the textured any-hit inlined into the extend / shadow kernels).
   tools/ah_repro.py base ahinl ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import numpy as np
    import torch
    import oracle
    import scenes_util as U
    from pathtracer_gaussiansplatting_amd import Renderer, make_ubo
    sc = U.features(textured=True)
    W, H, spp = 160, 120, 3
    refs = {}
    for use_lod in (0.0, 1.0):
        ubo = make_ubo(U.cornell_pose(W / H), sc, 0, ambient=(0.05, 0.05, 0.08, 1.0))
        ubo.use_lod, ubo.lod_factor = use_lod, 0.8
        acc = np.zeros((H, W, 4), np.float32)
        st = oracle.trace_camera(sc.desc(), ubo, W, H, acc, spp=spp)
        refs[use_lod] = (ubo, acc, st)
    ok = True
    for v in sys.argv[1:] or ["base"]:
        lib = os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs.so" if v == "base" else f"libptgs_{v}.so")
        r = Renderer(0, lib_path=lib)
        r.upload_scene(sc)
        for wavefront in (False, True):
            r.set_wavefront(wavefront)
            for use_lod, (ubo, ref, so) in refs.items():
                acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
                r.stats_reset()
                r.trace_camera(ubo, W, H, acc, spp=spp)
                torch.cuda.synchronize()
                st = r.stats()
                got = acc.cpu().numpy()
                nd = int(np.count_nonzero(np.any(got != ref, -1)))
                rays = (st.extension_rays, st.shadow_rays) == (so.extension_rays, so.shadow_rays)
                ok &= nd == 0 and rays
                print(f"{v:12s} {'wavefront' if wavefront else 'megakernel':10s} use_lod {use_lod}: {nd} pixels differ, "
                      f"rays {'equal' if rays else f'{st.extension_rays}+{st.shadow_rays} vs {so.extension_rays}+{so.shadow_rays}'}",
                      flush=True)
        r.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
