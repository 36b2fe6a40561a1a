#!/usr/bin/env python3
"""Check 3DGS library variants against the base library on the C2 workload (and GS_N / GS_W / GS_H;
GS_SORTED=2: the device Morton order with ids, so the published frame takes the fused front end):
sorted keys / values / ranges bit-exact and the image identical (or its relative L2 printed).
tools/gs_ab_check.py <variant> ...   (libptgs_<variant>.so next to libptgs.so)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def render(path, dg, ubo, W, H):
    import numpy as np
    import torch
    from pathtracer_gaussiansplatting_amd import Renderer
    r = Renderer(0, lib_path=path, publish_splat_buffers=True)
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    if os.environ.get("GS_SORTED", "0") == "2":  # device Morton order with ids (the fused front end's case)
        dg = r.sort_gaussians_spatial(dg)
    # a finished production frame first (no publish: it sizes the fused rows), then a published one
    r.splat_gaussians(dg, ubo, W, H, img, want_stats=True)
    st = r.splat_gaussians(dg, ubo, W, H, img, want_stats=True)
    print(f"  {os.path.basename(path)}: published frame {'fused' if st.fused else 'three launches'}", flush=True)
    torch.cuda.synchronize()
    b = r.splat_buffers()
    K = st.num_rendered
    keys = np.zeros(K, np.uint64)
    vals = np.zeros(K, np.uint32)
    rng = np.zeros(2 * b.num_tiles, np.uint32)
    r.copy_d2h(keys, b.sorted_keys, keys.nbytes)
    r.copy_d2h(vals, b.sorted_values, vals.nbytes)
    r.copy_d2h(rng, b.tile_ranges, rng.nbytes)
    out = img.cpu().numpy()
    r.close()
    return K, keys, vals, rng, out


def main():
    import numpy as np
    import torch
    from pathtracer_gaussiansplatting_amd import Camera, cornell_box_scene, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    n = int(os.environ.get("GS_N", "100000"))
    W, H = int(os.environ.get("GS_W", "1920")), int(os.environ.get("GS_H", "1080"))
    dg = {k: torch.from_numpy(v).cuda() for k, v in Y.gaussians_c2(n, seed=1).items()}
    ubo = make_ubo(Camera(aspect=W / H).look_at([0, 0, 0], [0, 0, -1]), cornell_box_scene(), 0)
    lib = os.path.join(ROOT, "pathtracer_gaussiansplatting_amd")
    base = render(os.path.join(lib, "libptgs.so"), dg, ubo, W, H)
    ok = True
    for v in sys.argv[1:]:
        got = render(os.path.join(lib, f"libptgs_{v}.so"), dg, ubo, W, H)
        same = [base[0] == got[0]] + [np.array_equal(a, b) for a, b in zip(base[1:4], got[1:4])]
        err = float(np.linalg.norm(got[4] - base[4]) / max(np.linalg.norm(base[4]), 1e-30))
        good = all(same) and err < 1e-6
        ok &= good
        print(f"{v:12s} K {got[0]} (base {base[0]})  keys/vals/ranges equal {same[1:]}  image rel L2 {err:.2e}  "
              f"{'OK' if good else 'MISMATCH'}", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
