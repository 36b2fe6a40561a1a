#!/usr/bin/env python3
"""Phase timeline of one C2 3DGS frame from a GS_STAMP build (libptgs_stamp.so: per-workgroup
s_memrealtime stamps, 100 MHz): fused front end (zero LDS / preprocess / count walk / reserve /
scatter walk) and blend (keys + sort + stage / evaluation / tail). GS_N, GS_SORTED as tools/gs_probe.py.
   tools/gs_stamps.py [libptgs_stamp.so]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stats(name, d):
    import numpy as np
    d = np.asarray(d, np.float64) * 0.01  # 10 ns ticks -> us
    print(f"  {name:28s} mean {d.mean():7.2f}  p50 {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f} us")


def main():
    import numpy as np
    import torch
    from pathtracer_gaussiansplatting_amd import Camera, Renderer, cornell_box_scene, make_ubo
    from pathtracer_gaussiansplatting_amd import synthetic as Y
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs_stamp.so")
    n = int(os.environ.get("GS_N", "100000"))
    W, H = 1920, 1080
    g = Y.gaussians_c2(n, seed=1)
    if os.environ.get("GS_SORTED", "0") == "1":
        m = g["means"]
        q = ((m - m.min(0)) / np.maximum(m.max(0) - m.min(0), 1e-30) * 1023).astype(np.uint64)
        code = np.zeros(len(m), np.uint64)
        for b in range(10):
            for a in range(3):
                code |= ((q[:, a] >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + a)
        g = {k: np.ascontiguousarray(v[np.argsort(code, kind="stable")]) for k, v in g.items()}
    dg = {k: torch.from_numpy(v).cuda() for k, v in g.items()}
    ubo = make_ubo(Camera(aspect=W / H).look_at([0, 0, 0], [0, 0, -1]), cornell_box_scene(), 0)
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    r = Renderer(0, lib_path=lib)
    if os.environ.get("GS_SORTED", "0") == "2":  # device Morton copy with ids (the bench's timed mode)
        dg = r.sort_gaussians_spatial(dg)
    rows = None
    if os.environ.get("GS_BAND"):  # band k of 8 equal tile-row bands, with chunk bounds
        k, gy = int(os.environ["GS_BAND"]), (H + 15) // 16
        rows = (gy * k // 8, gy * (k + 1) // 8)
        dg = dict(dg, chunk_bounds=r.gaussians_chunk_bounds(dg))
    for _ in range(5):  # (each finished before the next: the fused path starts once a frame has finished)
        r.splat_gaussians(dg, ubo, W, H, img, tile_rows=rows)
        torch.cuda.synchronize()
    r.splat_gaussians(dg, ubo, W, H, img, tile_rows=rows)
    torch.cuda.synchronize()
    st = r.splat_status()
    print(f"front end of the stamped frame: {'fused' if st.fused else 'three launches'} (touched runs {st.touched_runs})")
    dll = C.CDLL(lib)
    dll.ptgs_debug_stamps.argtypes = [C.c_int, C.c_void_p, C.c_uint]
    N8 = 65536 * 8
    fs = np.zeros(N8, np.uint64)
    bs = np.zeros(N8, np.uint64)
    assert dll.ptgs_debug_stamps(0, fs.ctypes.data, N8) == 0
    assert dll.ptgs_debug_stamps(1, bs.ctypes.data, N8) == 0
    fe = os.environ.get("PTGS_GS_FRONTEND", "default")
    chunks = (n + 255) // 256  # GS_FUSED_THREADS Gaussians per fused workgroup
    fall = fs.reshape(-1, 8).astype(np.int64)
    f = fall[:chunks]
    hlp = fall[chunks:chunks + 128]
    nb = 120 * 68 if rows is None else 120 * (rows[1] - rows[0])
    b = bs.reshape(-1, 8)[:nb].astype(np.int64)
    t0 = min(f[:, 0].min() if f[:, 0].any() else b[:, 0].min(), b[:, 0].min())
    print(f"n={n} sorted={os.environ.get('GS_SORTED', '0')} frontend={fe}")
    if st.fused:
        print(f"fused front end: {chunks} workgroups, span {(f[:, 5].max() - f[:, 0].min()) * 0.01:.2f} us, "
              f"last start {(f[:, 0].max() - f[:, 0].min()) * 0.01:.2f} us after the first")
        for k, nm in enumerate(["preprocess + rect + scan", "(sync)", "count walk", "reserve (atomics)", "scatter walk"]):
            stats(nm, f[:, k + 1] - f[:, k])
        if f[:, 6].any():  # (wave 0's own preprocess; the rect's barrier; the scans)
            stats("  preprocess (wave 0)", f[:, 6] - f[:, 0])
            stats("  rect + barrier", f[:, 7] - f[:, 6])
            stats("  zero + scan + 2 barriers", f[:, 1] - f[:, 7])
        stats("workgroup total", f[:, 5] - f[:, 0])
        print(f"  owner starts: first {0:.2f}, last {(f[:, 0].max() - f[:, 0].min()) * 0.01:.2f} us; "
              f"ends: median {(np.median(f[:, 5]) - f[:, 0].min()) * 0.01:.2f}, last {(f[:, 5].max() - f[:, 0].min()) * 0.01:.2f} us")
        hs = hlp[hlp[:, 0] > 0]
        if len(hs):
            print(f"  helpers: {len(hs)} stamped, starts {(hs[:, 0].min() - f[:, 0].min()) * 0.01:.2f} .. "
                  f"{(hs[:, 0].max() - f[:, 0].min()) * 0.01:.2f} us")
        print(f"  gap fused end -> first blend start {(b[:, 0].min() - f[:, 5].max()) * 0.01:.2f} us")
        for o in hs[-1:]:  # the tile-order workgroup (the extra last row; at C2 no helper workgroups launch)
            if o[5] > 0:
                print(f"  tile-order workgroup: starts {(o[0] - f[:, 0].min()) * 0.01:.2f} us, ends "
                      f"{(o[5] - f[:, 0].min()) * 0.01:.2f} us (owners' last end {(f[:, 5].max() - f[:, 0].min()) * 0.01:.2f} us)")
    print(f"blend: {len(b)} workgroups, span {(b[:, 3].max() - b[:, 0].min()) * 0.01:.2f} us, "
          f"last start {(b[:, 0].max() - b[:, 0].min()) * 0.01:.2f} us after the first")
    for k, nm in enumerate(["keys + sort + stage", "evaluation (wave 0)", "tail (slowest wave + store)"]):
        stats(nm, b[:, k + 1] - b[:, k])
    stats("workgroup total", b[:, 3] - b[:, 0])
    sm = b[b[:, 6] > 0]  # small tiles: the dependent loads before the rank (wave 0 waited on each)
    if len(sm):
        print(f"  small tiles ({len(sm)}): keys + sort + stage split")
        stats("  tile order load", sm[:, 4] - sm[:, 0])
        stats("  slot row + count", sm[:, 5] - sm[:, 4])
        stats("  records", sm[:, 6] - sm[:, 5])
        stats("  rank + stage + barrier", sm[:, 1] - sm[:, 6])
        stats("  evaluation", sm[:, 2] - sm[:, 1])
    # workgroup lifetimes by position in the blend's (heavy-first) tile order: where the slot-time goes
    life = (b[:, 3] - b[:, 0]) * 0.01
    edges = [0, 1000, 2000, 3000, 4000, 5000, 6000, 7000, len(b)]
    print("  lifetime by order position (workgroups: sum of lifetimes us, mean us): " + "; ".join(
        f"[{a}, {e}): {life[a:e].sum():.0f}, {life[a:e].mean():.2f}" for a, e in zip(edges, edges[1:]) if e > a))
    print(f"  sum of lifetimes {life.sum():.0f} us over {len(b)} workgroups (/ 2048 slots = {life.sum() / 2048:.2f} us)")
    # concurrency: workgroups resident over time
    ts = np.arange(b[:, 0].min(), b[:, 3].max(), 50)
    conc = [(np.count_nonzero((b[:, 0] <= t) & (b[:, 3] > t))) for t in ts]
    print("  resident blend workgroups every 0.5 us: " + " ".join(str(c) for c in conc[::2]))
    _ = t0
    r.close()


if __name__ == "__main__":
    main()
