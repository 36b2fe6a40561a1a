"""GPU BVH build timing on the C3 / C5 meshes (run under rocprofv3 --kernel-trace --stats for the
per-kernel split). Usage: python tools/bvh_build_prof.py [triangles ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import scenes_util as U
from pathtracer_gaussiansplatting_amd import FLAG_GPU_BVH, FLAG_GPU_LBVH, Renderer

lib = os.environ.get("PTGS_LIB")
r = Renderer(0, lib_path=os.path.join(os.path.dirname(__file__), "..", "pathtracer_gaussiansplatting_amd", f"libptgs_{lib}.so") if lib else None)
for n in [int(a) for a in sys.argv[1:]] or [250_000, 1_000_000]:
    sc = U.atrium(n)
    for flags, name in ((0, "host SAH"), (FLAG_GPU_BVH, "GPU SAH"), (FLAG_GPU_BVH | FLAG_GPU_LBVH, "GPU LBVH")):
        r.set_flags(flags)
        for k in range(3):
            t0 = time.perf_counter()
            r.upload_scene(sc)
            r.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            info = r.scene_info()
        print(f"{n} tris {name}: build_ms {info.build_ms:.2f} (upload call {dt:.1f} ms), {info.num_bvh_nodes} nodes, "
              f"depth {info.bvh_depth}", flush=True)
r.close()
