"""Build the native library libptgs.so (HIP kernels for gfx950 + the C-ABI host code).

Everything is compiled in-tree with hipcc so the .so travels with the repository snapshot to the
GPU box. Flags that are part of the parity contract (see csrc/detmath.h):
  -ffp-contract=off   no FMA contraction, so every float op rounds like the CPU oracle's
  (no -ffast-math)    IEEE division / sqrt (gfx950: v_div_scale/fixup, v_sqrt + fixup sequences)
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libptgs.so")

SOURCES = ["api.cpp", "bvh.cpp", "bvh_gpu.hip", "bvh_sah_gpu.hip", "bvh_collapse_gpu.hip", "capture.cpp", "capture_io.cpp", "comm.cpp", "jpeg.cpp", "scene.cpp", "textures.cpp",
           "pt_kernels.hip", "pt_wavefront.hip", "raster.hip", "splat.hip", "knn.hip", "gltf.cpp", "image_decode.cpp", "ply.cpp", "sampling.cpp"]
# pure host code (scene ingest): plain g++, no device pass
HOST_SOURCES = {"gltf.cpp", "image_decode.cpp", "ply.cpp", "sampling.cpp", "capture_io.cpp", "jpeg.cpp"}
# per-source extra flags. pt_kernels.hip: SimplifyCFG's common-store sinking merges stores to
# different Payload fields from the branches of closest_hit into one store through a phi of
# addresses, which SROA cannot split: the payload then stays a private (scratch) object.
# pt_wavefront.hip: the SLP vectorizer's horizontal-reduction seeding (-slp-vectorize-hor) turns the
# extend kernel's loop-carried ray-state phis into <2 x float> phis and, with the textured any-hit
# inlined, changes the traced rays (opt-bisect: slp-vectorizer on pt_wf_extend_kernel<false, true>;
# DESIGN.md §4 "-O3 any-hit miscompile", tools/ah_repro.py, tools/ah_variants.py). Without that seeding
# the inlined any-hit is bit-exact, so the any-hit is no longer called out of line.
# pt_kernels.hip: the same flag measured +3.1% on the megakernel (C3 at 16 spp: 4 917 vs 4 766 Mrays/s,
# images identical; -fno-slp-vectorize alike).
EXTRA = {"pt_kernels.hip": ["-mllvm", "-simplifycfg-sink-common=false", "-mllvm", "-slp-vectorize-hor=false"],
         "pt_wavefront.hip": ["-mllvm", "-simplifycfg-sink-common=false", "-mllvm", "-slp-vectorize-hor=false"]}
ARCH = os.environ.get("PTGS_ARCH", "gfx950")
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable", "-I", INCLUDE, "-I", CSRC]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build libptgs.so")


def _compile(src: str, defines: tuple = (), build_dir: str = BUILD) -> str:
    obj = os.path.join(build_dir, os.path.basename(src) + ".o")
    path = os.path.join(CSRC, src)
    deps = [path] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(INCLUDE, "ptgs", "ptgs.h"))
    if os.path.exists(obj) and all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in deps):
        return obj
    dflags = [f"-D{d}" for d in defines]
    cmd = [_hipcc()] + COMMON + dflags + EXTRA.get(src, []) + [f"--offload-arch={ARCH}", "-c", path, "-o", obj]
    if src in HOST_SOURCES:
        cmd = ["g++"] + COMMON + dflags + ["-c", path, "-o", obj]
    elif src.endswith(".cpp"):
        cmd = [_hipcc()] + COMMON + dflags + ["-x", "hip", f"--offload-arch={ARCH}", "-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose: bool = False, defines: tuple = (), variant: str = "") -> str:
    """Build libptgs.so (or, for A/B experiments, libptgs_<variant>.so with extra -D defines)."""
    build_dir = BUILD if not variant else BUILD + "_" + variant
    lib = LIB if not variant else os.path.join(HERE, f"libptgs_{variant}.so")
    os.makedirs(build_dir, exist_ok=True)
    with ThreadPoolExecutor(max_workers=min(6, os.cpu_count() or 2)) as ex:
        objs = list(ex.map(lambda s: _compile(s, tuple(defines), build_dir), SOURCES))
    if os.path.exists(lib) and all(os.path.getmtime(lib) >= os.path.getmtime(o) for o in objs):
        return lib
    tmp = lib + ".tmp"
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + [
        "-Wl,-Bsymbolic", "-Wl,-rpath,/opt/rocm/lib", "-L/opt/rocm/lib", "-lamdhip64", "-ldl", "-lz"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, lib)
    if verbose:
        print("built", lib)
    return lib


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
