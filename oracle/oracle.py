"""ctypes wrapper of the CPU ORACLE (oracle/ptgs_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module, and
only as the checker. The product (pathtracer_gaussiansplatting_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libptgs_oracle.so")

_FP = C.POINTER(C.c_float)
_P = C.c_void_p
_U = C.c_uint32


class OracleStats(C.Structure):
    _fields_ = [("extension_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("samples", C.c_uint64)]


def build() -> str:
    """Compile the oracle with its committed Makefile (gcc)."""
    r = subprocess.run(["make", "-s", "-C", HERE], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"oracle build failed:\n{r.stdout}\n{r.stderr}")
    return LIB


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.oracle_trace_camera.restype = C.c_int
        L.oracle_trace_camera.argtypes = [_P, _P, _U, _U, _U, _U, _U, _P, _U, _U, _U, C.c_int, C.POINTER(OracleStats)]
        L.oracle_trace_torus.restype = C.c_int
        L.oracle_trace_torus.argtypes = [_P, _P, _P, _P, _U, _P, C.c_int, C.POINTER(OracleStats)]
        L.oracle_camera_toroidal.restype = None
        L.oracle_camera_toroidal.argtypes = [C.c_float] * 8 + [_FP, _FP, _FP]
        L.oracle_mat4_inverse.restype = C.c_int
        L.oracle_mat4_inverse.argtypes = [_FP, _FP]
        L.oracle_encode_srgb8.restype = None
        L.oracle_encode_srgb8.argtypes = [_P, _U, _P]
        L.oracle_splat_points.restype = None
        L.oracle_splat_points.argtypes = [_P, _P, _P, _P, _U, _U, _U, _P, _P]
        L.oracle_splat_gaussians.restype = C.c_int
        L.oracle_trace_depth.restype = C.c_int
        L.oracle_trace_depth.argtypes = [_P, _P, _U, _U, _P, C.c_int]
        L.oracle_splat_gaussians.argtypes = [_P, _P, _P, _P, _P, _U, _P, _U, _U, _P, _P, _P, _U, _U, _P, _P, _P, _P, _P,
                                             C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.POINTER(C.c_uint32)), _P,
                                             _P]
        L.oracle_splat_gaussians_tight.restype = C.c_int
        L.oracle_splat_gaussians_tight.argtypes = L.oracle_splat_gaussians.argtypes
        L.oracle_free.restype = None
        L.oracle_free.argtypes = [_P]
        L.oracle_knn3_mean_dist2.restype = None
        L.oracle_knn3_mean_dist2.argtypes = [_P, _U, _P]
        L.oracle_sincos.restype = None
        L.oracle_sincos.argtypes = [C.c_float, _FP, _FP]
        L.oracle_exp2.restype = C.c_float
        L.oracle_exp2.argtypes = [C.c_float]
        L.oracle_log2.restype = C.c_float
        L.oracle_log2.argtypes = [C.c_float]
        _lib = L
    return _lib


def camera_toroidal(alpha, beta, radius, height, fov_deg, aspect, near=0.1, far=10000.0):
    view = np.zeros(16, np.float32)
    proj = np.zeros(16, np.float32)
    pos = np.zeros(3, np.float32)
    lib().oracle_camera_toroidal(alpha, beta, radius, height, fov_deg, aspect, near, far,
                                 view.ctypes.data_as(_FP), proj.ctypes.data_as(_FP), pos.ctypes.data_as(_FP))
    return view, proj, pos


def mat4_inverse(m):
    m = np.ascontiguousarray(m, np.float32)
    out = np.zeros(16, np.float32)
    if lib().oracle_mat4_inverse(m.ctypes.data_as(_FP), out.ctypes.data_as(_FP)) != 0:
        raise ValueError("singular")
    return out


def trace_camera(desc, ubo, width, height, accum: np.ndarray, spp=1, frame_stride=1, mode=0, rows=None,
                 row_stride=1, threads=0):
    """desc: pathtracer_gaussiansplatting_amd._abi.SceneDesc (host arrays); accum: (H, W, 4) float32, in/out."""
    assert accum.dtype == np.float32 and accum.flags.c_contiguous and accum.size == width * height * 4
    r0, r1 = (0, height) if rows is None else rows
    st = OracleStats()
    lib().oracle_trace_camera(C.addressof(desc), C.addressof(ubo), width, height, r0, r1, row_stride,
                              accum.ctypes.data, spp, frame_stride, mode, threads, C.byref(st))
    return st


def trace_torus(desc, ubo, push, samples: np.ndarray, hits: np.ndarray, threads=0):
    st = OracleStats()
    lib().oracle_trace_torus(C.addressof(desc), C.addressof(ubo), C.addressof(push), samples.ctypes.data,
                             len(samples), hits.ctypes.data, threads, C.byref(st))
    return st


def encode_srgb8(rgba: np.ndarray) -> np.ndarray:
    rgba = np.ascontiguousarray(rgba, np.float32)
    n = rgba.size // 4
    out = np.zeros(n, np.uint32)
    lib().oracle_encode_srgb8(rgba.ctypes.data, n, out.ctypes.data)
    return out


def splat_points(ubo, push, hits, samples, width, height, rgba8: np.ndarray, depth: np.ndarray):
    lib().oracle_splat_points(C.addressof(ubo), C.addressof(push), hits.ctypes.data, samples.ctypes.data,
                              len(hits), width, height, rgba8.ctypes.data, depth.ctypes.data)


def trace_depth(desc, ubo, width, height, threads=0) -> np.ndarray:
    """Primary-hit view depth per pixel ((H, W) float32, +inf on a miss)."""
    out = np.zeros((height, width), np.float32)
    lib().oracle_trace_depth(C.byref(desc), C.byref(ubo), width, height, out.ctypes.data, threads)
    return out


def splat_gaussians(g: dict, ubo, width, height, bg=(0.0, 0.0, 0.0), tile_rows=None, over=None, tight=False):
    """over=(depth (H, W) float32, under (H, W, 4) float32): the hybrid composite. tight: bin by the
    alpha >= 1/255 box as the product's stream-ordered (timed) frames do (oracle_splat_gaussians_tight);
    default: the 3-sigma rectangles of published / stats frames."""
    n = g["means"].shape[0]
    arrs = {k: np.ascontiguousarray(v, np.float32) for k, v in g.items()}
    radii = np.zeros(n, np.int32)
    touched = np.zeros(n, np.uint32)
    means2d = np.zeros(2 * n, np.float32)
    depths = np.zeros(n, np.float32)
    conic = np.zeros(4 * n, np.float32)
    gx, gy = (width + 15) // 16, (height + 15) // 16
    ranges = np.zeros(2 * gx * gy, np.uint32)
    image = np.zeros((height, width, 4), np.float32)
    bgc = np.asarray(bg, np.float32)
    kp = C.POINTER(C.c_uint64)()
    vp = C.POINTER(C.c_uint32)()
    t0, t1 = (0, 0xFFFFFFFF) if tile_rows is None else tile_rows
    dl = un = None
    if over is not None:
        dl = np.ascontiguousarray(over[0], np.float32)
        un = np.ascontiguousarray(over[1], np.float32)
    fn = lib().oracle_splat_gaussians_tight if tight else lib().oracle_splat_gaussians
    K = fn(arrs["means"].ctypes.data, arrs["scales"].ctypes.data,
                                     arrs["rotations"].ctypes.data, arrs["opacities"].ctypes.data,
                                     arrs["colors"].ctypes.data, n, C.addressof(ubo), width, height, bgc.ctypes.data,
                                     None if dl is None else dl.ctypes.data, None if un is None else un.ctypes.data,
                                     t0, t1, radii.ctypes.data, touched.ctypes.data, means2d.ctypes.data,
                                     depths.ctypes.data, conic.ctypes.data, C.byref(kp), C.byref(vp),
                                     ranges.ctypes.data, image.ctypes.data)
    keys = np.ctypeslib.as_array(kp, shape=(max(K, 1),))[:K].copy()
    vals = np.ctypeslib.as_array(vp, shape=(max(K, 1),))[:K].copy()
    lib().oracle_free(C.cast(kp, C.c_void_p))
    lib().oracle_free(C.cast(vp, C.c_void_p))
    return {"radii": radii, "touched": touched, "means2d": means2d, "depths": depths, "conic": conic,
            "keys": keys, "vals": vals, "ranges": ranges, "image": image, "K": K}


def knn3_mean_dist2(xyz: np.ndarray) -> np.ndarray:
    """Brute-force 3-NN mean squared distance (the distCUDA2 term of 3DGS initialisation)."""
    p = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    out = np.zeros(len(p), np.float32)
    lib().oracle_knn3_mean_dist2(p.ctypes.data, len(p), out.ctypes.data)
    return out


def gaussians_from_points(xyz: np.ndarray, rgb: np.ndarray | None) -> dict:
    """create_from_pcd in post-activation form (means, scales, rotations, opacities, colors)."""
    p = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    n = len(p)
    s = np.sqrt(np.maximum(knn3_mean_dist2(p), np.float32(1e-7))).astype(np.float32)
    rot = np.zeros((n, 4), np.float32)
    rot[:, 0] = 1.0
    col = (np.zeros((n, 3), np.float32) if rgb is None
           else (np.asarray(rgb, np.uint8).reshape(-1, 3).astype(np.float32) / np.float32(255.0)))
    return {"means": p.copy(), "scales": np.repeat(s[:, None], 3, 1), "rotations": rot,
            "opacities": np.full(n, 0.1, np.float32), "colors": col}
