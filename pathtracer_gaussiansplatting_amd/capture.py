"""Dataset capture (Engine::captureSceneData, Vulkan_Engine/engine.cpp:2658-2814) through the C-ABI:
ptgs_capture_dataset renders every toroidal view (one batched trace per view), writes
train/r_<i>.jpg, transforms_{train,test}.json and points3d.ply. The helpers expose the writers and the
pose generator on their own (host only, no GPU).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi


def _lib(lib=None):
    return lib if lib is not None else _abi.load_library(None)


def capture_poses(n: int, seed: int = 13, min_beta: float = -45.0, max_beta: float = 45.0, lib=None) -> np.ndarray:
    """(n, 2) float32 (alpha, beta) degrees: std::mt19937(seed) + uniform_real_distribution<double>."""
    out = np.zeros((n, 2), np.float32)
    rc = _lib(lib).ptgs_capture_poses(n, seed, min_beta, max_beta, _abi.fptr(out))
    if rc:
        raise _abi.PtgsError(f"ptgs_capture_poses: {rc}")
    return out


def inverse_glm(m, lib=None) -> np.ndarray:
    """glm::inverse of a column-major 4x4 (16 floats), float arithmetic as GLM does it."""
    src = np.ascontiguousarray(np.asarray(m, np.float32).reshape(16))
    out = np.zeros(16, np.float32)
    rc = _lib(lib).ptgs_mat4_inverse_glm(_abi.fptr(src), _abi.fptr(out))
    if rc:
        raise _abi.PtgsError("ptgs_mat4_inverse_glm: singular matrix")
    return out


def write_transforms_json(path: str, fov_y_deg: float, aspect: float, file_paths, transforms, lib=None):
    """transforms: (n, 16) column-major matrices (inverse view)."""
    T = np.ascontiguousarray(np.asarray(transforms, np.float32).reshape(-1, 16))
    arr = (C.c_char_p * max(len(file_paths), 1))(*[p.encode() for p in file_paths])
    rc = _lib(lib).ptgs_write_transforms_json(path.encode(), fov_y_deg, aspect, len(file_paths), arr,
                                              _abi.fptr(T) if len(T) else None)
    if rc:
        raise _abi.PtgsError(f"ptgs_write_transforms_json: {rc}")


def write_ply(path: str, hits: np.ndarray, lib=None) -> int:
    h = np.ascontiguousarray(hits, _abi.HITDATA_DTYPE)
    n = C.c_uint32()
    rc = _lib(lib).ptgs_write_ply(path.encode(), h.ctypes.data, len(h), C.byref(n))
    if rc:
        raise _abi.PtgsError(f"ptgs_write_ply: {rc}")
    return n.value


def read_ply(path: str, lib=None):
    """-> (xyz float32 (N, 3), normals float32 (N, 3), rgb uint8 (N, 3)) of a PLY point cloud."""
    L = _lib(lib)
    n = C.c_uint32()
    rc = L.ptgs_read_ply(path.encode(), None, None, None, 0, C.byref(n))
    if rc:
        raise _abi.PtgsError(f"ptgs_read_ply: {rc} ({path})")
    xyz = np.zeros((n.value, 3), np.float32)
    nrm = np.zeros((n.value, 3), np.float32)
    rgb = np.zeros((n.value, 3), np.uint8)
    rc = L.ptgs_read_ply(path.encode(), xyz.ctypes.data, nrm.ctypes.data, rgb.ctypes.data, n.value, C.byref(n))
    if rc:
        raise _abi.PtgsError(f"ptgs_read_ply: {rc} ({path})")
    return xyz, nrm, rgb


def write_jpeg(path: str, pixels: np.ndarray, quality: int = 90, lib=None):
    p = np.ascontiguousarray(pixels, np.uint8)
    comp = 1 if p.ndim == 2 else p.shape[2]
    rc = _lib(lib).ptgs_write_jpeg(path.encode(), p.ctypes.data, p.shape[1], p.shape[0], comp, quality)
    if rc:
        raise _abi.PtgsError(f"ptgs_write_jpeg: {rc}")


def capture_dataset(renderer, ubo, out_dir: str, width: int, height: int, samples=None, num_samples: int = 0,
                    torus_push=None, total_positions: int = 336, accumulation_steps: int = 512,
                    min_beta: float = -45.0, max_beta: float = 45.0, fov_deg: float = 60.0,
                    major_radius: float = 3.5, torus_height: float = 3.0, image_divisor: float = 2.0, seed: int = 13,
                    capture_images: bool = True, capture_pointcloud: bool = True, stream=None):
    """Run the capture on `renderer` (scene already uploaded). `ubo` supplies the lighting fields;
    `samples` is a device tensor of RaySamples for the point cloud."""
    os.makedirs(out_dir, exist_ok=True)
    d = _abi.CaptureDesc()
    d.out_dir = out_dir.encode()
    d.width, d.height = width, height
    d.total_positions, d.accumulation_steps = total_positions, accumulation_steps
    d.min_beta, d.max_beta, d.fov_deg = min_beta, max_beta, fov_deg
    d.major_radius, d.torus_height, d.image_divisor, d.seed = major_radius, torus_height, image_divisor, seed
    d.capture_images, d.capture_pointcloud = int(capture_images), int(capture_pointcloud)
    d.ubo = C.addressof(ubo)
    if torus_push is not None:
        d.torus = torus_push
    if samples is not None:
        d.samples = samples.data_ptr() if hasattr(samples, "data_ptr") else int(samples)
    d.num_samples = num_samples
    d.hip_stream = None if stream is None else int(stream.cuda_stream if hasattr(stream, "cuda_stream") else stream)
    rc = renderer.lib.ptgs_capture_dataset(renderer._h, C.byref(d))
    renderer._chk(rc, "ptgs_capture_dataset")
