"""MI355X-native renderer for the hot paths of FedericoCos/PathTracer_GaussianSplatting.

The product is the native library libptgs.so (HIP kernels for gfx950 behind the C-ABI in
include/ptgs/ptgs.h); this package is its Python binding plus the host-side scene/camera mirror.
"""
from ._abi import (ACCUM_RUNNING_MEAN, ACCUM_SUM, FLAG_COUNT_TRAVERSAL, FLAG_GPU_BVH, FLAG_GPU_LBVH, FLAG_PT_WAVEFRONT, FLAG_SPLAT_PUBLISH, FLAG_TIME_STAGES, HITDATA_DTYPE, MATERIAL_DTYPE,
                   PUNCTUAL_LIGHT_DTYPE, RAY_SAMPLE_DTYPE, VERTEX_DTYPE, PtgsError, RayPush, Ubo, load_library)
from .renderer import Renderer, torus_push
from .scene import Camera, CameraPose, Scene, SceneBuilder, cornell_box_scene, make_ubo, mat4_inverse

__all__ = [
    "ACCUM_RUNNING_MEAN", "ACCUM_SUM", "FLAG_COUNT_TRAVERSAL", "FLAG_GPU_BVH", "FLAG_GPU_LBVH", "FLAG_PT_WAVEFRONT", "FLAG_SPLAT_PUBLISH", "FLAG_TIME_STAGES", "HITDATA_DTYPE", "MATERIAL_DTYPE",
    "PUNCTUAL_LIGHT_DTYPE", "RAY_SAMPLE_DTYPE", "VERTEX_DTYPE", "PtgsError", "RayPush", "Ubo", "load_library",
    "Renderer", "torus_push", "Camera", "CameraPose", "Scene", "SceneBuilder", "cornell_box_scene", "make_ubo",
    "mat4_inverse",
]
