"""ctypes / numpy mirror of include/ptgs/ptgs.h and ptgs_host.h, and the loader of libptgs.so.

The native library is the product: there is no Python or CPU fallback. Loading fails loudly when
libptgs.so is missing or was built for another ABI version.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ABI_VERSION = 4
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libptgs.so")

PTGS_OK = 0
ERRORS = {-1: "PTGS_EINVAL", -2: "PTGS_EHIP", -3: "PTGS_ENOSCENE", -4: "PTGS_ERANGE", -5: "PTGS_EIO",
          -6: "PTGS_EINCOMPLETE", -7: "PTGS_EBADIDS"}
PTGS_EINVAL = -1
PTGS_EINCOMPLETE = -6
PTGS_EBADIDS = -7  # an earlier splat frame met ids >= count
ACCUM_RUNNING_MEAN = 0
ACCUM_SUM = 1
FLAG_COUNT_TRAVERSAL = 1
FLAG_TIME_STAGES = 2
FLAG_GPU_BVH = 4
FLAG_GPU_LBVH = 32
FLAG_SPLAT_PUBLISH = 8
FLAG_PT_WAVEFRONT = 16
FLAG_SPLAT_PUBLISH_TIGHT = 64  # tests: published frames bin like the stream-ordered (timed) frames
FLAG_SPLAT_OVERLAP = 128  # frames in flight: a splat call's front end overlaps the previous call's blend

# ---------------------------------------------------------------------------------------------
# numpy dtypes for the array structs (byte-compatible with Helpers/GeneralHeaders.h)
# ---------------------------------------------------------------------------------------------
VERTEX_DTYPE = np.dtype({
    "names": ["pos", "pad1", "normal", "pad2", "color", "pad3", "tangent", "tex_coord", "tex_coord_1"],
    "formats": [("<f4", 3), "<f4", ("<f4", 3), "<f4", ("<f4", 3), "<f4", ("<f4", 4), ("<f4", 2), ("<f4", 2)],
    "offsets": [0, 12, 16, 28, 32, 44, 48, 64, 72],
    "itemsize": 80,
})
MATERIAL_DTYPE = np.dtype({
    "names": ["base_color_factor", "uv_normal", "uv_emissive", "uv_albedo", "emissive_factor_and_pad",
              "metallic_factor", "roughness_factor", "occlusion_strength", "specular_factor",
              "specular_color_factor", "alpha_cutoff", "transmission_factor", "clearcoat_factor",
              "clearcoat_roughness_factor", "pad", "albedo_texture_index", "normal_texture_index",
              "metallic_roughness_texture_index", "emissive_texture_index", "occlusion_texture_index",
              "clearcoat_texture_index", "clearcoat_roughness_texture_index", "sg_id",
              "use_specular_glossiness_workflow"],
    "formats": [("<f4", 4), ("<f4", 16), ("<f4", 16), ("<f4", 16), ("<f4", 4), "<f4", "<f4", "<f4", "<f4",
                ("<f4", 3), "<f4", "<f4", "<f4", "<f4", "<f4", "<i4", "<i4", "<i4", "<i4", "<i4", "<i4", "<i4",
                "<i4", "<f4"],
    "offsets": [0, 16, 80, 144, 208, 224, 228, 232, 236, 240, 252, 256, 260, 264, 268, 272, 276, 280, 284,
                288, 292, 296, 300, 304],
    "itemsize": 308,
})
PUNCTUAL_LIGHT_DTYPE = np.dtype({
    "names": ["position", "intensity", "color", "range", "direction", "outer_cone_cos", "inner_cone_cos",
              "type", "padding"],
    "formats": [("<f4", 3), "<f4", ("<f4", 3), "<f4", ("<f4", 3), "<f4", "<f4", "<i4", ("<f4", 2)],
    "offsets": [0, 12, 16, 28, 32, 44, 48, 52, 56],
    "itemsize": 64,
})
MESH_INFO_DTYPE = np.dtype([("material_index", "<u4"), ("vertex_offset", "<u4"), ("index_offset", "<u4"),
                            ("_pad1", "<u4")])
LIGHT_TRIANGLE_DTYPE = np.dtype([("v0", "<u4"), ("v1", "<u4"), ("v2", "<u4"), ("material_index", "<u4")])
LIGHT_CDF_DTYPE = np.dtype([("cumulative_probability", "<f4"), ("triangle_index", "<u4"), ("padding", "<f4", 2)])
PUNCTUAL_CDF_DTYPE = np.dtype([("cumulative_probability", "<f4"), ("light_index", "<u4"), ("padding", "<f4", 2)])
HITDATA_DTYPE = np.dtype([("pos", "<f4", 3), ("flag", "<f4"), ("color", "<f4", 4), ("normal", "<f4", 3),
                          ("padding", "<f4")])
RAY_SAMPLE_DTYPE = np.dtype([("uv", "<f4", 2)])
PRIMITIVE_DTYPE = np.dtype([("first_index", "<u4"), ("index_count", "<u4"), ("material_index", "<i4")])

assert VERTEX_DTYPE.itemsize == 80 and MATERIAL_DTYPE.itemsize == 308 and PUNCTUAL_LIGHT_DTYPE.itemsize == 64
assert HITDATA_DTYPE.itemsize == 48 and RAY_SAMPLE_DTYPE.itemsize == 8


# ---------------------------------------------------------------------------------------------
# ctypes structs
# ---------------------------------------------------------------------------------------------
class Ubo(C.Structure):
    _fields_ = [("view", C.c_float * 16), ("proj", C.c_float * 16), ("camera_pos", C.c_float * 3),
                ("frame_count", C.c_uint32), ("ambient_light", C.c_float * 4), ("emissive_flux", C.c_float),
                ("punctual_flux", C.c_float), ("total_flux", C.c_float), ("p_emissive", C.c_float),
                ("fov", C.c_float), ("height", C.c_float), ("use_lod", C.c_float), ("lod_factor", C.c_float)]


class RayPush(C.Structure):
    _fields_ = [("model", C.c_float * 16), ("mode", C.c_int32), ("major_radius", C.c_float),
                ("minor_radius", C.c_float), ("height", C.c_float)]


class CaptureDesc(C.Structure):
    _fields_ = [("out_dir", C.c_char_p), ("width", C.c_uint32), ("height", C.c_uint32),
                ("total_positions", C.c_uint32), ("accumulation_steps", C.c_uint32), ("min_beta", C.c_float),
                ("max_beta", C.c_float), ("fov_deg", C.c_float), ("major_radius", C.c_float),
                ("torus_height", C.c_float), ("image_divisor", C.c_float), ("seed", C.c_uint32),
                ("capture_images", C.c_uint32), ("capture_pointcloud", C.c_uint32), ("ubo", C.c_void_p),
                ("torus", RayPush), ("samples", C.c_void_p), ("num_samples", C.c_uint32), ("hip_stream", C.c_void_p)]


class SceneDesc(C.Structure):
    _fields_ = [("vertices", C.c_void_p), ("num_vertices", C.c_uint32), ("indices", C.c_void_p),
                ("num_indices", C.c_uint32), ("meshes", C.c_void_p), ("mesh_index_count", C.c_void_p),
                ("num_meshes", C.c_uint32), ("materials", C.c_void_p), ("num_materials", C.c_uint32),
                ("light_triangles", C.c_void_p), ("num_light_triangles", C.c_uint32), ("light_cdf", C.c_void_p),
                ("num_light_cdf", C.c_uint32), ("punctual_lights", C.c_void_p), ("num_punctual_lights", C.c_uint32),
                ("punctual_cdf", C.c_void_p), ("num_punctual_cdf", C.c_uint32), ("blue_noise_rgba32f", C.c_void_p),
                ("blue_noise_size", C.c_uint32), ("textures", C.c_void_p), ("num_textures", C.c_uint32)]


class Texture(C.Structure):
    _fields_ = [("rgba8", C.c_void_p), ("width", C.c_uint32), ("height", C.c_uint32), ("srgb", C.c_uint32),
                ("reserved", C.c_uint32)]


class SceneSettings(C.Structure):
    """ptgs_scene_settings: Engine::loadScene settings (engine.cpp:1190-1255)."""
    _fields_ = [("ambient_light", C.c_float * 4), ("use_rt_box", C.c_int32), ("render_torus", C.c_int32),
                ("render_pointcloud", C.c_int32), ("torus_major_radius", C.c_float),
                ("torus_minor_radius", C.c_float), ("torus_height", C.c_float),
                ("torus_major_segments", C.c_int32), ("torus_minor_segments", C.c_int32),
                ("num_rays", C.c_uint32), ("use_lod", C.c_float), ("lod_factor", C.c_float),
                ("accumulation_steps", C.c_uint32), ("total_positions", C.c_uint32), ("min_beta", C.c_float),
                ("max_beta", C.c_float), ("image_divisor", C.c_float), ("capture_images", C.c_int32),
                ("capture_pointcloud", C.c_int32), ("num_objects", C.c_uint32)]


INGEST_MISSING_IMAGES_WHITE = 1


class SceneInfo(C.Structure):
    _fields_ = [("num_triangles", C.c_uint32), ("num_bvh_nodes", C.c_uint32), ("bvh_depth", C.c_uint32),
                ("max_leaf_size", C.c_uint32), ("build_ms", C.c_double), ("device_bytes", C.c_uint64)]


class TraceStats(C.Structure):
    _fields_ = [("extension_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("samples", C.c_uint64),
                ("node_visits", C.c_uint64), ("tri_tests", C.c_uint64), ("closest_hits", C.c_uint64)]


class Gaussians(C.Structure):
    _fields_ = [("means", C.c_void_p), ("scales", C.c_void_p), ("rotations", C.c_void_p),
                ("opacities", C.c_void_p), ("colors", C.c_void_p), ("count", C.c_uint32), ("ids", C.c_void_p),
                ("chunk_bounds", C.c_void_p)]


class SplatStats(C.Structure):
    _fields_ = [("num_rendered", C.c_uint32), ("tiles_x", C.c_uint32), ("tiles_y", C.c_uint32),
                ("num_visible", C.c_uint32), ("fused", C.c_uint32)]


class SplatStatus(C.Structure):
    """ptgs_splat_status: frames the stream-ordered splat left incomplete (spill pool exhausted), tiles
    it completed through the spill pool, buffer capacities."""
    _fields_ = [("frames", C.c_uint64), ("views", C.c_uint32 * 8), ("pair_capacity", C.c_uint32),
                ("last_pairs", C.c_uint32), ("touched_runs", C.c_uint32), ("fused", C.c_uint32),
                ("spilled_tiles", C.c_uint64), ("incomplete_tiles", C.c_uint64), ("spill_capacity", C.c_uint32),
                ("spill_demand", C.c_uint32)]


class SplatBuffers(C.Structure):
    _fields_ = [("radii", C.c_void_p), ("tiles_touched", C.c_void_p), ("sorted_keys", C.c_void_p),
                ("sorted_values", C.c_void_p), ("tile_ranges", C.c_void_p), ("means2d", C.c_void_p),
                ("depths", C.c_void_p), ("conic_opacity", C.c_void_p), ("num_gaussians", C.c_uint32),
                ("num_rendered", C.c_uint32), ("num_tiles", C.c_uint32)]


class BvhBuffers(C.Structure):
    _fields_ = [("nodes", C.c_void_p), ("num_nodes", C.c_uint32), ("triangles", C.c_void_p),
                ("num_triangles", C.c_uint32)]


assert C.sizeof(Ubo) == 192 and C.sizeof(RayPush) == 80

# (name, restype, argtypes) of every symbol include/ptgs/*.h declares
_P = C.c_void_p
_U = C.c_uint32
_I = C.c_int
_FP = C.POINTER(C.c_float)
SYMBOLS = {
    # ptgs.h
    "ptgs_abi_version": (_I, []),
    "ptgs_device_arch": (C.c_char_p, []),
    "ptgs_create": (_I, [_I, C.POINTER(_P)]),
    "ptgs_destroy": (None, [_P]),
    "ptgs_last_error": (C.c_char_p, [_P]),
    "ptgs_scene_upload": (_I, [_P, C.POINTER(SceneDesc)]),
    "ptgs_scene_get_info": (_I, [_P, C.POINTER(SceneInfo)]),
    "ptgs_scene_get_bvh": (_I, [_P, C.POINTER(BvhBuffers)]),
    "ptgs_trace_camera": (_I, [_P, C.POINTER(Ubo), _U, _U, _P, _U, _U, _U, _P]),
    "ptgs_trace_camera_rows": (_I, [_P, C.POINTER(Ubo), _U, _U, _U, _U, _P, _U, _U, _U, _P]),
    "ptgs_trace_torus": (_I, [_P, C.POINTER(Ubo), C.POINTER(RayPush), _P, _U, _P, _P]),
    "ptgs_trace_depth": (_I, [_P, C.POINTER(Ubo), _U, _U, _P, _P]),
    "ptgs_set_flags": (_I, [_P, _U]),
    "ptgs_stats_reset": (_I, [_P, _P]),
    "ptgs_stats_read": (_I, [_P, C.POINTER(TraceStats)]),
    "ptgs_splat_points": (_I, [_P, C.POINTER(Ubo), C.POINTER(RayPush), _P, _P, _U, _U, _U, _P, _P, _P]),
    "ptgs_splat_gaussians": (_I, [_P, C.POINTER(Gaussians), C.POINTER(Ubo), _U, _U, _FP, _U, _U, _P,
                                  C.POINTER(SplatStats), _P]),
    "ptgs_splat_gaussians_views": (_I, [_P, C.POINTER(Gaussians), _U, C.POINTER(Ubo), _U, _U, _FP,
                                        C.POINTER(C.c_void_p), _P]),
    "ptgs_splat_gaussians_over": (_I, [_P, C.POINTER(Gaussians), C.POINTER(Ubo), _U, _U, _P, _P, _U, _U, _P,
                                       C.POINTER(SplatStats), _P]),
    "ptgs_splat_get_buffers": (_I, [_P, C.POINTER(SplatBuffers)]),
    "ptgs_splat_get_tile_rows": (_I, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_uint32)]),
    "ptgs_splat_status_read": (_I, [_P, C.POINTER(SplatStatus), _P]),
    "ptgs_splat_reserve": (_I, [_P, _U]),
    "ptgs_gaussians_sort_spatial": (_I, [_P, C.POINTER(Gaussians), _P, _P, _P, _P, _P, _P, _P]),
    "ptgs_gaussians_chunk_bounds": (_I, [_P, C.POINTER(Gaussians), _P, _P]),
    "ptgs_trace_depth_rows": (_I, [_P, C.POINTER(Ubo), _U, _U, _U, _U, _P, _P]),
    "ptgs_knn3_mean_dist2": (_I, [_P, _P, _U, _P, _P]),
    "ptgs_gaussians_from_points": (_I, [_P, _P, _P, _U, _P, _P, _P, _P, _P, _P]),
    "ptgs_comm_unique_id": (_I, [_P]),
    "ptgs_comm_create": (_I, [_P, _P, C.c_int, C.c_int]),
    "ptgs_comm_destroy": (_I, [_P]),
    "ptgs_reduce_radiance": (_I, [_P, _P, C.c_size_t, C.c_int, _P]),
    "ptgs_allreduce_radiance": (_I, [_P, _P, C.c_size_t, _P]),
    "ptgs_gather_rows": (_I, [_P, _P, C.c_uint32, C.c_uint32, _P, C.c_int, _P]),
    "ptgs_reduce_scatter_rows": (_I, [_P, _P, C.c_uint32, C.c_uint32, _P, _P]),
    "ptgs_splat_stage_ms": (_I, [_P, _FP]),
    "ptgs_encode_srgb8": (_I, [_P, _P, _U, _U, _P, _P]),
    "ptgs_device_alloc": (_I, [_P, C.c_size_t, C.POINTER(_P)]),
    "ptgs_device_free": (_I, [_P, _P]),
    "ptgs_memcpy_h2d": (_I, [_P, _P, _P, C.c_size_t]),
    "ptgs_memcpy_d2h": (_I, [_P, _P, _P, C.c_size_t]),
    "ptgs_memset_d32": (_I, [_P, _P, _U, C.c_size_t, _P]),
    "ptgs_synchronize": (_I, [_P]),
    # ptgs_host.h
    "ptgs_camera_toroidal": (_I, [C.c_float] * 8 + [_FP, _FP, _FP]),
    "ptgs_camera_lookat": (_I, [_FP, _FP, _FP, _FP]),
    "ptgs_camera_perspective": (_I, [C.c_float] * 4 + [_FP]),
    "ptgs_mat4_inverse": (_I, [_FP, _FP]),
    "ptgs_mat4_inverse_glm": (_I, [_FP, _FP]),
    "ptgs_capture_poses": (_I, [_U, _U, C.c_float, C.c_float, _FP]),
    "ptgs_write_transforms_json": (_I, [C.c_char_p, C.c_float, C.c_float, _U, C.POINTER(C.c_char_p), _FP]),
    "ptgs_write_ply": (_I, [C.c_char_p, _P, _U, C.POINTER(C.c_uint32)]),
    "ptgs_write_jpeg": (_I, [C.c_char_p, _P, _U, _U, _U, C.c_int]),
    "ptgs_capture_dataset": (_I, [_P, _P]),
    "ptgs_builder_create": (_I, [C.POINTER(_P)]),
    "ptgs_builder_destroy": (None, [_P]),
    "ptgs_builder_add_rtbox_json": (_I, [_P, C.c_char_p]),
    "ptgs_builder_add_object": (_I, [_P, _P, _U, _P, _U, _P, _U, _P, _U, _P, _U, _U]),
    "ptgs_builder_finalize": (_I, [_P, C.POINTER(SceneDesc), C.POINTER(Ubo)]),
    "ptgs_builder_last_error": (C.c_char_p, [_P]),
    "ptgs_image_decode_rgba8": (_I, [_P, C.c_size_t, _P, C.c_size_t, C.POINTER(_U), C.POINTER(_U), C.POINTER(_U)]),
    "ptgs_read_ply": (_I, [C.c_char_p, _P, _P, _P, _U, C.POINTER(_U)]),
    "ptgs_generate_samples": (_I, [_I, _U, _P, _U, _P, _U, _U, _I, _P]),
    "ptgs_sort_samples": (_I, [_P, _U]),
    "ptgs_morton2d": (_U, [C.c_float, C.c_float]),
    "ptgs_builder_add_gltf": (_I, [_P, C.c_char_p, _FP, _FP, _FP, _U]),
    "ptgs_builder_add_punctual_light": (_I, [_P, _P]),
    "ptgs_builder_load_scene_json": (_I, [_P, C.c_char_p, C.c_char_p, _U, C.POINTER(SceneSettings)]),
}

_lib = None


class PtgsError(RuntimeError):
    def __init__(self, msg: str, code: int = 0):
        super().__init__(msg)
        self.code = code  # the PTGS_E* code (0: not from a library call)


def load_library(path: str | None = None) -> C.CDLL:
    """Load libptgs.so (raises PtgsError if missing). Imports torch first when available so the
    HIP runtime that torch already loaded (same soname libamdhip64.so.7) is the one we bind to."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise PtgsError(f"native library not built: {p} (run pathtracer_gaussiansplatting_amd/build.py)")
    try:
        import torch  # noqa: F401  (shares the HIP runtime)
    except Exception:
        pass
    lib = C.CDLL(p, mode=C.RTLD_GLOBAL if path is None else C.RTLD_LOCAL)
    for name, (res, args) in SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.ptgs_abi_version()
    if v != ABI_VERSION:
        raise PtgsError(f"libptgs ABI version {v} != expected {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str, err: str = "") -> None:
    if rc != PTGS_OK:
        raise PtgsError(f"{what} failed: {ERRORS.get(rc, rc)} {err}", rc)


def fptr(a: np.ndarray):
    return a.ctypes.data_as(_FP)
