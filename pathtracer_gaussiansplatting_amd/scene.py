"""Host-side mirror of the reference Engine's scene / camera API, over the C-ABI (ptgs_host.h).

  Camera.toroidal      -> Camera::updateToroidalAngles   Vulkan_Engine/camera.cpp:195-228
  SceneBuilder         -> Engine::createRTBox / loadScene / createGlobalBindlessBuffers
                          Vulkan_Engine/engine.cpp:181-335, :1172-1352, :1658-1860
  make_ubo             -> Engine::updateUniformBuffer    Vulkan_Engine/engine.cpp:2123-2140
Everything here is host code in the native library (no GPU needed).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

from . import _abi
from ._abi import (HITDATA_DTYPE, LIGHT_CDF_DTYPE, LIGHT_TRIANGLE_DTYPE, MATERIAL_DTYPE, MESH_INFO_DTYPE,
                   PRIMITIVE_DTYPE, PUNCTUAL_CDF_DTYPE, PUNCTUAL_LIGHT_DTYPE, VERTEX_DTYPE, Ubo, fptr)

SCENES_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")


def _lib():
    return _abi.load_library()


@dataclass
class CameraPose:
    view: np.ndarray  # (16,) float32 column-major
    proj: np.ndarray  # (16,) float32 column-major
    position: np.ndarray  # (3,) float32
    fov_deg: float
    aspect: float


class Camera:
    """The reference's Camera (camera.cpp). fov 60 deg, near 0.1, far 1e4 (GeneralHeaders.h:442-445)."""

    def __init__(self, aspect: float, fov_deg: float = 60.0, near: float = 0.1, far: float = 10000.0):
        self.aspect = float(aspect)
        self.fov_deg = float(fov_deg)
        self.near = float(near)
        self.far = float(far)

    def toroidal(self, alpha_deg: float, beta_deg: float, radius: float, height: float) -> CameraPose:
        view = np.zeros(16, np.float32)
        proj = np.zeros(16, np.float32)
        pos = np.zeros(3, np.float32)
        rc = _lib().ptgs_camera_toroidal(alpha_deg, beta_deg, radius, height, self.fov_deg, self.aspect, self.near,
                                         self.far, fptr(view), fptr(proj), fptr(pos))
        _abi.check(rc, "ptgs_camera_toroidal")
        return CameraPose(view, proj, pos, self.fov_deg, self.aspect)

    def look_at(self, eye, center, up=(0.0, 1.0, 0.0)) -> CameraPose:
        e = np.asarray(eye, np.float32)
        c = np.asarray(center, np.float32)
        u = np.asarray(up, np.float32)
        view = np.zeros(16, np.float32)
        proj = np.zeros(16, np.float32)
        _abi.check(_lib().ptgs_camera_lookat(fptr(e), fptr(c), fptr(u), fptr(view)), "ptgs_camera_lookat")
        _abi.check(_lib().ptgs_camera_perspective(np.float32(np.radians(self.fov_deg)), self.aspect, self.near,
                                                  self.far, fptr(proj)), "ptgs_camera_perspective")
        return CameraPose(view, proj, e.copy(), self.fov_deg, self.aspect)


def mat4_inverse(m: np.ndarray) -> np.ndarray:
    m = np.ascontiguousarray(m, np.float32)
    out = np.zeros(16, np.float32)
    _abi.check(_lib().ptgs_mat4_inverse(fptr(m), fptr(out)), "ptgs_mat4_inverse")
    return out


def transform_matrix_rows(view: np.ndarray) -> np.ndarray:
    """saveTransformsJson (engine.cpp:2816-2847): rows of inverse(view), written as m[col][row]."""
    inv = mat4_inverse(view).reshape(4, 4)  # [col][row]
    return inv.T.copy()


@dataclass
class Scene:
    """Flattened scene in the reference layouts (what createGlobalBindlessBuffers uploads)."""
    vertices: np.ndarray
    indices: np.ndarray
    meshes: np.ndarray
    mesh_index_count: np.ndarray
    materials: np.ndarray
    light_triangles: np.ndarray
    light_cdf: np.ndarray
    punctual_lights: np.ndarray
    punctual_cdf: np.ndarray
    emissive_flux: float
    punctual_flux: float
    total_flux: float
    p_emissive: float
    blue_noise: np.ndarray | None = None  # (S, S, 4) float32
    # global_textures[]: (rgba8 (H, W, 4) uint8, srgb) pairs; material texture indices index this list
    # (index 0 is the reference's default white texture, gameobject.cpp:347-349)
    textures: list = field(default_factory=list)
    _keep: list = field(default_factory=list, repr=False)

    @property
    def num_triangles(self) -> int:
        c = self.mesh_index_count
        return int(np.sum(np.where(c >= 3, c // 3, 0)))

    def desc(self) -> _abi.SceneDesc:
        if self.blue_noise is None:
            raise ValueError("scene has no blue-noise texture (scene.blue_noise = blue_noise.generate(...))")
        bn = np.ascontiguousarray(self.blue_noise, np.float32)
        arrays = [np.ascontiguousarray(a) for a in (self.vertices, self.indices, self.meshes, self.mesh_index_count,
                                                    self.materials, self.light_triangles, self.light_cdf,
                                                    self.punctual_lights, self.punctual_cdf)]
        self._keep = arrays + [bn]
        v, i, m, mc, mat, lt, lc, pl, pc = arrays
        d = _abi.SceneDesc()
        d.vertices, d.num_vertices = v.ctypes.data, len(v)
        d.indices, d.num_indices = i.ctypes.data, len(i)
        d.meshes, d.mesh_index_count, d.num_meshes = m.ctypes.data, mc.ctypes.data, len(m)
        d.materials, d.num_materials = mat.ctypes.data, len(mat)
        d.light_triangles, d.num_light_triangles = lt.ctypes.data, len(lt)
        d.light_cdf, d.num_light_cdf = lc.ctypes.data, len(lc)
        d.punctual_lights, d.num_punctual_lights = pl.ctypes.data, len(pl)
        d.punctual_cdf, d.num_punctual_cdf = pc.ctypes.data, len(pc)
        d.blue_noise_rgba32f, d.blue_noise_size = bn.ctypes.data, bn.shape[0]
        if self.textures:
            pix = [np.ascontiguousarray(t[0], np.uint8) for t in self.textures]
            tex = (_abi.Texture * len(pix))()
            for k, (img, (_, srgb)) in enumerate(zip(pix, self.textures)):
                if img.ndim != 3 or img.shape[2] != 4:
                    raise ValueError(f"texture {k}: expected (H, W, 4) uint8, got {img.shape}")
                tex[k].rgba8, tex[k].height, tex[k].width, tex[k].srgb = img.ctypes.data, img.shape[0], img.shape[1], int(bool(srgb))
            self._keep += pix + [tex]
            d.textures, d.num_textures = C.cast(tex, C.c_void_p), len(pix)
        return d


def default_material() -> np.ndarray:
    """Material defaults (GeneralHeaders.h:202-235) in MaterialPushConstant layout."""
    m = np.zeros(1, MATERIAL_DTYPE)
    m["base_color_factor"] = 1.0
    eye = np.eye(4, dtype=np.float32).reshape(16)
    m["uv_normal"] = eye
    m["uv_emissive"] = eye
    m["uv_albedo"] = eye
    m["metallic_factor"] = 1.0
    m["roughness_factor"] = 1.0
    m["occlusion_strength"] = 1.0
    m["specular_factor"] = 0.5
    m["specular_color_factor"] = 1.0
    m["sg_id"] = -1
    return m


class SceneBuilder:
    """Objects are aggregated in insertion order, then the rt-box (engine.cpp:1749-1755)."""

    def __init__(self):
        h = C.c_void_p()
        _abi.check(_lib().ptgs_builder_create(C.byref(h)), "ptgs_builder_create")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            _lib().ptgs_builder_destroy(self._h)
            self._h = None

    def _err(self) -> str:
        return (_lib().ptgs_builder_last_error(self._h) or b"").decode()

    def add_rtbox_json(self, path: str) -> "SceneBuilder":
        rc = _lib().ptgs_builder_add_rtbox_json(self._h, path.encode())
        _abi.check(rc, "ptgs_builder_add_rtbox_json", self._err())
        return self

    def add_object(self, vertices: np.ndarray, indices: np.ndarray, prims: np.ndarray, materials: np.ndarray,
                   lights: np.ndarray | None = None, num_textures: int = 1) -> "SceneBuilder":
        v = np.ascontiguousarray(vertices, VERTEX_DTYPE)
        i = np.ascontiguousarray(indices, np.uint32)
        p = np.ascontiguousarray(prims, PRIMITIVE_DTYPE)
        m = np.ascontiguousarray(materials, MATERIAL_DTYPE)
        lt = np.ascontiguousarray(lights if lights is not None else np.zeros(0, PUNCTUAL_LIGHT_DTYPE),
                                  PUNCTUAL_LIGHT_DTYPE)
        rc = _lib().ptgs_builder_add_object(self._h, v.ctypes.data, len(v), i.ctypes.data, len(i), p.ctypes.data,
                                            len(p), m.ctypes.data, len(m), lt.ctypes.data, len(lt), num_textures)
        _abi.check(rc, "ptgs_builder_add_object", self._err())
        return self

    def add_gltf(self, path: str, position=None, rotation_deg=None, scale=None,
                 missing_images_white: bool = False) -> "SceneBuilder":
        """One glTF / GLB model (Gameobject::loadModel) placed as a scene-JSON object entry."""
        def v3(x):
            return None if x is None else (C.c_float * 3)(*[float(t) for t in x])
        flags = _abi.INGEST_MISSING_IMAGES_WHITE if missing_images_white else 0
        rc = _lib().ptgs_builder_add_gltf(self._h, path.encode(), v3(position), v3(rotation_deg), v3(scale), flags)
        _abi.check(rc, "ptgs_builder_add_gltf", self._err())
        return self

    def add_punctual_light(self, light) -> "SceneBuilder":
        """A scene-level light (the settings "sun"): PUNCTUAL_LIGHT_DTYPE record."""
        lt = np.ascontiguousarray(np.asarray(light, PUNCTUAL_LIGHT_DTYPE).reshape(1))
        _abi.check(_lib().ptgs_builder_add_punctual_light(self._h, lt.ctypes.data), "ptgs_builder_add_punctual_light",
                   self._err())
        return self

    def load_scene_json(self, path: str, root_dir: str | None = None,
                        missing_images_white: bool = False) -> _abi.SceneSettings:
        """Engine::loadScene: every object of the scene JSON (+ rt-box); returns the settings."""
        st = _abi.SceneSettings()
        flags = _abi.INGEST_MISSING_IMAGES_WHITE if missing_images_white else 0
        rc = _lib().ptgs_builder_load_scene_json(self._h, path.encode(), None if root_dir is None else root_dir.encode(),
                                                 flags, C.byref(st))
        _abi.check(rc, "ptgs_builder_load_scene_json", self._err())
        return st

    def finalize(self) -> Scene:
        d = _abi.SceneDesc()
        ubo = Ubo()
        rc = _lib().ptgs_builder_finalize(self._h, C.byref(d), C.byref(ubo))
        _abi.check(rc, "ptgs_builder_finalize", self._err())

        def arr(ptr, n, dt):
            if n == 0:
                return np.zeros(0, dt)
            buf = (C.c_char * (n * dt.itemsize)).from_address(ptr)
            return np.frombuffer(bytes(buf), dtype=dt).copy()

        textures = []
        if d.num_textures:
            tex = (_abi.Texture * d.num_textures).from_address(d.textures)
            for t in tex:
                px = arr(t.rgba8, t.width * t.height * 4, np.dtype(np.uint8)).reshape(t.height, t.width, 4)
                textures.append((px, bool(t.srgb)))

        return Scene(
            vertices=arr(d.vertices, d.num_vertices, VERTEX_DTYPE),
            indices=arr(d.indices, d.num_indices, np.dtype("<u4")),
            meshes=arr(d.meshes, d.num_meshes, MESH_INFO_DTYPE),
            mesh_index_count=arr(d.mesh_index_count, d.num_meshes, np.dtype("<u4")),
            materials=arr(d.materials, d.num_materials, MATERIAL_DTYPE),
            light_triangles=arr(d.light_triangles, d.num_light_triangles, LIGHT_TRIANGLE_DTYPE),
            light_cdf=arr(d.light_cdf, d.num_light_cdf, LIGHT_CDF_DTYPE),
            punctual_lights=arr(d.punctual_lights, d.num_punctual_lights, PUNCTUAL_LIGHT_DTYPE),
            punctual_cdf=arr(d.punctual_cdf, d.num_punctual_cdf, PUNCTUAL_CDF_DTYPE),
            emissive_flux=ubo.emissive_flux, punctual_flux=ubo.punctual_flux, total_flux=ubo.total_flux,
            p_emissive=ubo.p_emissive, textures=textures)


def make_ubo(pose: CameraPose, scene: Scene, frame_count: int, ambient=(0.0, 0.0, 0.0, 1.0),
             height: float = 720.0, use_lod: float = 0.0, lod_factor: float = 1.0) -> Ubo:
    """Engine::updateUniformBuffer (engine.cpp:2123-2140) + the light fields of createGlobalBindlessBuffers."""
    u = Ubo()
    u.view[:] = [float(x) for x in pose.view]
    u.proj[:] = [float(x) for x in pose.proj]
    u.camera_pos[:] = [float(x) for x in pose.position]
    u.frame_count = int(frame_count)
    u.ambient_light[:] = [float(x) for x in ambient]
    u.emissive_flux = scene.emissive_flux
    u.punctual_flux = scene.punctual_flux
    u.total_flux = scene.total_flux
    u.p_emissive = scene.p_emissive
    u.fov = float(np.float32(np.radians(pose.fov_deg)))
    u.height = float(height)
    u.use_lod = float(use_lod)
    u.lod_factor = float(lod_factor)
    return u


def cornell_box_scene() -> Scene:
    """rt-box of showcase/subjects/bunny_box.json (objects [] — bunny.bin is a missing blob)."""
    return SceneBuilder().add_rtbox_json(os.path.join(SCENES_DIR, "cornell_box.json")).finalize()


def new_hitdata(n: int) -> np.ndarray:
    return np.zeros(n, HITDATA_DTYPE)


def decode_image(data: bytes) -> np.ndarray:
    """PNG / JPEG bytes -> (H, W, 4) uint8 with stbi_load(..., STBI_rgb_alpha) semantics."""
    lib = _lib()
    w, h, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
    _abi.check(lib.ptgs_image_decode_rgba8(data, len(data), None, 0, C.byref(w), C.byref(h), C.byref(c)),
               "ptgs_image_decode_rgba8")
    out = np.empty((h.value, w.value, 4), np.uint8)
    _abi.check(lib.ptgs_image_decode_rgba8(data, len(data), out.ctypes.data, out.nbytes, C.byref(w), C.byref(h),
                                           C.byref(c)), "ptgs_image_decode_rgba8")
    return out
