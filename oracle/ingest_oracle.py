"""ingest_oracle.py — CPU ORACLE for scene ingest (test infrastructure only; never imported by the
product package).

An independent Python restatement of the reference's asset path, used by tests/ to check
ptgs_builder_add_gltf / ptgs_builder_load_scene_json / ptgs_image_decode_rgba8:

  Gameobject::loadModel          Vulkan_Engine/gameobject.cpp:198-273
    computeGlobalNodeTransforms  :65-159   (animation 0, frame 0)
    loadLights                   :798-851  (KHR_lights_punctual)
    scanTextureFormats           :275-342, loadTextures :344-368, getTextureIndex :370-378
    loadMaterials                :380-517  (+ getTextureTransform :11-47)
    loadGeometry / processNode   :519-560, loadPrimitive :562-795 (dedup, duplicated indices,
                                 CPU skinning, emissive triangles)
  Engine::loadScene              engine.cpp:1172-1352 (settings, sun, T*R*S bake)
  Engine::createRTBox            engine.cpp:181-335
  createGlobalBindlessBuffers    engine.cpp:1658-1860 (aggregation + light CDFs)

Arithmetic: numpy float32 (IEEE single, one rounding per operation) in the operation order of the
GLM functions the reference calls; cosf / sinf come from the C library through ctypes (the same
functions std::cos(float) binds to). JSON via the json module, images via PIL with
stbi_load(..., STBI_rgb_alpha)'s conventions applied on top (16-bit -> >> 8).

Parity status: pinned by nothing from the reference itself (it holds no ingest outputs, and building
its tinygltf/stb/GLM as a checker was refused in this environment — DESIGN.md §4). PNG texels are
exact by construction; JPEG texels are PIL/libjpeg's, within a tolerance of stb's decoder.
"""
from __future__ import annotations

import base64
import ctypes
import json
import math
import os
import urllib.parse

import numpy as np

F = np.float32
_libm = ctypes.CDLL("libm.so.6")
_libm.cosf.restype = ctypes.c_float
_libm.cosf.argtypes = [ctypes.c_float]
_libm.sinf.restype = ctypes.c_float
_libm.sinf.argtypes = [ctypes.c_float]


def cosf(x):
    return F(_libm.cosf(float(x)))


def sinf(x):
    return F(_libm.sinf(float(x)))


# ----------------------------------------------------------------------------------------------
# GLM in float32, operation order preserved. Matrices: m[col][row] (4x4 float32 arrays).
# ----------------------------------------------------------------------------------------------
def ident():
    return np.eye(4, dtype=F)


def mat_mul(a, b):
    r = np.zeros((4, 4), F)
    for i in range(4):
        for k in range(4):
            s = F(a[0][k] * b[i][0]) + F(a[1][k] * b[i][1])
            s = F(s + F(a[2][k] * b[i][2]))
            r[i][k] = F(s + F(a[3][k] * b[i][3]))
    return r


def translate(m, v):
    r = m.copy()
    for k in range(4):
        s = F(m[0][k] * v[0]) + F(m[1][k] * v[1])
        s = F(s + F(m[2][k] * v[2]))
        r[3][k] = F(s + m[3][k])
    return r


def scale_m(m, v):
    r = m.copy()
    for i in range(3):
        r[i] = m[i] * F(v[i])
    return r


def mat4_cast(q):  # q = (w, x, y, z) float32
    w, x, y, z = (F(t) for t in q)
    qxx, qyy, qzz = x * x, y * y, z * z
    qxz, qxy, qyz = x * z, x * y, y * z
    qwx, qwy, qwz = w * x, w * y, w * z
    one, two = F(1), F(2)
    r = ident()
    r[0][0] = one - two * (qyy + qzz)
    r[0][1] = two * (qxy + qwz)
    r[0][2] = two * (qxz - qwy)
    r[1][0] = two * (qxy - qwz)
    r[1][1] = one - two * (qxx + qzz)
    r[1][2] = two * (qyz + qwx)
    r[2][0] = two * (qxz + qwy)
    r[2][1] = two * (qyz - qwx)
    r[2][2] = one - two * (qxx + qyy)
    return r


def trs(t, q, s):
    return mat_mul(mat_mul(translate(ident(), t), mat4_cast(q)), scale_m(ident(), s))


def rotate(m, angle, v):
    a = F(angle)
    c, s = cosf(a), sinf(a)
    axis = normalize3(np.array(v, F))
    temp = (F(1) - c) * axis
    R = np.zeros((3, 3), F)
    R[0][0] = c + temp[0] * axis[0]
    R[0][1] = temp[0] * axis[1] + s * axis[2]
    R[0][2] = temp[0] * axis[2] - s * axis[1]
    R[1][0] = temp[1] * axis[0] - s * axis[2]
    R[1][1] = c + temp[1] * axis[1]
    R[1][2] = temp[1] * axis[2] + s * axis[0]
    R[2][0] = temp[2] * axis[0] + s * axis[1]
    R[2][1] = temp[2] * axis[1] - s * axis[0]
    R[2][2] = c + temp[2] * axis[2]
    r = np.zeros((4, 4), F)
    for i in range(3):
        r[i] = (m[0] * R[i][0] + m[1] * R[i][1]) + m[2] * R[i][2]
    r[3] = m[3]
    return r


def dot3(x, y, z):
    return F(F(x * x) + F(y * y)) + F(z * z) if np.isscalar(x) else (x * x + y * y) + z * z


def normalize3(v):  # single vec3 (float32 array)
    d = (F(v[0] * v[0]) + F(v[1] * v[1])) + F(v[2] * v[2])
    return v * (F(1) / np.sqrt(F(d)))


def inverse3(m):  # compute_inverse<3,3>
    m = m.astype(F)
    det = (m[0][0] * (m[1][1] * m[2][2] - m[2][1] * m[1][2])
           - m[1][0] * (m[0][1] * m[2][2] - m[2][1] * m[0][2])) + m[2][0] * (m[0][1] * m[1][2] - m[1][1] * m[0][2])
    ood = F(1) / det
    r = np.zeros((3, 3), F)
    r[0][0] = +(m[1][1] * m[2][2] - m[2][1] * m[1][2]) * ood
    r[1][0] = -(m[1][0] * m[2][2] - m[2][0] * m[1][2]) * ood
    r[2][0] = +(m[1][0] * m[2][1] - m[2][0] * m[1][1]) * ood
    r[0][1] = -(m[0][1] * m[2][2] - m[2][1] * m[0][2]) * ood
    r[1][1] = +(m[0][0] * m[2][2] - m[2][0] * m[0][2]) * ood
    r[2][1] = -(m[0][0] * m[2][1] - m[2][0] * m[0][1]) * ood
    r[0][2] = +(m[0][1] * m[1][2] - m[1][1] * m[0][2]) * ood
    r[1][2] = -(m[0][0] * m[1][2] - m[1][0] * m[0][2]) * ood
    r[2][2] = +(m[0][0] * m[1][1] - m[1][0] * m[0][1]) * ood
    return r


def inverse4_batch(m):
    """compute_inverse<4,4> on (N, 4, 4) float32 [col][row] matrices."""
    g = lambda c, r: m[:, c, r]  # noqa: E731
    c00 = g(2, 2) * g(3, 3) - g(3, 2) * g(2, 3)
    c02 = g(1, 2) * g(3, 3) - g(3, 2) * g(1, 3)
    c03 = g(1, 2) * g(2, 3) - g(2, 2) * g(1, 3)
    c04 = g(2, 1) * g(3, 3) - g(3, 1) * g(2, 3)
    c06 = g(1, 1) * g(3, 3) - g(3, 1) * g(1, 3)
    c07 = g(1, 1) * g(2, 3) - g(2, 1) * g(1, 3)
    c08 = g(2, 1) * g(3, 2) - g(3, 1) * g(2, 2)
    c10 = g(1, 1) * g(3, 2) - g(3, 1) * g(1, 2)
    c11 = g(1, 1) * g(2, 2) - g(2, 1) * g(1, 2)
    c12 = g(2, 0) * g(3, 3) - g(3, 0) * g(2, 3)
    c14 = g(1, 0) * g(3, 3) - g(3, 0) * g(1, 3)
    c15 = g(1, 0) * g(2, 3) - g(2, 0) * g(1, 3)
    c16 = g(2, 0) * g(3, 2) - g(3, 0) * g(2, 2)
    c18 = g(1, 0) * g(3, 2) - g(3, 0) * g(1, 2)
    c19 = g(1, 0) * g(2, 2) - g(2, 0) * g(1, 2)
    c20 = g(2, 0) * g(3, 1) - g(3, 0) * g(2, 1)
    c22 = g(1, 0) * g(3, 1) - g(3, 0) * g(1, 1)
    c23 = g(1, 0) * g(2, 1) - g(2, 0) * g(1, 1)
    st = lambda *a: np.stack(a, axis=1)  # noqa: E731
    fac0, fac1, fac2 = st(c00, c00, c02, c03), st(c04, c04, c06, c07), st(c08, c08, c10, c11)
    fac3, fac4, fac5 = st(c12, c12, c14, c15), st(c16, c16, c18, c19), st(c20, c20, c22, c23)
    vec0 = st(g(1, 0), g(0, 0), g(0, 0), g(0, 0))
    vec1 = st(g(1, 1), g(0, 1), g(0, 1), g(0, 1))
    vec2 = st(g(1, 2), g(0, 2), g(0, 2), g(0, 2))
    vec3 = st(g(1, 3), g(0, 3), g(0, 3), g(0, 3))
    inv0 = (vec1 * fac0 - vec2 * fac1) + vec3 * fac2
    inv1 = (vec0 * fac0 - vec2 * fac3) + vec3 * fac4
    inv2 = (vec0 * fac1 - vec1 * fac3) + vec3 * fac5
    inv3 = (vec0 * fac2 - vec1 * fac4) + vec2 * fac5
    sa = np.array([1, -1, 1, -1], F)
    sb = np.array([-1, 1, -1, 1], F)
    inv = np.stack([inv0 * sa, inv1 * sb, inv2 * sa, inv3 * sb], axis=1)  # [n, col, row]
    row0 = inv[:, :, 0]
    dot0 = m[:, 0, :] * row0
    dot1 = (dot0[:, 0] + dot0[:, 1]) + (dot0[:, 2] + dot0[:, 3])
    ood = F(1) / dot1
    return inv * ood[:, None, None]


def apply_point(M, x, y, z):
    """(M * vec4(p, 1)).xyz on arrays: (m0*x + m1*y) + (m2*z + m3*1)."""
    one = F(1)
    return [(M[0][k] * x + M[1][k] * y) + (M[2][k] * z + M[3][k] * one) for k in range(3)]


def apply_dir4(M, x, y, z, w):
    return [(M[0][k] * x + M[1][k] * y) + (M[2][k] * z + M[3][k] * w) for k in range(3)]


def apply3(M3, x, y, z):
    """mat3 * vec3: (m[0][k] x + m[1][k] y) + m[2][k] z."""
    return [(M3[0][k] * x + M3[1][k] * y) + M3[2][k] * z for k in range(3)]


def normalize_arr(x, y, z):
    d = (x * x + y * y) + z * z
    inv = F(1) / np.sqrt(d)
    return x * inv, y * inv, z * inv


def length3(x, y, z):
    return np.sqrt((x * x + y * y) + z * z)


def cross_arr(a, b):
    return (a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1])


# ----------------------------------------------------------------------------------------------
# layouts (GeneralHeaders.h; the same numpy dtypes the product exposes are rebuilt here)
# ----------------------------------------------------------------------------------------------
VERTEX = np.dtype([("pos", "<f4", 3), ("pad1", "<f4"), ("normal", "<f4", 3), ("pad2", "<f4"),
                   ("color", "<f4", 3), ("pad3", "<f4"), ("tangent", "<f4", 4), ("tex_coord", "<f4", 2),
                   ("tex_coord_1", "<f4", 2)])
MATERIAL = np.dtype([("base_color_factor", "<f4", 4), ("uv_normal", "<f4", 16), ("uv_emissive", "<f4", 16),
                     ("uv_albedo", "<f4", 16), ("emissive_factor_and_pad", "<f4", 4), ("metallic_factor", "<f4"),
                     ("roughness_factor", "<f4"), ("occlusion_strength", "<f4"), ("specular_factor", "<f4"),
                     ("specular_color_factor", "<f4", 3), ("alpha_cutoff", "<f4"), ("transmission_factor", "<f4"),
                     ("clearcoat_factor", "<f4"), ("clearcoat_roughness_factor", "<f4"), ("pad", "<f4"),
                     ("albedo_texture_index", "<i4"), ("normal_texture_index", "<i4"),
                     ("metallic_roughness_texture_index", "<i4"), ("emissive_texture_index", "<i4"),
                     ("occlusion_texture_index", "<i4"), ("clearcoat_texture_index", "<i4"),
                     ("clearcoat_roughness_texture_index", "<i4"), ("sg_id", "<i4"),
                     ("use_specular_glossiness_workflow", "<f4")])
PLIGHT = np.dtype([("position", "<f4", 3), ("intensity", "<f4"), ("color", "<f4", 3), ("range", "<f4"),
                   ("direction", "<f4", 3), ("outer_cone_cos", "<f4"), ("inner_cone_cos", "<f4"), ("type", "<i4"),
                   ("padding", "<f4", 2)])
assert VERTEX.itemsize == 80 and MATERIAL.itemsize == 308 and PLIGHT.itemsize == 64


def default_material():
    """Material{} (GeneralHeaders.h:202-235) in the MaterialPushConstant layout."""
    m = np.zeros((), MATERIAL)
    m["base_color_factor"] = 1.0
    eye = np.eye(4, dtype=F).reshape(16)
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


class GltfObject:
    """One Gameobject after loadModel (model space) — vertices/indices/prims/materials/lights/etris/textures."""

    def __init__(self):
        self.vertices = []
        self.indices = []
        self.prims = []       # (first_index, index_count, material_index)
        self.materials = []
        self.lights = []
        self.etris = []       # (i0, i1, i2, mat, area)
        self.textures = []    # (rgba (H, W, 4) uint8, srgb, exact)


# ----------------------------------------------------------------------------------------------
# images: PIL + stbi_load(..., 4) conventions
# ----------------------------------------------------------------------------------------------
def decode_image(data: bytes):
    """-> (rgba uint8 (H, W, 4), exact) ; exact = False for JPEG (libjpeg vs stb rounding)."""
    import io

    from PIL import Image
    im = Image.open(io.BytesIO(data))
    im.load()
    exact = im.format == "PNG"
    if im.mode in ("I;16", "I;16B", "I;16L", "I"):
        g = (np.asarray(im).astype(np.uint32) >> 8).astype(np.uint8)
        a = np.full(g.shape, 255, np.uint8)
        if "transparency" in im.info:
            a[np.asarray(im) == im.info["transparency"]] = 0
        return np.stack([g, g, g, a], axis=-1), exact
    return np.asarray(im.convert("RGBA")).copy(), exact


# ----------------------------------------------------------------------------------------------
# glTF
# ----------------------------------------------------------------------------------------------
def _load_uri(uri: str, base: str) -> bytes:
    if uri.startswith("data:"):
        return base64.b64decode(uri.split(",", 1)[1])
    p = os.path.join(base, uri)
    if not os.path.exists(p):
        p = os.path.join(base, urllib.parse.unquote(uri))
    with open(p, "rb") as f:
        return f.read()


def _read_glb(path):
    raw = open(path, "rb").read()
    assert raw[:4] == b"glTF"
    total = int.from_bytes(raw[8:12], "little")
    o, js, binc = 12, None, None
    while o + 8 <= total:
        n = int.from_bytes(raw[o:o + 4], "little")
        t = int.from_bytes(raw[o + 4:o + 8], "little")
        if t == 0x4E4F534A and js is None:
            js = json.loads(raw[o + 8:o + 8 + n])
        elif t == 0x004E4942 and binc is None:
            binc = raw[o + 8:o + 8 + n]
        o += 8 + ((n + 3) & ~3)
    return js, binc


_CSIZE = {5120: 1, 5121: 1, 5122: 2, 5123: 2, 5125: 4, 5126: 4}
_NCOMP = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4, "MAT2": 4, "MAT3": 9, "MAT4": 16}


class _Model:
    def __init__(self, path):
        self.base = os.path.dirname(path)
        if path.endswith(".glb"):
            self.j, binc = _read_glb(path)
        else:
            self.j, binc = json.load(open(path)), None
        self.buffers = []
        for i, b in enumerate(self.j.get("buffers", [])):
            self.buffers.append(binc if ("uri" not in b and binc is not None) else _load_uri(b["uri"], self.base))

    def accessor(self, ai, default_stride=0):
        """-> (bytes view starting at element 0, stride, count, componentType, accessor dict)"""
        a = self.j["accessors"][ai]
        bv = self.j["bufferViews"][a["bufferView"]]
        buf = self.buffers[bv["buffer"]]
        off = bv.get("byteOffset", 0) + a.get("byteOffset", 0)
        tight = _CSIZE[a["componentType"]] * _NCOMP[a["type"]]
        stride = bv.get("byteStride", 0) or default_stride or tight
        return memoryview(buf)[off:], stride, a["count"], a["componentType"], a

    def floats(self, ai, n, default_stride):
        mv, stride, count, ct, _ = self.accessor(ai, default_stride)
        out = np.zeros((count, n), F)
        for i in range(count):
            out[i] = np.frombuffer(mv[i * stride:i * stride + 4 * n], "<f4")
        return out


def _tex_source(m, ti):
    tex = m.j.get("textures", [])
    return tex[ti].get("source", -1) if 0 <= ti < len(tex) else -1


def _tex_id(m, ti):
    if ti is not None and 0 <= ti < len(m.j.get("textures", [])):
        s = _tex_source(m, ti)
        if 0 <= s < len(m.j.get("images", [])):
            return s + 1
    return 0


def _tex_transform(info):
    ext = (info or {}).get("extensions", {}).get("KHR_texture_transform")
    if ext is None:
        return None
    off = ext.get("offset", [0.0, 0.0])
    sc = ext.get("scale", [1.0, 1.0])
    rot = F(ext.get("rotation", 0.0))
    S = scale_m(ident(), [F(sc[0]), F(sc[1]), F(1)])
    R = rotate(ident(), -rot, [0.0, 0.0, 1.0])
    T = translate(ident(), [F(off[0]), F(off[1]), F(0)])
    return mat_mul(mat_mul(T, R), S).reshape(16)


def _materials(m):
    out = []
    for mt in m.j.get("materials", []):
        x = default_material()
        transparent = mt.get("alphaMode", "OPAQUE") == "BLEND"
        if mt.get("alphaMode") == "MASK":
            x["alpha_cutoff"] = F(mt.get("alphaCutoff", 0.5))
        ext = mt.get("extensions", {})
        pbr = mt.get("pbrMetallicRoughness", {})
        sg = ext.get("KHR_materials_pbrSpecularGlossiness")
        if sg is not None:
            x["use_specular_glossiness_workflow"] = 1.0
            x["base_color_factor"] = [F(t) for t in sg.get("diffuseFactor", [1.0, 1.0, 1.0, 1.0])]
            x["roughness_factor"] = F(sg.get("glossinessFactor", 1.0))
            if "diffuseTexture" in sg:
                x["albedo_texture_index"] = _tex_id(m, sg["diffuseTexture"].get("index"))
            if "specularGlossinessTexture" in sg:
                x["sg_id"] = _tex_id(m, sg["specularGlossinessTexture"].get("index"))
        else:
            x["base_color_factor"] = [F(t) for t in pbr.get("baseColorFactor", [1.0, 1.0, 1.0, 1.0])]
            x["metallic_factor"] = F(pbr.get("metallicFactor", 1.0))
            x["roughness_factor"] = F(pbr.get("roughnessFactor", 1.0))
            bct = pbr.get("baseColorTexture")
            x["albedo_texture_index"] = _tex_id(m, (bct or {}).get("index"))
            tt = _tex_transform(bct)
            if tt is not None:
                x["uv_albedo"] = tt
            x["metallic_roughness_texture_index"] = _tex_id(m, pbr.get("metallicRoughnessTexture", {}).get("index"))
        ef = np.array([F(t) for t in mt.get("emissiveFactor", [0.0, 0.0, 0.0])], F)
        es = ext.get("KHR_materials_emissive_strength")
        if es is not None and "emissiveStrength" in es:
            ef = ef * F(es["emissiveStrength"])
        x["emissive_factor_and_pad"] = [ef[0], ef[1], ef[2], 0.0]
        x["normal_texture_index"] = _tex_id(m, mt.get("normalTexture", {}).get("index"))
        x["occlusion_texture_index"] = _tex_id(m, mt.get("occlusionTexture", {}).get("index"))
        x["emissive_texture_index"] = _tex_id(m, mt.get("emissiveTexture", {}).get("index"))
        x["occlusion_strength"] = F(mt.get("occlusionTexture", {}).get("strength", 1.0))
        x["specular_color_factor"] = 1.0
        x["specular_factor"] = 0.5
        sp = ext.get("KHR_materials_specular")
        if sp is not None:
            if "specularFactor" in sp:
                x["specular_factor"] = F(sp["specularFactor"])
            c = sp.get("specularColorFactor")
            if isinstance(c, list) and len(c) >= 3:
                x["specular_color_factor"] = [F(t) for t in c[:3]]
        for key, field_name in (("normalTexture", "uv_normal"), ("emissiveTexture", "uv_emissive")):
            tt = _tex_transform(mt.get(key))
            if tt is not None:
                x[field_name] = tt
        tr = ext.get("KHR_materials_transmission")
        if tr is not None:
            if "transmissionFactor" in tr:
                x["transmission_factor"] = F(tr["transmissionFactor"])
            if x["transmission_factor"] > 0 or "transmissionTexture" in tr:
                transparent = True
        cc = ext.get("KHR_materials_clearcoat")
        if cc is not None:
            if "clearcoatFactor" in cc:
                x["clearcoat_factor"] = F(cc["clearcoatFactor"])
            if "clearcoatRoughnessFactor" in cc:
                x["clearcoat_roughness_factor"] = F(cc["clearcoatRoughnessFactor"])
            if "clearcoatTexture" in cc:
                x["clearcoat_texture_index"] = _tex_id(m, cc["clearcoatTexture"].get("index"))
            if "clearcoatRoughnessTexture" in cc:
                x["clearcoat_roughness_texture_index"] = _tex_id(m, cc["clearcoatRoughnessTexture"].get("index"))
        x["pad"] = 1.0 if transparent else 0.0
        out.append(x)
    if not out:
        out.append(default_material())
    return out


def _formats(m):
    f = {}

    def put(info, srgb):
        s = _tex_source(m, (info or {}).get("index", -1))
        if s >= 0:
            f[s] = srgb

    mats = m.j.get("materials", [])
    for mt in mats:
        pbr = mt.get("pbrMetallicRoughness", {})
        ext = mt.get("extensions", {})
        put(pbr.get("baseColorTexture"), 1)
        put(mt.get("emissiveTexture"), 1)
        put(mt.get("normalTexture"), 0)
        put(pbr.get("metallicRoughnessTexture"), 0)
        put(mt.get("occlusionTexture"), 0)
        tr = ext.get("KHR_materials_transmission", {})
        put(tr.get("transmissionTexture"), 0)
        cc = ext.get("KHR_materials_clearcoat", {})
        put(cc.get("clearcoatTexture"), 0)
        put(cc.get("clearcoatRoughnessTexture"), 0)
    for mt in mats:
        sg = mt.get("extensions", {}).get("KHR_materials_pbrSpecularGlossiness")
        if sg is not None:
            put(sg.get("specularGlossinessTexture"), 1)
            put(sg.get("diffuseTexture"), 1)
    return f


def _node_trs(n, anim=None):
    t = [F(v) for v in n["translation"]] if len(n.get("translation", [])) == 3 else [F(0)] * 3
    q = n.get("rotation", [])
    r = (F(q[3]), F(q[0]), F(q[1]), F(q[2])) if len(q) == 4 else (F(1), F(0), F(0), F(0))
    s = [F(v) for v in n["scale"]] if len(n.get("scale", [])) == 3 else [F(1)] * 3
    if anim:
        t = anim.get("t", t)
        r = anim.get("r", r)
        s = anim.get("s", s)
    return trs(t, r, s)


def _node_matrix(n):
    return np.array([F(v) for v in n["matrix"]], F).reshape(4, 4)


def _globals(m, scene_index):
    nodes = m.j.get("nodes", [])
    g = [ident() for _ in nodes]
    anims = {}
    if m.j.get("animations"):
        a = m.j["animations"][0]
        for ch in a.get("channels", []):
            node = ch.get("target", {}).get("node", -1)
            path = ch.get("target", {}).get("path", "")
            out_acc = a["samplers"][ch["sampler"]]["output"]
            if path == "translation":
                v = m.floats(out_acc, 3, 12)[0]
                anims.setdefault(node, {})["t"] = [v[0], v[1], v[2]]
            elif path == "rotation":
                v = m.floats(out_acc, 4, 16)[0]
                anims.setdefault(node, {})["r"] = (v[3], v[0], v[1], v[2])
            elif path == "scale":
                v = m.floats(out_acc, 3, 12)[0]
                anims.setdefault(node, {})["s"] = [v[0], v[1], v[2]]

    def walk(ni, parent):
        n = nodes[ni]
        if len(n.get("matrix", [])) == 16:
            local = _node_matrix(n) if ni not in anims else ident()
        else:
            local = _node_trs(n, anims.get(ni))
        gm = mat_mul(parent, local)
        g[ni] = gm
        for c in n.get("children", []):
            walk(c, gm)

    for r in m.j["scenes"][scene_index].get("nodes", []):
        walk(r, ident())
    return g


def _lights(m, g):
    lights = m.j.get("extensions", {}).get("KHR_lights_punctual", {}).get("lights", [])
    out = []
    for i, n in enumerate(m.j.get("nodes", [])):
        li = n.get("extensions", {}).get("KHR_lights_punctual", {}).get("light", None)
        if li is None or not (0 <= li < len(lights)):
            continue
        L = lights[li]
        x = np.zeros((), PLIGHT)
        T = g[i]
        x["position"] = T[3][:3]
        d = apply_dir4(T, F(0), F(0), F(-1), F(0))
        x["direction"] = normalize3(np.array(d, F))
        x["color"] = [F(c) for c in L["color"]] if L.get("color") else [1.0, 1.0, 1.0]
        x["intensity"] = F(L.get("intensity", 1.0))
        x["range"] = F(L.get("range", 0.0))
        t = L.get("type", "")
        if t == "directional":
            x["type"] = 1
        elif t == "spot":
            x["type"] = 2
            sp = L.get("spot", {})
            x["inner_cone_cos"] = F(math.cos(sp.get("innerConeAngle", 0.0)))
            x["outer_cone_cos"] = F(math.cos(sp.get("outerConeAngle", 0.7853981634)))
        out.append(x)
    return out


def load_gltf(path: str, missing_images_white: bool = False) -> GltfObject:
    """Gameobject::loadModel (model-space object, before the scene bake)."""
    m = _Model(path)
    si = m.j.get("scene", -1)
    si = si if si > -1 else 0
    g = _globals(m, si)
    obj = GltfObject()
    obj.lights = _lights(m, g)
    skin = []
    if m.j.get("skins"):
        sk = m.j["skins"][0]
        skin = [ident() for _ in sk["joints"]]
        if sk.get("inverseBindMatrices", -1) > -1:
            ibm = m.floats(sk["inverseBindMatrices"], 16, 64)
            for i, jn in enumerate(sk["joints"]):
                skin[i] = mat_mul(g[jn], ibm[i].reshape(4, 4))
    fm = _formats(m)
    obj.textures.append((np.array([[[255, 255, 255, 255]]], np.uint8), True, True))
    for i, im in enumerate(m.j.get("images", [])):
        try:
            if "uri" in im:
                data = _load_uri(im["uri"], m.base)
            else:
                bv = m.j["bufferViews"][im["bufferView"]]
                o = bv.get("byteOffset", 0)
                data = bytes(m.buffers[bv["buffer"]][o:o + bv["byteLength"]])
            rgba, exact = decode_image(data)
        except (OSError, KeyError):
            if not missing_images_white:
                raise
            rgba, exact = np.array([[[255, 255, 255, 255]]], np.uint8), True
        obj.textures.append((rgba, bool(fm.get(i, 1)), exact))
    obj.materials = _materials(m)
    uniq = {}

    def primitive(prim, T):
        mi = prim.get("material", -1)
        mi = mi if mi >= 0 else 0
        e = obj.materials[mi]["emissive_factor_and_pad"]
        emissive = length3(F(e[0]), F(e[1]), F(e[2])) > F(0.001)
        at = prim["attributes"]
        if "indices" in prim:
            mv, stride, count, ct, _ = m.accessor(prim["indices"], {5123: 2, 5125: 4}.get(
                m.j["accessors"][prim["indices"]]["componentType"], 1))
            dt = {5123: "<u2", 5125: "<u4"}.get(ct, "u1")
            idx = np.frombuffer(mv[:count * np.dtype(dt).itemsize], dt).astype(np.int64)
        else:
            idx = np.arange(m.j["accessors"][at["POSITION"]]["count"])
        n = len(idx)
        pos = m.floats(at["POSITION"], 3, 12)[idx]
        nrm = m.floats(at["NORMAL"], 3, 12)[idx] if "NORMAL" in at else np.tile(np.array([0, 1, 0], F), (n, 1))
        tan = m.floats(at["TANGENT"], 4, 16)[idx] if "TANGENT" in at else np.tile(np.array([1, 0, 0, 0], F), (n, 1))
        uv0 = m.floats(at["TEXCOORD_0"], 2, 8)[idx] if "TEXCOORD_0" in at else np.zeros((n, 2), F)
        uv1 = m.floats(at["TEXCOORD_1"], 2, 8)[idx] if "TEXCOORD_1" in at else uv0.copy()
        has_skin = bool(skin) and "JOINTS_0" in at and "WEIGHTS_0" in at
        x, y, z = pos[:, 0], pos[:, 1], pos[:, 2]
        nx, ny, nz = nrm[:, 0], nrm[:, 1], nrm[:, 2]
        tx, ty, tz = tan[:, 0], tan[:, 1], tan[:, 2]
        tw = tan[:, 3]
        if has_skin:
            jmv, js, jc, jct, _ = m.accessor(at["JOINTS_0"])
            jd = "<u2" if jct == 5123 else "u1"
            J = np.array([np.frombuffer(jmv[i * js:i * js + 4 * np.dtype(jd).itemsize], jd) for i in idx], np.int64)
            wmv, ws, wc, wct, _ = m.accessor(at["WEIGHTS_0"])
            if wct == 5126:
                W = np.array([np.frombuffer(wmv[i * ws:i * ws + 16], "<f4") for i in idx], F)
            else:
                W = np.tile(np.array([1, 0, 0, 0], F), (n, 1))
            s = ((W[:, 0] + W[:, 1]) + W[:, 2]) + W[:, 3]
            ok = s > 0
            W = np.where(ok[:, None], W / np.where(ok, s, F(1))[:, None], np.array([1, 0, 0, 0], F))
            SK = np.stack(skin).astype(F)
            S = ((SK[J[:, 0]] * W[:, 0, None, None] + SK[J[:, 1]] * W[:, 1, None, None])
                 + SK[J[:, 2]] * W[:, 2, None, None]) + SK[J[:, 3]] * W[:, 3, None, None]
            one = F(1)
            px = [(S[:, 0, k] * x + S[:, 1, k] * y) + (S[:, 2, k] * z + S[:, 3, k] * one) for k in range(3)]
            Inv = inverse4_batch(S)
            # mat3(transpose(inverse(S))) * n : element [c][r] of the transpose = Inv[r][c]
            nn = [(Inv[:, k, 0] * nx + Inv[:, k, 1] * ny) + Inv[:, k, 2] * nz for k in range(3)]
            nn = normalize_arr(*nn)
            tt = [(S[:, 0, k] * tx + S[:, 1, k] * ty) + S[:, 2, k] * tz for k in range(3)]
            tt = normalize_arr(*tt)
        else:
            px = apply_point(T, x, y, z)
            NM = inverse3(T[:3, :3]).T
            nn = normalize_arr(*apply3(NM, nx, ny, nz))
            tt = normalize_arr(*apply3(T[:3, :3], tx, ty, tz))
        use_t = tw != 0
        tx2 = np.where(use_t, tt[0], tx)
        ty2 = np.where(use_t, tt[1], ty)
        tz2 = np.where(use_t, tt[2], tz)
        local = []
        for i in range(n):
            v = np.zeros((), VERTEX)
            v["pos"] = [px[0][i], px[1][i], px[2][i]]
            v["normal"] = [nn[0][i], nn[1][i], nn[2][i]]
            v["color"] = 1.0
            v["tangent"] = [tx2[i], ty2[i], tz2[i], tw[i]]
            v["tex_coord"] = uv0[i]
            v["tex_coord_1"] = uv1[i]
            key = tuple(float(t) for t in (*v["pos"], *v["color"], *v["tex_coord"], *v["tangent"], *v["normal"]))
            if key in uniq:
                local.append(uniq[key])
                continue
            obj.vertices.append(v)
            if any(t != t for t in key):
                local.append(0)
            else:
                uniq[key] = len(obj.vertices) - 1
                local.append(len(obj.vertices) - 1)
        first = len(obj.indices)
        obj.indices += local
        for k in range(0, len(local) - 2, 3):
            i0, i1, i2 = local[k], local[k + 1], local[k + 2]
            obj.indices += [i0, i1, i2]
            if emissive:
                p = [obj.vertices[i]["pos"].astype(F) for i in (i0, i1, i2)]
                c = cross_arr(p[1] - p[0], p[2] - p[0])
                area = F(0.5) * length3(F(c[0]), F(c[1]), F(c[2]))
                if area > F(1e-6):
                    obj.etris.append((i0, i1, i2, mi, area))
        obj.prims.append((first, n, mi))

    nodes = m.j.get("nodes", [])

    def node(ni, parent):
        n = nodes[ni]
        local = mat_mul(parent, _node_matrix(n) if len(n.get("matrix", [])) == 16 else _node_trs(n))
        T = parent if n.get("skin", -1) >= 0 else local
        if n.get("mesh", -1) >= 0:
            for prim in m.j["meshes"][n["mesh"]]["primitives"]:
                primitive(prim, T)
        for c in n.get("children", []):
            node(c, local)

    for r in m.j["scenes"][si].get("nodes", []):
        node(r, ident())
    return obj


def bake(obj: GltfObject, position=(0, 0, 0), rotation_deg=(0, 0, 0), scale=(1, 1, 1)):
    """Engine::loadScene STEP 1-3 (engine.cpp:1271-1331)."""
    k = F(0.01745329251994329576923690768489)
    e = [F(r) * k for r in rotation_deg]
    half = F(0.5)
    cx, cy, cz = (cosf(t * half) for t in e)
    sx, sy, sz = (sinf(t * half) for t in e)
    q = ((cx * cy) * cz + (sx * sy) * sz, (sx * cy) * cz - (cx * sy) * sz,
         (cx * sy) * cz + (sx * cy) * sz, (cx * cy) * sz - (sx * sy) * cz)
    T = trs([F(t) for t in position], q, [F(t) for t in scale])
    NM = inverse3(T[:3, :3]).T
    if obj.vertices:
        V = np.array(obj.vertices, VERTEX)
        p = apply_point(T, V["pos"][:, 0], V["pos"][:, 1], V["pos"][:, 2])
        n = normalize_arr(*apply3(NM, V["normal"][:, 0], V["normal"][:, 1], V["normal"][:, 2]))
        t = normalize_arr(*apply3(T[:3, :3], V["tangent"][:, 0], V["tangent"][:, 1], V["tangent"][:, 2]))
        V["pos"] = np.stack(p, 1)
        V["normal"] = np.stack(n, 1)
        V["tangent"][:, :3] = np.stack(t, 1)
        obj.vertices = list(V)
    sf = length3(T[0][0], T[0][1], T[0][2])
    for L in obj.lights:
        p = apply_point(T, L["position"][0], L["position"][1], L["position"][2])
        d = normalize3(np.array(apply3(NM, L["direction"][0], L["direction"][1], L["direction"][2]), F))
        L["position"] = p
        L["direction"] = d
        if L["range"] > 0:
            L["range"] = F(L["range"]) * sf
        L["intensity"] = F(L["intensity"]) * (sf * sf)
    et = []
    for (i0, i1, i2, mi, _) in obj.etris:
        p = [obj.vertices[i]["pos"].astype(F) for i in (i0, i1, i2)]
        c = cross_arr(p[1] - p[0], p[2] - p[0])
        et.append((i0, i1, i2, mi, F(0.5) * length3(F(c[0]), F(c[1]), F(c[2]))))
    obj.etris = et
    return obj


def rtbox(path: str) -> GltfObject:
    """Engine::createRTBox (engine.cpp:181-335)."""
    cfg = json.load(open(path))
    pos = [F(v) for v in cfg["position"]]
    dim = [F(v) for v in cfg["dimensions"]]
    w, h, d = dim[0] / F(2), dim[1], dim[2] / F(2)
    yb, yt = pos[1], pos[1] + h
    X0, X1, Z0, Z1 = pos[0] - w, pos[0] + w, pos[2] - d, pos[2] + d
    P = [(X0, yb, Z0), (X1, yb, Z0), (X1, yb, Z1), (X0, yb, Z1), (X0, yt, Z0), (X1, yt, Z0), (X1, yt, Z1), (X0, yt, Z1),
         (X0, yb, Z0), (X1, yb, Z0), (X1, yt, Z0), (X0, yt, Z0), (X0, yb, Z1), (X0, yb, Z0), (X0, yt, Z0), (X0, yt, Z1),
         (X1, yb, Z0), (X1, yb, Z1), (X1, yt, Z1), (X1, yt, Z0), (X0, yb, Z1), (X1, yb, Z1), (X1, yt, Z1), (X0, yt, Z1)]
    N = [(0, 1, 0), (0, -1, 0), (0, 0, 1), (1, 0, 0), (-1, 0, 0), (0, 0, -1)]
    o = GltfObject()
    for i in range(24):
        v = np.zeros((), VERTEX)
        v["pos"] = P[i]
        v["normal"] = N[i // 4]
        v["color"] = 1.0
        v["tangent"] = [1, 0, 0, 0]
        o.vertices.append(v)
    o.indices = [0, 3, 2, 2, 1, 0, 4, 5, 6, 6, 7, 4, 8, 9, 10, 10, 11, 8,
                 12, 13, 14, 14, 15, 12, 16, 17, 18, 18, 19, 16, 20, 21, 22, 22, 23, 20]
    for i, name in enumerate(["floor", "ceiling", "back_wall", "left_wall", "right_wall", "front_wall"]):
        panel = cfg["panels"][name]
        mt = panel["material"]
        x = default_material()
        bc = [F(c) for c in mt["base_color"]]
        x["base_color_factor"] = [bc[0], bc[1], bc[2], 1.0]
        x["metallic_factor"] = F(mt.get("metallic", 0.0))
        x["roughness_factor"] = F(mt.get("roughness", 1.0))
        inten = F(panel.get("light", {}).get("intensity", 0.0))
        x["emissive_factor_and_pad"] = [bc[0] * inten, bc[1] * inten, bc[2] * inten, 0.0]
        o.materials.append(x)
        o.prims.append((i * 6, 6, i))
    for k in range(0, 36, 3):
        mi = k // 6
        e = o.materials[mi]["emissive_factor_and_pad"]
        if length3(F(e[0]), F(e[1]), F(e[2])) < F(0.00001):
            continue
        i0, i1, i2 = o.indices[k:k + 3]
        p = [o.vertices[i]["pos"].astype(F) for i in (i0, i1, i2)]
        c = cross_arr(p[1] - p[0], p[2] - p[0])
        o.etris.append((i0, i1, i2, mi, F(0.5) * length3(F(c[0]), F(c[1]), F(c[2]))))
    o.textures = [(np.array([[[125, 125, 125, 255]]], np.uint8), True, True)]
    return o


def flatten(objects, rt=None, suns=()):
    """createGlobalBindlessBuffers (engine.cpp:1658-1860) -> dict of arrays + fluxes."""
    allobj = list(objects) + ([rt] if rt is not None else [])
    V, I, meshes, counts, mats, ltris, flux, plights, textures = [], [], [], [], [], [], [], list(suns), []
    emit_tex = any(len(o.textures) for o in objects)
    tex_off = 0
    for o in allobj:
        if not o.vertices:
            continue
        voff, ioff, moff = len(V), len(I), len(mats)
        V += list(o.vertices)
        I += list(o.indices)
        for x in o.materials:
            y = x.copy()
            for f in ("albedo_texture_index", "normal_texture_index", "metallic_roughness_texture_index",
                      "emissive_texture_index", "occlusion_texture_index", "clearcoat_texture_index",
                      "clearcoat_roughness_texture_index", "sg_id"):
                y[f] = int(y[f]) + tex_off
            mats.append(y)
        for (first, count, mi) in o.prims:
            meshes.append((moff + mi, voff, ioff + first, 0))
            counts.append(count)
        for (i0, i1, i2, mi, area) in o.etris:
            ltris.append((voff + i0, voff + i1, voff + i2, moff + mi))
            e = o.materials[mi]["emissive_factor_and_pad"]
            flux.append(F(area) * length3(F(e[0]), F(e[1]), F(e[2])))
        plights += [L for L in o.lights if L["intensity"] > 0]
        if emit_tex:
            textures += [(t[0], t[1], t[2]) for t in o.textures]
        tex_off += max(len(o.textures), 1)
    emissive_flux = F(0)
    cdf = []
    if ltris:
        for f in flux:
            emissive_flux = F(emissive_flux + f)
        run = F(0)
        for i, f in enumerate(flux):
            run = F(run + f)
            cdf.append((F(run / emissive_flux) if emissive_flux > 0 else F(0), i))
        cdf[-1] = (F(1), cdf[-1][1])
    else:
        ltris = [(0, 0, 0, 0)]
        cdf = [(F(1), 0)]
    punctual = F(0)
    pcdf = []
    if plights:
        pf = [F(L["intensity"]) * F(400.0) if L["type"] == 1 else F(L["intensity"]) * F(12.566) for L in plights]
        for f in pf:
            punctual = F(punctual + f)
        run = F(0)
        for i, f in enumerate(pf):
            run = F(run + f)
            pcdf.append((F(run / punctual) if punctual > 0 else F(0), i))
    else:
        plights = [np.zeros((), PLIGHT)]
        pcdf = [(F(1), 0)]
    total = F(emissive_flux + punctual)
    p_em = F(0)
    if emissive_flux > 0 and punctual > 0:
        p = F(emissive_flux / total)
        p_em = F(min(max(p, F(0.1)), F(0.9)))
    return dict(vertices=np.array(V, VERTEX), indices=np.array(I, np.uint32),
                meshes=np.array(meshes, np.uint32).reshape(-1, 4), mesh_index_count=np.array(counts, np.uint32),
                materials=np.array(mats, MATERIAL), light_triangles=np.array(ltris, np.uint32).reshape(-1, 4),
                light_cdf=cdf, punctual_lights=np.array(plights, PLIGHT), punctual_cdf=pcdf,
                emissive_flux=emissive_flux, punctual_flux=punctual, total_flux=total, p_emissive=p_em,
                textures=textures)


def load_scene_json(path: str, root_dir: str = "", missing_images_white: bool = False):
    """Engine::loadScene -> (flatten(...) dict, settings dict)."""
    j = json.load(open(os.path.join(root_dir, path)))
    if "scene" in j and "objects" not in j and "settings" not in j:
        j = json.load(open(os.path.join(root_dir, j["scene"])))
    st = j.get("settings", {})
    settings = dict(ambient_light=st.get("ambient_light", [0.0, 0.0, 0.0, 1.0]), use_rt_box=st.get("use_rt_box", False),
                    accumulation_steps=st.get("accumulation_steps", 512), total_positions=st.get("total_positions", 336),
                    min_beta=st.get("min_beta", -45.0), max_beta=st.get("max_beta", 45.0),
                    image_divisor=st.get("image_divisor", 2.0), use_lod=st.get("use_lod", 0.0),
                    lod_factor=st.get("lod_factor", 1.0))
    ts = st.get("torus_settings", {})
    settings.update(torus_major_radius=ts.get("major_radius", 16.0), torus_minor_radius=ts.get("minor_radius", 1.0),
                    torus_height=ts.get("height", 8.0), num_rays=ts.get("num_rays", 1000000))
    suns = []
    if "sun" in st:
        s = st["sun"]
        L = np.zeros((), PLIGHT)
        L["color"] = s["color"]
        L["direction"] = s["direction"]
        L["intensity"] = F(s.get("intensity", 1.0))
        L["type"] = 1
        suns.append(L)
    objs = []
    for od in j.get("objects", []):
        o = load_gltf(os.path.join(root_dir, od["model"]), missing_images_white)
        objs.append(bake(o, od.get("position", [0, 0, 0]), od.get("rotation", [0, 0, 0]), od.get("scale", [1, 1, 1])))
    rt = None
    if st.get("use_rt_box", False) and st.get("rt_box_file"):
        rt = rtbox(os.path.join(root_dir, st["rt_box_file"]))
    return flatten(objs, rt, suns), settings
