"""Generate the scene-ingest fixtures in this directory (run: python tests/golden/ingest/make_fixtures.py).

Everything here is synthetic (the reference's own assets are mostly missing blobs and too large to
commit): small PNG / JPEG textures covering the decoder's formats, a glTF 2.0 model exercising every
branch of Gameobject::loadModel the reference has (node hierarchy with matrix and TRS nodes, frame-0
animation, a skin, the KHR material extensions, texture transforms, punctual lights, u8/u16/u32
indices, interleaved and default attributes, duplicated vertices), the same model as .glb, a second
model with a data: URI buffer, an rt-box JSON and a scene JSON tying them together.
Deterministic: re-running reproduces the committed bytes.
"""
from __future__ import annotations

import base64
import io
import json
import math
import os
import struct
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
RNG = np.random.default_rng(20240611)


# ------------------------------------------------------------------ PNG writer (own, so every colour
# type / bit depth / interlace / tRNS combination can be produced; expected stb output is computed
# from the source samples in tests/test_ingest.py)
def _chunk(tag: bytes, body: bytes) -> bytes:
    return struct.pack(">I", len(body)) + tag + body + struct.pack(">I", zlib.crc32(tag + body) & 0xFFFFFFFF)


def _pack_row(samples: np.ndarray, depth: int) -> bytes:
    s = samples.astype(np.uint32).ravel()
    if depth == 16:
        return s.astype(">u2").tobytes()
    if depth == 8:
        return s.astype(np.uint8).tobytes()
    per = 8 // depth
    out = bytearray((len(s) * depth + 7) // 8)
    for i, v in enumerate(s):
        out[i // per] |= int(v) << (8 - depth - (i % per) * depth)
    return bytes(out)


def _filter_rows(rows: list[bytes], bpp: int, rng) -> bytes:
    """Apply a pseudo-random filter type per row (exercises all five unfilters)."""
    out = bytearray()
    prev = bytes(len(rows[0])) if rows else b""
    for r in rows:
        f = int(rng.integers(0, 5))
        cur = bytearray(len(r))
        for i in range(len(r)):
            a = r[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            if f == 0:
                p = 0
            elif f == 1:
                p = a
            elif f == 2:
                p = b
            elif f == 3:
                p = (a + b) >> 1
            else:
                pp = a + b - c
                pa, pb, pc = abs(pp - a), abs(pp - b), abs(pp - c)
                p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            cur[i] = (r[i] - p) & 255
        out.append(f)
        out += cur
        prev = r
    return bytes(out)


def write_png(path, samples: np.ndarray, color: int, depth: int, interlace: bool = False, palette=None, trns=None):
    """samples: (H, W, C) integer array at the file's bit depth."""
    h, w, c = samples.shape
    ihdr = struct.pack(">IIBBBBB", w, h, depth, color, 0, 0, 1 if interlace else 0)
    bpp = max(1, c * depth // 8)
    rng = np.random.default_rng(w * 1000 + h * 10 + color + depth)
    raw = b""
    passes = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)] \
        if interlace else [(0, 0, 1, 1)]
    for x0, y0, dx, dy in passes:
        sub = samples[y0::dy, x0::dx]
        if sub.size == 0:
            continue
        rows = [_pack_row(sub[j], depth) for j in range(sub.shape[0])]
        raw += _filter_rows(rows, bpp, rng)
    data = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr)
    if palette is not None:
        data += _chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).ravel()))
    if trns is not None:
        data += _chunk(b"tRNS", trns)
    data += _chunk(b"tEXt", b"Comment\x00ptgs ingest fixture")  # ancillary chunk: skipped
    comp = zlib.compress(raw, 9)
    data += _chunk(b"IDAT", comp[: len(comp) // 2]) + _chunk(b"IDAT", comp[len(comp) // 2:])  # split IDAT
    data += _chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(data)


def smooth_rgb(w, h, seed):
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    r = np.random.default_rng(seed)
    ph = r.uniform(0, 6.28, 3)
    img = np.stack([127 + 110 * np.sin(x * 0.37 + ph[0]) * np.cos(y * 0.21),
                    127 + 110 * np.cos(x * 0.19 - y * 0.31 + ph[1]),
                    127 + 100 * np.sin((x + y) * 0.25 + ph[2])], -1)
    return np.clip(img + r.normal(0, 6, img.shape), 0, 255).astype(np.uint8)


IMAGES = {}  # name -> dict(kind, expected stb RGBA uint8 (H, W, 4) or None for JPEG)


def make_images():
    d = os.path.join(HERE, "images")
    os.makedirs(d, exist_ok=True)

    def reg(name, expected):
        IMAGES[name] = expected

    # RGBA8, odd size, all filters
    a = RNG.integers(0, 256, (13, 17, 4)).astype(np.uint8)
    write_png(os.path.join(d, "rgba8.png"), a, 6, 8)
    reg("rgba8.png", a)
    # RGB8 with a tRNS key (8-bit key = low byte of the 16-bit field)
    rgb = RNG.integers(0, 4, (11, 9, 3)).astype(np.uint8) * 60
    key = (60, 0, 120)
    write_png(os.path.join(d, "rgb8_trns.png"), rgb, 2, 8, trns=struct.pack(">HHH", *key))
    exp = np.concatenate([rgb, np.full(rgb.shape[:2] + (1,), 255, np.uint8)], -1)
    exp[(rgb == np.array(key, np.uint8)).all(-1), 3] = 0
    reg("rgb8_trns.png", exp)
    # palette 4-bit with partial tRNS
    pal = RNG.integers(0, 256, (12, 3)).astype(np.uint8)
    idx = RNG.integers(0, 12, (10, 15, 1)).astype(np.uint8)
    alpha = bytes([0, 128, 255, 7])
    write_png(os.path.join(d, "pal4_trns.png"), idx, 3, 4, palette=pal, trns=alpha)
    palA = np.concatenate([pal, np.full((12, 1), 255, np.uint8)], -1)
    palA[:4, 3] = np.frombuffer(alpha, np.uint8)
    reg("pal4_trns.png", palA[idx[..., 0]])
    # grey 1/2/4-bit (scaled by 0xff / 0x55 / 0x11)
    for depth, scale in ((1, 0xFF), (2, 0x55), (4, 0x11)):
        g = RNG.integers(0, 1 << depth, (9, 19, 1)).astype(np.uint8)
        write_png(os.path.join(d, f"grey{depth}.png"), g, 0, depth)
        v = (g[..., 0].astype(np.int32) * scale).astype(np.uint8)
        reg(f"grey{depth}.png", np.stack([v, v, v, np.full_like(v, 255)], -1))
    # grey 8 + alpha, Adam7 interlaced
    ga = RNG.integers(0, 256, (21, 19, 2)).astype(np.uint8)
    write_png(os.path.join(d, "greya8_adam7.png"), ga, 4, 8, interlace=True)
    reg("greya8_adam7.png", np.stack([ga[..., 0], ga[..., 0], ga[..., 0], ga[..., 1]], -1))
    # RGB 16-bit, interlaced, with a 16-bit key
    r16 = RNG.integers(0, 4, (7, 6, 3)).astype(np.uint16) * 16000 + 7
    k16 = (16007, 7, 32007)
    write_png(os.path.join(d, "rgb16_adam7_trns.png"), r16, 2, 16, interlace=True, trns=struct.pack(">HHH", *k16))
    e = np.concatenate([(r16 >> 8).astype(np.uint8), np.full(r16.shape[:2] + (1,), 255, np.uint8)], -1)
    e[(r16 == np.array(k16, np.uint16)).all(-1), 3] = 0
    reg("rgb16_adam7_trns.png", e)
    # grey 16
    g16 = RNG.integers(0, 65536, (5, 8, 1)).astype(np.uint16)
    write_png(os.path.join(d, "grey16.png"), g16, 0, 16)
    v = (g16[..., 0] >> 8).astype(np.uint8)
    reg("grey16.png", np.stack([v, v, v, np.full_like(v, 255)], -1))

    # JPEG: expected values come from the decoder under test vs PIL within a tolerance
    from PIL import Image
    base = smooth_rgb(37, 29, 1)
    for name, kw in (("q90_444.jpg", dict(quality=90, subsampling=0)),
                     ("q75_422.jpg", dict(quality=75, subsampling=1)),
                     ("q80_420.jpg", dict(quality=80, subsampling=2)),
                     ("q85_420_prog.jpg", dict(quality=85, subsampling=2, progressive=True)),
                     ("q85_444_prog.jpg", dict(quality=85, subsampling=0, progressive=True)),
                     ("q70_420_restart.jpg", dict(quality=70, subsampling=2, restart_marker_blocks=3))):
        Image.fromarray(base).save(os.path.join(d, name), "JPEG", **kw)
        reg(name, None)
    Image.fromarray(base[..., 1]).save(os.path.join(d, "grey_q85.jpg"), "JPEG", quality=85)
    reg("grey_q85.jpg", None)
    Image.fromarray(smooth_rgb(1, 1, 3)).save(os.path.join(d, "one_pixel.jpg"), "JPEG", quality=95)
    reg("one_pixel.jpg", None)
    # the glTF textures
    Image.fromarray(smooth_rgb(16, 16, 5)).save(os.path.join(d, "albedo.jpg"), "JPEG", quality=90, subsampling=2)
    Image.fromarray(smooth_rgb(12, 8, 6)).save(os.path.join(d, "emissive.jpg"), "JPEG", quality=90, subsampling=0)
    n = np.zeros((8, 8, 3), np.uint8)
    n[..., 0], n[..., 1], n[..., 2] = 128 + RNG.integers(-20, 20, (8, 8)), 128 + RNG.integers(-20, 20, (8, 8)), 230
    write_png(os.path.join(d, "normal.png"), n, 2, 8)
    mr = RNG.integers(0, 256, (8, 8, 3)).astype(np.uint8)
    write_png(os.path.join(d, "metal_rough.png"), mr, 2, 8)
    write_png(os.path.join(d, "sg.png"), RNG.integers(0, 256, (4, 4, 4)).astype(np.uint8), 6, 8)
    write_png(os.path.join(d, "cutout.png"), RNG.integers(0, 256, (8, 8, 2)).astype(np.uint8), 4, 8)


# ------------------------------------------------------------------ glTF builder
class Gltf:
    def __init__(self):
        self.j = {"asset": {"version": "2.0", "generator": "ptgs ingest fixture"}, "buffers": [], "bufferViews": [],
                  "accessors": [], "meshes": [], "nodes": [], "materials": [], "textures": [], "images": [],
                  "samplers": [{}]}
        self.bin = bytearray()

    def _align(self, n=4):
        while len(self.bin) % n:
            self.bin.append(0)

    def view(self, data: bytes, stride: int = 0, target: int | None = None) -> int:
        self._align(4)
        bv = {"buffer": 0, "byteOffset": len(self.bin), "byteLength": len(data)}
        if stride:
            bv["byteStride"] = stride
        if target:
            bv["target"] = target
        self.bin += data
        self.j["bufferViews"].append(bv)
        return len(self.j["bufferViews"]) - 1

    def accessor(self, bv: int, ctype: int, count: int, typ: str, offset: int = 0, minmax=None) -> int:
        a = {"bufferView": bv, "componentType": ctype, "count": count, "type": typ}
        if offset:
            a["byteOffset"] = offset
        if minmax is not None:
            a["min"], a["max"] = minmax
        self.j["accessors"].append(a)
        return len(self.j["accessors"]) - 1

    def floats(self, arr, typ) -> int:
        arr = np.ascontiguousarray(arr, "<f4")
        return self.accessor(self.view(arr.tobytes()), 5126, arr.shape[0], typ)

    def image(self, uri) -> int:
        self.j["images"].append({"uri": uri})
        self.j["textures"].append({"sampler": 0, "source": len(self.j["images"]) - 1})
        return len(self.j["textures"]) - 1


def box_geometry():
    P, N, T, UV = [], [], [], []
    faces = [((0, 0, 1), (1, 0, 0)), ((0, 0, -1), (-1, 0, 0)), ((1, 0, 0), (0, 0, -1)),
             ((-1, 0, 0), (0, 0, 1)), ((0, 1, 0), (1, 0, 0)), ((0, -1, 0), (1, 0, 0))]
    idx = []
    for f, (n, t) in enumerate(faces):
        n, t = np.array(n, float), np.array(t, float)
        b = np.cross(n, t)
        base = len(P)
        for (u, v) in ((0, 0), (1, 0), (1, 1), (0, 1)):
            p = n * 0.5 + t * (u - 0.5) + b * (v - 0.5)
            P.append(p)
            N.append(n)
            T.append(list(t) + [1.0 if f % 2 == 0 else -1.0])
            UV.append((u * 1.5 - 0.25, v * 2.0))
        idx += [base, base + 1, base + 2, base, base + 2, base + 3]
    return np.array(P), np.array(N), np.array(T), np.array(UV), np.array(idx)


def quat(axis, angle):
    a = np.array(axis, float)
    a /= np.linalg.norm(a)
    s = math.sin(angle / 2)
    return [a[0] * s, a[1] * s, a[2] * s, math.cos(angle / 2)]


def make_features(g: Gltf):
    t_alb = g.image("images/albedo.jpg")
    t_nrm = g.image("images/normal.png")
    t_mr = g.image("images/metal_rough.png")
    t_em = g.image("images/emissive.jpg")
    t_sg = g.image("images/sg.png")
    t_cut = g.image("images/cutout.png")
    # an image only referenced as clearcoat (UNORM) and one unreferenced image (stays sRGB)
    t_cc = g.image("images/q75_422.jpg")
    g.j["images"].append({"uri": "images/grey4.png"})
    tt = {"KHR_texture_transform": {"offset": [0.25, -0.5], "scale": [2.0, 0.5], "rotation": 0.3}}
    M = g.j["materials"]
    M.append({"name": "metal_rough_textured",
              "pbrMetallicRoughness": {"baseColorFactor": [0.9, 0.8, 0.7, 1.0], "metallicFactor": 0.3,
                                       "roughnessFactor": 0.6,
                                       "baseColorTexture": {"index": t_alb, "extensions": tt},
                                       "metallicRoughnessTexture": {"index": t_mr}},
              "normalTexture": {"index": t_nrm, "scale": 1.0,
                                "extensions": {"KHR_texture_transform": {"scale": [3.0, 3.0]}}},
              "occlusionTexture": {"index": t_mr, "strength": 0.5}})
    M.append({"name": "clearcoat_transmission",
              "pbrMetallicRoughness": {"baseColorFactor": [0.2, 0.5, 0.9, 1.0], "metallicFactor": 0.0,
                                       "roughnessFactor": 0.1},
              "extensions": {"KHR_materials_clearcoat": {"clearcoatFactor": 0.8, "clearcoatRoughnessFactor": 0.2,
                                                         "clearcoatTexture": {"index": t_cc},
                                                         "clearcoatRoughnessTexture": {"index": t_mr}},
                             "KHR_materials_transmission": {"transmissionFactor": 0.0,
                                                            "transmissionTexture": {"index": t_mr}}},
              "doubleSided": True})
    M.append({"name": "spec_gloss",
              "extensions": {"KHR_materials_pbrSpecularGlossiness": {
                  "diffuseFactor": [0.7, 0.6, 0.5, 1.0], "specularFactor": [0.3, 0.3, 0.3],
                  "glossinessFactor": 0.55, "diffuseTexture": {"index": t_alb},
                  "specularGlossinessTexture": {"index": t_sg}}}})
    M.append({"name": "emitter", "emissiveFactor": [1.0, 0.8, 0.6],
              "emissiveTexture": {"index": t_em, "extensions": {"KHR_texture_transform": {"offset": [0.1, 0.2]}}},
              "pbrMetallicRoughness": {"baseColorFactor": [0.1, 0.1, 0.1, 1.0]},
              "extensions": {"KHR_materials_emissive_strength": {"emissiveStrength": 6},
                             "KHR_materials_specular": {"specularFactor": 0.7,
                                                        "specularColorFactor": [1.0, 0.9, 0.8]}}})
    M.append({"name": "skin_glass", "pbrMetallicRoughness": {"baseColorFactor": [0.95, 0.95, 0.95, 1.0],
                                                               "metallicFactor": 0.0, "roughnessFactor": 0.05},
              "extensions": {"KHR_materials_transmission": {"transmissionFactor": 0.9}}})
    M.append({"name": "mask", "alphaMode": "MASK", "alphaCutoff": 0.4,
              "pbrMetallicRoughness": {"baseColorTexture": {"index": t_cut}}})
    M.append({"name": "blend", "alphaMode": "BLEND", "pbrMetallicRoughness": {"baseColorFactor": [1, 1, 1, 0.5]}})

    # mesh 0: box, interleaved POSITION/NORMAL/TANGENT/TEXCOORD_0 (stride 48), u16 indices, 2 primitives
    P, N, T, UV, idx = box_geometry()
    inter = np.zeros((24, 12), "<f4")
    inter[:, 0:3], inter[:, 3:6], inter[:, 6:10], inter[:, 10:12] = P, N, T, UV
    bv = g.view(inter.tobytes(), stride=48, target=34962)
    a_p = g.accessor(bv, 5126, 24, "VEC3", 0, ([-0.5] * 3, [0.5] * 3))
    a_n = g.accessor(bv, 5126, 24, "VEC3", 12)
    a_t = g.accessor(bv, 5126, 24, "VEC4", 24)
    a_uv = g.accessor(bv, 5126, 24, "VEC2", 40)
    ib = g.view(idx.astype("<u2").tobytes())
    a_i0 = g.accessor(ib, 5123, 18, "SCALAR")
    a_i1 = g.accessor(ib, 5123, 18, "SCALAR", 36)
    attrs = {"POSITION": a_p, "NORMAL": a_n, "TANGENT": a_t, "TEXCOORD_0": a_uv}
    g.j["meshes"].append({"name": "box", "primitives": [{"attributes": attrs, "indices": a_i0, "material": 0},
                                                         {"attributes": attrs, "indices": a_i1, "material": 1}]})
    # mesh 1: quad, POSITION only, u8 indices with a repeated corner (dedup), MASK + spec-gloss
    qp = np.array([[-1, 0, -1], [1, 0, -1], [1, 0, 1], [-1, 0, 1], [1, 0, -1], [-1, 0, 1]], "<f4")
    a_qp = g.floats(qp, "VEC3")
    a_qi = g.accessor(g.view(np.array([0, 1, 2, 4, 2, 3, 0, 2, 5], np.uint8).tobytes()), 5121, 9, "SCALAR")
    g.j["meshes"].append({"name": "quad", "primitives": [{"attributes": {"POSITION": a_qp}, "indices": a_qi,
                                                          "material": 2},
                                                         {"attributes": {"POSITION": a_qp}, "indices": a_qi,
                                                          "material": 5}]})
    # mesh 2: emitter plane, u32 indices, TEXCOORD_1, a degenerate (zero-area) triangle
    ep = np.array([[-0.5, 0, -0.5], [0.5, 0, -0.5], [0.5, 0, 0.5], [-0.5, 0, 0.5], [0.5, 0, 0.5]], "<f4")
    en = np.tile(np.array([[0, -1, 0]], "<f4"), (5, 1))
    euv = np.array([[0, 0], [1, 0], [1, 1], [0, 1], [1, 1]], "<f4")
    euv1 = euv[:, ::-1] * 0.5
    a_ei = g.accessor(g.view(np.array([0, 2, 1, 0, 3, 2, 2, 4, 2], "<u4").tobytes()), 5125, 9, "SCALAR")
    g.j["meshes"].append({"name": "emitter", "primitives": [{"attributes": {
        "POSITION": g.floats(ep, "VEC3"), "NORMAL": g.floats(en, "VEC3"), "TEXCOORD_0": g.floats(euv, "VEC2"),
        "TEXCOORD_1": g.floats(euv1, "VEC2")}, "indices": a_ei, "material": 3}]})
    # mesh 3: skinned strip (2 joints, u8 joints, unnormalised float weights), BLEND second primitive
    sp = np.array([[x, y, 0] for y in (0.0, 0.6, 1.2) for x in (-0.2, 0.2)], "<f4")
    sn = np.tile(np.array([[0, 0, 1]], "<f4"), (6, 1))
    sj = np.array([[0, 1, 0, 0]] * 6, np.uint8)
    sw = np.array([[1.0, 0.0, 0, 0], [2.0, 0.0, 0, 0], [0.5, 0.5, 0, 0], [0.3, 0.9, 0, 0],
                   [0.0, 1.0, 0, 0], [0.0, 0.0, 0, 0]], "<f4")
    st = np.array([[1, 0, 0, 1]] * 6, "<f4")
    a_si = g.accessor(g.view(np.array([0, 1, 3, 0, 3, 2, 2, 3, 5, 2, 5, 4], "<u2").tobytes()), 5123, 12, "SCALAR")
    sattr = {"POSITION": g.floats(sp, "VEC3"), "NORMAL": g.floats(sn, "VEC3"), "TANGENT": g.floats(st, "VEC4"),
             "JOINTS_0": g.accessor(g.view(sj.tobytes()), 5121, 6, "VEC4"), "WEIGHTS_0": g.floats(sw, "VEC4")}
    g.j["meshes"].append({"name": "strip", "primitives": [{"attributes": sattr, "indices": a_si, "material": 4},
                                                           {"attributes": sattr, "indices": a_si, "material": 6}]})
    # nodes
    ry = 0.6
    box_m = [math.cos(ry), 0, -math.sin(ry), 0, 0, 1, 0, 0, math.sin(ry), 0, math.cos(ry), 0, 0.3, 0.5, -0.2, 1]
    nodes = g.j["nodes"]
    nodes.append({"name": "root", "translation": [0.5, -0.25, 1.0], "rotation": quat((1, 2, 3), 0.7),
                  "scale": [1.5, 0.75, 1.25], "children": [1, 2, 3, 5]})                      # 0
    nodes.append({"name": "box", "matrix": box_m, "mesh": 0, "children": [4]})                  # 1
    nodes.append({"name": "quad", "translation": [0, -0.6, 0], "scale": [0.8, 1, 0.6], "mesh": 1})  # 2
    nodes.append({"name": "emitter", "translation": [0, 1.4, 0], "mesh": 2})                    # 3
    nodes.append({"name": "point", "translation": [0, 1.0, 0],
                  "extensions": {"KHR_lights_punctual": {"light": 0}}})                            # 4
    nodes.append({"name": "spot", "translation": [1, 1, 0], "rotation": quat((1, 0, 0), -1.2),
                  "extensions": {"KHR_lights_punctual": {"light": 1}}})                            # 5
    nodes.append({"name": "sun", "matrix": [1, 0, 0, 0, 0, 0.8, 0.6, 0, 0, -0.6, 0.8, 0, 0, 5, 0, 1],
                  "extensions": {"KHR_lights_punctual": {"light": 2}}})                            # 6
    nodes.append({"name": "skinned", "translation": [9, 9, 9], "mesh": 3, "skin": 0})          # 7 (own T unused)
    nodes.append({"name": "joint0", "translation": [-0.8, 0.2, 0.4], "children": [9]})       # 8
    nodes.append({"name": "joint1", "translation": [0, 0.6, 0], "rotation": quat((0, 0, 1), 0.2)})  # 9
    nodes.append({"name": "off", "extensions": {"KHR_lights_punctual": {"light": 3}}})        # 10 (not in scene)
    ibm = np.zeros((2, 16), "<f4")
    ibm[0] = np.eye(4, dtype="<f4").ravel()
    ibm[1] = np.eye(4, dtype="<f4").ravel()
    ibm[1][13] = -0.6
    g.j["skins"] = [{"joints": [8, 9], "inverseBindMatrices": g.floats(ibm, "MAT4")}]
    # animation 0, frame 0 overrides joint1's rotation and joint0's translation (times 0, 1)
    tin = g.floats(np.array([[0.0], [1.0]], "<f4"), "SCALAR")
    rot_out = g.floats(np.array([quat((0, 0, 1), 0.5), quat((0, 0, 1), 0.9)], "<f4"), "VEC4")
    tr_out = g.floats(np.array([[-0.7, 0.1, 0.4], [0, 0, 0]], "<f4"), "VEC3")
    g.j["animations"] = [{"samplers": [{"input": tin, "output": rot_out}, {"input": tin, "output": tr_out}],
                          "channels": [{"sampler": 0, "target": {"node": 9, "path": "rotation"}},
                                       {"sampler": 1, "target": {"node": 8, "path": "translation"}}]}]
    g.j["extensions"] = {"KHR_lights_punctual": {"lights": [
        {"type": "point", "color": [1.0, 0.9, 0.7], "intensity": 15.0, "range": 4.0},
        {"type": "spot", "intensity": 40.0, "spot": {"innerConeAngle": 0.2, "outerConeAngle": 0.6}},
        {"type": "directional", "color": [0.9, 0.95, 1.0], "intensity": 0.8},
        {"type": "point", "intensity": 0.0}]}}
    g.j["extensionsUsed"] = ["KHR_texture_transform", "KHR_lights_punctual", "KHR_materials_clearcoat",
                             "KHR_materials_transmission", "KHR_materials_pbrSpecularGlossiness",
                             "KHR_materials_emissive_strength", "KHR_materials_specular"]
    g.j["scenes"] = [{"nodes": [10]}, {"nodes": [0, 6, 7, 8]}]
    g.j["scene"] = 1


def write_gltf(g: Gltf, name: str, glb: bool = False):
    g._align(4)
    j = json.loads(json.dumps(g.j))
    if glb:
        j["buffers"] = [{"byteLength": len(g.bin)}]
        js = json.dumps(j, separators=(",", ":")).encode()
        js += b" " * ((4 - len(js) % 4) % 4)
        body = struct.pack("<II", len(js), 0x4E4F534A) + js + struct.pack("<II", len(g.bin), 0x004E4942) + bytes(g.bin)
        with open(os.path.join(HERE, name), "wb") as f:
            f.write(b"glTF" + struct.pack("<II", 2, 12 + len(body)) + body)
        return
    binname = name.replace(".gltf", ".bin")
    j["buffers"] = [{"uri": binname, "byteLength": len(g.bin)}]
    with open(os.path.join(HERE, binname), "wb") as f:
        f.write(bytes(g.bin))
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(j, f, indent=1)


def make_lamp():
    """A second model: data: URI buffer, no materials, a default-coloured light, a non-square node scale."""
    g = Gltf()
    p = np.array([[0, 0, 0], [0.4, 0, 0], [0, 0.4, 0], [0, 0, 0.4]], "<f4")
    a_p = g.floats(p, "VEC3")
    a_i = g.accessor(g.view(np.array([0, 2, 1, 0, 1, 3, 0, 3, 2, 1, 2, 3], "<u2").tobytes()), 5123, 12, "SCALAR")
    del g.j["materials"], g.j["textures"], g.j["images"], g.j["samplers"]
    g.j["meshes"] = [{"primitives": [{"attributes": {"POSITION": a_p}, "indices": a_i}]}]
    g.j["nodes"] = [{"mesh": 0, "scale": [1, 2, 1], "children": [1]},
                    {"translation": [0, 0.5, 0], "extensions": {"KHR_lights_punctual": {"light": 0}}}]
    g.j["extensions"] = {"KHR_lights_punctual": {"lights": [{"type": "point", "range": 2.5}]}}
    g.j["scenes"] = [{"nodes": [0]}]
    g._align(4)
    j = json.loads(json.dumps(g.j))
    j["buffers"] = [{"byteLength": len(g.bin),
                     "uri": "data:application/octet-stream;base64," + base64.b64encode(bytes(g.bin)).decode()}]
    with open(os.path.join(HERE, "lamp.gltf"), "w") as f:
        json.dump(j, f, indent=1)


def main():
    make_images()
    g = Gltf()
    make_features(g)
    write_gltf(g, "features.gltf")
    write_gltf(g, "features.glb", glb=True)
    make_lamp()
    rt = {"position": [0, -2.5, 0], "dimensions": [9, 7, 9], "panels": {
        "floor": {"material": {"base_color": [0.8, 0.8, 0.8], "metallic": 0.0, "roughness": 1.0},
                  "light": {"intensity": 0.0}},
        "ceiling": {"material": {"base_color": [0.9, 0.9, 0.9]}, "light": {"intensity": 1.5}},
        "back_wall": {"material": {"base_color": [0.7, 0.7, 0.7], "roughness": 0.8}, "light": {"intensity": 0.0}},
        "left_wall": {"material": {"base_color": [0.1, 0.7, 0.1]}, "light": {"intensity": 0.0}},
        "right_wall": {"material": {"base_color": [0.7, 0.1, 0.1], "metallic": 0.5}, "light": {"intensity": 0.0}},
        "front_wall": {"material": {"base_color": [0.6, 0.6, 0.6]}, "light": {"intensity": 0.0}}}}
    with open(os.path.join(HERE, "rtbox.json"), "w") as f:
        json.dump(rt, f, indent=1)
    scene = {"settings": {"use_rt_box": True, "rt_box_file": "rtbox.json", "ambient_light": [0.2, 0.25, 0.3, 1.0],
                          "sun": {"color": [1.0, 0.95, 0.9], "direction": [0.3, -1.0, 0.2], "intensity": 2.0},
                          "torus_settings": {"major_radius": 3.5, "minor_radius": 1.0, "height": 1.0,
                                             "num_rays": 4096},
                          "use_lod": 1.0, "lod_factor": 0.5, "accumulation_steps": 8, "total_positions": 6,
                          "min_beta": -20, "max_beta": 35.5, "image_divisor": 2, "capture_pointcloud": False},
             "objects": [{"model": "features.gltf", "position": [0.2, -1.0, -0.5], "scale": [1.2, 1.2, 1.2],
                          "rotation": [10.0, -30.0, 5.0]},
                         {"model": "lamp.gltf", "position": [-2.0, -2.5, 1.0], "scale": [2, 2, 2]},
                         {"model": "features.glb", "position": [2.0, -2.0, 1.5], "rotation": [0, 90, 0],
                          "scale": [0.5, 0.7, 0.5]}]}
    with open(os.path.join(HERE, "scene.json"), "w") as f:
        json.dump(scene, f, indent=1)
    with open(os.path.join(HERE, "main_scene.json"), "w") as f:
        json.dump({"scene": "scene.json"}, f)
    np.savez_compressed(os.path.join(HERE, "png_expected.npz"), **{k: v for k, v in IMAGES.items() if v is not None})


if __name__ == "__main__":
    main()
