"""Test scenes (seeded, small enough for the CPU oracle in seconds)."""
from __future__ import annotations

import os

import numpy as np

from pathtracer_gaussiansplatting_amd import scene as S
from pathtracer_gaussiansplatting_amd import synthetic as Y
from pathtracer_gaussiansplatting_amd._abi import PRIMITIVE_DTYPE, PUNCTUAL_LIGHT_DTYPE, VERTEX_DTYPE

_BN = {}


def blue_noise(size=1024):
    if size not in _BN:
        _BN[size] = Y.blue_noise(size)
    return _BN[size]


def cornell():
    sc = S.cornell_box_scene()
    sc.blue_noise = blue_noise()
    return sc


def cornell_pose(aspect=1.0):
    # first mt19937(13) draw of captureSceneData (engine.cpp:2673-2681), R=3.5, h=3
    return S.Camera(aspect=aspect).toroidal(218.6429, 21.5660, 3.5, 3.0)


def _sphere(center, r, nu=24, nv=16):
    th = np.linspace(0, np.pi, nv + 1)
    ph = np.linspace(0, 2 * np.pi, nu, endpoint=False)
    T, P = np.meshgrid(th, ph, indexing="ij")
    n = np.stack([np.sin(T) * np.cos(P), np.cos(T), np.sin(T) * np.sin(P)], -1).reshape(-1, 3)
    pos = np.asarray(center) + r * n
    i = np.arange(nv)[:, None] * nu + np.arange(nu)[None, :]
    j = np.arange(nv)[:, None] * nu + (np.arange(nu)[None, :] + 1) % nu
    tri = np.stack([np.stack([i, i + nu, j + nu], -1), np.stack([i, j + nu, j], -1)], -2).reshape(-1, 3)
    return pos, n, tri


def _mat(**kw):
    m = S.default_material()
    for k, v in kw.items():
        m[k] = v
    return m


def _tex_rgba(h, w, seed, lo=0, hi=256):
    rng = np.random.default_rng(seed)
    return rng.integers(lo, hi, (h, w, 4), dtype=np.int64).astype(np.uint8)


def feature_textures():
    """global_textures[] for features(textured=True): sizes and formats chosen to cover odd mip chains,
    both formats, repeat wrapping (UVs outside [0, 1]) and texture alpha."""
    yy, xx = np.mgrid[0:64, 0:48]
    checker = ((yy // 8 + xx // 8) % 2).astype(np.float64)
    albedo = np.zeros((64, 48, 4), np.uint8)
    albedo[..., 0] = 60 + 180 * checker
    albedo[..., 1] = 40 + 120 * (xx / 47.0)
    albedo[..., 2] = 200 - 150 * checker
    albedo[..., 3] = np.where((yy // 4) % 3 == 0, 40, 230)  # alpha stripes for BLEND / MASK
    ny, nx = np.mgrid[0:32, 0:32] * (2 * np.pi / 32)
    n = np.stack([0.5 * np.sin(nx), 0.5 * np.cos(ny), np.ones_like(nx)], -1)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    nmap = np.zeros((32, 32, 4), np.uint8)
    nmap[..., :3] = np.round((n * 0.5 + 0.5) * 255)
    nmap[..., 3] = 255
    return [
        (np.full((1, 1, 4), 255, np.uint8), True),  # 0: default white (gameobject.cpp:347-349)
        (albedo, True),                             # 1: base colour (sRGB) with alpha
        (nmap, False),                              # 2: normal map (UNORM)
        (_tex_rgba(16, 16, 3), False),              # 3: metal-rough (UNORM: g rough, b metal)
        (_tex_rgba(8, 8, 4, 64), True),             # 4: emissive (sRGB)
        (_tex_rgba(16, 16, 5), True),               # 5: spec-gloss (sRGB: rgb spec, a gloss)
        (_tex_rgba(16, 16, 6), False),              # 6: clearcoat (UNORM r)
        (_tex_rgba(3, 5, 7), True),                 # 7: odd 5x3 base colour (mip chain 5x3 -> 2x1 -> 1x1)
        (_tex_rgba(9, 7, 8), False),                # 8: clearcoat roughness (UNORM r)
    ]


def _planar_uv(pos):
    return np.stack([pos[:, 0] * 0.7 + pos[:, 2] * 0.3, pos[:, 1] * 0.9 - pos[:, 2] * 0.4], -1)


def features(with_punctual=True, transparent=True, textured=False):
    objs = []
    # (mesh, material)
    objs.append((Y._box([-2.0, 1.0, -1.5], [0.8, 1.0, 0.8]), _mat(transmission_factor=1.0, metallic_factor=0.0,
                                                                roughness_factor=0.05,
                                                                base_color_factor=[0.9, 0.95, 1.0, 1.0])))
    objs.append((_sphere([1.5, 1.2, -1.0], 1.1), _mat(clearcoat_factor=1.0, clearcoat_roughness_factor=0.1,
                                                     metallic_factor=0.0, roughness_factor=0.6,
                                                     base_color_factor=[0.2, 0.3, 0.8, 1.0])))
    objs.append((_sphere([0.0, 0.8, 1.8], 0.8), _mat(metallic_factor=1.0, roughness_factor=0.2,
                                                    base_color_factor=[0.95, 0.7, 0.3, 1.0])))
    objs.append((Y._box([-1.0, 0.5, 2.5], [0.5, 0.5, 0.5]),
                 _mat(use_specular_glossiness_workflow=1.0, specular_color_factor=[0.6, 0.6, 0.6],
                      roughness_factor=0.7, base_color_factor=[0.5, 0.8, 0.5, 1.0], metallic_factor=0.0)))
    objs.append((Y._box([2.8, 0.4, 2.0], [0.4, 0.4, 0.4]), _mat(emissive_factor_and_pad=[4.0, 2.0, 1.0, 0.0],
                                                               metallic_factor=0.0)))
    if transparent:
        objs.append((Y._box([0.5, 2.5, 0.0], [0.6, 0.2, 0.6]), _mat(pad=1.0, base_color_factor=[1.0, 1.0, 1.0, 0.5],
                                                                   metallic_factor=0.0)))
        objs.append((Y._box([-0.5, 3.2, -0.5], [0.4, 0.1, 0.4]),
                     _mat(pad=1.0, alpha_cutoff=0.5, base_color_factor=[1.0, 0.2, 0.2, 0.3], metallic_factor=0.0)))
    tex_ids = []
    if textured:  # global indices into feature_textures(), set on the flattened materials below
        tex_ids = [dict(normal_texture_index=2),
                   dict(albedo_texture_index=1, normal_texture_index=2, clearcoat_texture_index=6,
                        clearcoat_roughness_texture_index=8),
                   dict(albedo_texture_index=7, metallic_roughness_texture_index=3),
                   dict(albedo_texture_index=1, sg_id=5),
                   dict(emissive_texture_index=4),
                   dict(albedo_texture_index=1),
                   dict(albedo_texture_index=1)]
        uvn = np.eye(4, dtype=np.float32)
        uvn[0, 0], uvn[1, 1], uvn[3, 0], uvn[3, 1] = 1.5, 0.75, 0.25, -0.5  # column-major: m[12], m[13]
        objs[1][1]["uv_normal"] = uvn.reshape(-1)
        uve = np.eye(4, dtype=np.float32)
        uve[0, 0], uve[3, 1] = 2.0, 0.3
        objs[4][1]["uv_emissive"] = uve.reshape(-1)
    b = S.SceneBuilder()
    for k, ((pos, nrm, tri), m) in enumerate(objs):
        v = np.zeros(len(pos), VERTEX_DTYPE)
        v["pos"] = pos
        v["normal"] = nrm
        v["color"] = 1.0
        v["tangent"] = [1.0, 0.0, 0.0, 0.0]
        if textured:
            v["tex_coord"] = _planar_uv(np.asarray(pos, np.float32))
            v["tangent"] = [0.0, 0.0, 1.0, -1.0 if k % 2 else 1.0]
        idx = tri.reshape(-1).astype(np.uint32)
        prims = np.zeros(1, PRIMITIVE_DTYPE)
        prims["index_count"] = len(idx)
        b.add_object(v, idx, prims, m)
    if with_punctual:
        lights = np.zeros(3, PUNCTUAL_LIGHT_DTYPE)
        lights[0]["position"] = [0.0, 6.0, 0.0]
        lights[0]["color"] = [1.0, 0.9, 0.8]
        lights[0]["intensity"] = 20.0
        lights[0]["range"] = 30.0
        lights[0]["type"] = 0
        lights[1]["position"] = [-3.0, 5.0, 3.0]
        lights[1]["direction"] = [0.5, -1.0, -0.5]
        lights[1]["color"] = [0.6, 0.8, 1.0]
        lights[1]["intensity"] = 30.0
        lights[1]["inner_cone_cos"] = 0.95
        lights[1]["outer_cone_cos"] = 0.8
        lights[1]["type"] = 2
        lights[2]["direction"] = [0.2, -1.0, 0.1]
        lights[2]["color"] = [1.0, 1.0, 1.0]
        lights[2]["intensity"] = 0.05
        lights[2]["type"] = 1
        v = np.zeros(3, VERTEX_DTYPE)
        v["pos"] = [[50, 50, 50], [50.1, 50, 50], [50, 50.1, 50]]
        # a far-away degenerate carrier object for the lights (never visible: behind the box walls)
        prims = np.zeros(0, PRIMITIVE_DTYPE)
        b.add_object(v, np.zeros(0, np.uint32), prims, S.default_material(), lights)
    b.add_rtbox_json(os.path.join(S.SCENES_DIR, "cornell_box.json"))
    sc = b.finalize()
    sc.blue_noise = blue_noise()
    if textured:
        sc.textures = feature_textures()
        tex_fields = ("albedo_texture_index", "normal_texture_index", "metallic_roughness_texture_index",
                      "emissive_texture_index", "occlusion_texture_index", "clearcoat_texture_index",
                      "clearcoat_roughness_texture_index", "sg_id")
        for key in tex_fields:  # the builder offset every object's default texture: one shared table here
            sc.materials[key] = 0
        for k, ids in enumerate(tex_ids):  # one material per object, in object order
            for key, val in ids.items():
                sc.materials[k][key] = val
    return sc


def atrium(target_tris=250_000):
    sc = Y.atrium_scene(target_tris=target_tris, seed=2)
    sc.blue_noise = blue_noise()
    return sc


def atrium_pose(aspect=16 / 9):
    return S.Camera(aspect=aspect).look_at([-15.0, 4.0, 5.0], [10.0, 3.0, -3.0])


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
