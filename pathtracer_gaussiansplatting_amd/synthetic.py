"""Seeded synthetic inputs of the shapes named in BASELINE.json (nothing large is committed).

  blue_noise()        the missing blue-noise blob (.MISSING_LARGE_BLOBS:1) — a deterministic hash
                      texture decoded with the stbi_loadf convention (RGB^2.2, A linear;
                      Helpers/stb_image.h:1858-1872 via Vulkan_Engine/image.cpp:10)
  atrium_scene()      C3: "250k-tri Sponza-like" procedural atrium
  gaussians_c2()      C2/C4: synthetic Gaussians in a camera-space box
  torus_samples()     RaySample (u,v) inputs for the toroidal tracer (the reference's generators,
                      Vulkan_Engine/sampling.cpp, via ptgs_generate_samples)
"""
from __future__ import annotations

import numpy as np

from ._abi import MATERIAL_DTYPE, PRIMITIVE_DTYPE, PUNCTUAL_LIGHT_DTYPE, RAY_SAMPLE_DTYPE, VERTEX_DTYPE
from .scene import Scene, SceneBuilder, default_material


def _hash32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def blue_noise_rgba8(size: int = 1024, seed: int = 0x5EED) -> np.ndarray:
    """(size, size, 4) uint8 substitute for blue_noise/1024_1024/LDR_RGBA_0.png."""
    with np.errstate(over="ignore"):
        y, x = np.mgrid[0:size, 0:size].astype(np.uint32)
        out = np.empty((size, size, 4), np.uint8)
        for c in range(4):
            h = _hash32(x * np.uint32(73856093) ^ y * np.uint32(19349663) ^ np.uint32((seed * 83492791 + c * 2654435761) & 0xFFFFFFFF))
            out[..., c] = (h >> np.uint32(24)).astype(np.uint8)
    return out


def blue_noise(size: int = 1024, seed: int = 0x5EED) -> np.ndarray:
    """stbi_loadf decode: (v/255)^2.2 for RGB (pow in double, like stb's pow()), A = v/255."""
    px = blue_noise_rgba8(size, seed)
    f = px.astype(np.float32) / np.float32(255.0)
    out = np.empty(f.shape, np.float32)
    out[..., :3] = np.power(f[..., :3].astype(np.float64), 2.2).astype(np.float32)
    out[..., 3] = f[..., 3]
    return out


# ---------------------------------------------------------------------------------------------
# procedural geometry helpers
# ---------------------------------------------------------------------------------------------
class _Mesh:
    def __init__(self):
        self.pos, self.nrm, self.idx, self.prims = [], [], [], []
        self.nv = 0
        self.ni = 0

    def add(self, pos: np.ndarray, nrm: np.ndarray, tri: np.ndarray, material: int):
        tri = tri.astype(np.uint32) + np.uint32(self.nv)
        self.pos.append(pos.astype(np.float32))
        self.nrm.append(nrm.astype(np.float32))
        flat = tri.reshape(-1)
        self.idx.append(flat)
        self.prims.append((self.ni, len(flat), material))
        self.nv += len(pos)
        self.ni += len(flat)

    def ntris(self) -> int:
        return self.ni // 3


def _grid(origin, du, dv, nu, nv):
    """quad grid with nu x nv cells spanning origin + [0,1]du + [0,1]dv"""
    origin, du, dv = (np.asarray(a, np.float64) for a in (origin, du, dv))
    s = np.linspace(0.0, 1.0, nu + 1)
    t = np.linspace(0.0, 1.0, nv + 1)
    S, T = np.meshgrid(s, t, indexing="ij")
    pos = origin + S[..., None] * du + T[..., None] * dv
    n = np.cross(du, dv)
    n = n / np.linalg.norm(n)
    pos = pos.reshape(-1, 3)
    nrm = np.broadcast_to(n, pos.shape)
    i = np.arange(nu)[:, None] * (nv + 1) + np.arange(nv)[None, :]
    a, b, c, d = i, i + (nv + 1), i + (nv + 2), i + 1
    tri = np.stack([np.stack([a, b, c], -1), np.stack([a, c, d], -1)], -2).reshape(-1, 3)
    return pos, nrm, tri


def _cylinder(center, radius, height, nseg, nring):
    cx, cy, cz = center
    ang = np.linspace(0.0, 2 * np.pi, nseg, endpoint=False)
    hs = np.linspace(0.0, height, nring + 1)
    A, Hh = np.meshgrid(ang, hs, indexing="ij")
    pos = np.stack([cx + radius * np.cos(A), cy + Hh, cz + radius * np.sin(A)], -1).reshape(-1, 3)
    nrm = np.stack([np.cos(A), np.zeros_like(A), np.sin(A)], -1).reshape(-1, 3)
    i = np.arange(nseg)[:, None] * (nring + 1) + np.arange(nring)[None, :]
    j = ((np.arange(nseg)[:, None] + 1) % nseg) * (nring + 1) + np.arange(nring)[None, :]
    tri = np.stack([np.stack([i, i + 1, j + 1], -1), np.stack([i, j + 1, j], -1)], -2).reshape(-1, 3)
    return pos, nrm, tri


def _arch(p0, p1, y0, radius_tube, nseg, ntube):
    """half-torus arch between two column tops"""
    p0, p1 = np.asarray(p0, np.float64), np.asarray(p1, np.float64)
    c = 0.5 * (p0 + p1)
    span = np.linalg.norm(p1 - p0)
    R = 0.5 * span
    ax = (p1 - p0) / span
    th = np.linspace(0.0, np.pi, nseg + 1)
    ph = np.linspace(0.0, 2 * np.pi, ntube, endpoint=False)
    TH, PH = np.meshgrid(th, ph, indexing="ij")
    ring = (np.cos(TH)[..., None] * ax[None, None, :] * -1.0 + np.sin(TH)[..., None] * np.array([0.0, 1.0, 0.0]))
    side = np.cross(ax, [0.0, 1.0, 0.0])
    side = side / np.linalg.norm(side)
    nrm = np.cos(PH)[..., None] * ring + np.sin(PH)[..., None] * side
    pos = np.array([c[0], y0, c[2]]) + R * ring + radius_tube * nrm
    pos = pos.reshape(-1, 3)
    nrm = nrm.reshape(-1, 3)
    i = np.arange(nseg)[:, None] * ntube + np.arange(ntube)[None, :]
    i1 = np.arange(nseg)[:, None] * ntube + (np.arange(ntube)[None, :] + 1) % ntube
    tri = np.stack([np.stack([i, i + ntube, i1 + ntube], -1), np.stack([i, i1 + ntube, i1], -1)], -2).reshape(-1, 3)
    return pos, nrm, tri


def _box(center, half):
    c = np.asarray(center, np.float64)
    h = np.asarray(half, np.float64)
    pos, nrm, tri = [], [], []
    k = 0
    for axis in range(3):
        for sgn in (-1.0, 1.0):
            n = np.zeros(3)
            n[axis] = sgn
            u = np.zeros(3)
            u[(axis + 1) % 3] = 2 * h[(axis + 1) % 3]
            v = np.zeros(3)
            v[(axis + 2) % 3] = 2 * h[(axis + 2) % 3]
            o = c + n * h - 0.5 * u - 0.5 * v
            if sgn < 0:
                u, v = v, u
                o = c + n * h - 0.5 * u - 0.5 * v
            p = np.array([o, o + u, o + u + v, o + v])
            pos.append(p)
            nrm.append(np.broadcast_to(n, (4, 3)))
            tri.append(np.array([[0, 1, 2], [0, 2, 3]]) + k)
            k += 4
    return np.concatenate(pos), np.concatenate(nrm), np.concatenate(tri)


def _materials(rng: np.random.Generator, n: int) -> np.ndarray:
    mats = np.concatenate([default_material() for _ in range(n)])
    mats["base_color_factor"][:, :3] = rng.uniform(0.2, 0.9, (n, 3)).astype(np.float32)
    mats["roughness_factor"] = rng.uniform(0.05, 1.0, n).astype(np.float32)
    mats["metallic_factor"] = (rng.uniform(0.0, 1.0, n) < 0.2).astype(np.float32)
    return mats


def atrium_scene(target_tris: int = 250_000, seed: int = 2, with_sun: bool = True) -> Scene:
    """C3: 36 x 15 x 16 m atrium, tessellated floor/walls, 2 x 12 columns + arches, filler boxes to
    exactly `target_tris`, one emissive ceiling quad + one directional sun (both NEE branches and
    the p_emissive clamp)."""
    rng = np.random.default_rng(seed)
    NMAT = 48
    mats = _materials(rng, NMAT)
    # material 0: emissive light panel (non-metal, rough)
    mats[0]["base_color_factor"][:3] = 1.0
    mats[0]["emissive_factor_and_pad"][:3] = 8.0
    mats[0]["metallic_factor"] = 0.0
    mats[0]["roughness_factor"] = 1.0
    m = _Mesh()
    X, Y, Z = 36.0, 15.0, 16.0
    x0, z0 = -X / 2, -Z / 2
    # floor / walls / ceiling frame (open skylight in the middle of the roof)
    m.add(*_grid([x0, 0, z0], [0, 0, Z], [X, 0, 0], 96, 64), material=1)
    m.add(*_grid([x0, 0, z0], [X, 0, 0], [0, Y, 0], 96, 40), material=2)  # back
    m.add(*_grid([x0, 0, -z0], [0, Y, 0], [X, 0, 0], 96, 40), material=2)  # front
    m.add(*_grid([x0, 0, z0], [0, Y, 0], [0, 0, Z], 40, 48), material=3)  # left
    m.add(*_grid([-x0, 0, z0], [0, 0, Z], [0, Y, 0], 48, 40), material=3)  # right
    m.add(*_grid([x0, Y, z0], [X, 0, 0], [0, 0, 4.0], 64, 8), material=4)  # roof band back
    m.add(*_grid([x0, Y, -z0 - 4.0], [X, 0, 0], [0, 0, 4.0], 64, 8), material=4)  # roof band front
    # emissive panel hanging under the roof band
    m.add(*_grid([-4.0, Y - 0.5, z0 + 1.0], [8.0, 0, 0], [0, 0, 2.0], 1, 1), material=0)
    # 2 x 12 columns + arches
    xs = np.linspace(x0 + 3.0, -x0 - 3.0, 12)
    for zc in (z0 + 4.5, -z0 - 4.5):
        for k, xc in enumerate(xs):
            m.add(*_cylinder((xc, 0.0, zc), 0.45, 9.0, 48, 40), material=5 + k % 6)
        for k in range(11):
            m.add(*_arch((xs[k], 0, zc), (xs[k + 1], 0, zc), 9.0, 0.35, 48, 16), material=11 + k % 6)
    # filler boxes ("clutter"), 12 triangles each, to reach exactly target_tris
    remaining = target_tris - m.ntris()
    if remaining < 0:
        raise ValueError(f"base atrium already has {m.ntris()} triangles > {target_tris}")
    nbox, rest = divmod(remaining, 12)
    for b in range(nbox):
        c = [rng.uniform(x0 + 1, -x0 - 1), rng.uniform(0.1, 6.0), rng.uniform(z0 + 1, -z0 - 1)]
        h = rng.uniform(0.05, 0.35, 3)
        m.add(*_box(c, h), material=17 + int(rng.integers(0, NMAT - 17)))
    if rest:
        # a strip of `rest` small triangles on the floor
        p = np.array([[x0 + 1 + 0.1 * k, 0.01, z0 + 1] for k in range(rest + 2)], np.float64)
        p[1::2, 2] += 0.1
        tri = np.array([[k, k + 1, k + 2] for k in range(rest)])
        m.add(p, np.broadcast_to([0.0, 1.0, 0.0], p.shape), tri, material=1)
    assert m.ntris() == target_tris, (m.ntris(), target_tris)

    pos = np.concatenate(m.pos)
    nrm = np.concatenate(m.nrm)
    verts = np.zeros(len(pos), VERTEX_DTYPE)
    verts["pos"] = pos
    verts["normal"] = nrm
    verts["color"] = 1.0
    verts["tangent"] = [1.0, 0.0, 0.0, 0.0]
    idx = np.concatenate(m.idx).astype(np.uint32)
    prims = np.zeros(len(m.prims), PRIMITIVE_DTYPE)
    prims["first_index"] = [p[0] for p in m.prims]
    prims["index_count"] = [p[1] for p in m.prims]
    prims["material_index"] = [p[2] for p in m.prims]
    lights = np.zeros(1 if with_sun else 0, PUNCTUAL_LIGHT_DTYPE)
    if with_sun:
        d = np.array([0.3, -1.0, 0.25])
        lights[0]["direction"] = (d / np.linalg.norm(d)).astype(np.float32)
        lights[0]["color"] = [1.0, 0.95, 0.85]
        lights[0]["intensity"] = 10.0
        lights[0]["type"] = 1
    return SceneBuilder().add_object(verts, idx, prims, mats, lights).finalize()


def gaussians_c2(n: int = 100_000, seed: int = 1) -> dict:
    """SoA Gaussians in the camera-space box x in [-4,4], y in [-2.25,2.25], z in [-12,-4] (the
    camera is the identity view at the origin looking down -Z)."""
    rng = np.random.default_rng(seed)
    means = np.stack([rng.uniform(-4.0, 4.0, n), rng.uniform(-2.25, 2.25, n), rng.uniform(-12.0, -4.0, n)], -1)
    log_scales = rng.uniform(np.log(0.005), np.log(0.05), (n, 3))
    rots = rng.normal(size=(n, 4))
    return {
        "means": means.astype(np.float32),
        "scales": np.exp(log_scales).astype(np.float32),
        "rotations": rots.astype(np.float32),
        "opacities": rng.uniform(0.05, 0.95, n).astype(np.float32),
        "colors": rng.uniform(0.0, 1.0, (n, 3)).astype(np.float32),
    }


def gaussians_in_view(n: int, seed: int, ubo) -> dict:
    """gaussians_c2 placed in the world frame of the camera `ubo` (BASELINE C4 / C5: the Gaussians sit
    in the path-traced mesh's view frustum, some in front of and some behind the mesh)."""
    g = gaussians_c2(n, seed=seed)
    view = np.array(ubo.view, np.float64).reshape(4, 4).T  # column-major -> row-major
    inv = np.linalg.inv(view)
    m = g["means"].astype(np.float64)
    g["means"] = (m @ inv[:3, :3].T + inv[:3, 3]).astype(np.float32)
    return g


def torus_samples(n: int, method: int = 0, seed: int = 13) -> np.ndarray:
    """The reference's own RaySample generator (default: RANDOM with seed 13, sampling.cpp:164-179),
    Morton-sorted as the Engine uploads it (product: ptgs_generate_samples)."""
    from .sampling import update_sampling
    return update_sampling(method, n, seed=seed)
