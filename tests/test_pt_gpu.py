"""Path-tracer parity: HIP kernels (through the C-ABI) vs the CPU oracle on the same seeded inputs.

Bar (BASELINE.json north_star): relative L2 < 1e-4 on linear RGBA32F; extension/shadow ray counts
(integers) bit-exact. In practice the arithmetic contract makes the images bit-identical; the tests
report the number of differing pixels so a regression is visible before it breaks the bound.
"""
import numpy as np
import pytest

import scenes_util as U
from pathtracer_gaussiansplatting_amd import ACCUM_RUNNING_MEAN, ACCUM_SUM, make_ubo

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-4



def _gpu_render(renderer, scene, ubo, W, H, spp, frame_stride=1, mode=ACCUM_RUNNING_MEAN, rows=None, init=None):
    renderer.upload_scene(scene)
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    if init is not None:
        acc.copy_(torch.from_numpy(init))
    renderer.stats_reset()
    renderer.trace_camera(ubo, W, H, acc, spp=spp, frame_stride=frame_stride, mode=mode, rows=rows)
    torch.cuda.synchronize()
    st = renderer.stats()
    return acc.cpu().numpy(), st


def _oracle_render(oracle_lib, scene, ubo, W, H, spp, frame_stride=1, mode=ACCUM_RUNNING_MEAN, rows=None, init=None):
    acc = np.zeros((H, W, 4), np.float32) if init is None else init.copy()
    st = oracle_lib.trace_camera(scene.desc(), ubo, W, H, acc, spp=spp, frame_stride=frame_stride, mode=mode,
                                 rows=rows)
    return acc, st


def _compare(gpu, ref, st_g, st_o, tol=TOL):
    err = U.rel_l2(gpu[..., :3], ref[..., :3])
    ndiff = int(np.count_nonzero(np.any(gpu != ref, axis=-1)))
    assert err < tol, f"rel L2 {err:.3e} ({ndiff} pixels differ)"
    assert st_g.extension_rays == st_o.extension_rays, (st_g.extension_rays, st_o.extension_rays)
    assert st_g.shadow_rays == st_o.shadow_rays, (st_g.shadow_rays, st_o.shadow_rays)
    return err, ndiff


def test_cornell_256_1spp(pt, oracle_lib):
    """C1: Cornell box (rt-box of bunny_box.json), 256x256, 1 spp, frame 0."""
    sc = U.cornell()
    ubo = make_ubo(U.cornell_pose(), sc, 0)
    g, sg = _gpu_render(pt, sc, ubo, 256, 256, 1)
    o, so = _oracle_render(oracle_lib, sc, ubo, 256, 256, 1)
    err, nd = _compare(g, o, sg, so)
    assert sg.samples == 256 * 256
    assert np.all(g[..., 3] == 1.0)
    print(f"cornell rel L2 {err:.2e}, {nd} pixels differ, ext {sg.extension_rays} shadow {sg.shadow_rays}")


def test_counts_after_a_smaller_call(pt, oracle_lib):
    """Ray counts of a call that follows a smaller one on the same context (the wavefront workspace
    is reused with a larger grid: a previous call's per-bounce work flags must not be counted as
    partial ray counts)."""
    sc = U.cornell()
    ubo = make_ubo(U.cornell_pose(), sc, 0)
    _gpu_render(pt, sc, ubo, 24, 24, 3)
    g, sg = _gpu_render(pt, sc, ubo, 192, 192, 2)
    o, so = _oracle_render(oracle_lib, sc, ubo, 192, 192, 2)
    _compare(g, o, sg, so)
    assert sg.samples == 192 * 192 * 2


def test_cornell_running_mean(pt, oracle_lib):
    """frames 3..6 on top of an existing accumulator (mix(prev, cur, 1/(n+1)), raygen_camera.rgen:80-87)."""
    sc = U.cornell()
    rng = np.random.default_rng(0)
    init = rng.uniform(0, 1, (64, 96, 4)).astype(np.float32)
    ubo = make_ubo(U.cornell_pose(96 / 64), sc, 3)
    g, sg = _gpu_render(pt, sc, ubo, 96, 64, 4, init=init)
    o, so = _oracle_render(oracle_lib, sc, ubo, 96, 64, 4, init=init)
    _compare(g, o, sg, so)


def test_features_all_branches(pt, oracle_lib):
    """glass, clearcoat, metal, spec-gloss, emissive object, BLEND/MASK any-hit, point/spot/sun."""
    sc = U.features()
    ubo = make_ubo(U.cornell_pose(160 / 120), sc, 0, ambient=(0.05, 0.05, 0.08, 1.0))
    g, sg = _gpu_render(pt, sc, ubo, 160, 120, 3)
    o, so = _oracle_render(oracle_lib, sc, ubo, 160, 120, 3)
    err, nd = _compare(g, o, sg, so)
    print(f"features rel L2 {err:.2e}, {nd} pixels differ")


@pytest.mark.parametrize("use_lod", [0.0, 1.0])
def test_features_textured(pt, oracle_lib, use_lod):
    """closesthit.rchit texture paths: base colour / spec-gloss / metal-rough / clearcoat (+ roughness) /
    emissive (uv_emissive) samples, tangent-space normal map (uv_normal, lod_factor, computeLOD with
    use_lod), texture alpha in any-hit, odd mip chains, repeat wrapping."""
    sc = U.features(textured=True)
    ubo = make_ubo(U.cornell_pose(160 / 120), sc, 0, ambient=(0.05, 0.05, 0.08, 1.0))
    ubo.use_lod = use_lod
    ubo.lod_factor = 0.8
    g, sg = _gpu_render(pt, sc, ubo, 160, 120, 3)
    o, so = _oracle_render(oracle_lib, sc, ubo, 160, 120, 3)
    err, nd = _compare(g, o, sg, so)
    print(f"textured (use_lod {use_lod}) rel L2 {err:.2e}, {nd} pixels differ")
    plain = U.features()
    o2, _ = _oracle_render(oracle_lib, plain, make_ubo(U.cornell_pose(160 / 120), plain, 0,
                                                        ambient=(0.05, 0.05, 0.08, 1.0)), 160, 120, 3)
    assert U.rel_l2(o, o2) > 1e-2  # the textures change the image


def test_atrium_250k(pt, oracle_lib):
    """C3 scene (250k triangles, sun + emissive panel) at a reduced resolution."""
    sc = U.atrium()
    ubo = make_ubo(U.atrium_pose(), sc, 0, ambient=(0.3, 0.4, 0.5, 1.0))
    g, sg = _gpu_render(pt, sc, ubo, 160, 90, 2)
    o, so = _oracle_render(oracle_lib, sc, ubo, 160, 90, 2)
    err, nd = _compare(g, o, sg, so)
    print(f"atrium rel L2 {err:.2e}, {nd} pixels differ")


@pytest.mark.parametrize("tries", ["4:4:38", "3:3:38", "3:2:38", "2:4:38"])
def test_tree_shapes_render_the_same_image(pt, oracle_lib, tries, monkeypatch):
    """The hits do not depend on the tree (closest hit with the lower-id tie rule, padded boxes, the near /
    far slab test): the C3 scene uploaded with other leaf sizes / fan-outs (api.cpp PTGS_BVH_TRIES, incl.
    the 2-wide nodes whose empty slots hold point boxes at 1e30) renders bit for bit the default tree's
    image and the oracle's."""
    sc = U.atrium()
    ubo = make_ubo(U.atrium_pose(), sc, 0, ambient=(0.3, 0.4, 0.5, 1.0))
    monkeypatch.delenv("PTGS_BVH_TRIES", raising=False)
    g0, s0 = _gpu_render(pt, sc, ubo, 160, 90, 2)
    info0 = pt.scene_info()
    monkeypatch.setenv("PTGS_BVH_TRIES", tries)
    g1, s1 = _gpu_render(pt, sc, ubo, 160, 90, 2)
    info1 = pt.scene_info()
    monkeypatch.delenv("PTGS_BVH_TRIES")
    leaf = int(tries.split(":")[0])
    assert info1.max_leaf_size <= leaf and (info1.num_bvh_nodes, info1.max_leaf_size) != (info0.num_bvh_nodes,
                                                                                          info0.max_leaf_size)
    assert np.array_equal(g0, g1), f"tree {tries}: {int(np.count_nonzero(np.any(g0 != g1, -1)))} pixels differ"
    assert (s0.extension_rays, s0.shadow_rays) == (s1.extension_rays, s1.shadow_rays)
    o, so = _oracle_render(oracle_lib, sc, ubo, 160, 90, 2)
    _compare(g1, o, s1, so)


def test_sample_shard_sum_mode(pt, oracle_lib):
    """§8e sample-index shard: rank g of G renders frames g, g+G, ... in SUM mode."""
    sc = U.cornell()
    ubo = make_ubo(U.cornell_pose(), sc, 1)
    g, sg = _gpu_render(pt, sc, ubo, 64, 64, 3, frame_stride=4, mode=ACCUM_SUM)
    o, so = _oracle_render(oracle_lib, sc, ubo, 64, 64, 3, frame_stride=4, mode=ACCUM_SUM)
    _compare(g, o, sg, so)
    assert np.all(g[..., 3] == 3.0)


def test_tile_schedule_and_lane_pairs(pt, oracle_lib):
    """Launches of >= 4M pixel-samples record each tile's time and the next launch of the same grid
    renders the tiles longest first (PtSched); with spp >= 2 two lanes share a pixel (even / odd
    samples, folded in sample order). The first launch (row-major order) and the second (heavy-first)
    are bit-identical and equal the oracle, odd spp included (the last odd lane idles)."""
    sc = U.cornell()
    W = H = 512
    spp = 17  # 512 * 512 * 17 = 4.46M pixel-samples: above PTGS_PT_SCHED_MIN
    ubo = make_ubo(U.cornell_pose(), sc, 0)
    g1, s1 = _gpu_render(pt, sc, ubo, W, H, spp)
    g2, s2 = _gpu_render(pt, sc, ubo, W, H, spp)
    assert np.array_equal(g1, g2)
    assert (s1.extension_rays, s1.shadow_rays, s1.samples) == (s2.extension_rays, s2.shadow_rays, s2.samples)
    o, so = _oracle_render(oracle_lib, sc, ubo, W, H, spp)
    err, nd = _compare(g2, o, s2, so)
    assert s2.samples == W * H * spp
    print(f"scheduled cornell {W}x{H} {spp} spp: rel L2 {err:.2e}, {nd} pixels differ")


def test_row_range(pt, oracle_lib):
    sc = U.cornell()
    ubo = make_ubo(U.cornell_pose(), sc, 0)
    g, sg = _gpu_render(pt, sc, ubo, 64, 64, 1, rows=(10, 37))
    o, so = _oracle_render(oracle_lib, sc, ubo, 64, 64, 1, rows=(10, 37))
    _compare(g, o, sg, so)
    assert np.all(g[:10] == 0) and np.all(g[37:] == 0)


def test_native_rccl_reduce_single_rank(renderer):
    """ptgs_comm_create / ptgs_reduce_radiance / ptgs_allreduce_radiance through the C-ABI on a
    one-rank RCCL communicator (the box has one GPU): the SUM over one rank is the identity."""
    from pathtracer_gaussiansplatting_amd import dist as D
    rank, world = D.init_native_comm(renderer)
    assert (rank, world) == (0, 1)
    x = torch.arange(4096 * 4, dtype=torch.float32, device="cuda").reshape(4096, 4)
    ref = x.clone()
    renderer.reduce_radiance(x, root=0)
    renderer.allreduce_radiance(x)
    img = torch.arange(16 * 8 * 4, dtype=torch.float32, device="cuda").reshape(16, 8, 4)
    renderer.gather_rows(img, [(0, 16)], root=0)  # ptgs_gather_rows: the root's own rows stay in place
    torch.cuda.synchronize()
    assert torch.equal(x, ref)
    assert torch.equal(img.flatten(), torch.arange(16 * 8 * 4, dtype=torch.float32, device="cuda"))
    from pathtracer_gaussiansplatting_amd import PtgsError
    with pytest.raises(PtgsError):
        renderer.gather_rows(img, [(0, 17)], root=0)  # rows beyond the image
    renderer.comm_destroy()


def _bvh_arrays(renderer):
    """(BVH4 nodes as u32 [n, 32], triangle records as u32 [t, 12]) of the uploaded scene."""
    bb = renderer.bvh_buffers()
    nodes = np.zeros((bb.num_nodes, 32), np.uint32)
    tris = np.zeros((bb.num_triangles, 12), np.uint32)
    renderer.copy_d2h(nodes, bb.nodes, nodes.nbytes)
    renderer.copy_d2h(tris, bb.triangles, tris.nbytes)
    return nodes, tris


def _leaf_sets_equal(nodes, tris_a, tris_b):
    """Every leaf range of the 4-wide nodes holds the same triangle records in both arrays (the
    order inside a leaf may differ)."""
    links = nodes[:, 24:28].view(np.int32).reshape(-1)
    boxes_lo_x = nodes[:, 0:4].view(np.float32).reshape(-1)
    leaves = links[(links < 0) & (boxes_lo_x < 1e29)]
    L = (~leaves).astype(np.uint32)
    first, count = L & 0x07FFFFFF, (L >> 27) + 1
    for f, c in zip(first.tolist(), count.tolist()):
        ra = tris_a[f:f + c]
        rb = tris_b[f:f + c]
        ka = np.lexsort(ra.T[::-1])
        kb = np.lexsort(rb.T[::-1])
        if not np.array_equal(ra[ka], rb[kb]):
            return False
    return int(count.sum()) == tris_a.shape[0]


@pytest.mark.parametrize("scene", ["features", "atrium"])
def test_gpu_sah_bvh_is_the_host_tree(renderer, oracle_lib, scene):
    """PTGS_FLAG_GPU_BVH: the binned-SAH build on the GPU (bvh_sah_gpu.hip) reproduces the host build
    (bvh.cpp): the 4-wide nodes are identical word for word (boxes, links, leaf ranges) and every
    leaf holds the same triangles; the image equals the oracle's bit for bit."""
    from pathtracer_gaussiansplatting_amd import FLAG_GPU_BVH
    sc = U.features() if scene == "features" else U.atrium()
    pose = U.cornell_pose(160 / 120) if scene == "features" else U.atrium_pose()
    ubo = make_ubo(pose, sc, 0, ambient=(0.3, 0.4, 0.5, 1.0))
    renderer.upload_scene(sc)
    info_h = renderer.scene_info()
    nodes_h, tris_h = _bvh_arrays(renderer)
    renderer.set_flags(FLAG_GPU_BVH)
    try:
        gpu, st_g = _gpu_render(renderer, sc, ubo, 160, 120, 2)
        info_g = renderer.scene_info()
        nodes_g, tris_g = _bvh_arrays(renderer)
    finally:
        renderer.set_flags(0)
    assert (info_g.num_bvh_nodes, info_g.bvh_depth) == (info_h.num_bvh_nodes, info_h.bvh_depth)
    assert np.array_equal(nodes_g, nodes_h), f"{int(np.count_nonzero(np.any(nodes_g != nodes_h, 1)))} nodes differ"
    assert _leaf_sets_equal(nodes_h, tris_h, tris_g)
    o, so = _oracle_render(oracle_lib, sc, ubo, 160, 120, 2)
    _compare(gpu, o, st_g, so)
    assert np.array_equal(gpu, o)
    print(f"{scene}: host SAH {info_h.build_ms:.1f} ms, GPU SAH {info_g.build_ms:.2f} ms "
          f"({info_g.num_bvh_nodes} 4-wide nodes, depth {info_g.bvh_depth})")


@pytest.mark.parametrize("scene", ["features", "atrium"])
def test_gpu_lbvh_vs_oracle(renderer, oracle_lib, scene):
    """PTGS_FLAG_GPU_BVH | PTGS_FLAG_GPU_LBVH (linear BVH on the GPU): the image and ray counts equal
    the oracle's (its own median-split BVH): hits do not depend on the tree (closest-hit tie rule,
    conservative boxes)."""
    from pathtracer_gaussiansplatting_amd import FLAG_GPU_BVH, FLAG_GPU_LBVH
    sc = U.features() if scene == "features" else U.atrium()
    pose = U.cornell_pose(160 / 120) if scene == "features" else U.atrium_pose()
    ubo = make_ubo(pose, sc, 0, ambient=(0.3, 0.4, 0.5, 1.0))
    renderer.set_flags(FLAG_GPU_BVH | FLAG_GPU_LBVH)
    try:
        gpu, st_g = _gpu_render(renderer, sc, ubo, 160, 120, 2)
        info_g = renderer.scene_info()
    finally:
        renderer.set_flags(0)
    o, so = _oracle_render(oracle_lib, sc, ubo, 160, 120, 2)
    _compare(gpu, o, st_g, so)
    assert np.array_equal(gpu, o)
    print(f"{scene}: GPU LBVH {info_g.build_ms:.2f} ms ({info_g.num_bvh_nodes} nodes, depth {info_g.bvh_depth})")


def test_ingested_scene_json(pt, oracle_lib):
    """§8f #3: the scene-JSON fixture (three glTF models incl. .glb, skin, lights, every material
    extension and texture format, rt-box, sun) loaded by ptgs_builder_load_scene_json, then path
    traced on the GPU vs the oracle on the same flattened scene (textures and settings included)."""
    import os

    from pathtracer_gaussiansplatting_amd import Camera
    from pathtracer_gaussiansplatting_amd.scene import SceneBuilder
    fix = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ingest")
    b = SceneBuilder()
    st = b.load_scene_json("main_scene.json", root_dir=fix)
    sc = b.finalize()
    sc.blue_noise = U.blue_noise()
    assert len(sc.textures) > 10 and sc.num_triangles > 60
    W, H = 160, 120
    pose = Camera(aspect=W / H).look_at([0.0, 0.2, 4.3], [0.2, -1.2, 0.0])
    ubo = make_ubo(pose, sc, 0, ambient=tuple(st.ambient_light), height=H, use_lod=st.use_lod,
                   lod_factor=st.lod_factor)
    g, sg = _gpu_render(pt, sc, ubo, W, H, 4)
    o, so = _oracle_render(oracle_lib, sc, ubo, W, H, 4)
    err, nd = _compare(g, o, sg, so)
    print(f"ingested scene rel L2 {err:.2e}, {nd} pixels differ")
    assert float(g[..., :3].mean()) > 1e-3


def test_bvh_node_window_guard(pt, monkeypatch):
    """the traversal addresses 4-wide nodes through a buffer descriptor with 32-bit offsets
    (2 GiB, ~16.7M nodes). ptgs_scene_upload refuses a larger tree with PTGS_ERANGE instead of tracing
    zero boxes; PTGS_BVH_NODE_LIMIT lowers the limit so a small scene exercises the refusal."""
    from pathtracer_gaussiansplatting_amd._abi import PtgsError
    sc = U.cornell()
    monkeypatch.setenv("PTGS_BVH_NODE_LIMIT", "1")
    with pytest.raises(PtgsError, match="PTGS_ERANGE"):
        pt.upload_scene(sc)
    monkeypatch.delenv("PTGS_BVH_NODE_LIMIT")
    info = pt.upload_scene(sc)
    assert info.num_bvh_nodes > 1
