"""3DGS initialisation from a point cloud (§8f #3) on the GPU: ptgs_knn3_mean_dist2 /
ptgs_gaussians_from_points against the brute-force oracle (bit-exact: the pruning is exact and the
f32 expressions are the same), and at 1M points against an independent float64 k-d tree.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle as OR  # noqa: E402

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _clouds():
    r = np.random.default_rng(7)
    yield "one", np.zeros((1, 3), np.float32)
    yield "two", np.array([[0, 0, 0], [1, 2, 2]], np.float32)
    yield "three", r.normal(size=(3, 3)).astype(np.float32)
    yield "four", r.normal(size=(4, 3)).astype(np.float32)
    yield "gauss_1000", r.normal(size=(1000, 3)).astype(np.float32)
    clustered = np.concatenate([r.normal(size=(3000, 3)) * 0.02 + c for c in r.uniform(-5, 5, (5, 3))])
    yield "clusters_15000", clustered.astype(np.float32)
    dup = r.normal(size=(4097, 3)).astype(np.float32)
    dup[100:200] = dup[5]  # 101 coincident points
    yield "dups_4097", dup
    plane = np.zeros((6000, 3), np.float32)
    plane[:, :2] = r.uniform(-1, 1, (6000, 2))  # degenerate bounds on one axis
    yield "plane_6000", plane
    grid = np.stack(np.meshgrid(np.arange(17), np.arange(13), np.arange(11), indexing="ij"), -1).reshape(-1, 3)
    yield "grid_ties", grid.astype(np.float32) * 0.5  # many equal distances


@pytest.mark.parametrize("name,pts", list(_clouds()), ids=[c[0] for c in _clouds()])
def test_knn3_bit_exact(renderer, name, pts):
    x = torch.from_numpy(pts).cuda()
    d = torch.empty(len(pts), dtype=torch.float32, device="cuda")
    renderer.knn3_mean_dist2(x, d)
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    ref = OR.knn3_mean_dist2(pts)
    assert np.array_equal(got, ref), (name, int(np.count_nonzero(got != ref)))


def test_gaussians_from_points_bit_exact(renderer):
    r = np.random.default_rng(9)
    pts = r.normal(size=(5000, 3)).astype(np.float32) * np.array([4, 1, 2], np.float32)
    rgb = r.integers(0, 256, (5000, 3)).astype(np.uint8)
    g = renderer.gaussians_from_points(torch.from_numpy(pts).cuda(), torch.from_numpy(rgb).cuda())
    torch.cuda.synchronize()
    ref = OR.gaussians_from_points(pts, rgb)
    for k in ("means", "scales", "rotations", "opacities", "colors"):
        assert np.array_equal(g[k].cpu().numpy(), ref[k]), k


def test_knn3_million_points_vs_kdtree(renderer):
    """Full-size cloud (1M points): against scipy's float64 k-d tree (the f32 oracle is O(N^2))."""
    spatial = pytest.importorskip("scipy.spatial")
    r = np.random.default_rng(13)
    n = 1 << 20
    pts = np.concatenate([r.normal(size=(n // 2, 3)) * np.array([8, 2, 8]),
                          r.uniform(-10, 10, (n - n // 2, 3))]).astype(np.float32)
    x = torch.from_numpy(pts).cuda()
    d = torch.empty(n, dtype=torch.float32, device="cuda")
    renderer.knn3_mean_dist2(x, d)  # warm-up (module load, allocations)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    renderer.knn3_mean_dist2(x, d)
    ev1.record()
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    sub = r.choice(n, 20000, replace=False)
    tree = spatial.cKDTree(pts.astype(np.float64))
    dd, _ = tree.query(pts[sub].astype(np.float64), k=4)
    ref = (dd[:, 1:] ** 2).mean(1)
    assert np.allclose(got[sub], ref, rtol=5e-5, atol=1e-12)
    print(f"knn3 1M points: {ev0.elapsed_time(ev1):.2f} ms (incl. sort + synchronise)")
