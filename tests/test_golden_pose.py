"""Pose KAT: the reference's only golden vectors, dataset/transforms_{train,test}.json
(copied to tests/golden/). They are reproducible from mt19937(13) draws -> Camera::updateToroidalAngles
(R=3.5, h=3, showcase/subjects/bunny.json) -> inverse(view) (engine.cpp:2673-2681, :2759-2761,
camera.cpp:195-228), written row-wise as m[col][row] (engine.cpp:2833-2839).

Pins both the oracle's camera restatement and the product's host camera (the ubo.view boundary).
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

from mt19937 import capture_poses

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TOL = 2e-5


def _frames():
    train = json.load(open(os.path.join(GOLDEN, "transforms_train.json")))
    test = json.load(open(os.path.join(GOLDEN, "transforms_test.json")))
    frames = {}
    for f in train["frames"] + test["frames"]:
        frames[int(f["file_path"].split("_")[-1])] = np.array(f["transform_matrix"], np.float64)
    return frames, train, test


def test_golden_split_and_count():
    frames, train, test = _frames()
    assert len(train["frames"]) == 48 and len(test["frames"]) == 16
    assert sorted(frames) == list(range(64))
    # i % 4 == 0 -> test split (engine.cpp:2763)
    assert all(int(f["file_path"].split("_")[-1]) % 4 == 0 for f in test["frames"])


def test_mt19937_reference_first_pose():
    (a, b), = capture_poses(1)
    assert abs(a - 218.6429) < 1e-3 and abs(b - 21.5660) < 1e-3


@pytest.mark.parametrize("which", ["oracle", "product"])
def test_pose_kat(which, oracle_lib, native_lib):
    frames, _, _ = _frames()
    poses = capture_poses(64)
    worst = 0.0
    for i, (alpha, beta) in enumerate(poses):
        if which == "oracle":
            view, _, _ = oracle_lib.camera_toroidal(alpha, beta, 3.5, 3.0, 60.0, 16 / 9)
            inv = oracle_lib.mat4_inverse(view).reshape(4, 4)  # [col][row]
        else:
            from pathtracer_gaussiansplatting_amd import Camera, mat4_inverse
            pose = Camera(aspect=16 / 9).toroidal(alpha, beta, 3.5, 3.0)
            inv = mat4_inverse(pose.view).reshape(4, 4)
        rows = inv.T
        worst = max(worst, float(np.max(np.abs(rows - frames[i]))))
    assert worst < TOL, worst


def test_camera_angle_x_convention():
    """saveTransformsJson: camera_angle_x = 2*atan(tan(fov_y/2)*aspect) (engine.cpp:2819-2825)."""
    _, train, _ = _frames()
    fov_x = train["camera_angle_x"]
    aspect = 16 / 9
    fov_y = 2 * np.arctan(np.tan(fov_x / 2) / aspect)
    assert 85.0 < np.degrees(fov_y) < 87.0  # the capture ran with fov_y ~86 deg


GOLDEN_FOV_DEG = 86.5008544921875  # the golden capture's camera fov (a zoomed state): the float whose
                                   # camera_angle_x = 2 atan(tan(fov_y / 2) * 16/9) is the golden value


def _capture_transforms(native_lib, n=64):
    from pathtracer_gaussiansplatting_amd import capture
    poses = capture.capture_poses(n, seed=13, min_beta=-30.0, max_beta=30.0, lib=native_lib)
    train, test = ([], []), ([], [])
    view = (C.c_float * 16)()
    proj = (C.c_float * 16)()
    for i, (a, b) in enumerate(poses):
        native_lib.ptgs_camera_toroidal(float(a), float(b), 3.5, 3.0, GOLDEN_FOV_DEG, 16 / 9, 0.1, 10000.0,
                                        view, proj, None)
        inv = capture.inverse_glm(np.frombuffer(view, np.float32), lib=native_lib)
        dst = test if i % 4 == 0 else train
        dst[0].append(f"./train/r_{i}")
        dst[1].append(inv)
    return train, test


def test_product_capture_poses_match_mt19937_emulation(native_lib):
    """ptgs_capture_poses (std::mt19937 + uniform_real_distribution<double>, as the reference) vs the
    Python emulation used by the oracle tests."""
    from pathtracer_gaussiansplatting_amd import capture
    got = capture.capture_poses(64, seed=13, min_beta=-30.0, max_beta=30.0, lib=native_lib)
    ref = np.array(capture_poses(64), np.float32)
    assert np.array_equal(got, ref)


def test_golden_transforms_bytes(native_lib, tmp_path):
    """The whole capture-side pose chain — mt19937 draws, updateToroidalAngles, glm::inverse restated,
    the nlohmann dump(4) writer — reproduces dataset/transforms_train.json and transforms_test.json
    byte for byte (camera.cpp's unqualified cos / sin of the toroidal position are the double C
    library functions: with float cosf / sinf pose 36 came out 2 ulps off)."""
    from pathtracer_gaussiansplatting_amd import capture
    train, test = _capture_transforms(native_lib)
    p_train, p_test = str(tmp_path / "train.json"), str(tmp_path / "test.json")
    capture.write_transforms_json(p_train, GOLDEN_FOV_DEG, 16 / 9, train[0], np.array(train[1]), lib=native_lib)
    capture.write_transforms_json(p_test, GOLDEN_FOV_DEG, 16 / 9, test[0], np.array(test[1]), lib=native_lib)
    assert open(p_train, "rb").read() == open(os.path.join(GOLDEN, "transforms_train.json"), "rb").read()
    assert open(p_test, "rb").read() == open(os.path.join(GOLDEN, "transforms_test.json"), "rb").read()


def test_ply_and_jpeg_writers(native_lib, tmp_path):
    from pathtracer_gaussiansplatting_amd import capture
    from pathtracer_gaussiansplatting_amd._abi import HITDATA_DTYPE
    hits = np.zeros(5, HITDATA_DTYPE)
    hits["flag"] = [1.0, -1.0, 2.0, 0.0, 0.5]
    hits["pos"] = np.arange(15, dtype=np.float32).reshape(5, 3) * 0.125
    hits["normal"] = [0.0, 1.0, 0.0]
    hits["color"] = [[0.5, 1.0, 0.999, 1.0]] * 5
    p = str(tmp_path / "p.ply")
    assert capture.write_ply(p, hits, lib=native_lib) == 3
    lines = open(p).read().splitlines()
    assert lines[0] == "ply" and lines[2] == "element vertex 3" and lines[12] == "end_header"
    assert lines[13] == "0 0.125 0.25 0 1 0 127 255 254"  # int(c * 255) truncates
    assert lines[15] == "1.5 1.625 1.75 0 1 0 127 255 254" and len(lines) == 16
    PIL = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(2)
    yy, xx = np.mgrid[0:45, 0:70]
    img = np.stack([xx * 3, yy * 5, (xx + yy) * 2, np.full_like(xx, 255)], -1).astype(np.uint8)
    img[10:20, 10:30, :3] = rng.integers(0, 256, (10, 20, 3))
    for q in (90, 95):
        j = str(tmp_path / f"i{q}.jpg")
        capture.write_jpeg(j, img, quality=q, lib=native_lib)
        dec = np.asarray(PIL.open(j).convert("RGB")).astype(np.float64)
        assert dec.shape == (45, 70, 3)
        smooth = np.ones((45, 70), bool)
        smooth[8:22, 8:32] = False
        mse = np.mean((dec[smooth] - img[..., :3][smooth]) ** 2)
        assert 10 * np.log10(255.0 ** 2 / mse) > 35.0, mse
