"""Torus RaySample generators (product: ptgs_generate_samples, csrc/sampling.cpp) against the
independent Python restatement (oracle/sampling_oracle.py) of Vulkan_Engine/sampling.cpp:5-434 and
the libstdc++ algorithms it calls. Bit-for-bit: every uv, in the Morton order the reference uploads.
Host code only (no GPU)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import sampling_oracle as O
from pathtracer_gaussiansplatting_amd import HITDATA_DTYPE
from pathtracer_gaussiansplatting_amd import sampling as S

SIZES = [0, 1, 2, 3, 16, 17, 100, 1021, 4096]


def _same(got: np.ndarray, ref: np.ndarray):
    g = np.ascontiguousarray(got["uv"], np.float32).reshape(-1, 2)
    assert g.shape == ref.shape
    assert np.array_equal(g.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("method", [S.RANDOM, S.UNIFORM, S.STRATIFIED, S.LHS, S.HALTON])
@pytest.mark.parametrize("n", SIZES)
def test_generators_bit_exact(native_lib, method, n):
    _same(S.update_sampling(method, n), O.generate(method, n))


def test_generators_other_seed(native_lib):
    for m in (S.RANDOM, S.STRATIFIED, S.LHS):
        got = S.update_sampling(m, 777, seed=99)
        ref = {S.RANDOM: O.gen_random, S.STRATIFIED: O.gen_stratified, S.LHS: O.gen_lhs}[m](777, seed=99)
        _same(got, np.array(ref, np.float32).reshape(-1, 2))


def _prev_hits(prev: np.ndarray, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    h = np.zeros(len(prev), HITDATA_DTYPE)
    h["flag"] = np.where(rng.random(len(prev)) < 0.6, 1.0, -1.0)
    h["color"] = rng.random((len(prev), 4)).astype(np.float32)
    # a structured region so the gradient map is not flat
    uv = prev["uv"]
    h["color"][uv[:, 0] > 0.5, :3] *= 0.1
    return h


@pytest.mark.parametrize("method", [S.IMP_COL, S.IMP_HIT])
@pytest.mark.parametrize("res", [256, 16])
def test_importance_resamplers_bit_exact(native_lib, method, res):
    prev = S.update_sampling(S.HALTON, 3000)
    hits = _prev_hits(prev, 5)
    got = S.update_sampling(method, 2000, prev, hits, grid_resolution=res)
    pu = [(np.float32(a), np.float32(b)) for a, b in prev["uv"]]
    if method == S.IMP_COL:
        ref = O.gen_importance_color(2000, pu, hits["color"], res=res)
    else:
        ref = O.gen_importance_hits(2000, pu, hits["flag"], res=res)
    _same(got, np.array(ref, np.float32).reshape(-1, 2))


def test_importance_shorter_hits_and_fallback(native_lib):
    prev = S.update_sampling(S.RANDOM, 500)
    hits = _prev_hits(prev, 6)[:300]  # binning stops at the shorter of the two (sampling.cpp:77, :221)
    got = S.update_sampling(S.IMP_HIT, 400, prev, hits)
    pu = [(np.float32(a), np.float32(b)) for a, b in prev["uv"]]
    _same(got, np.array(O.gen_importance_hits(400, pu, hits["flag"]), np.float32).reshape(-1, 2))
    # no previous samples: Halton fallback (sampling.cpp:389-392)
    _same(S.update_sampling(S.IMP_COL, 321), O.generate(S.HALTON, 321))


def test_morton_sort_ties(native_lib):
    """std::sort is not stable: equal Morton codes must come out in introsort's order."""
    rng = np.random.default_rng(3)
    cells = rng.integers(0, 40, (3000, 2))
    uv = ((cells + rng.random((3000, 2)) * 0.5) / np.float32(32768.0)).astype(np.float32)
    uv[::7] = np.float32(2.0)  # clamped to 32767 on both axes (many equal keys)
    uv[::11] = np.float32(-1.0)
    got = S.sort_samples(uv)
    ref = np.array(O.sort_samples([(np.float32(a), np.float32(b)) for a, b in uv]), np.float32)
    _same(got, ref)
    assert S.morton2d(1.0, 1.0) == O.morton2d(np.float32(1.0), np.float32(1.0)) == 0x3FFFFFFF


def test_invalid_arguments(native_lib):
    from pathtracer_gaussiansplatting_amd import PtgsError
    with pytest.raises(PtgsError):
        S.update_sampling(7, 10)
    with pytest.raises(PtgsError):
        S.update_sampling(S.IMP_COL, 10, np.zeros((4, 2), np.float32), None, grid_resolution=-3)


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_gxx_argument_order(tmp_path):
    """The oracle's RANDOM draws v before u because g++ evaluates glm::vec2(dis(gen), dis(gen))'s
    arguments right to left (sampling.cpp:175): checked on this image's g++ with a two-argument
    constructor of the same shape."""
    src = tmp_path / "order.cpp"
    src.write_text(
        "#include <cstdio>\n#include <random>\n"
        "struct V2 { float x, y; V2(float a, float b) : x(a), y(b) {} };\n"
        "int main() { std::mt19937 g(13); std::uniform_real_distribution<float> d(0.0f, 1.0f);\n"
        "  V2 v(d(g), d(g)); std::mt19937 h(13); float a = d(h); float b = d(h);\n"
        "  std::printf(\"%d\\n\", (v.y == a && v.x == b) ? 1 : 0); }\n")
    exe = tmp_path / "order"
    subprocess.run(["g++", "-O2", "-o", str(exe), str(src)], check=True)
    assert subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.strip() == "1"
