"""Torus RaySample generators — binding of ptgs_generate_samples (csrc/sampling.cpp), mirroring the
reference's `Sampling` namespace (Vulkan_Engine/sampling.h, sampling.cpp:5-434).

`update_sampling(method, n, samples, hits)` is Sampling::updateSampling's generation step: it returns
the n Morton-sorted RaySamples the Engine would upload for sampling method `method` (the index into
sampling_methods, GeneralHeaders.h:552-560). The importance methods resample from the previous samples
and the HitData read back after tracing them; with no previous samples they fall back to Halton.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import HITDATA_DTYPE, RAY_SAMPLE_DTYPE

RANDOM, UNIFORM, STRATIFIED, LHS, HALTON, IMP_COL, IMP_HIT = range(7)
METHOD_NAMES = ("RANDOM", "UNIFORM", "STRATIFIED", "LHS", "HALTON", "IMP_COL", "IMP_HIT")
REFERENCE_SEED = 13  # sampling.cpp:3
GRID_RESOLUTION = 256  # sampling.h:17, :29


def _as_samples(a) -> np.ndarray:
    a = np.asarray(a)
    if a.dtype == RAY_SAMPLE_DTYPE:
        return np.ascontiguousarray(a)
    uv = np.ascontiguousarray(a, dtype=np.float32).reshape(-1, 2)
    out = np.zeros(len(uv), RAY_SAMPLE_DTYPE)
    out["uv"] = uv
    return out


def update_sampling(method: int, n: int, prev_samples=None, prev_hits=None, seed: int = REFERENCE_SEED,
                    grid_resolution: int = GRID_RESOLUTION) -> np.ndarray:
    """n RaySamples (RAY_SAMPLE_DTYPE) for `method`. prev_samples: RaySamples or an (m, 2) float32 array;
    prev_hits: HITDATA_DTYPE records of those samples (importance methods only)."""
    lib = _abi.load_library()
    out = np.zeros(int(n), RAY_SAMPLE_DTYPE)
    ps = _as_samples(prev_samples) if prev_samples is not None else np.zeros(0, RAY_SAMPLE_DTYPE)
    ph = np.ascontiguousarray(prev_hits, dtype=HITDATA_DTYPE) if prev_hits is not None else np.zeros(0, HITDATA_DTYPE)
    rc = lib.ptgs_generate_samples(int(method), int(n), ps.ctypes.data if len(ps) else None, len(ps),
                                   ph.ctypes.data if len(ph) else None, len(ph), int(seed), int(grid_resolution),
                                   out.ctypes.data if len(out) else None)
    _abi.check(rc, f"ptgs_generate_samples({METHOD_NAMES[method] if 0 <= method < 7 else method})")
    return out


def sort_samples(samples) -> np.ndarray:
    """Sampling::sortSamples: Morton order (std::sort, not stable)."""
    s = _as_samples(samples).copy()
    _abi.check(_abi.load_library().ptgs_sort_samples(s.ctypes.data if len(s) else None, len(s)), "ptgs_sort_samples")
    return s


def morton2d(u: float, v: float) -> int:
    return int(_abi.load_library().ptgs_morton2d(C.c_float(u), C.c_float(v)))
