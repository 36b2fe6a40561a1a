"""CPU ORACLE of the torus RaySample generators — TEST INFRASTRUCTURE ONLY.

Only tests/ use this module, and only as the checker of the product's `ptgs_generate_samples`
(pathtracer_gaussiansplatting_amd/csrc/sampling.cpp).

Restates Vulkan_Engine/sampling.cpp:5-434 (the reference's CPU sample generators for the toroidal
data-collection tracer) in pure Python + numpy float32 scalars, one rounding per C++ float operation,
together with the parts of the C++ standard library those generators call. The reference builds with
the system g++ (Makefile:1-2, setup.sh); the library algorithms below follow libstdc++ of GCC 11 (the
g++ 11.4 of this image), cited by header:line under /usr/include/c++/11:
  std::mt19937                               bits/random.h (Matsumoto-Nishimura MT19937)
  generate_canonical<float, 24>              bits/random.tcc:3348-3378: one 32-bit draw, x / 2^32
  uniform_int_distribution (32-bit engine)   bits/uniform_int_dist.h:246-316: Lemire's method
  std::shuffle                               bits/stl_algo.h:3704-3792: pairs of swaps per draw
  std::sort                                  bits/stl_algo.h:1795-1959 + bits/stl_heap.h:130-426:
                                             introsort (median of 3, threshold 16, heapsort fallback)
std::sort is not stable: equal Morton codes keep the order introsort leaves them in, so the exact
algorithm matters for bit-for-bit sample order. glm::vec2(dis(gen), dis(gen)) (sampling.cpp:175)
evaluates its arguments right to left under g++ (tests/test_sampling.py::test_gxx_argument_order).
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32
ONE = f32(1.0)
TWO32 = f32(4294967296.0)

# sampling_methods order, GeneralHeaders.h:552-560 (engine.cpp:772-790 key bindings)
RANDOM, UNIFORM, STRATIFIED, LHS, HALTON, IMP_COL, IMP_HIT = range(7)


class MT19937:
    """std::mt19937 (32-bit Mersenne twister, default seeding)."""

    def __init__(self, seed: int):
        mt = [0] * 624
        mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.mt = mt
        self.idx = 624

    def _twist(self):
        mt = self.mt
        for i in range(624):
            y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
            v = mt[(i + 397) % 624] ^ (y >> 1)
            if y & 1:
                v ^= 0x9908B0DF
            mt[i] = v
        self.idx = 0

    def __call__(self) -> int:
        if self.idx >= 624:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF


def uniform01(gen: MT19937) -> np.float32:
    """std::uniform_real_distribution<float>(0, 1)(gen): generate_canonical<float, 24> = float(x) / 2^32
    (one draw), clamped below 1 (random.tcc:3362-3378); then * (1 - 0) + 0."""
    r = f32(gen()) / TWO32
    if r >= ONE:
        r = np.nextafter(ONE, f32(0.0))
    return r * f32(1.0) + f32(0.0)


def uniform_int(gen: MT19937, a: int, b: int) -> int:
    """uniform_int_distribution<unsigned long>{a, b}(gen) for b - a < 2^32 - 1 (uniform_int_dist.h:294-316,
    Lemire's nearly divisionless method with a 64-bit product)."""
    erange = (b - a + 1) & 0xFFFFFFFF
    product = gen() * erange
    low = product & 0xFFFFFFFF
    if low < erange:
        threshold = ((1 << 32) - erange) % erange
        while low < threshold:
            product = gen() * erange
            low = product & 0xFFFFFFFF
    return (product >> 32) + a


def shuffle(a: list, gen: MT19937) -> None:
    """std::shuffle (stl_algo.h:3726-3792)."""
    n = len(a)
    if n == 0:
        return
    if (0xFFFFFFFF // n) >= n:
        i = 1
        if n % 2 == 0:
            j = uniform_int(gen, 0, 1)
            a[i], a[j] = a[j], a[i]
            i += 1
        while i != n:
            swap_range = i + 1
            x = uniform_int(gen, 0, swap_range * (swap_range + 1) - 1)
            p1, p2 = x // (swap_range + 1), x % (swap_range + 1)
            a[i], a[p1] = a[p1], a[i]
            i += 1
            a[i], a[p2] = a[p2], a[i]
            i += 1
        return
    for i in range(1, n):
        j = uniform_int(gen, 0, i)
        a[i], a[j] = a[j], a[i]


# ---- std::sort (libstdc++ introsort) over a list of (key, payload) with comp = key < key ----------
def _push_heap(a, first, hole, top, value):
    parent = (hole - 1) // 2
    while hole > top and a[first + parent][0] < value[0]:
        a[first + hole] = a[first + parent]
        hole = parent
        parent = (hole - 1) // 2
    a[first + hole] = value


def _adjust_heap(a, first, hole, length, value):
    top = hole
    second = hole
    while second < (length - 1) // 2:
        second = 2 * (second + 1)
        if a[first + second][0] < a[first + second - 1][0]:
            second -= 1
        a[first + hole] = a[first + second]
        hole = second
    if (length & 1) == 0 and second == (length - 2) // 2:
        second = 2 * (second + 1)
        a[first + hole] = a[first + second - 1]
        hole = second - 1
    _push_heap(a, first, hole, top, value)


def _pop_heap(a, first, last, result):
    value = a[result]
    a[result] = a[first]
    _adjust_heap(a, first, 0, last - first, value)


def _make_heap(a, first, last):
    length = last - first
    if length < 2:
        return
    parent = (length - 2) // 2
    while True:
        _adjust_heap(a, first, parent, length, a[first + parent])
        if parent == 0:
            return
        parent -= 1


def _partial_sort_all(a, first, last):  # __partial_sort(first, last, last): heap_select + sort_heap
    _make_heap(a, first, last)
    while last - first > 1:
        last -= 1
        _pop_heap(a, first, last, last)


def _move_median_to_first(a, result, i, j, k):
    A, B, C = a[i][0], a[j][0], a[k][0]
    if A < B:
        if B < C:
            s = j
        elif A < C:
            s = k
        else:
            s = i
    elif A < C:
        s = i
    elif B < C:
        s = k
    else:
        s = j
    a[result], a[s] = a[s], a[result]


def _unguarded_partition(a, first, last, pivot):
    pk = a[pivot][0]
    while True:
        while a[first][0] < pk:
            first += 1
        last -= 1
        while pk < a[last][0]:
            last -= 1
        if not first < last:
            return first
        a[first], a[last] = a[last], a[first]
        first += 1


def _introsort_loop(a, first, last, depth):
    while last - first > 16:
        if depth == 0:
            _partial_sort_all(a, first, last)
            return
        depth -= 1
        mid = first + (last - first) // 2
        _move_median_to_first(a, first, first + 1, mid, last - 1)
        cut = _unguarded_partition(a, first + 1, last, first)
        _introsort_loop(a, cut, last, depth)
        last = cut


def _unguarded_linear_insert(a, last):
    val = a[last]
    nxt = last - 1
    while val[0] < a[nxt][0]:
        a[last] = a[nxt]
        last = nxt
        nxt -= 1
    a[last] = val


def _insertion_sort(a, first, last):
    if first == last:
        return
    for i in range(first + 1, last):
        if a[i][0] < a[first][0]:
            val = a[i]
            a[first + 1:i + 1] = a[first:i]
            a[first] = val
        else:
            _unguarded_linear_insert(a, i)


def std_sort(a: list) -> None:
    """std::sort(begin, end, comp) on (key, payload) pairs (stl_algo.h:1946-1959)."""
    n = len(a)
    if n == 0:
        return
    _introsort_loop(a, 0, n, (n.bit_length() - 1) * 2)
    if n > 16:
        _insertion_sort(a, 0, 16)
        for i in range(16, n):
            _unguarded_linear_insert(a, i)
    else:
        _insertion_sort(a, 0, n)


# ---- sampling.cpp -----------------------------------------------------------------------------------
def _expand_bits(v: int) -> int:  # sampling.cpp:335-343
    x = v
    x = (x | (x << 8)) & 0x00FF00FF
    x = (x | (x << 4)) & 0x0F0F0F0F
    x = (x | (x << 2)) & 0x33333333
    x = (x | (x << 1)) & 0x55555555
    return x


def morton2d(u: np.float32, v: np.float32) -> int:  # sampling.cpp:346-354 (std::clamp, then (uint16_t))
    x = u * f32(32768.0)
    x = f32(0.0) if x < f32(0.0) else (f32(32767.0) if f32(32767.0) < x else x)
    y = v * f32(32768.0)
    y = f32(0.0) if y < f32(0.0) else (f32(32767.0) if f32(32767.0) < y else y)
    return (_expand_bits(int(x)) | (_expand_bits(int(y)) << 1)) & 0xFFFFFFFF


def sort_samples(uv: list) -> list:  # sampling.cpp:356-361
    a = [(morton2d(u, v), (u, v)) for (u, v) in uv]
    std_sort(a)
    return [p for _, p in a]


def halton(index: int, base: int) -> np.float32:  # sampling.cpp:5-16
    f = f32(1.0)
    r = f32(0.0)
    while index > 0:
        f = f / f32(base)
        r = r + f * f32(index % base)
        index = index // base
    return r


def _grid_dims(n: int):  # sampling.cpp:40-41 / :187-188
    cols = int(math.ceil(math.sqrt(float(n))))
    if cols == 0:  # n == 0: the reference divides 0.f / 0 but never uses rows
        return 0, 0
    rows = int(math.ceil(f32(n) / f32(cols)))
    return cols, rows


def gen_halton(n):  # :18-32
    return sort_samples([(halton(i + 1, 2), halton(i + 1, 3)) for i in range(n)])


def gen_stratified(n, seed=13):  # :34-61
    cols, rows = _grid_dims(n)
    g = MT19937(seed)
    out = []
    for i in range(n):
        y, x = i // cols, i % cols
        u = (f32(x) + uniform01(g)) / f32(cols)
        v = (f32(y) + uniform01(g)) / f32(rows)
        out.append((u, v))
    return sort_samples(out)


def gen_random(n, seed=13):  # :164-179; glm::vec2(dis(gen), dis(gen)): g++ draws v first
    g = MT19937(seed)
    out = []
    for _ in range(n):
        v = uniform01(g)
        u = uniform01(g)
        out.append((u, v))
    return sort_samples(out)


def gen_uniform(n):  # :181-204
    cols, rows = _grid_dims(n)
    out = []
    for i in range(n):
        y, x = i // cols, i % cols
        out.append(((f32(x) + f32(0.5)) / f32(cols), (f32(y) + f32(0.5)) / f32(rows)))
    return sort_samples(out)


def gen_lhs(n, seed=13):  # :292-333
    ui = list(range(n))
    vi = list(range(n))
    g = MT19937(seed)
    shuffle(ui, g)
    shuffle(vi, g)
    out = []
    for i in range(n):
        u = (f32(ui[i]) + uniform01(g)) / f32(n)
        v = (f32(vi[i]) + uniform01(g)) / f32(n)
        out.append((u, v))
    return sort_samples(out)


def _bin(uvx: np.float32, res: int) -> int:
    k = int(uvx * f32(res))  # static_cast<int>(uv * grid_resolution): truncation
    return min(max(k, 0), res - 1)


def _inverse_cdf_samples(n, importance, res, seed):  # :120-161 / :253-290
    total = f32(0.0)
    for w in importance:
        total = total + w
    cdf = np.zeros(len(importance), np.float32)
    s = f32(0.0)
    for i, w in enumerate(importance):
        s = s + w
        cdf[i] = s
    cdf = (cdf / total).astype(np.float32)
    g = MT19937(seed)
    out = []
    for _ in range(n):
        r = uniform01(g)
        idx = int(np.searchsorted(cdf, r, side="left"))  # std::lower_bound
        y, x = idx // res, idx % res
        u = (f32(x) + uniform01(g)) / f32(res)
        v = (f32(y) + uniform01(g)) / f32(res)
        out.append((u, v))
    return sort_samples(out)


def gen_importance_color(n, prev_uv, prev_rgba, res=256, seed=13):  # :63-161
    cells = res * res
    col = [[f32(0.0)] * 3 for _ in range(cells)]
    cnt = [f32(0.0)] * cells
    for i in range(len(prev_uv)):
        if i >= len(prev_rgba):
            break
        x, y = _bin(prev_uv[i][0], res), _bin(prev_uv[i][1], res)
        k = y * res + x
        for c in range(3):
            col[k][c] = col[k][c] + f32(prev_rgba[i][c])
        cnt[k] = cnt[k] + f32(1.0)
    for k in range(cells):
        if cnt[k] > f32(0.0):
            col[k] = [col[k][c] / cnt[k] for c in range(3)]

    def lum(x, y):
        if x < 0 or x >= res or y < 0 or y >= res:
            return f32(0.0)
        c = col[y * res + x]
        return (f32(0.2126) * c[0] + f32(0.7152) * c[1]) + f32(0.0722) * c[2]

    imp = []
    for y in range(res):
        for x in range(res):
            dx = lum(x + 1, y) - lum(x - 1, y)
            dy = lum(x, y + 1) - lum(x, y - 1)
            grad = np.sqrt(dx * dx + dy * dy, dtype=np.float32)
            imp.append(grad + f32(0.05))
    return _inverse_cdf_samples(n, imp, res, seed)


def gen_importance_hits(n, prev_uv, prev_flags, res=256, seed=13):  # :207-290
    cells = res * res
    hits = [f32(0.0)] * cells
    cnt = [f32(0.0)] * cells
    for i in range(len(prev_uv)):
        if i >= len(prev_flags):
            break
        x, y = _bin(prev_uv[i][0], res), _bin(prev_uv[i][1], res)
        k = y * res + x
        hits[k] = hits[k] + (f32(1.0) if f32(prev_flags[i]) > f32(0.0) else f32(0.0))
        cnt[k] = cnt[k] + f32(1.0)
    imp = []
    for k in range(cells):
        ratio = hits[k] / cnt[k] if cnt[k] > f32(0.0) else f32(0.0)
        imp.append(ratio + f32(0.01))
    return _inverse_cdf_samples(n, imp, res, seed)


def generate(method: int, n: int, prev_uv=None, prev_hits=None) -> np.ndarray:
    """Sampling::updateSampling (sampling.cpp:366-419) -> (n, 2) float32 uv array.
    prev_uv: (m, 2) float32; prev_hits: HitData records (fields 'color' (m, 4) and 'flag' (m,))."""
    if method == HALTON:
        uv = gen_halton(n)
    elif method == LHS:
        uv = gen_lhs(n)
    elif method == STRATIFIED:
        uv = gen_stratified(n)
    elif method == RANDOM:
        uv = gen_random(n)
    elif method == UNIFORM:
        uv = gen_uniform(n)
    elif prev_uv is None or len(prev_uv) == 0:  # :390-392: fall back to Halton
        uv = gen_halton(n)
    else:
        pu = [(f32(a), f32(b)) for a, b in np.asarray(prev_uv, np.float32).reshape(-1, 2)]
        if method == IMP_COL:
            uv = gen_importance_color(n, pu, np.asarray(prev_hits["color"], np.float32))
        elif method == IMP_HIT:
            uv = gen_importance_hits(n, pu, np.asarray(prev_hits["flag"], np.float32))
        else:
            raise ValueError(f"unknown sampling method {method}")
    return np.array(uv, np.float32).reshape(-1, 2)
