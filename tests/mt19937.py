"""std::mt19937 + libstdc++ std::uniform_real_distribution<double> (test helper).

Reproduces Engine::captureSceneData's pose draws (Vulkan_Engine/engine.cpp:2673-2681):
    std::mt19937 gen(13); alpha = U(0, 360); beta = U(min_beta, max_beta)
libstdc++ generate_canonical<double, 53> consumes two 32-bit draws: (x0 + x1 * 2^32) / 2^64.
"""


class MT19937:
    def __init__(self, seed: int):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            self.mt[i] = (1812433253 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.idx = 624

    def _twist(self):
        for i in range(624):
            y = (self.mt[i] & 0x80000000) | (self.mt[(i + 1) % 624] & 0x7FFFFFFF)
            v = self.mt[(i + 397) % 624] ^ (y >> 1)
            if y & 1:
                v ^= 0x9908B0DF
            self.mt[i] = v
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


def uniform_real(gen: MT19937, a: float, b: float) -> float:
    x0 = gen()
    x1 = gen()
    u = (x0 + x1 * 4294967296.0) / 18446744073709551616.0
    if u >= 1.0:
        u = 1.0 - 2.0 ** -53
    return a + (b - a) * u


def capture_poses(n: int, min_beta: float = -30.0, max_beta: float = 30.0, seed: int = 13):
    """[(alpha, beta)] as floats, in capture order i = 0..n-1."""
    import numpy as np
    g = MT19937(seed)
    out = []
    for _ in range(n):
        a = uniform_real(g, 0.0, 360.0)
        b = uniform_real(g, float(np.float32(min_beta)), float(np.float32(max_beta)))
        out.append((float(np.float32(a)), float(np.float32(b))))
    return out
