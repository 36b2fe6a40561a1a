// hostmath.h — host-side matrix helpers for the boundary (C++).
#pragma once

#include <cmath>
#include <cstring>

namespace ptgs {

// Inverse of a column-major 4x4 float matrix, computed in double (Gauss-Jordan, partial
// pivoting) and rounded to float once. Replaces the per-pixel GLSL inverse(ubo.view) /
// inverse(ubo.proj) of raygen_camera.rgen:32-34 (hoisted to the host, SURVEY §7 hard part #1).
// Returns false for a singular matrix.
inline bool inverse4(const float* m, float* out) {
  double a[4][8];
  for (int r = 0; r < 4; ++r) {
    for (int c = 0; c < 4; ++c) a[r][c] = (double)m[c * 4 + r];
    for (int c = 0; c < 4; ++c) a[r][4 + c] = (r == c) ? 1.0 : 0.0;
  }
  for (int col = 0; col < 4; ++col) {
    int piv = col;
    double best = std::fabs(a[col][col]);
    for (int r = col + 1; r < 4; ++r) {
      double v = std::fabs(a[r][col]);
      if (v > best) { best = v; piv = r; }
    }
    if (best == 0.0) return false;
    if (piv != col) {
      for (int c = 0; c < 8; ++c) { double t = a[col][c]; a[col][c] = a[piv][c]; a[piv][c] = t; }
    }
    double inv = 1.0 / a[col][col];
    for (int c = 0; c < 8; ++c) a[col][c] *= inv;
    for (int r = 0; r < 4; ++r) {
      if (r == col) continue;
      double f = a[r][col];
      if (f == 0.0) continue;
      for (int c = 0; c < 8; ++c) a[r][c] -= f * a[col][c];
    }
  }
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) out[c * 4 + r] = (float)a[r][4 + c];
  return true;
}

}  // namespace ptgs
