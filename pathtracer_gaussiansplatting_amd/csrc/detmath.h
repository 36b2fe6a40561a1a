// detmath.h — deterministic float32 arithmetic shared by every kernel of the renderer.
//
// Why: Monte-Carlo parity at 1e-4 relative L2 (SURVEY.md §7 "hard parts" #1) needs every
// pixel's path to be the same path as the CPU oracle's, so every float op must round the same
// way. Rules (and the build flags that enforce them, see build.py): IEEE add/sub/mul/div/sqrt
// only, -ffp-contract=off (no FMA contraction), no fast-math; transcendentals are the
// polynomial implementations below instead of ocml/libm (whose last bits differ). The oracle
// (oracle/ptgs_oracle.c) restates the same functions independently in C.
//
// GLSL built-ins are defined here with an explicit evaluation order (GLSL leaves it to the
// implementation): dot = (x*x' + y*y') + z*z', normalize = v / length(v), mix = x*(1-a) + y*a,
// mat*vec = ((c0*x + c1*y) + c2*z) + c3*w, pow(x,5) = (x*x)*(x*x)*x.
#pragma once

#ifdef __HIPCC__
#define PTGS_HD __host__ __device__ __forceinline__
#else
#define PTGS_HD inline
#endif

#include <stdint.h>

namespace ptgs {

struct v2 { float x, y; };
struct v3 { float x, y, z; };
struct v4 { float x, y, z, w; };

PTGS_HD v2 mk2(float x, float y) { v2 r; r.x = x; r.y = y; return r; }
PTGS_HD v3 mk3(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
PTGS_HD v3 mk3(float s) { return mk3(s, s, s); }
// component-wise c ? a : b (a ?: between two v3 values can lower to a select between two stack
// copies: a dynamically addressed private object, i.e. scratch traffic in the path-tracer kernel)
PTGS_HD v3 sel3(bool c, v3 a, v3 b) { return mk3(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }
PTGS_HD v4 mk4(float x, float y, float z, float w) { v4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }

PTGS_HD v3 operator+(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
PTGS_HD v3 operator-(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
PTGS_HD v3 operator*(v3 a, v3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
PTGS_HD v3 operator/(v3 a, v3 b) { return mk3(a.x / b.x, a.y / b.y, a.z / b.z); }
PTGS_HD v3 operator*(v3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
PTGS_HD v3 operator*(float s, v3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
PTGS_HD v3 operator/(v3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
PTGS_HD v3 operator-(v3 a) { return mk3(-a.x, -a.y, -a.z); }
PTGS_HD v3 operator+(v3 a, float s) { return mk3(a.x + s, a.y + s, a.z + s); }
PTGS_HD v3 operator-(float s, v3 a) { return mk3(s - a.x, s - a.y, s - a.z); }

PTGS_HD float fminx(float a, float b) { return b < a ? b : a; }   // GLSL min (no NaN games)
PTGS_HD float fmaxx(float a, float b) { return a < b ? b : a; }   // GLSL max
PTGS_HD float clampf(float x, float lo, float hi) { return fminx(fmaxx(x, lo), hi); }
PTGS_HD v3 vmin(v3 a, float s) { return mk3(fminx(a.x, s), fminx(a.y, s), fminx(a.z, s)); }
PTGS_HD float dot3(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
PTGS_HD v3 cross3(v3 a, v3 b) {
  return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
PTGS_HD float sqrtx(float x) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_sqrtf(x);  // correctly rounded on gfx950 (v_sqrt + fixup; checked in the .s)
#else
  return __builtin_sqrtf(x);
#endif
}
PTGS_HD float length3(v3 v) { return sqrtx(dot3(v, v)); }
PTGS_HD v3 normalize3(v3 v) { return v / length3(v); }
PTGS_HD float floorx(float x) { return __builtin_floorf(x); }
PTGS_HD float fractx(float x) { return x - floorx(x); }
PTGS_HD float absx(float x) { return __builtin_fabsf(x); }
PTGS_HD float mixf(float x, float y, float a) { return x * (1.0f - a) + y * a; }
PTGS_HD v3 mix3(v3 x, v3 y, float a) { return mk3(mixf(x.x, y.x, a), mixf(x.y, y.y, a), mixf(x.z, y.z, a)); }
PTGS_HD float signx(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
PTGS_HD float maxc(v3 v) { return fmaxx(fmaxx(v.x, v.y), v.z); }
PTGS_HD float pow5(float x) { float x2 = x * x; return (x2 * x2) * x; }
PTGS_HD float pow4(float x) { float x2 = x * x; return x2 * x2; }

// reflect(I, N) = I - 2*dot(N,I)*N  (GLSL.std.450 Reflect)
PTGS_HD v3 reflect3(v3 i, v3 n) { float d = 2.0f * dot3(n, i); return i - n * d; }
// refract(I, N, eta) (GLSL.std.450 Refract)
PTGS_HD v3 refract3(v3 i, v3 n, float eta) {
  float ni = dot3(n, i);
  float k = 1.0f - eta * eta * (1.0f - ni * ni);
  if (k < 0.0f) return mk3(0.0f);
  return i * eta - n * (eta * ni + sqrtx(k));
}

// 2^n for integer n in [-126, 127]
PTGS_HD float ldexp_pos(int n) {
  union { uint32_t u; float f; } c;
  c.u = (uint32_t)(n + 127) << 23;
  return c.f;
}

// sin/cos: Cody-Waite reduction by pi/2 (3-part constant, exact k*C1 for |k| < 2^15) and
// Cephes single-precision minimax polynomials on [-pi/4, pi/4]. Arguments on the path are
// bounded (2*pi*[0,1], torus angles), max error ~2 ulp vs libm.
PTGS_HD void sincosx(float x, float* s, float* c) {
  float k = floorx(x * 0.636619772367581343f + 0.5f);
  int q = (int)k;
  float r = x - k * 1.5703125f;
  r = r - k * 4.837512969970703125e-4f;
  r = r - k * 7.54978995489188216e-8f;
  float z = r * r;
  float sp = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
  float cp = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z
             - 0.5f * z + 1.0f;
  int qm = q & 3;
  float so, co;
  if (qm == 0) { so = sp; co = cp; }
  else if (qm == 1) { so = cp; co = -sp; }
  else if (qm == 2) { so = -sp; co = -cp; }
  else { so = -cp; co = sp; }
  *s = so; *c = co;
}
PTGS_HD float sinx(float x) { float s, c; sincosx(x, &s, &c); return s; }
PTGS_HD float cosx(float x) { float s, c; sincosx(x, &s, &c); return c; }

// exp2 on [-126, 128): n = round(x), f in [-0.5, 0.5], degree-6 polynomial for 2^f.
PTGS_HD float exp2x(float x) {
  if (x < -126.0f) return 0.0f;
  if (x > 127.99f) x = 127.99f;
  float n = floorx(x + 0.5f);
  float f = x - n;
  float p = 1.535336188319500e-4f;
  p = p * f + 1.339887440266574e-3f;
  p = p * f + 9.618437357674640e-3f;
  p = p * f + 5.550332471162809e-2f;
  p = p * f + 2.402264791363012e-1f;
  p = p * f + 6.931472028550421e-1f;
  p = p * f + 1.0f;
  int ni = (int)n;
  if (ni > 127) { p = p * 2.0f; ni -= 1; }
  return p * ldexp_pos(ni);
}
PTGS_HD float expx(float x) { return exp2x(x * 1.44269504088896341f); }

// log2 for x > 0 (finite): x = m*2^e with m in [sqrt(1/2), sqrt(2)), atanh series in s=(m-1)/(m+1).
PTGS_HD float log2x(float x) {
  if (!(x > 0.0f)) return -1.0e30f;
  union { float f; uint32_t u; } c; c.f = x;
  int e = (int)((c.u >> 23) & 0xffu) - 127;
  if (e == -127) {  // subnormal: rescale
    c.f = x * 8388608.0f;
    e = (int)((c.u >> 23) & 0xffu) - 127 - 23;
  }
  c.u = (c.u & 0x007fffffu) | 0x3f800000u;
  float m = c.f;
  if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
  float s = (m - 1.0f) / (m + 1.0f);
  float s2 = s * s;
  float p = 0.2222222222f;
  p = p * s2 + 0.2857142857f;
  p = p * s2 + 0.4f;
  p = p * s2 + 0.6666666667f;
  p = p * s2 + 2.0f;
  float ln = s * p;  // ln(m), |s| <= 0.1716
  return (float)e + ln * 1.44269504088896341f;
}
PTGS_HD float powx(float x, float y) { return exp2x(y * log2x(x)); }
PTGS_HD float tanx(float x) { float s, c; sincosx(x, &s, &c); return s / c; }

}  // namespace ptgs
