// Float vector / matrix helpers for the scene ingest, each written in the operation order of the
// GLM functions the reference calls (GLM 0.9.9, the copy the reference vendors under
// Helpers/tinygltf-release/examples/common/glm): results round exactly as the reference's
// (IEEE f32, no FMA contraction — build flag -ffp-contract=off). Column-major: m.c[col][row].
#pragma once
#include <cmath>

namespace ptgs {
namespace glm {

struct vec3 { float x = 0, y = 0, z = 0; };
struct vec4 { float x = 0, y = 0, z = 0, w = 0; };
struct quat { float w = 1, x = 0, y = 0, z = 0; };
struct mat3 { float c[3][3]; };
struct mat4 { float c[4][4]; };

inline vec3 v3(float x, float y, float z) { vec3 r; r.x = x; r.y = y; r.z = z; return r; }
inline vec4 v4(float x, float y, float z, float w) { vec4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
inline vec3 xyz(const vec4& v) { return v3(v.x, v.y, v.z); }

inline vec3 operator+(const vec3& a, const vec3& b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline vec3 operator-(const vec3& a, const vec3& b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline vec3 operator*(const vec3& a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
inline vec3 operator*(float s, const vec3& a) { return v3(s * a.x, s * a.y, s * a.z); }
inline vec4 operator*(const vec4& a, float s) { return v4(a.x * s, a.y * s, a.z * s, a.w * s); }
inline vec4 operator+(const vec4& a, const vec4& b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// compute_dot<vec3>: tmp = a * b; (tmp.x + tmp.y) + tmp.z
inline float dot(const vec3& a, const vec3& b) {
  float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
  return (tx + ty) + tz;
}
inline float length(const vec3& v) { return std::sqrt(dot(v, v)); }
// normalize = v * inversesqrt(dot(v, v)), inversesqrt(x) = 1 / sqrt(x)
inline vec3 normalize(const vec3& v) { return v * (1.0f / std::sqrt(dot(v, v))); }
inline vec3 cross(const vec3& a, const vec3& b) {
  return v3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
inline vec3 min(const vec3& a, const vec3& b) {  // glm::min(x, y) = (y < x) ? y : x
  return v3(b.x < a.x ? b.x : a.x, b.y < a.y ? b.y : a.y, b.z < a.z ? b.z : a.z);
}
inline vec3 max(const vec3& a, const vec3& b) {  // glm::max(x, y) = (x < y) ? y : x
  return v3(a.x < b.x ? b.x : a.x, a.y < b.y ? b.y : a.y, a.z < b.z ? b.z : a.z);
}

inline mat4 identity4() {
  mat4 m;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) m.c[i][j] = i == j ? 1.0f : 0.0f;
  return m;
}
inline mat3 identity3() {
  mat3 m;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) m.c[i][j] = i == j ? 1.0f : 0.0f;
  return m;
}

// mat4 * mat4: Result[i] = ((A0 * B[i][0] + A1 * B[i][1]) + A2 * B[i][2]) + A3 * B[i][3]
inline mat4 mul(const mat4& a, const mat4& b) {
  mat4 r;
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 4; ++k) {
      float s = a.c[0][k] * b.c[i][0] + a.c[1][k] * b.c[i][1];
      s = s + a.c[2][k] * b.c[i][2];
      r.c[i][k] = s + a.c[3][k] * b.c[i][3];
    }
  return r;
}
// mat4 * vec4: (m0 * v0 + m1 * v1) + (m2 * v2 + m3 * v3)
inline vec4 mul(const mat4& m, const vec4& v) {
  float r[4];
  const float vv[4] = {v.x, v.y, v.z, v.w};
  for (int k = 0; k < 4; ++k) {
    float a0 = m.c[0][k] * vv[0] + m.c[1][k] * vv[1];
    float a1 = m.c[2][k] * vv[2] + m.c[3][k] * vv[3];
    r[k] = a0 + a1;
  }
  return v4(r[0], r[1], r[2], r[3]);
}
// mat3 * vec3: ((m[0][k] * x + m[1][k] * y) + m[2][k] * z)
inline vec3 mul(const mat3& m, const vec3& v) {
  float r[3];
  for (int k = 0; k < 3; ++k) r[k] = (m.c[0][k] * v.x + m.c[1][k] * v.y) + m.c[2][k] * v.z;
  return v3(r[0], r[1], r[2]);
}
// scalar * mat4 and mat4 + mat4 (skinning blend)
inline mat4 scale(const mat4& m, float s) {
  mat4 r;
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 4; ++k) r.c[i][k] = m.c[i][k] * s;
  return r;
}
inline mat4 add(const mat4& a, const mat4& b) {
  mat4 r;
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 4; ++k) r.c[i][k] = a.c[i][k] + b.c[i][k];
  return r;
}
inline mat3 upper3(const mat4& m) {
  mat3 r;
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) r.c[i][k] = m.c[i][k];
  return r;
}
inline mat3 transpose(const mat3& m) {
  mat3 r;
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) r.c[i][k] = m.c[k][i];
  return r;
}
inline mat4 transpose(const mat4& m) {
  mat4 r;
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 4; ++k) r.c[i][k] = m.c[k][i];
  return r;
}
// compute_inverse<3, 3>
inline mat3 inverse(const mat3& mm) {
  const float(*m)[3] = mm.c;
  float ood = 1.0f / (+m[0][0] * (m[1][1] * m[2][2] - m[2][1] * m[1][2])
                      - m[1][0] * (m[0][1] * m[2][2] - m[2][1] * m[0][2])
                      + m[2][0] * (m[0][1] * m[1][2] - m[1][1] * m[0][2]));
  mat3 r;
  r.c[0][0] = +(m[1][1] * m[2][2] - m[2][1] * m[1][2]) * ood;
  r.c[1][0] = -(m[1][0] * m[2][2] - m[2][0] * m[1][2]) * ood;
  r.c[2][0] = +(m[1][0] * m[2][1] - m[2][0] * m[1][1]) * ood;
  r.c[0][1] = -(m[0][1] * m[2][2] - m[2][1] * m[0][2]) * ood;
  r.c[1][1] = +(m[0][0] * m[2][2] - m[2][0] * m[0][2]) * ood;
  r.c[2][1] = -(m[0][0] * m[2][1] - m[2][0] * m[0][1]) * ood;
  r.c[0][2] = +(m[0][1] * m[1][2] - m[1][1] * m[0][2]) * ood;
  r.c[1][2] = -(m[0][0] * m[1][2] - m[1][0] * m[0][2]) * ood;
  r.c[2][2] = +(m[0][0] * m[1][1] - m[1][0] * m[0][1]) * ood;
  return r;
}
// translate(m, v): Result[3] = ((m0 * v0 + m1 * v1) + m2 * v2) + m3
inline mat4 translate(const mat4& m, const vec3& v) {
  mat4 r = m;
  for (int k = 0; k < 4; ++k) {
    float s = m.c[0][k] * v.x + m.c[1][k] * v.y;
    s = s + m.c[2][k] * v.z;
    r.c[3][k] = s + m.c[3][k];
  }
  return r;
}
// scale(m, v): Result[i] = m[i] * v[i] (i < 3), Result[3] = m[3]
inline mat4 scale(const mat4& m, const vec3& v) {
  mat4 r = m;
  const float s[3] = {v.x, v.y, v.z};
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 4; ++k) r.c[i][k] = m.c[i][k] * s[i];
  return r;
}
// rotate(m, angle, axis)
inline mat4 rotate(const mat4& m, float angle, const vec3& v) {
  float c = std::cos(angle), s = std::sin(angle);
  vec3 axis = normalize(v);
  vec3 temp = (1.0f - c) * axis;
  float R[3][3];
  R[0][0] = c + temp.x * axis.x;
  R[0][1] = temp.x * axis.y + s * axis.z;
  R[0][2] = temp.x * axis.z - s * axis.y;
  R[1][0] = temp.y * axis.x - s * axis.z;
  R[1][1] = c + temp.y * axis.y;
  R[1][2] = temp.y * axis.z + s * axis.x;
  R[2][0] = temp.z * axis.x + s * axis.y;
  R[2][1] = temp.z * axis.y - s * axis.x;
  R[2][2] = c + temp.z * axis.z;
  mat4 r;
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 4; ++k) {
      float t = m.c[0][k] * R[i][0] + m.c[1][k] * R[i][1];
      r.c[i][k] = t + m.c[2][k] * R[i][2];
    }
  for (int k = 0; k < 4; ++k) r.c[3][k] = m.c[3][k];
  return r;
}
// mat3_cast / mat4_cast
inline mat4 mat4_cast(const quat& q) {
  float qxx = q.x * q.x, qyy = q.y * q.y, qzz = q.z * q.z;
  float qxz = q.x * q.z, qxy = q.x * q.y, qyz = q.y * q.z;
  float qwx = q.w * q.x, qwy = q.w * q.y, qwz = q.w * q.z;
  mat4 r = identity4();
  r.c[0][0] = 1.0f - 2.0f * (qyy + qzz);
  r.c[0][1] = 2.0f * (qxy + qwz);
  r.c[0][2] = 2.0f * (qxz - qwy);
  r.c[1][0] = 2.0f * (qxy - qwz);
  r.c[1][1] = 1.0f - 2.0f * (qxx + qzz);
  r.c[1][2] = 2.0f * (qyz + qwx);
  r.c[2][0] = 2.0f * (qxz + qwy);
  r.c[2][1] = 2.0f * (qyz - qwx);
  r.c[2][2] = 1.0f - 2.0f * (qxx + qyy);
  return r;
}
// quat(vec3 eulerAngle) (radians): c = cos(e * 0.5), s = sin(e * 0.5)
inline quat quat_from_euler(const vec3& e) {
  float cx = std::cos(e.x * 0.5f), cy = std::cos(e.y * 0.5f), cz = std::cos(e.z * 0.5f);
  float sx = std::sin(e.x * 0.5f), sy = std::sin(e.y * 0.5f), sz = std::sin(e.z * 0.5f);
  quat q;
  q.w = cx * cy * cz + sx * sy * sz;
  q.x = sx * cy * cz - cx * sy * sz;
  q.y = cx * sy * cz + sx * cy * sz;
  q.z = cx * cy * sz - sx * sy * cz;
  return q;
}
// glm::radians(vec3)
inline vec3 radians(const vec3& d) {
  const float k = (float)0.01745329251994329576923690768489;
  return v3(d.x * k, d.y * k, d.z * k);
}
// translate(I, t) * mat4_cast(r) * scale(I, s)  (getNodeTransform, updateModelMatrix)
inline mat4 trs(const vec3& t, const quat& r, const vec3& s) {
  return mul(mul(translate(identity4(), t), mat4_cast(r)), scale(identity4(), s));
}

}  // namespace glm
}  // namespace ptgs
