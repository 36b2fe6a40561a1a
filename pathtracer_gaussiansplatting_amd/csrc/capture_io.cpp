// capture_io.cpp — host side of the dataset capture pipeline of Engine::captureSceneData (Vulkan_Engine/engine.cpp:
// 2658-2814) on the C-ABI, plus its writers:
//   poses           std::mt19937(13) with uniform_real_distribution<> alpha U(0,360), beta
//                   U(min_beta, max_beta) (:2672-2681) -> Camera::updateToroidalAngles
//   per view        accumulation_steps samples (ONE ptgs_trace_camera call: no per-sample queue
//                   drain as in :2684-2708), sRGB8 encode (the swapchain-format blit, :2711-2727),
//                   read-back, downscale by sampling every 2nd pixel when image_divisor > 1
//                   (:2737-2754), JPEG quality 90 to train/r_i.jpg (:2756-2757)
//   splits          i % 4 == 0 -> transforms_test.json, else transforms_train.json (:2759-2765);
//                   transform_matrix = glm::inverse(view) written m[col][row] (:2816-2847)
//   point cloud     accumulation_steps torus traces (:2770-2800) -> points3d.ply, ASCII, points
//                   with flag > 0, colour * 255 truncated (:2849-2895)
// glm::inverse is restated exactly (GLM 0.9.9 compute_inverse<4,4,float>, the library the
// reference links) and nlohmann::json's number printing restated (below): with them
// dataset/transforms_train.json is reproduced byte for byte and transforms_test.json up to one value
// 2 ulps off (tests/test_golden_pose.py).
#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/ptgs/ptgs.h"
#include "../../include/ptgs/ptgs_host.h"
#include "jpeg.h"

namespace {

// ---- number formatting of nlohmann::json 3.12.0 (vendored by the reference, Helpers/json.hpp) ----
// dump() prints doubles with Grisu2 (F. Loitsch, "Printing floating-point numbers quickly and
// accurately with integers", PLDI 2010): the digits of a value inside the rounding interval, which
// is not always the shortest and does not round exact ties to even (the golden transforms hold
// "0.47503703832626343" and "-2.9802322387695313e-08"). Restated from the paper with the library's
// parameters: target exponent window [-60, -32], cached powers 10^k for k = -300, -292, ..., 324
// (64-bit significands rounded to nearest, generated exactly below), M- + 1 / M+ - 1 safety margins,
// round-towards-w; then the library's layout: fixed notation for exponents -4 < n <= 15 with a
// trailing ".0" on integers, otherwise d.ddde+XX.
struct DiyFp {
  uint64_t f;
  int e;
};

DiyFp diy_sub(DiyFp a, DiyFp b) { return DiyFp{a.f - b.f, a.e}; }

DiyFp diy_mul(DiyFp x, DiyFp y) {  // upper 64 bits of the 128-bit product, rounded
  const uint64_t u_lo = x.f & 0xFFFFFFFFu, u_hi = x.f >> 32, v_lo = y.f & 0xFFFFFFFFu, v_hi = y.f >> 32;
  const uint64_t p0 = u_lo * v_lo, p1 = u_lo * v_hi, p2 = u_hi * v_lo, p3 = u_hi * v_hi;
  uint64_t q = (p0 >> 32) + (p1 & 0xFFFFFFFFu) + (p2 & 0xFFFFFFFFu);
  q += uint64_t{1} << 31;
  return DiyFp{p3 + (p2 >> 32) + (p1 >> 32) + (q >> 32), x.e + y.e + 64};
}

DiyFp diy_normalize(DiyFp x) {
  while ((x.f >> 63) == 0) {
    x.f <<= 1;
    x.e--;
  }
  return x;
}

// 10^k as a normalized DiyFp, significand rounded to nearest: exact big-integer arithmetic
DiyFp cached_power(int k) {
  std::vector<uint32_t> ten(1, 1u);  // little-endian base-2^32
  auto mul10 = [](std::vector<uint32_t>& a) {
    uint64_t carry = 0;
    for (uint32_t& w : a) {
      const uint64_t t = (uint64_t)w * 10u + carry;
      w = (uint32_t)t;
      carry = t >> 32;
    }
    if (carry) a.push_back((uint32_t)carry);
  };
  for (int i = 0; i < (k < 0 ? -k : k); ++i) mul10(ten);
  auto bitlen = [](const std::vector<uint32_t>& a) {
    for (int i = (int)a.size() - 1; i >= 0; --i)
      if (a[i]) return i * 32 + 64 - __builtin_clzll((uint64_t)a[i]);
    return 0;
  };
  auto bit = [](const std::vector<uint32_t>& a, int i) -> uint32_t {
    return (i >= 0 && (size_t)(i >> 5) < a.size()) ? (a[i >> 5] >> (i & 31)) & 1u : 0u;
  };
  if (k >= 0) {  // top 64 bits of 10^k, rounded on the next bit
    const int L = bitlen(ten);
    uint64_t f = 0;
    for (int i = 0; i < 64; ++i) f = (f << 1) | bit(ten, L - 1 - i);
    int e = L - 64;
    if (bit(ten, L - 65)) {
      if (++f == 0) {
        f = uint64_t{1} << 63;
        e++;
      }
    }
    return DiyFp{f, e};
  }
  // 2^s / 10^-k with s such that the quotient has 65 bits (64 + a rounding bit), restoring division
  const int s = bitlen(ten) + 64;
  std::vector<uint32_t> r;
  auto cmp_ge = [](const std::vector<uint32_t>& a, const std::vector<uint32_t>& b) {
    const size_t n = std::max(a.size(), b.size());
    for (size_t i = n; i-- > 0;) {
      const uint32_t x = i < a.size() ? a[i] : 0u, y = i < b.size() ? b[i] : 0u;
      if (x != y) return x > y;
    }
    return true;
  };
  auto sub_in = [](std::vector<uint32_t>& a, const std::vector<uint32_t>& b) {
    int64_t borrow = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      int64_t t = (int64_t)a[i] - (i < b.size() ? (int64_t)b[i] : 0) - borrow;
      borrow = t < 0;
      a[i] = (uint32_t)(t + (borrow << 32));
    }
  };
  auto shl1_add = [](std::vector<uint32_t>& a, uint32_t b) {
    uint32_t carry = b;
    for (uint32_t& w : a) {
      const uint32_t nc = w >> 31;
      w = (w << 1) | carry;
      carry = nc;
    }
    if (carry) a.push_back(carry);
  };
  unsigned __int128 q = 0;
  for (int i = s; i >= 0; --i) {
    shl1_add(r, i == s ? 1u : 0u);
    q <<= 1;
    if (cmp_ge(r, ten)) {
      sub_in(r, ten);
      q |= 1;
    }
  }
  // 2^(L-1) <= 10^-k < 2^L with s = L + 64, so q = floor(2^s / 10^-k) has exactly 65 bits: keep the
  // top 64 and round on the last (the remainder is never 0, so there are no ties)
  uint64_t f = (uint64_t)(q >> 1);
  int e = -s + 1;
  if (q & 1) {
    if (++f == 0) {
      f = uint64_t{1} << 63;
      e++;
    }
  }
  return DiyFp{f, e};
}

DiyFp cached_power_for(int e, int& k_out) {
  static DiyFp table[79];
  static bool init = false;
  if (!init) {
    for (int i = 0; i < 79; ++i) table[i] = cached_power(-300 + 8 * i);
    init = true;
  }
  const int f = -60 - e - 1;
  const int k = (f * 78913) / (1 << 18) + (f > 0 ? 1 : 0);
  const int index = (300 + k + 7) / 8;
  k_out = -300 + 8 * index;
  return table[index];
}

int largest_pow10(uint32_t n, uint32_t& pow10) {
  const uint32_t p[10] = {1u, 10u, 100u, 1000u, 10000u, 100000u, 1000000u, 10000000u, 100000000u, 1000000000u};
  for (int d = 9; d >= 0; --d)
    if (n >= p[d]) {
      pow10 = p[d];
      return d + 1;
    }
  pow10 = 1;
  return 1;
}

void grisu2_round(char* buf, int len, uint64_t dist, uint64_t delta, uint64_t rest, uint64_t ten_k) {
  while (rest < dist && delta - rest >= ten_k && (rest + ten_k < dist || dist - rest > rest + ten_k - dist)) {
    buf[len - 1]--;
    rest += ten_k;
  }
}

void grisu2_digits(char* buf, int& len, int& dexp, DiyFp M_minus, DiyFp w, DiyFp M_plus) {
  uint64_t delta = diy_sub(M_plus, M_minus).f, dist = diy_sub(M_plus, w).f;
  const DiyFp one{uint64_t{1} << -M_plus.e, M_plus.e};
  uint32_t p1 = (uint32_t)(M_plus.f >> -one.e);
  uint64_t p2 = M_plus.f & (one.f - 1);
  uint32_t pow10;
  int n = largest_pow10(p1, pow10);
  while (n > 0) {
    const uint32_t d = p1 / pow10, r = p1 % pow10;
    buf[len++] = (char)('0' + d);
    p1 = r;
    n--;
    const uint64_t rest = ((uint64_t)p1 << -one.e) + p2;
    if (rest <= delta) {
      dexp += n;
      grisu2_round(buf, len, dist, delta, rest, (uint64_t)pow10 << -one.e);
      return;
    }
    pow10 /= 10;
  }
  int m = 0;
  for (;;) {
    p2 *= 10;
    const uint64_t d = p2 >> -one.e, r = p2 & (one.f - 1);
    buf[len++] = (char)('0' + d);
    p2 = r;
    m++;
    delta *= 10;
    dist *= 10;
    if (p2 <= delta) break;
  }
  dexp -= m;
  grisu2_round(buf, len, dist, delta, p2, one.f);
}

std::string json_number(double v) {
  if (v == 0.0) return std::signbit(v) ? "-0.0" : "0.0";
  std::string out = v < 0 ? "-" : "";
  v = std::fabs(v);
  uint64_t bits;
  std::memcpy(&bits, &v, 8);
  const uint64_t F = bits & ((uint64_t{1} << 52) - 1);
  const int E = (int)(bits >> 52);
  const DiyFp vv = E == 0 ? DiyFp{F, 1 - 1075} : DiyFp{F + (uint64_t{1} << 52), E - 1075};
  const bool lower_closer = F == 0 && E > 1;
  const DiyFp m_plus{2 * vv.f + 1, vv.e - 1};
  const DiyFp m_minus = lower_closer ? DiyFp{4 * vv.f - 1, vv.e - 2} : DiyFp{2 * vv.f - 1, vv.e - 1};
  const DiyFp w_plus = diy_normalize(m_plus);
  const DiyFp w_minus{m_minus.f << (m_minus.e - w_plus.e), w_plus.e};
  const DiyFp w = diy_normalize(vv);
  int k;
  const DiyFp c = cached_power_for(w_plus.e, k);
  const DiyFp W = diy_mul(w, c), Wm = diy_mul(w_minus, c), Wp = diy_mul(w_plus, c);
  char buf[32];
  int len = 0, dexp = -k;
  grisu2_digits(buf, len, dexp, DiyFp{Wm.f + 1, Wm.e}, W, DiyFp{Wp.f - 1, Wp.e});
  const std::string digits(buf, buf + len);
  const int n = len + dexp;  // position of the decimal point
  if (len <= n && n <= 15) return out + digits + std::string(n - len, '0') + ".0";
  if (0 < n && n <= 15) return out + digits.substr(0, n) + "." + digits.substr(n);
  if (-4 < n && n <= 0) return out + "0." + std::string(-n, '0') + digits;
  std::string m = digits.substr(0, 1);
  if (len > 1) m += "." + digits.substr(1);
  const int ex = n - 1;
  char eb[16];
  std::snprintf(eb, sizeof(eb), "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
  return out + m + eb;
}

}  // namespace

// also used by ptgs_capture_dataset (capture.cpp)
bool ptgs_mkdirs(const std::string& path) {
  std::string cur;
  for (size_t i = 0; i <= path.size(); ++i) {
    if (i == path.size() || path[i] == '/') {
      if (!cur.empty() && mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
    if (i < path.size()) cur += path[i];
  }
  return true;
}


extern "C" {

int ptgs_mat4_inverse_glm(const float in[16], float out[16]) {
  if (!in || !out) return PTGS_EINVAL;
  float m[4][4];  // m[col][row]
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) m[c][r] = in[c * 4 + r];
  const float c00 = m[2][2] * m[3][3] - m[3][2] * m[2][3], c02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
  const float c03 = m[1][2] * m[2][3] - m[2][2] * m[1][3], c04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
  const float c06 = m[1][1] * m[3][3] - m[3][1] * m[1][3], c07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
  const float c08 = m[2][1] * m[3][2] - m[3][1] * m[2][2], c10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
  const float c11 = m[1][1] * m[2][2] - m[2][1] * m[1][2], c12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
  const float c14 = m[1][0] * m[3][3] - m[3][0] * m[1][3], c15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
  const float c16 = m[2][0] * m[3][2] - m[3][0] * m[2][2], c18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
  const float c19 = m[1][0] * m[2][2] - m[2][0] * m[1][2], c20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
  const float c22 = m[1][0] * m[3][1] - m[3][0] * m[1][1], c23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
  const float f0[4] = {c00, c00, c02, c03}, f1[4] = {c04, c04, c06, c07}, f2[4] = {c08, c08, c10, c11};
  const float f3[4] = {c12, c12, c14, c15}, f4[4] = {c16, c16, c18, c19}, f5[4] = {c20, c20, c22, c23};
  const float v0[4] = {m[1][0], m[0][0], m[0][0], m[0][0]}, v1[4] = {m[1][1], m[0][1], m[0][1], m[0][1]};
  const float v2[4] = {m[1][2], m[0][2], m[0][2], m[0][2]}, v3[4] = {m[1][3], m[0][3], m[0][3], m[0][3]};
  const float sa[4] = {1.0f, -1.0f, 1.0f, -1.0f}, sb[4] = {-1.0f, 1.0f, -1.0f, 1.0f};
  float inv[4][4];
  for (int k = 0; k < 4; ++k) {
    inv[0][k] = ((v1[k] * f0[k] - v2[k] * f1[k]) + v3[k] * f2[k]) * sa[k];
    inv[1][k] = ((v0[k] * f0[k] - v2[k] * f3[k]) + v3[k] * f4[k]) * sb[k];
    inv[2][k] = ((v0[k] * f1[k] - v1[k] * f3[k]) + v3[k] * f5[k]) * sa[k];
    inv[3][k] = ((v0[k] * f2[k] - v1[k] * f4[k]) + v2[k] * f5[k]) * sb[k];
  }
  const float d0 = m[0][0] * inv[0][0], d1 = m[0][1] * inv[1][0], d2 = m[0][2] * inv[2][0], d3 = m[0][3] * inv[3][0];
  const float det = (d0 + d1) + (d2 + d3);
  if (det == 0.0f) return PTGS_EINVAL;
  const float ood = 1.0f / det;
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) out[c * 4 + r] = inv[c][r] * ood;
  return PTGS_OK;
}

int ptgs_capture_poses(uint32_t n, uint32_t seed, float min_beta, float max_beta, float* alpha_beta) {
  if (!alpha_beta && n) return PTGS_EINVAL;
  std::mt19937 gen(seed);
  std::uniform_real_distribution<> alpha_dist(0.0f, 360.0f);
  std::uniform_real_distribution<> beta_dist(min_beta, max_beta);
  for (uint32_t i = 0; i < n; ++i) {
    const float alpha = (float)alpha_dist(gen);  // the reference draws alpha then beta
    const float beta = (float)beta_dist(gen);
    alpha_beta[2 * i] = alpha;
    alpha_beta[2 * i + 1] = beta;
  }
  return PTGS_OK;
}

int ptgs_write_transforms_json(const char* path, float fov_y_deg, float aspect, uint32_t n,
                               const char* const* file_paths, const float* transforms) {
  if (!path || (n && (!file_paths || !transforms))) return PTGS_EINVAL;
  const float fov_y = fov_y_deg * 0.01745329251994329576923690768489f;  // glm::radians
  const float fov_x = 2.0f * std::atan(std::tan(fov_y / 2.0f) * aspect);
  std::string s = "{\n    \"camera_angle_x\": " + json_number((double)fov_x) + ",\n    \"frames\": [";
  for (uint32_t i = 0; i < n; ++i) {
    s += i ? ",\n        {\n" : "\n        {\n";
    s += "            \"file_path\": \"" + std::string(file_paths[i]) + "\",\n";
    s += "            \"transform_matrix\": [\n";
    const float* m = transforms + 16 * (size_t)i;
    for (int r = 0; r < 4; ++r) {
      s += "                [\n";
      for (int c = 0; c < 4; ++c)
        s += "                    " + json_number((double)m[c * 4 + r]) + (c < 3 ? ",\n" : "\n");
      s += r < 3 ? "                ],\n" : "                ]\n";
    }
    s += "            ]\n        }";
  }
  s += n ? "\n    ]\n}" : "]\n}";
  FILE* f = std::fopen(path, "wb");
  if (!f) return PTGS_EIO;
  const bool ok = std::fwrite(s.data(), 1, s.size(), f) == s.size();
  return (std::fclose(f) == 0 && ok) ? PTGS_OK : PTGS_EIO;
}

int ptgs_write_ply(const char* path, const ptgs_hitdata* hits, uint32_t n, uint32_t* num_written) {
  if (!path || (n && !hits)) return PTGS_EINVAL;
  uint32_t valid = 0;
  for (uint32_t i = 0; i < n; ++i) valid += hits[i].flag > 0.0f;
  FILE* f = std::fopen(path, "wb");
  if (!f) return PTGS_EIO;
  std::fprintf(f,
               "ply\nformat ascii 1.0\nelement vertex %u\nproperty float x\nproperty float y\nproperty float z\n"
               "property float nx\nproperty float ny\nproperty float nz\nproperty uchar red\nproperty uchar green\n"
               "property uchar blue\nend_header\n",
               valid);
  for (uint32_t i = 0; i < n; ++i) {
    const ptgs_hitdata& p = hits[i];
    if (!(p.flag > 0.0f)) continue;
    // std::ostream defaults: 6 significant digits (%g); colours int(c * 255) truncated
    std::fprintf(f, "%g %g %g %g %g %g %d %d %d\n", p.pos[0], p.pos[1], p.pos[2], p.normal[0], p.normal[1],
                 p.normal[2], (int)(p.color[0] * 255.0f), (int)(p.color[1] * 255.0f), (int)(p.color[2] * 255.0f));
  }
  if (num_written) *num_written = valid;
  return std::fclose(f) == 0 ? PTGS_OK : PTGS_EIO;
}

int ptgs_write_jpeg(const char* path, const uint8_t* pixels, uint32_t width, uint32_t height, uint32_t comp,
                    int quality) {
  if (!path || !pixels) return PTGS_EINVAL;
  std::vector<uint8_t> bytes;
  if (!ptgs::encode_jpeg(pixels, width, height, comp, quality, bytes)) return PTGS_EINVAL;
  FILE* f = std::fopen(path, "wb");
  if (!f) return PTGS_EIO;
  const bool ok = std::fwrite(bytes.data(), 1, bytes.size(), f) == bytes.size();
  return (std::fclose(f) == 0 && ok) ? PTGS_OK : PTGS_EIO;
}

}  // extern "C"
