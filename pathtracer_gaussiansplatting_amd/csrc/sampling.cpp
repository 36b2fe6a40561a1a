// Torus RaySample generators: the CPU side of the reference's data-collection tracer
// (Vulkan_Engine/sampling.cpp:5-434, Sampling::updateSampling). The generated uv sequence feeds
// ptgs_trace_torus (rt_datacollect/raygen.rgen) in the Morton order the reference uploads.
//
// Bit-for-bit contract with the reference build (plain g++, libstdc++): std::mt19937 +
// std::uniform_real_distribution<float>, std::shuffle and std::sort are the library's own (this file
// is compiled by g++ against the same libstdc++), every float operation is evaluated in the
// reference's order (-ffp-contract=off), and glm::vec2(dis(gen), dis(gen)) draws v before u, the
// argument order g++ evaluates (sampling.cpp:175).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#include "ptgs/ptgs_host.h"

namespace {

struct UV {
  float u, v;
};

// Sampling::halton, sampling.cpp:5-16
float halton(int index, int base) {
  float f = 1.f;
  float r = 0.f;
  while (index > 0) {
    f = f / (float)base;
    r = r + f * (float)(index % base);
    index = index / base;
  }
  return r;
}

// expandBits / morton2D, sampling.cpp:335-354 (15 bits per axis, clamp to 32767)
uint32_t expand_bits(uint16_t v) {
  uint32_t x = v;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}

uint32_t morton2d(float u, float v) {
  const float x = std::clamp(u * 32768.0f, 0.0f, 32767.0f);
  const float y = std::clamp(v * 32768.0f, 0.0f, 32767.0f);
  return expand_bits((uint16_t)x) | (expand_bits((uint16_t)y) << 1);
}

// Sampling::sortSamples, sampling.cpp:356-361. The reference's comparator recomputes both codes per
// comparison; std::sort's moves depend only on the comparison outcomes, so sorting (code, uv) records
// by code yields the same permutation (ties included: std::sort is not stable, its tie order is what
// introsort leaves, reproduced here by running the same library algorithm on the same outcomes).
struct Keyed {
  uint32_t key;
  UV uv;
};

void sort_samples(std::vector<UV>& s) {
  std::vector<Keyed> k(s.size());
  for (size_t i = 0; i < s.size(); ++i) k[i] = {morton2d(s[i].u, s[i].v), s[i]};
  std::sort(k.begin(), k.end(), [](const Keyed& a, const Keyed& b) { return a.key < b.key; });
  for (size_t i = 0; i < s.size(); ++i) s[i] = k[i].uv;
}

// uniform grid of Uniform / Stratified (sampling.cpp:40-41, :187-188)
void grid_dims(int n, int& cols, int& rows) {
  cols = static_cast<int>(std::ceil(std::sqrt(n)));
  if (cols == 0) {  // n == 0: the reference computes 0.f / 0 here but never uses rows
    rows = 0;
    return;
  }
  rows = static_cast<int>(std::ceil(static_cast<float>(n) / cols));
}

void gen_halton(std::vector<UV>& s, int n) {  // sampling.cpp:18-32
  s.resize(n);
  for (int i = 0; i < n; i++) s[i] = {halton(i + 1, 2), halton(i + 1, 3)};
  sort_samples(s);
}

void gen_stratified(std::vector<UV>& s, int n, uint32_t seed) {  // sampling.cpp:34-61
  s.resize(n);
  int cols, rows;
  grid_dims(n, cols, rows);
  std::mt19937 gen(seed);
  std::uniform_real_distribution<float> dis(0.0f, 1.0f);
  for (int i = 0; i < n; i++) {
    const int y = i / cols, x = i % cols;
    const float u = (x + dis(gen)) / cols;
    const float v = (y + dis(gen)) / rows;
    s[i] = {u, v};
  }
  sort_samples(s);
}

void gen_random(std::vector<UV>& s, int n, uint32_t seed) {  // sampling.cpp:164-179
  s.resize(n);
  std::mt19937 gen(seed);
  std::uniform_real_distribution<float> dis(0.0f, 1.0f);
  for (int i = 0; i < n; i++) {
    const float v = dis(gen);  // glm::vec2(dis(gen), dis(gen)) under g++: right argument first
    const float u = dis(gen);
    s[i] = {u, v};
  }
  sort_samples(s);
}

void gen_uniform(std::vector<UV>& s, int n) {  // sampling.cpp:181-204
  s.resize(n);
  int cols, rows;
  grid_dims(n, cols, rows);
  for (int i = 0; i < n; i++) {
    const int y = i / cols, x = i % cols;
    s[i] = {(static_cast<float>(x) + 0.5f) / cols, (static_cast<float>(y) + 0.5f) / rows};
  }
  sort_samples(s);
}

void gen_lhs(std::vector<UV>& s, int n, uint32_t seed) {  // sampling.cpp:292-333
  s.resize(n);
  std::vector<int> ui(n), vi(n);
  std::iota(ui.begin(), ui.end(), 0);
  std::iota(vi.begin(), vi.end(), 0);
  std::mt19937 gen(seed);
  std::shuffle(ui.begin(), ui.end(), gen);
  std::shuffle(vi.begin(), vi.end(), gen);
  std::uniform_real_distribution<float> dis(0.0f, 1.0f);
  for (int i = 0; i < n; i++) {
    const float u = (ui[i] + dis(gen)) / static_cast<float>(n);
    const float v = (vi[i] + dis(gen)) / static_cast<float>(n);
    s[i] = {u, v};
  }
  sort_samples(s);
}

int grid_cell(float uv, int res) {  // std::clamp(static_cast<int>(uv * res), 0, res - 1)
  return std::clamp(static_cast<int>(uv * res), 0, res - 1);
}

// inverse-transform resampling over an importance grid (sampling.cpp:110-161 / :241-290)
void inverse_cdf_samples(std::vector<UV>& s, int n, const std::vector<float>& importance, float total_weight,
                         int res, uint32_t seed) {
  std::vector<float> cdf(importance.size());
  float current_sum = 0.0f;
  for (size_t i = 0; i < importance.size(); i++) {
    current_sum += importance[i];
    cdf[i] = current_sum;
  }
  for (size_t i = 0; i < cdf.size(); i++) cdf[i] /= total_weight;
  s.assign(n, UV{0.0f, 0.0f});
  std::mt19937 gen(seed);
  std::uniform_real_distribution<float> dis(0.0f, 1.0f);
  for (int i = 0; i < n; i++) {
    const float r = dis(gen);
    const int idx = static_cast<int>(std::lower_bound(cdf.begin(), cdf.end(), r) - cdf.begin());
    const int y = idx / res, x = idx % res;
    const float u = (x + dis(gen)) / static_cast<float>(res);
    const float v = (y + dis(gen)) / static_cast<float>(res);
    s[i] = {u, v};
  }
  sort_samples(s);
}

// Sampling::generateImportanceSamples, sampling.cpp:63-161 (colour-gradient importance)
void gen_importance_color(std::vector<UV>& s, int n, const std::vector<UV>& prev, const ptgs_hitdata* hits,
                          size_t n_hits, int res, uint32_t seed) {
  const size_t cells = (size_t)res * res;
  std::vector<float> col(3 * cells, 0.0f), cnt(cells, 0.0f);
  for (size_t i = 0; i < prev.size(); i++) {
    if (i >= n_hits) break;
    const int x = grid_cell(prev[i].u, res), y = grid_cell(prev[i].v, res);
    const size_t k = (size_t)y * res + x;
    for (int c = 0; c < 3; ++c) col[3 * k + c] += hits[i].color[c];
    cnt[k] += 1.0f;
  }
  for (size_t k = 0; k < cells; k++)
    if (cnt[k] > 0.0f)
      for (int c = 0; c < 3; ++c) col[3 * k + c] /= cnt[k];
  auto lum = [&](int x, int y) -> float {
    if (x < 0 || x >= res || y < 0 || y >= res) return 0.0f;
    const float* c = &col[3 * ((size_t)y * res + x)];
    return 0.2126f * c[0] + 0.7152f * c[1] + 0.0722f * c[2];
  };
  std::vector<float> imp(cells, 0.0f);
  float total = 0.0f;
  for (int y = 0; y < res; y++)
    for (int x = 0; x < res; x++) {
      const float dx = lum(x + 1, y) - lum(x - 1, y);
      const float dy = lum(x, y + 1) - lum(x, y - 1);
      const float w = std::sqrt(dx * dx + dy * dy) + 0.05f;
      imp[(size_t)y * res + x] = w;
      total += w;
    }
  inverse_cdf_samples(s, n, imp, total, res, seed);
}

// Sampling::generateHitBasedImportanceSamples, sampling.cpp:207-290 (hit-ratio importance)
void gen_importance_hits(std::vector<UV>& s, int n, const std::vector<UV>& prev, const ptgs_hitdata* hits,
                         size_t n_hits, int res, uint32_t seed) {
  const size_t cells = (size_t)res * res;
  std::vector<float> hit(cells, 0.0f), cnt(cells, 0.0f);
  for (size_t i = 0; i < prev.size(); i++) {
    if (i >= n_hits) break;
    const int x = grid_cell(prev[i].u, res), y = grid_cell(prev[i].v, res);
    const size_t k = (size_t)y * res + x;
    hit[k] += (hits[i].flag > 0.0f) ? 1.0f : 0.0f;
    cnt[k] += 1.0f;
  }
  std::vector<float> imp(cells, 0.0f);
  float total = 0.0f;
  for (size_t k = 0; k < cells; k++) {
    const float ratio = cnt[k] > 0.0f ? hit[k] / cnt[k] : 0.0f;
    const float w = ratio + 0.01f;
    imp[k] = w;
    total += w;
  }
  inverse_cdf_samples(s, n, imp, total, res, seed);
}

}  // namespace

extern "C" {

uint32_t ptgs_morton2d(float u, float v) { return morton2d(u, v); }

int ptgs_sort_samples(ptgs_ray_sample* samples, uint32_t n) {
  if (n && !samples) return PTGS_EINVAL;
  std::vector<UV> s(n);
  std::memcpy(s.data(), samples, sizeof(UV) * n);
  sort_samples(s);
  std::memcpy(samples, s.data(), sizeof(UV) * n);
  return PTGS_OK;
}

int ptgs_generate_samples(int method, uint32_t n, const ptgs_ray_sample* prev_samples, uint32_t n_prev,
                          const ptgs_hitdata* prev_hits, uint32_t n_prev_hits, uint32_t seed, int grid_resolution,
                          ptgs_ray_sample* out) {
  if (n > 0x7FFFFFFFu || (n && !out)) return PTGS_EINVAL;
  if (method < PTGS_SAMPLING_RANDOM || method > PTGS_SAMPLING_IMP_HIT) return PTGS_EINVAL;
  if (grid_resolution == 0) grid_resolution = 256;  // sampling.h:17, :29 default
  const bool importance = method == PTGS_SAMPLING_IMP_COL || method == PTGS_SAMPLING_IMP_HIT;
  if (importance && n_prev > 0) {
    if (!prev_samples || (n_prev_hits && !prev_hits) || grid_resolution < 1 || grid_resolution > 8192)
      return PTGS_EINVAL;
  }
  try {
    std::vector<UV> s;
    const int N = (int)n;
    switch (method) {
      case PTGS_SAMPLING_HALTON: gen_halton(s, N); break;
      case PTGS_SAMPLING_LHS: gen_lhs(s, N, seed); break;
      case PTGS_SAMPLING_STRATIFIED: gen_stratified(s, N, seed); break;
      case PTGS_SAMPLING_RANDOM: gen_random(s, N, seed); break;
      case PTGS_SAMPLING_UNIFORM: gen_uniform(s, N); break;
      default:
        if (n_prev == 0) {  // sampling.cpp:389-392: no previous samples -> Halton fallback
          gen_halton(s, N);
        } else {
          // the previous samples are read in full before the output is written (out may alias them)
          std::vector<UV> prev(n_prev);
          std::memcpy(prev.data(), prev_samples, sizeof(UV) * n_prev);
          if (method == PTGS_SAMPLING_IMP_COL)
            gen_importance_color(s, N, prev, prev_hits, n_prev_hits, grid_resolution, seed);
          else
            gen_importance_hits(s, N, prev, prev_hits, n_prev_hits, grid_resolution, seed);
        }
    }
    if (n) std::memcpy(out, s.data(), sizeof(UV) * n);
  } catch (...) {
    return PTGS_ERANGE;  // allocation failure
  }
  return PTGS_OK;
}

}  // extern "C"
