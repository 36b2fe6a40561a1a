// bvh.cpp — binned-SAH BVH2 builder (host, C++). See bvh.h for the device layout.
#include "bvh.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

#ifndef PTGS_BVH_CT
#define PTGS_BVH_CT 0.125f
#endif
#ifndef PTGS_BVH_BINS
#define PTGS_BVH_BINS 32  // (bvh_sah_gpu.hip reproduces this builder with 32 bins)
#endif

namespace ptgs {

namespace {

struct Box {
  float lo[3], hi[3];
  void reset() {
    for (int a = 0; a < 3; ++a) { lo[a] = std::numeric_limits<float>::infinity(); hi[a] = -lo[a]; }
  }
  void grow(const float* p) {
    for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], p[a]); hi[a] = std::max(hi[a], p[a]); }
  }
  void grow(const Box& b) {
    for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], b.lo[a]); hi[a] = std::max(hi[a], b.hi[a]); }
  }
  float area() const {
    float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (dx < 0 || dy < 0 || dz < 0) return 0.0f;
    return 2.0f * (dx * dy + dy * dz + dz * dx);
  }
};

struct Ref {
  Box box;
  float c[3];
  uint32_t tri;
};

struct Builder {
  const std::vector<BuildTri>& tris;
  std::vector<Ref> refs;
  std::vector<float>& nodes;
  int max_leaf;
  uint32_t max_depth = 31;
  uint32_t depth = 0, max_leaf_seen = 0;
  float pad_abs;

  Builder(const std::vector<BuildTri>& t, std::vector<float>& n, int ml) : tris(t), nodes(n), max_leaf(ml) {}

  // Padding keeps the device slab test conservative w.r.t. the Moller-Trumbore rounding:
  // relative 1e-5 of the box extent plus an absolute term from the scene's coordinate scale.
  void padded(const Box& b, float* lo, float* hi) const {
    float ext = std::max(b.hi[0] - b.lo[0], std::max(b.hi[1] - b.lo[1], b.hi[2] - b.lo[2]));
    float p = ext * 1e-5f + pad_abs;
    for (int a = 0; a < 3; ++a) { lo[a] = b.lo[a] - p; hi[a] = b.hi[a] + p; }
  }

  int32_t make_leaf(uint32_t begin, uint32_t count) {
    max_leaf_seen = std::max(max_leaf_seen, count);
    uint32_t L = ((count - 1u) << 27) | begin;
    return ~(int32_t)L;
  }

  Box range_box(uint32_t b, uint32_t e) const {
    Box bb; bb.reset();
    for (uint32_t i = b; i < e; ++i) bb.grow(refs[i].box);
    return bb;
  }

  // returns child encoding; writes its bounds to out_box
  int32_t build(uint32_t begin, uint32_t end, uint32_t d, Box& out_box) {
    depth = std::max(depth, d);
    uint32_t n = end - begin;
    out_box = range_box(begin, end);
    if (n <= (uint32_t)max_leaf && !(d == 0 && n > 1)) return make_leaf(begin, n);

    Box cb; cb.reset();
    for (uint32_t i = begin; i < end; ++i) cb.grow(refs[i].c);
    int axis = 0;
    float ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = cb.hi[a] - cb.lo[a];
    if (ext[1] > ext[axis]) axis = 1;
    if (ext[2] > ext[axis]) axis = 2;

    uint32_t mid = begin + n / 2;
    bool split_found = false;
    // Depth budget: SAH splits only while d + ceil(log2(n / leaf)) stays below max_depth; past that,
    // balanced splits halve n per level, so the tree depth never exceeds max_depth (the kernels'
    // LDS traversal stack, PTGS_STACK - 1).
    uint32_t need = 0;
    while (((uint64_t)max_leaf << need) < n) need++;
    if (ext[axis] > 0.0f && d + need + 1 < max_depth) {
      const int NB = PTGS_BVH_BINS;
      float best_cost = std::numeric_limits<float>::infinity();
      int best_axis = -1, best_bin = -1;
      for (int a = 0; a < 3; ++a) {
        if (!(ext[a] > 0.0f)) continue;
        Box bins[NB]; uint32_t cnt[NB];
        for (int k = 0; k < NB; ++k) { bins[k].reset(); cnt[k] = 0; }
        float scale = NB / ext[a];
        for (uint32_t i = begin; i < end; ++i) {
          int k = (int)((refs[i].c[a] - cb.lo[a]) * scale);
          k = std::min(NB - 1, std::max(0, k));
          bins[k].grow(refs[i].box); cnt[k]++;
        }
        float rarea[NB]; uint32_t rcnt[NB];
        Box acc; acc.reset(); uint32_t c = 0;
        for (int k = NB - 1; k > 0; --k) { acc.grow(bins[k]); c += cnt[k]; rarea[k] = acc.area(); rcnt[k] = c; }
        acc.reset(); c = 0;
        for (int k = 0; k < NB - 1; ++k) {
          acc.grow(bins[k]); c += cnt[k];
          if (c == 0 || rcnt[k + 1] == 0) continue;
          float cost = acc.area() * c + rarea[k + 1] * rcnt[k + 1];
          if (cost < best_cost) { best_cost = cost; best_axis = a; best_bin = k; }
        }
      }
      if (best_axis >= 0) {
        float leaf_cost = out_box.area() * n;
        float split_cost = PTGS_BVH_CT * out_box.area() + best_cost;  // traversal step vs tri test
        if (n <= (uint32_t)max_leaf && leaf_cost <= split_cost && d > 0) return make_leaf(begin, n);
        float scale = NB / ext[best_axis];
        float lo = cb.lo[best_axis];
        auto it = std::partition(refs.begin() + begin, refs.begin() + end, [&](const Ref& r) {
          int k = (int)((r.c[best_axis] - lo) * scale);
          k = std::min(NB - 1, std::max(0, k));
          return k <= best_bin;
        });
        mid = (uint32_t)(it - refs.begin());
        split_found = (mid > begin && mid < end);
      }
    }
    if (!split_found) {
      // degenerate centroids: median split by index order along the widest axis
      mid = begin + n / 2;
      std::nth_element(refs.begin() + begin, refs.begin() + mid, refs.begin() + end,
                       [&](const Ref& x, const Ref& y) { return x.c[axis] < y.c[axis]; });
      if (n == 1) {
        // single triangle: both children are the same leaf (never an empty box)
        uint32_t idx = (uint32_t)(nodes.size() / 16);
        nodes.resize(nodes.size() + 16);
        int32_t leaf = make_leaf(begin, 1);
        write_node(idx, out_box, leaf, out_box, leaf);
        return (int32_t)idx;
      }
    }
    uint32_t idx = (uint32_t)(nodes.size() / 16);
    nodes.resize(nodes.size() + 16);
    Box b0, b1;
    int32_t c0 = build(begin, mid, d + 1, b0);
    int32_t c1 = build(mid, end, d + 1, b1);
    write_node(idx, b0, c0, b1, c1);
    return (int32_t)idx;
  }

  void write_node(uint32_t idx, const Box& b0, int32_t c0, const Box& b1, int32_t c1) {
    float lo0[3], hi0[3], lo1[3], hi1[3];
    padded(b0, lo0, hi0);
    padded(b1, lo1, hi1);
    float* f = nodes.data() + 16u * idx;
    f[0] = lo0[0]; f[1] = hi0[0]; f[2] = lo0[1]; f[3] = hi0[1];
    f[4] = lo1[0]; f[5] = hi1[0]; f[6] = lo1[1]; f[7] = hi1[1];
    f[8] = lo0[2]; f[9] = hi0[2]; f[10] = lo1[2]; f[11] = hi1[2];
    std::memcpy(&f[12], &c0, 4);
    std::memcpy(&f[13], &c1, 4);
    f[14] = 0.0f; f[15] = 0.0f;
  }
};

}  // namespace

void build_bvh(const std::vector<BuildTri>& tris, int max_leaf_size, uint32_t max_depth, BvhOut& out) {
  out.nodes.clear();
  out.tris.clear();
  out.tri_flags.clear();
  max_leaf_size = std::max(1, std::min(16, max_leaf_size));
  Builder b(tris, out.nodes, max_leaf_size);
  b.max_depth = max_depth;
  float maxabs = 0.0f;
  b.refs.resize(tris.size());
  for (size_t i = 0; i < tris.size(); ++i) {
    Ref& r = b.refs[i];
    r.box.reset();
    r.box.grow(tris[i].v0); r.box.grow(tris[i].v1); r.box.grow(tris[i].v2);
    for (int a = 0; a < 3; ++a) {
      r.c[a] = 0.5f * (r.box.lo[a] + r.box.hi[a]);
      maxabs = std::max(maxabs, std::max(std::fabs(r.box.lo[a]), std::fabs(r.box.hi[a])));
    }
    r.tri = (uint32_t)i;
  }
  b.pad_abs = maxabs * 4e-7f + 1e-30f;
  if (tris.empty()) {
    // a root whose two children are empty leaves far away: every ray misses
    out.nodes.assign(16, 0.0f);
    float* f = out.nodes.data();
    for (int k = 0; k < 12; ++k) f[k] = 1e30f;  // point boxes far beyond tmax = 1e4
    int32_t leaf = ~(int32_t)0;  // count 1 at triangle 0 — never reached (boxes are inverted)
    std::memcpy(&f[12], &leaf, 4);
    std::memcpy(&f[13], &leaf, 4);
    out.tris.assign(12, 0.0f);
    out.tri_flags.assign(1, 0u);
    out.num_nodes = 1;
    return;
  }
  Box root_box;
  b.build(0, (uint32_t)tris.size(), 0, root_box);
  out.num_nodes = (uint32_t)(out.nodes.size() / 16);
  out.depth = b.depth;
  out.max_leaf = b.max_leaf_seen;
  out.tris.resize(tris.size() * 12);
  out.tri_flags.resize(tris.size());
  for (size_t k = 0; k < b.refs.size(); ++k) {
    const BuildTri& t = tris[b.refs[k].tri];
    float* f = out.tris.data() + 12 * k;
    f[0] = t.v0[0]; f[1] = t.v0[1]; f[2] = t.v0[2];
    std::memcpy(&f[3], &t.mesh, 4);
    f[4] = t.v1[0] - t.v0[0]; f[5] = t.v1[1] - t.v0[1]; f[6] = t.v1[2] - t.v0[2];
    std::memcpy(&f[7], &t.prim, 4);
    f[8] = t.v2[0] - t.v0[0]; f[9] = t.v2[1] - t.v0[1]; f[10] = t.v2[2] - t.v0[2];
    std::memcpy(&f[11], &t.gid, 4);
    out.tri_flags[k] = t.flags;
  }
}

namespace {
struct Ent4 {
  float lo[3], hi[3];
  int32_t ref;
};
void bvh2_children(const float* n, Ent4 e[2]) {
  int32_t c0, c1;
  std::memcpy(&c0, &n[12], 4);
  std::memcpy(&c1, &n[13], 4);
  e[0] = Ent4{{n[0], n[2], n[8]}, {n[1], n[3], n[9]}, c0};
  e[1] = Ent4{{n[4], n[6], n[10]}, {n[5], n[7], n[11]}, c1};
}
float ent_area(const Ent4& e) {
  float d[3];
  for (int a = 0; a < 3; ++a) d[a] = std::max(0.0f, e.hi[a] - e.lo[a]);
  return d[0] * d[1] + d[1] * d[2] + d[2] * d[0];
}
}  // namespace

void collapse_bvh4(const std::vector<float>& n2, std::vector<float>& n4, uint32_t& num4, uint32_t& max_stack,
                   uint32_t& depth4, int max_children) {
  n4.clear();
  std::vector<std::pair<int32_t, uint32_t>> queue;  // (BVH2 node, BVH4 slot), breadth first
  std::vector<std::vector<uint32_t>> kids;          // interior BVH4 children per node
  std::vector<uint32_t> ncount;                     // non-empty children per node
  queue.push_back({0, 0u});
  n4.assign(32, 0.0f);
  kids.emplace_back();
  ncount.push_back(0);
  for (size_t q = 0; q < queue.size(); ++q) {
    const int32_t b2 = queue[q].first;
    const uint32_t slot = queue[q].second;
    Ent4 list[4];
    int cnt = 2;
    bvh2_children(&n2[16 * (size_t)b2], list);
    while (cnt < max_children) {
      int best = -1;
      float ba = -1.0f;
      for (int k = 0; k < cnt; ++k)
        if (list[k].ref >= 0 && ent_area(list[k]) > ba) { ba = ent_area(list[k]); best = k; }
      if (best < 0) break;
      Ent4 sub[2];
      bvh2_children(&n2[16 * (size_t)list[best].ref], sub);
      list[best] = sub[0];
      list[cnt++] = sub[1];
    }
    float* f = &n4[32 * (size_t)slot];
    for (int j = 0; j < 4; ++j) {
      int32_t child = 0;
      if (j < cnt) {
        for (int a = 0; a < 3; ++a) {
          f[(2 * a) * 4 + j] = list[j].lo[a];
          f[(2 * a + 1) * 4 + j] = list[j].hi[a];
        }
        if (list[j].ref >= 0) {
          const uint32_t ni = (uint32_t)(n4.size() / 32);
          n4.resize(n4.size() + 32, 0.0f);
          f = &n4[32 * (size_t)slot];  // (resize may move the storage)
          queue.push_back({list[j].ref, ni});
          kids.emplace_back();
          ncount.push_back(0);
          kids[slot].push_back(ni);
          child = (int32_t)ni;
        } else {
          child = list[j].ref;
        }
      } else {
        for (int a = 0; a < 6; ++a) f[a * 4 + j] = 1e30f;  // empty: a point box no ray reaches
      }
      std::memcpy(&f[24 + j], &child, 4);
    }
    ncount[slot] = (uint32_t)cnt;
  }
  num4 = (uint32_t)(n4.size() / 32);
  // stack need and depth, children after parents (breadth-first order): reverse pass
  std::vector<uint32_t> need(num4, 0), dep(num4, 1);
  for (size_t i = num4; i-- > 0;) {
    uint32_t m = 0, d = 0;
    for (uint32_t k : kids[i]) { m = std::max(m, need[k]); d = std::max(d, dep[k]); }
    need[i] = (ncount[i] - 1) + m;
    dep[i] = 1 + d;
  }
  max_stack = need[0];
  depth4 = dep[0];
}

}  // namespace ptgs
