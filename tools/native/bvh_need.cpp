// bvh_need: the host SAH build + 4-wide collapse of a triangle soup (raw float32 x 9 per triangle),
// printing, per leaf size, the collapsed tree's worst-case traversal stack need and depth (the
// quantities api.cpp's kBvhTries compares with the stack capacity). Host code only (bvh.cpp).
//   g++ -O2 -std=c++17 -I pathtracer_gaussiansplatting_amd/csrc tools/native/bvh_need.cpp \
//       pathtracer_gaussiansplatting_amd/csrc/bvh.cpp -o /tmp/bvh_need && /tmp/bvh_need tris.f32 [max_depth]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "bvh.h"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 1;
  std::vector<float> v;
  float buf[9];
  while (std::fread(buf, sizeof(float), 9, f) == 9) v.insert(v.end(), buf, buf + 9);
  std::fclose(f);
  const uint32_t max_depth = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 38u;
  std::vector<ptgs::BuildTri> tris(v.size() / 9);
  for (size_t i = 0; i < tris.size(); ++i) {
    for (int k = 0; k < 3; ++k) {
      tris[i].v0[k] = v[9 * i + k];
      tris[i].v1[k] = v[9 * i + 3 + k];
      tris[i].v2[k] = v[9 * i + 6 + k];
    }
    tris[i].mesh = 0;
    tris[i].prim = (uint32_t)i;
    tris[i].gid = (uint32_t)i;
    tris[i].flags = 0;
  }
  for (int leaf : {2, 3, 4}) {
    ptgs::BvhOut out;
    ptgs::build_bvh(tris, leaf, max_depth, out);
    for (int fan : {4}) {
      std::vector<float> n4;
      uint32_t num4 = 0, need = 0, dep4 = 0;
      ptgs::collapse_bvh4(out.nodes, n4, num4, need, dep4, fan);
      std::printf("%zu tris leaf %d: bvh2 nodes %u depth %u | %d-wide nodes %u depth %u worst-case stack %u\n",
                  tris.size(), leaf, out.num_nodes, out.depth, fan, num4, dep4, need);
    }
  }
  return 0;
}
