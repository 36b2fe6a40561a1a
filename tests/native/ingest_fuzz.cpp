// ingest_fuzz.cpp — the hand-written parsers of untrusted input (PNG incl. Adam7 / 16-bit / tRNS,
// baseline + progressive JPEG, glTF / GLB, scene / rt-box JSON, ASCII + binary PLY) and the torus
// sample generators, built with AddressSanitizer + UndefinedBehaviorSanitizer
// (tests/native/Makefile, driven by tests/test_sanitize.py) and run over the committed fixtures plus
// deterministic mutations of them (byte flips, truncation, extreme integers, number substitution
// in the text formats). A parser may accept or reject a mutated file; any sanitizer report aborts
// the process (-fno-sanitize-recover=all), which fails the test.
//
// Usage: ingest_fuzz <fixture dir> <scratch dir> <mutations per file> [rng seed]
#include <dirent.h>
#include <stdint.h>
#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ptgs/ptgs.h"
#include "ptgs/ptgs_host.h"

namespace {

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint32_t rnd() {  // xorshift64*
  g_rng ^= g_rng >> 12;
  g_rng ^= g_rng << 25;
  g_rng ^= g_rng >> 27;
  return (uint32_t)((g_rng * 0x2545F4914F6CDD1Dull) >> 32);
}

std::vector<uint8_t> read_file(const std::string& p) {
  std::vector<uint8_t> v;
  FILE* f = fopen(p.c_str(), "rb");
  if (!f) return v;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  v.resize(n > 0 ? (size_t)n : 0);
  if (n > 0 && fread(v.data(), 1, v.size(), f) != v.size()) v.clear();
  fclose(f);
  return v;
}

void write_file(const std::string& p, const std::vector<uint8_t>& v) {
  FILE* f = fopen(p.c_str(), "wb");
  if (!f) {
    perror(p.c_str());
    exit(2);
  }
  if (!v.empty()) fwrite(v.data(), 1, v.size(), f);
  fclose(f);
}

bool is_text(const std::string& name) {
  for (const char* s : {".json", ".gltf", ".ply.txt"})
    if (name.size() >= strlen(s) && name.compare(name.size() - strlen(s), strlen(s), s) == 0) return true;
  return false;
}

// one mutation of `in`: kind chosen at random; text files also get number substitutions
std::vector<uint8_t> mutate(const std::vector<uint8_t>& in, bool text) {
  std::vector<uint8_t> v = in;
  if (v.empty()) return v;
  const uint32_t kind = rnd() % (text ? 6u : 4u);
  switch (kind) {
    case 0: {  // flip 1-8 random bytes
      const uint32_t k = 1 + rnd() % 8;
      for (uint32_t i = 0; i < k; ++i) v[rnd() % v.size()] ^= (uint8_t)(1u << (rnd() % 8));
      break;
    }
    case 1:  // truncate
      v.resize(rnd() % v.size());
      break;
    case 2: {  // an extreme 32-bit integer at a random offset (sizes, counts, offsets in headers)
      static const uint32_t ext[] = {0xFFFFFFFFu, 0x7FFFFFFFu, 0x80000000u, 0x00010000u, 0u, 0x40000000u};
      const uint32_t x = ext[rnd() % 6];
      const size_t at = rnd() % v.size();
      for (int b = 0; b < 4 && at + b < v.size(); ++b) v[at + b] = (uint8_t)(rnd() & 1 ? x >> (8 * b) : x >> (8 * (3 - b)));
      break;
    }
    case 3: {  // duplicate or delete a random span
      const size_t a = rnd() % v.size(), n = 1 + rnd() % 64;
      if (rnd() & 1) {
        v.insert(v.begin() + a, in.begin() + a, in.begin() + std::min(in.size(), a + n));
      } else {
        v.erase(v.begin() + a, v.begin() + std::min(v.size(), a + n));
      }
      break;
    }
    default: {  // text: replace the number that starts at / after a random offset
      static const char* nums[] = {"-1", "4294967296", "1e300", "-1e300", "18446744073709551615", "nan", "0",
                                   "2147483647", "1.5", "-0", "9999999999999", "1e-320", "\"x\"", "[]", "{}"};
      size_t a = rnd() % v.size();
      while (a < v.size() && !((v[a] >= '0' && v[a] <= '9') || v[a] == '-')) ++a;
      if (a >= v.size()) break;
      size_t b = a + 1;
      while (b < v.size() && ((v[b] >= '0' && v[b] <= '9') || v[b] == '.' || v[b] == 'e' || v[b] == '-' || v[b] == '+')) ++b;
      const char* s = nums[rnd() % (sizeof(nums) / sizeof(nums[0]))];
      v.erase(v.begin() + a, v.begin() + b);
      v.insert(v.begin() + a, s, s + strlen(s));
      break;
    }
  }
  return v;
}

std::vector<uint8_t> g_pixels(64u << 20);

int decode_image(const std::vector<uint8_t>& v) {
  uint32_t w = 0, h = 0, c = 0;
  return ptgs_image_decode_rgba8(v.data(), v.size(), g_pixels.data(), g_pixels.size(), &w, &h, &c);
}

int load_gltf(const std::string& path) {
  ptgs_scene_builder* b = nullptr;
  if (ptgs_builder_create(&b)) return -1;
  const float pos[3] = {0, 0, 0}, rot[3] = {0, 30, 0}, scl[3] = {1, 1, 1};
  int rc = ptgs_builder_add_gltf(b, path.c_str(), pos, rot, scl, PTGS_INGEST_MISSING_IMAGES_WHITE);
  if (rc == 0) {
    ptgs_scene_desc d;
    ptgs_ubo u;
    rc = ptgs_builder_finalize(b, &d, &u);
  }
  ptgs_builder_destroy(b);
  return rc;
}

int load_scene(const std::string& path, const std::string& root) {
  ptgs_scene_builder* b = nullptr;
  if (ptgs_builder_create(&b)) return -1;
  ptgs_scene_settings st;
  int rc = ptgs_builder_load_scene_json(b, path.c_str(), root.c_str(), PTGS_INGEST_MISSING_IMAGES_WHITE, &st);
  if (rc == 0) {
    ptgs_scene_desc d;
    ptgs_ubo u;
    rc = ptgs_builder_finalize(b, &d, &u);
  }
  if (rc && getenv("FUZZ_VERBOSE")) fprintf(stderr, "scene %s: %s\n", path.c_str(), ptgs_builder_last_error(b));
  ptgs_builder_destroy(b);
  return rc;
}

int load_rtbox(const std::string& path) {
  ptgs_scene_builder* b = nullptr;
  if (ptgs_builder_create(&b)) return -1;
  int rc = ptgs_builder_add_rtbox_json(b, path.c_str());
  ptgs_builder_destroy(b);
  return rc;
}

int read_ply(const std::string& path) {
  uint32_t n = 0;
  int rc = ptgs_read_ply(path.c_str(), nullptr, nullptr, nullptr, 0, &n);
  if (rc || n > (1u << 20)) return rc;
  std::vector<float> xyz(3 * (size_t)n + 3), nrm(3 * (size_t)n + 3);
  std::vector<uint8_t> rgb(3 * (size_t)n + 3);
  return ptgs_read_ply(path.c_str(), xyz.data(), nrm.data(), rgb.data(), n, &n);
}

// small PLY seeds: the ASCII layout Engine::savePly writes, and binary little / big endian
void make_ply_seeds(const std::string& dir, std::vector<std::string>& out) {
  std::string a = "ply\nformat ascii 1.0\nelement vertex 4\nproperty float x\nproperty float y\nproperty float z\n"
                  "property float nx\nproperty float ny\nproperty float nz\nproperty uchar red\nproperty uchar green\n"
                  "property uchar blue\nend_header\n";
  for (int i = 0; i < 4; ++i) a += std::to_string(i) + " 0.5 -1.25 0 1 0 " + std::to_string(10 * i) + " 20 30\n";
  write_file(dir + "/seed_ascii.ply.txt", std::vector<uint8_t>(a.begin(), a.end()));
  out.push_back(dir + "/seed_ascii.ply.txt");
  for (int be = 0; be < 2; ++be) {
    std::string h = std::string("ply\nformat ") + (be ? "binary_big_endian" : "binary_little_endian") +
                    " 1.0\nelement vertex 3\n"
                    "property float x\nproperty float y\nproperty float z\nproperty float f_dc_0\n"
                    "property float f_dc_1\nproperty float f_dc_2\nelement face 1\n"
                    "property list uchar int vertex_indices\nend_header\n";
    std::vector<uint8_t> v(h.begin(), h.end());
    for (int i = 0; i < 18; ++i) {
      float f = 0.25f * (float)i - 1.0f;
      uint8_t b[4];
      memcpy(b, &f, 4);
      if (be) std::swap(b[0], b[3]), std::swap(b[1], b[2]);
      v.insert(v.end(), b, b + 4);
    }
    const uint8_t face[13] = {3, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 2};
    v.insert(v.end(), face, face + 13);
    const std::string p = dir + (be ? "/seed_be.ply" : "/seed_le.ply");
    write_file(p, v);
    out.push_back(p);
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <fixture dir> <scratch dir> <mutations per file>\n", argv[0]);
    return 2;
  }
  const std::string fix = argv[1], tmp = argv[2];
  const int M = atoi(argv[3]);
  if (argc > 4) g_rng ^= strtoull(argv[4], nullptr, 10) * 0xD1B54A32D192ED03ull;
  mkdir(tmp.c_str(), 0755);
  long runs = 0, accepted = 0;

  // images (in memory)
  std::vector<std::string> images;
  if (DIR* d = opendir((fix + "/images").c_str())) {
    while (dirent* e = readdir(d))
      if (e->d_name[0] != '.') images.push_back(fix + "/images/" + e->d_name);
    closedir(d);
  }
  for (const std::string& p : images) {
    const std::vector<uint8_t> seed = read_file(p);
    if (decode_image(seed) != 0) {
      fprintf(stderr, "fixture %s does not decode\n", p.c_str());
      return 1;
    }
    for (int k = 0; k < M; ++k, ++runs) accepted += decode_image(mutate(seed, false)) == 0;
  }
  // glTF / GLB: mutate the model file; its buffers / images stay the fixtures' (same directory)
  for (const char* name : {"features.gltf", "features.glb", "lamp.gltf"}) {
    const std::vector<uint8_t> seed = read_file(fix + "/" + name);
    if (load_gltf(fix + "/" + name) != 0) {
      fprintf(stderr, "fixture %s does not load\n", name);
      return 1;
    }
    const std::string ext = strrchr(name, '.');
    const std::string mp = fix + "/_fuzz_model" + ext;  // beside the fixture: relative URIs resolve
    for (int k = 0; k < M; ++k, ++runs) {
      write_file(mp, mutate(seed, ext == ".gltf"));
      accepted += load_gltf(mp) == 0;
    }
    remove(mp.c_str());
  }
  // the .bin buffer of features.gltf (accessor bounds against a damaged buffer)
  {
    const std::vector<uint8_t> bin = read_file(fix + "/features.bin");
    std::vector<uint8_t> g = read_file(fix + "/features.gltf");
    std::string gs(g.begin(), g.end());
    const size_t at = gs.find("features.bin");
    if (at != std::string::npos) {
      gs.replace(at, 12, "_fuzz_buf.bin");
      write_file(fix + "/_fuzz_bufref.gltf", std::vector<uint8_t>(gs.begin(), gs.end()));
      for (int k = 0; k < M; ++k, ++runs) {
        write_file(fix + "/_fuzz_buf.bin", mutate(bin, false));
        accepted += load_gltf(fix + "/_fuzz_bufref.gltf") == 0;
      }
      remove((fix + "/_fuzz_buf.bin").c_str());
      remove((fix + "/_fuzz_bufref.gltf").c_str());
    }
  }
  // scene JSON (models resolve against the fixture root) and the rt-box JSON
  {
    const std::vector<uint8_t> seed = read_file(fix + "/scene.json");
    if (load_scene("scene.json", fix) != 0) {
      fprintf(stderr, "fixture scene.json does not load\n");
      return 1;
    }
    for (int k = 0; k < M; ++k, ++runs) {
      write_file(fix + "/_fuzz_scene.json", mutate(seed, true));
      accepted += load_scene("_fuzz_scene.json", fix) == 0;
    }
    remove((fix + "/_fuzz_scene.json").c_str());
    const std::vector<uint8_t> rb = read_file(fix + "/rtbox.json");
    for (int k = 0; k < M; ++k, ++runs) {
      write_file(tmp + "/rtbox.json", mutate(rb, true));
      accepted += load_rtbox(tmp + "/rtbox.json") == 0;
    }
  }
  // PLY
  {
    std::vector<std::string> seeds;
    make_ply_seeds(tmp, seeds);
    for (const std::string& p : seeds) {
      const std::vector<uint8_t> seed = read_file(p);
      if (read_ply(p) != 0) {
        fprintf(stderr, "seed %s does not read\n", p.c_str());
        return 1;
      }
      const bool text = p.find("ascii") != std::string::npos;
      for (int k = 0; k < M; ++k, ++runs) {
        write_file(tmp + "/m.ply", mutate(seed, text));
        accepted += read_ply(tmp + "/m.ply") == 0;
      }
    }
  }
  // torus sample generators and importance resamplers on damaged previous hits
  {
    std::vector<ptgs_ray_sample> s(4096), o(4096);
    std::vector<ptgs_hitdata> h(4096);
    for (int m = 0; m <= PTGS_SAMPLING_IMP_HIT; ++m) {
      for (uint32_t n : {0u, 1u, 7u, 1000u, 4096u}) {
        ++runs;
        accepted += ptgs_generate_samples(m, n, nullptr, 0, nullptr, 0, 13, 0, o.data()) == 0;
      }
    }
    for (int k = 0; k < M; ++k, ++runs) {
      uint8_t* raw = reinterpret_cast<uint8_t*>(h.data());
      for (size_t i = 0; i < h.size() * sizeof(ptgs_hitdata); ++i) raw[i] = (uint8_t)rnd();
      uint8_t* rs = reinterpret_cast<uint8_t*>(s.data());
      for (size_t i = 0; i < s.size() * sizeof(ptgs_ray_sample); ++i) rs[i] = (uint8_t)rnd();
      const uint32_t n = rnd() % 4097, np = rnd() % 4097;
      const int method = PTGS_SAMPLING_IMP_COL + (int)(rnd() & 1);
      accepted += ptgs_generate_samples(method, n, s.data(), np, h.data(), rnd() % 4097, 13, (int)(rnd() % 300) - 10,
                                        o.data()) == 0;
    }
  }
  // writers (capture_io.cpp): JPEG of odd sizes decoded back, PLY written and re-read, transforms JSON
  {
    for (int k = 0; k < 24; ++k, ++runs) {
      const uint32_t w = 1 + rnd() % 37, h = 1 + rnd() % 29, comp = (rnd() & 1) ? 3u : 4u;
      std::vector<uint8_t> px((size_t)w * h * comp);
      for (uint8_t& b : px) b = (uint8_t)rnd();
      if (ptgs_write_jpeg((tmp + "/w.jpg").c_str(), px.data(), w, h, comp, 50 + (int)(rnd() % 51)) != 0) return 1;
      accepted += decode_image(read_file(tmp + "/w.jpg")) == 0;
    }
    std::vector<ptgs_hitdata> h(257);
    uint8_t* raw = reinterpret_cast<uint8_t*>(h.data());
    for (size_t i = 0; i < h.size() * sizeof(ptgs_hitdata); ++i) raw[i] = (uint8_t)rnd();
    uint32_t nw = 0;
    if (ptgs_write_ply((tmp + "/w.ply").c_str(), h.data(), (uint32_t)h.size(), &nw) != 0) return 1;
    ++runs;
    accepted += read_ply(tmp + "/w.ply") == 0;
    std::vector<float> view(16 * 5);
    for (float& f : view) f = (float)(int32_t)rnd() * 1e-7f;
    const char* names[5] = {"a", "b", "c", "d", "e"};
    if (ptgs_write_transforms_json((tmp + "/t.json").c_str(), 45.0f, 1.5f, 5, names, view.data()) != 0) return 1;
    ++runs;
  }
  printf("ingest_fuzz: %ld runs, %ld accepted, no sanitizer report\n", runs, accepted);
  return 0;
}
