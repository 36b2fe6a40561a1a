// gltf.cpp — scene ingest: glTF 2.0 models and the reference's scene JSON into the scene builder.
//
//   ptgs_builder_add_gltf         Gameobject::loadModel (Vulkan_Engine/gameobject.cpp:198-273) + the
//                                 per-object bake of Engine::loadScene (engine.cpp:1265-1345)
//   ptgs_builder_load_scene_json  Engine::loadScene (engine.cpp:1172-1352)
//   ptgs_builder_add_punctual_light  the settings "sun" (engine.cpp:1225-1242)
//   ptgs_image_decode_rgba8       Image::createTextureImage's decode (image.cpp:12)
//
// Behaviour restated from the reference (each item cites the line it follows):
//   * node globals at animation 0 / frame 0 for lights and skin joints (gameobject.cpp:65-159);
//     mesh placement walks the hierarchy without animation (:519-560); skinned meshes use the
//     parent transform and are CPU-skinned with weight-normalised joint blends (:666-719)
//   * one default white texture per model, then model.images in order, sRGB unless only ever used
//     as a linear map (scanTextureFormats :275-342); texture ids are image index + 1 (:370-378)
//   * materials (:380-517): metal-rough or KHR_materials_pbrSpecularGlossiness (glossiness kept in
//     roughness_factor, specular colour reset to 1), emissive strength, KHR_materials_specular,
//     transmission (=> transparent), clearcoat, KHR_texture_transform on base colour / normal /
//     emissive, alpha MASK cutoff, BLEND => transparent
//   * vertices deduplicated on (pos, colour, uv0, tangent, normal) by float equality — uv1 is not
//     compared (GeneralHeaders.h:92-94) — and each primitive's index list appended twice, only the
//     first copy referenced (:750-766); emissive triangles with area > 1e-6 (:777-790)
//   * KHR_lights_punctual on nodes (:798-851)
//   * the scene-JSON transform T * R(euler degrees) * S baked into vertices, normals, tangents
//     (unconditionally) and lights (range * s, intensity * s^2), emissive areas recomputed
// All float math goes through glm_lite.h (GLM's operation order, no FMA contraction).
// Extensions beyond the reference (which would throw or read out of bounds): .glb containers,
// data: URIs and bufferView images, non-indexed primitives (sequential indices), bounds checks.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/ptgs/ptgs_host.h"
#include "glm_lite.h"
#include "image_decode.h"
#include "json.h"
#include "scene_builder.h"

using ptgs::JVal;
namespace G = ptgs::glm;

namespace {

// unaligned little-endian loads from accessor data
inline uint32_t ld_u16(const uint8_t* p) {
  uint16_t v;
  memcpy(&v, p, 2);
  return v;
}
inline uint32_t ld_u32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}


struct LoadError {
  std::string msg;
};
[[noreturn]] void fail(const std::string& m) { throw LoadError{m}; }

std::string dir_of(const std::string& path) {
  size_t k = path.find_last_of('/');
  return k == std::string::npos ? std::string() : path.substr(0, k + 1);
}

std::string join_path(const std::string& root, const std::string& rel) {
  if (root.empty() || (!rel.empty() && rel[0] == '/')) return rel;
  return root.back() == '/' ? root + rel : root + "/" + rel;
}

std::string percent_decode(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && isxdigit((unsigned char)s[i + 1]) && isxdigit((unsigned char)s[i + 2])) {
      o.push_back((char)strtol(s.substr(i + 1, 2).c_str(), nullptr, 16));
      i += 2;
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

bool base64_decode(const std::string& in, size_t start, std::vector<uint8_t>& out) {
  auto val = [](char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+' || c == '-') return 62;
    if (c == '/' || c == '_') return 63;
    return -1;
  };
  out.clear();
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = start; i < in.size(); ++i) {
    char c = in[i];
    if (c == '=') break;
    int v = val(c);
    if (v < 0) {
      if (c == '\n' || c == '\r' || c == ' ') continue;
      return false;
    }
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((uint8_t)(acc >> bits));
    }
  }
  return true;
}

// Resolve a glTF uri (file relative to the model, or data:) into bytes.
bool load_uri(const std::string& uri, const std::string& base, std::vector<uint8_t>& out) {
  if (uri.compare(0, 5, "data:") == 0) {
    size_t comma = uri.find(',');
    if (comma == std::string::npos || uri.find(";base64") == std::string::npos) return false;
    return base64_decode(uri, comma + 1, out);
  }
  if (ptgs::read_file(base + uri, out)) return true;
  std::string dec = percent_decode(uri);
  return dec != uri && ptgs::read_file(base + dec, out);
}

const JVal& req(const JVal& o, const char* key, const char* what) {
  const JVal* v = o.get(key);
  if (!v) fail(std::string(what) + " lacks \"" + key + "\"");
  return *v;
}

const JVal* arr_at(const JVal& root, const char* key, int i) {
  const JVal* a = root.get(key);
  return (a && i >= 0) ? a->at((size_t)i) : nullptr;
}

// -------------------------------------------------------------------------------------------------
struct Model {
  JVal doc;
  std::vector<std::vector<uint8_t>> buffers;
  std::string base;
  size_t n_nodes = 0, n_images = 0, n_textures = 0;

  const JVal* node(int i) const { return arr_at(doc, "nodes", i); }

  // Raw view of an accessor: pointer to element 0, element stride, element count
  struct View {
    const uint8_t* p = nullptr;
    size_t stride = 0, count = 0;
    int ctype = 0;
  };
  static int comp_size(int ct) {
    switch (ct) {
      case 5120: case 5121: return 1;
      case 5122: case 5123: return 2;
      case 5125: case 5126: return 4;
      default: return 0;
    }
  }
  static int type_count(const std::string& t) {
    if (t == "SCALAR") return 1;
    if (t == "VEC2") return 2;
    if (t == "VEC3") return 3;
    if (t == "VEC4") return 4;
    if (t == "MAT2") return 4;
    if (t == "MAT3") return 9;
    if (t == "MAT4") return 16;
    return 0;
  }
  // default_stride: 0 = tinygltf's Accessor::ByteStride (tight packing of the accessor's element),
  // otherwise the stride gameobject.cpp assumes when bufferView.byteStride is 0 (sizeof(glm::vecN)).
  // elem_bytes: bytes actually read per element (for the bounds check).
  View view(int acc_index, size_t default_stride, size_t elem_bytes, const char* what) const {
    const JVal* acc = arr_at(doc, "accessors", acc_index);
    if (!acc) fail(std::string(what) + ": accessor index out of range");
    // count / offsets / stride are untrusted JSON numbers: anything but an integer in [0, 2^32) is
    // rejected before the cast (a double -> size_t cast of a negative or huge value is UB)
    auto size_field = [&](const JVal* j) -> size_t {
      const double d = ptgs::jdouble(j, 0);
      if (!(d >= 0.0 && d < 4294967296.0) || d != (double)(uint64_t)d)
        fail(std::string(what) + ": accessor count/offset/stride is not an integer in [0, 2^32)");
      return (size_t)d;
    };
    View v;
    v.count = size_field(acc->get("count"));
    v.ctype = ptgs::jint(acc->get("componentType"), 0);
    int bvi = ptgs::jint(acc->get("bufferView"), -1);
    if (bvi < 0) fail(std::string(what) + ": accessor without bufferView (sparse-only accessors unsupported)");
    const JVal* bv = arr_at(doc, "bufferViews", bvi);
    if (!bv) fail(std::string(what) + ": bufferView index out of range");
    int bi = ptgs::jint(bv->get("buffer"), -1);
    if (bi < 0 || (size_t)bi >= buffers.size()) fail(std::string(what) + ": buffer index out of range");
    size_t off = size_field(bv->get("byteOffset")) + size_field(acc->get("byteOffset"));
    size_t bvstride = size_field(bv->get("byteStride"));
    size_t tight = (size_t)comp_size(v.ctype) * type_count(ptgs::jstr(acc->get("type"), ""));
    v.stride = bvstride ? bvstride : (default_stride ? default_stride : tight);
    const std::vector<uint8_t>& buf = buffers[bi];
    // overflow-free form of off + (count - 1) * stride + elem_bytes <= size
    if (v.count) {
      bool ok = off <= buf.size() && elem_bytes <= buf.size() - off;
      if (ok && v.count > 1 && v.stride) ok = (v.count - 1) <= (buf.size() - off - elem_bytes) / v.stride;
      if (!ok) fail(std::string(what) + ": accessor reads past the end of its buffer");
    }
    v.p = buf.data() + off;
    return v;
  }
};

void load_model_file(const std::string& path, Model& m) {
  std::vector<uint8_t> bytes;
  bool glb;
  std::string ext = path.substr(path.find_last_of('.') + 1);  // gameobject.cpp:205-213
  if (ext == "gltf") glb = false;
  else if (ext == "glb") glb = true;
  else fail("Failed to load glTF: Unknown file extension for " + path);
  if (!ptgs::read_file(path, bytes)) fail("cannot open " + path);
  m.base = dir_of(path);
  const char* json = (const char*)bytes.data();
  size_t json_len = bytes.size();
  std::vector<uint8_t> bin;
  bool have_bin = false;
  if (glb) {
    auto rd32 = [&](size_t o) {
      return (uint32_t)bytes[o] | (uint32_t)bytes[o + 1] << 8 | (uint32_t)bytes[o + 2] << 16 | (uint32_t)bytes[o + 3] << 24;
    };
    if (bytes.size() < 20 || memcmp(bytes.data(), "glTF", 4) || rd32(4) != 2) fail("not a glTF 2.0 binary: " + path);
    size_t total = std::min<size_t>(rd32(8), bytes.size());
    size_t o = 12;
    json = nullptr;
    while (o + 8 <= total) {
      uint32_t len = rd32(o), type = rd32(o + 4);
      if (o + 8 + (size_t)len > total) fail("truncated GLB chunk in " + path);
      if (type == 0x4E4F534Au && !json) { json = (const char*)bytes.data() + o + 8; json_len = len; }
      else if (type == 0x004E4942u && !have_bin) { bin.assign(bytes.begin() + o + 8, bytes.begin() + o + 8 + len); have_bin = true; }
      o += 8 + (size_t)((len + 3) & ~3u);
    }
    if (!json) fail("GLB without a JSON chunk: " + path);
  }
  if (!ptgs::parse_json(json, json_len, m.doc) || m.doc.kind != JVal::OBJ) fail("bad JSON in " + path);
  const JVal* bufs = m.doc.get("buffers");
  for (size_t i = 0; bufs && i < bufs->size(); ++i) {
    const JVal& b = bufs->arr[i];
    std::vector<uint8_t> data;
    std::string uri = ptgs::jstr(b.get("uri"), "");
    if (uri.empty()) {
      if (!(glb && i == 0 && have_bin)) fail("buffer " + std::to_string(i) + " has no uri");
      data = bin;
    } else if (!load_uri(uri, m.base, data)) {
      fail("cannot load buffer '" + uri + "' of " + path);
    }
    size_t need = (size_t)ptgs::jdouble(b.get("byteLength"), 0);
    if (data.size() < need) fail("buffer '" + uri + "' is shorter than its byteLength");
    m.buffers.push_back(std::move(data));
  }
  const JVal* nodes = m.doc.get("nodes");
  m.n_nodes = nodes ? nodes->size() : 0;
  const JVal* imgs = m.doc.get("images");
  m.n_images = imgs ? imgs->size() : 0;
  const JVal* texs = m.doc.get("textures");
  m.n_textures = texs ? texs->size() : 0;
}

G::vec3 jvec3(const JVal* a, G::vec3 def) {
  if (!a || a->kind != JVal::ARR || a->size() < 3) return def;
  return G::v3((float)ptgs::jdouble(a->at(0), 0), (float)ptgs::jdouble(a->at(1), 0), (float)ptgs::jdouble(a->at(2), 0));
}

G::mat4 jmat4(const JVal& a) {  // glm::make_mat4(double*) then float conversion
  G::mat4 r;
  for (int i = 0; i < 16; ++i) r.c[i / 4][i % 4] = (float)ptgs::jdouble(a.at((size_t)i), 0);
  return r;
}

// getNodeTransform (gameobject.cpp:547-560): matrix, else T * R * S from the fields of exact size
G::mat4 node_local(const JVal& n) {
  const JVal* mat = n.get("matrix");
  if (mat && mat->size() == 16) return jmat4(*mat);
  G::vec3 t = G::v3(0, 0, 0), s = G::v3(1, 1, 1);
  G::quat r;
  const JVal* tt = n.get("translation");
  if (tt && tt->size() == 3) t = jvec3(tt, t);
  const JVal* q = n.get("rotation");
  if (q && q->size() == 4) {
    r.x = (float)ptgs::jdouble(q->at(0), 0); r.y = (float)ptgs::jdouble(q->at(1), 0);
    r.z = (float)ptgs::jdouble(q->at(2), 0); r.w = (float)ptgs::jdouble(q->at(3), 1);
  }
  const JVal* ss = n.get("scale");
  if (ss && ss->size() == 3) s = jvec3(ss, s);
  return G::trs(t, r, s);
}

int scene_index(const Model& m) {
  const JVal* scenes = m.doc.get("scenes");
  if (!scenes || scenes->kind != JVal::ARR || scenes->arr.empty()) fail("glTF has no scenes!");
  int ds = ptgs::jint(m.doc.get("scene"), -1);
  int si = ds > -1 ? ds : 0;
  if ((size_t)si >= scenes->arr.size()) fail("default scene index out of range");
  return si;
}

// computeGlobalNodeTransforms (gameobject.cpp:65-159)
void global_transforms(const Model& m, std::vector<G::mat4>& globals) {
  globals.assign(m.n_nodes, G::identity4());
  struct TRS { G::vec3 t, s; G::quat r; bool ht = false, hr = false, hs = false; };
  std::map<int, TRS> anim;
  const JVal* anims = m.doc.get("animations");
  if (anims && anims->size() > 0) {
    const JVal& a = anims->arr[0];
    const JVal* chans = a.get("channels");
    const JVal* samplers = a.get("samplers");
    for (size_t i = 0; chans && i < chans->size(); ++i) {
      const JVal& ch = chans->arr[i];
      const JVal* tgt = ch.get("target");
      int node = tgt ? ptgs::jint(tgt->get("node"), -1) : -1;
      std::string pathk = tgt ? ptgs::jstr(tgt->get("path"), "") : "";
      const JVal* smp = samplers ? samplers->at((size_t)ptgs::jint(ch.get("sampler"), -1)) : nullptr;
      if (!smp) fail("animation channel with a bad sampler");
      int out_acc = ptgs::jint(smp->get("output"), -1);
      // getDataValue<T>: element 0, raw floats
      if (pathk == "translation") {
        Model::View v = m.view(out_acc, 12, 12, "animation output");
        if (!v.count) continue;
        float f[3];
        memcpy(f, v.p, 12);  // (accessor data need not be 4-byte aligned in a damaged file)
        anim[node].t = G::v3(f[0], f[1], f[2]);
        anim[node].ht = true;
      } else if (pathk == "rotation") {
        Model::View v = m.view(out_acc, 16, 16, "animation output");
        if (!v.count) continue;
        float f[4];
        memcpy(f, v.p, 16);
        anim[node].r.x = f[0]; anim[node].r.y = f[1]; anim[node].r.z = f[2]; anim[node].r.w = f[3];
        anim[node].hr = true;
      } else if (pathk == "scale") {
        Model::View v = m.view(out_acc, 12, 12, "animation output");
        if (!v.count) continue;
        float f[3];
        memcpy(f, v.p, 12);
        anim[node].s = G::v3(f[0], f[1], f[2]);
        anim[node].hs = true;
      }
    }
  }
  std::vector<char> on_stack(m.n_nodes, 0);
  std::function<void(int, const G::mat4&)> walk = [&](int ni, const G::mat4& parent) {
    const JVal* n = m.node(ni);
    if (!n) fail("node index out of range");
    if (on_stack[ni]) fail("cycle in the node hierarchy");
    on_stack[ni] = 1;
    G::mat4 local = G::identity4();
    const JVal* mat = n->get("matrix");
    if (mat && mat->size() == 16) {
      if (!anim.count(ni)) local = jmat4(*mat);  // an animated matrix node falls back to identity
    } else {
      G::vec3 t = G::v3(0, 0, 0), s = G::v3(1, 1, 1);
      G::quat r;
      const JVal* tt = n->get("translation");
      if (tt && tt->size() == 3) t = jvec3(tt, t);
      const JVal* q = n->get("rotation");
      if (q && q->size() == 4) {
        r.x = (float)ptgs::jdouble(q->at(0), 0); r.y = (float)ptgs::jdouble(q->at(1), 0);
        r.z = (float)ptgs::jdouble(q->at(2), 0); r.w = (float)ptgs::jdouble(q->at(3), 1);
      }
      const JVal* ss = n->get("scale");
      if (ss && ss->size() == 3) s = jvec3(ss, s);
      auto it = anim.find(ni);
      if (it != anim.end()) {
        if (it->second.ht) t = it->second.t;
        if (it->second.hr) r = it->second.r;
        if (it->second.hs) s = it->second.s;
      }
      local = G::trs(t, r, s);
    }
    G::mat4 global = G::mul(parent, local);
    globals[ni] = global;
    const JVal* ch = n->get("children");
    for (size_t i = 0; ch && i < ch->size(); ++i) walk(ptgs::jint(ch->at(i), -1), global);
    on_stack[ni] = 0;
  };
  const size_t si = (size_t)scene_index(m);  // (validates "scenes" before it is dereferenced)
  const JVal& sc = m.doc.get("scenes")->arr[si];
  const JVal* roots = sc.get("nodes");
  for (size_t i = 0; roots && i < roots->size(); ++i) walk(ptgs::jint(roots->at(i), -1), G::identity4());
}

// loadLights (gameobject.cpp:798-851)
void load_lights(const Model& m, const std::vector<G::mat4>& globals, std::vector<ptgs_punctual_light>& out) {
  const JVal* ext = m.doc.get("extensions");
  const JVal* kl = ext ? ext->get("KHR_lights_punctual") : nullptr;
  const JVal* lights = kl ? kl->get("lights") : nullptr;
  size_t nl = lights ? lights->size() : 0;
  for (size_t i = 0; i < m.n_nodes; ++i) {
    const JVal* n = m.node((int)i);
    const JVal* ne = n->get("extensions");
    const JVal* nk = ne ? ne->get("KHR_lights_punctual") : nullptr;
    if (!nk || !nk->has("light")) continue;
    int li = ptgs::jint(nk->get("light"), -1);
    if (li < 0 || (size_t)li >= nl) continue;
    const JVal& L = lights->arr[(size_t)li];
    ptgs_punctual_light l;
    memset(&l, 0, sizeof(l));
    const G::mat4& T = globals[i];
    l.position[0] = T.c[3][0]; l.position[1] = T.c[3][1]; l.position[2] = T.c[3][2];
    G::vec3 d = G::normalize(G::xyz(G::mul(T, G::v4(0, 0, -1, 0))));
    l.direction[0] = d.x; l.direction[1] = d.y; l.direction[2] = d.z;
    l.color[0] = l.color[1] = l.color[2] = 1.0f;
    const JVal* col = L.get("color");
    if (col && col->size() > 0) {
      l.color[0] = (float)ptgs::jdouble(col->at(0), 0);
      l.color[1] = (float)ptgs::jdouble(col->at(1), 0);
      l.color[2] = (float)ptgs::jdouble(col->at(2), 0);
    }
    l.intensity = (float)ptgs::jdouble(L.get("intensity"), 1.0);
    l.range = (float)ptgs::jdouble(L.get("range"), 0.0);
    std::string type = ptgs::jstr(L.get("type"), "");
    if (type == "directional") {
      l.type = 1;
    } else if (type == "point") {
      l.type = 0;
    } else if (type == "spot") {
      l.type = 2;
      const JVal* spot = L.get("spot");
      double inner = spot ? ptgs::jdouble(spot->get("innerConeAngle"), 0.0) : 0.0;
      double outer = spot ? ptgs::jdouble(spot->get("outerConeAngle"), 0.7853981634) : 0.7853981634;
      l.inner_cone_cos = (float)std::cos(inner);
      l.outer_cone_cos = (float)std::cos(outer);
    }
    out.push_back(l);
  }
}

int tex_source(const Model& m, int tex_index) {  // getImageSourceIndex
  const JVal* t = arr_at(m.doc, "textures", tex_index);
  if (!t || tex_index < 0 || (size_t)tex_index >= m.n_textures) return -1;
  return ptgs::jint(t->get("source"), -1);
}

int texture_id(const Model& m, int tex_index) {  // getTextureIndex (:370-378)
  if (tex_index >= 0 && (size_t)tex_index < m.n_textures) {
    int src = tex_source(m, tex_index);
    if (src >= 0 && (size_t)src < m.n_images) return src + 1;
  }
  return 0;
}

int info_index(const JVal* info) { return info ? ptgs::jint(info->get("index"), -1) : -1; }

// scanTextureFormats (:275-342): 1 = sRGB, 0 = UNORM
std::map<int, uint32_t> texture_formats(const Model& m) {
  std::map<int, uint32_t> f;
  const JVal* mats = m.doc.get("materials");
  size_t nm = mats ? mats->size() : 0;
  auto set = [&](const JVal* info, uint32_t srgb) {
    int src = tex_source(m, info_index(info));
    if (src >= 0) f[src] = srgb;
  };
  for (size_t i = 0; i < nm; ++i) {
    const JVal& mt = mats->arr[i];
    const JVal* pbr = mt.get("pbrMetallicRoughness");
    set(pbr ? pbr->get("baseColorTexture") : nullptr, 1);
    set(mt.get("emissiveTexture"), 1);
    set(mt.get("normalTexture"), 0);
    set(pbr ? pbr->get("metallicRoughnessTexture") : nullptr, 0);
    set(mt.get("occlusionTexture"), 0);
    const JVal* ex = mt.get("extensions");
    const JVal* tr = ex ? ex->get("KHR_materials_transmission") : nullptr;
    if (tr && tr->has("transmissionTexture")) set(tr->get("transmissionTexture"), 0);
    const JVal* cc = ex ? ex->get("KHR_materials_clearcoat") : nullptr;
    if (cc && cc->has("clearcoatTexture")) set(cc->get("clearcoatTexture"), 0);
    if (cc && cc->has("clearcoatRoughnessTexture")) set(cc->get("clearcoatRoughnessTexture"), 0);
  }
  for (size_t i = 0; i < nm; ++i) {
    const JVal* ex = mats->arr[i].get("extensions");
    const JVal* sg = ex ? ex->get("KHR_materials_pbrSpecularGlossiness") : nullptr;
    if (!sg) continue;
    if (sg->has("specularGlossinessTexture")) set(sg->get("specularGlossinessTexture"), 1);
    if (sg->has("diffuseTexture")) set(sg->get("diffuseTexture"), 1);
  }
  return f;
}

// getTextureTransform (gameobject.cpp:11-47): T * R(-rotation about z) * S
bool texture_transform(const JVal* info, float out[16]) {
  const JVal* ex = info ? info->get("extensions") : nullptr;
  const JVal* tt = ex ? ex->get("KHR_texture_transform") : nullptr;
  if (!tt) return false;
  float ox = 0, oy = 0, sx = 1, sy = 1, rot = 0;
  if (const JVal* o = tt->get("offset")) { ox = (float)ptgs::jdouble(o->at(0), 0); oy = (float)ptgs::jdouble(o->at(1), 0); }
  if (const JVal* s = tt->get("scale")) { sx = (float)ptgs::jdouble(s->at(0), 0); sy = (float)ptgs::jdouble(s->at(1), 0); }
  if (tt->has("rotation")) rot = (float)ptgs::jdouble(tt->get("rotation"), 0);
  G::mat4 S = G::scale(G::identity4(), G::v3(sx, sy, 1.0f));
  G::mat4 R = G::rotate(G::identity4(), -rot, G::v3(0, 0, 1));
  G::mat4 T = G::translate(G::identity4(), G::v3(ox, oy, 0.0f));
  G::mat4 M = G::mul(G::mul(T, R), S);
  for (int i = 0; i < 16; ++i) out[i] = M.c[i / 4][i % 4];
  return true;
}

// loadMaterials (:380-517) in the MaterialPushConstant layout (engine.cpp:1694-1718), texture ids
// object-relative; `pad` carries is_transparent.
void load_materials(const Model& m, std::vector<ptgs_material>& out) {
  const JVal* mats = m.doc.get("materials");
  size_t nm = mats ? mats->size() : 0;
  for (size_t i = 0; i < nm; ++i) {
    const JVal& mt = mats->arr[i];
    ptgs_material x = ptgs_default_material();
    x.albedo_texture_index = x.normal_texture_index = x.metallic_roughness_texture_index = 0;
    x.occlusion_texture_index = x.emissive_texture_index = 0;
    x.clearcoat_texture_index = x.clearcoat_roughness_texture_index = 0;
    x.sg_id = -1;
    std::string alpha_mode = ptgs::jstr(mt.get("alphaMode"), "OPAQUE");
    bool transparent = alpha_mode == "BLEND";
    if (alpha_mode == "MASK") x.alpha_cutoff = (float)ptgs::jdouble(mt.get("alphaCutoff"), 0.5);
    const JVal* ex = mt.get("extensions");
    const JVal* pbr = mt.get("pbrMetallicRoughness");
    const JVal* sg = ex ? ex->get("KHR_materials_pbrSpecularGlossiness") : nullptr;
    if (sg) {
      x.use_specular_glossiness_workflow = 1.0f;
      if (const JVal* f = sg->get("diffuseFactor")) {
        for (int k = 0; k < 4; ++k) x.base_color_factor[k] = (float)ptgs::jdouble(f->at((size_t)k), 0);
      } else {
        for (int k = 0; k < 4; ++k) x.base_color_factor[k] = 1.0f;
      }
      // specularFactor is stored then overwritten by the unconditional reset below (:465)
      x.roughness_factor = sg->has("glossinessFactor") ? (float)ptgs::jdouble(sg->get("glossinessFactor"), 1.0) : 1.0f;
      if (sg->has("diffuseTexture")) x.albedo_texture_index = texture_id(m, info_index(sg->get("diffuseTexture")));
      if (sg->has("specularGlossinessTexture"))
        x.sg_id = texture_id(m, info_index(sg->get("specularGlossinessTexture")));
    } else {
      const JVal* bcf = pbr ? pbr->get("baseColorFactor") : nullptr;
      for (int k = 0; k < 4; ++k) x.base_color_factor[k] = bcf ? (float)ptgs::jdouble(bcf->at((size_t)k), 1.0) : 1.0f;
      x.metallic_factor = (float)(pbr ? ptgs::jdouble(pbr->get("metallicFactor"), 1.0) : 1.0);
      x.roughness_factor = (float)(pbr ? ptgs::jdouble(pbr->get("roughnessFactor"), 1.0) : 1.0);
      const JVal* bct = pbr ? pbr->get("baseColorTexture") : nullptr;
      x.albedo_texture_index = texture_id(m, info_index(bct));
      texture_transform(bct, x.uv_albedo);
      x.metallic_roughness_texture_index = texture_id(m, info_index(pbr ? pbr->get("metallicRoughnessTexture") : nullptr));
    }
    G::vec3 ef = jvec3(mt.get("emissiveFactor"), G::v3(0, 0, 0));
    const JVal* es = ex ? ex->get("KHR_materials_emissive_strength") : nullptr;
    if (es && es->has("emissiveStrength")) {
      float s = (float)ptgs::jdouble(es->get("emissiveStrength"), 1.0);
      ef = G::v3(ef.x * s, ef.y * s, ef.z * s);
    }
    x.emissive_factor_and_pad[0] = ef.x; x.emissive_factor_and_pad[1] = ef.y; x.emissive_factor_and_pad[2] = ef.z;
    x.emissive_factor_and_pad[3] = 0.0f;
    x.normal_texture_index = texture_id(m, info_index(mt.get("normalTexture")));
    x.occlusion_texture_index = texture_id(m, info_index(mt.get("occlusionTexture")));
    x.emissive_texture_index = texture_id(m, info_index(mt.get("emissiveTexture")));
    const JVal* occ = mt.get("occlusionTexture");
    x.occlusion_strength = (float)(occ ? ptgs::jdouble(occ->get("strength"), 1.0) : 1.0);
    x.specular_color_factor[0] = x.specular_color_factor[1] = x.specular_color_factor[2] = 1.0f;
    x.specular_factor = 0.5f;
    const JVal* sp = ex ? ex->get("KHR_materials_specular") : nullptr;
    if (sp) {
      if (sp->has("specularFactor")) x.specular_factor = (float)ptgs::jdouble(sp->get("specularFactor"), 0.5);
      const JVal* c = sp->get("specularColorFactor");
      if (c && c->kind == JVal::ARR && c->size() >= 3)
        for (int k = 0; k < 3; ++k) x.specular_color_factor[k] = (float)ptgs::jdouble(c->at((size_t)k), 1.0);
    }
    texture_transform(mt.get("normalTexture"), x.uv_normal);
    texture_transform(mt.get("emissiveTexture"), x.uv_emissive);
    const JVal* tr = ex ? ex->get("KHR_materials_transmission") : nullptr;
    if (tr) {
      if (tr->has("transmissionFactor")) x.transmission_factor = (float)ptgs::jdouble(tr->get("transmissionFactor"), 0.0);
      // transmission_texture_index is resolved by the reference but never reaches the GPU (engine.cpp:1694-1718)
      if (x.transmission_factor > 0.0f || tr->has("transmissionTexture")) transparent = true;
    }
    const JVal* cc = ex ? ex->get("KHR_materials_clearcoat") : nullptr;
    if (cc) {
      if (cc->has("clearcoatFactor")) x.clearcoat_factor = (float)ptgs::jdouble(cc->get("clearcoatFactor"), 0.0);
      if (cc->has("clearcoatRoughnessFactor"))
        x.clearcoat_roughness_factor = (float)ptgs::jdouble(cc->get("clearcoatRoughnessFactor"), 0.0);
      if (cc->has("clearcoatTexture")) x.clearcoat_texture_index = texture_id(m, info_index(cc->get("clearcoatTexture")));
      if (cc->has("clearcoatRoughnessTexture"))
        x.clearcoat_roughness_texture_index = texture_id(m, info_index(cc->get("clearcoatRoughnessTexture")));
    }
    x.pad = transparent ? 1.0f : 0.0f;
    out.push_back(x);
  }
  if (out.empty()) {
    ptgs_material x = ptgs_default_material();
    x.albedo_texture_index = 0;
    x.sg_id = -1;
    out.push_back(x);
  }
}

// Vertex identity for deduplication: Vertex::operator== (GeneralHeaders.h:92-94) compares pos,
// color, tex_coord, tangent and normal with float ==; the hash folds -0 into +0 so that equal keys
// hash alike (std::hash<float> does the same).
struct VKey {
  float f[15];
};
struct VKeyHash {
  size_t operator()(const VKey& k) const {
    size_t h = 1469598103934665603ull;
    for (float x : k.f) {
      uint32_t u;
      float y = x == 0.0f ? 0.0f : x;
      memcpy(&u, &y, 4);
      h = (h ^ u) * 1099511628211ull;
    }
    return h;
  }
};
struct VKeyEq {
  bool operator()(const VKey& a, const VKey& b) const {
    for (int i = 0; i < 15; ++i)
      if (!(a.f[i] == b.f[i])) return false;
    return true;
  }
};
VKey vkey(const ptgs_vertex& v) {
  VKey k;
  const float* src[5] = {v.pos, v.color, v.tex_coord, v.tangent, v.normal};
  const int n[5] = {3, 3, 2, 4, 3};
  int o = 0;
  for (int s = 0; s < 5; ++s)
    for (int i = 0; i < n[s]; ++i) k.f[o++] = src[s][i];
  return k;
}

struct Loader {
  const Model& m;
  ptgs_scene_builder::Object& obj;
  std::vector<G::mat4> skin;
  std::unordered_map<VKey, uint32_t, VKeyHash, VKeyEq> uniq;

  uint32_t add_vertex(const ptgs_vertex& v) {
    VKey k = vkey(v);
    auto it = uniq.find(k);
    if (it != uniq.end()) return it->second;
    uint32_t id = (uint32_t)obj.vertices.size();
    obj.vertices.push_back(v);
    bool nan = false;
    for (float x : k.f) nan |= (x != x);
    // a key holding NaN never compares equal: the reference's second map lookup then inserts a
    // fresh entry whose value is 0, so such a corner references vertex 0
    if (nan) return 0;
    uniq.emplace(k, id);
    return id;
  }

  // loadPrimitive (:562-795)
  void primitive(const JVal& prim, const G::mat4& transform) {
    int mi = ptgs::jint(prim.get("material"), -1);
    int material_index = mi >= 0 ? mi : 0;
    if ((size_t)material_index >= obj.materials.size()) fail("primitive material index out of range");
    const float* e = obj.materials[(size_t)material_index].emissive_factor_and_pad;
    bool is_emissive = G::length(G::v3(e[0], e[1], e[2])) > 0.001f;
    const JVal& attrs = req(prim, "attributes", "primitive");
    if (!attrs.has("POSITION")) fail("primitive without POSITION");
    auto attr_view = [&](const char* name, size_t def_stride, size_t bytes) {
      Model::View v = m.view(ptgs::jint(attrs.get(name), -1), def_stride, bytes, name);
      if (v.ctype != 5126) fail(std::string(name) + ": only float attributes are supported");
      return v;
    };
    Model::View pos = attr_view("POSITION", 12, 12);
    Model::View nrm, tan, uv0, uv1, jnt, wgt;
    if (attrs.has("NORMAL")) nrm = attr_view("NORMAL", 12, 12);
    if (attrs.has("TANGENT")) tan = attr_view("TANGENT", 16, 16);
    if (attrs.has("TEXCOORD_0")) uv0 = attr_view("TEXCOORD_0", 8, 8);
    if (attrs.has("TEXCOORD_1")) uv1 = attr_view("TEXCOORD_1", 8, 8);
    bool has_skin = !skin.empty() && attrs.has("JOINTS_0") && attrs.has("WEIGHTS_0");
    if (has_skin) {
      // element sizes from the accessor types (tinygltf ByteStride)
      jnt = m.view(ptgs::jint(attrs.get("JOINTS_0"), -1), 0, 4, "JOINTS_0");
      if (jnt.ctype == 5123) jnt = m.view(ptgs::jint(attrs.get("JOINTS_0"), -1), 0, 8, "JOINTS_0");
      wgt = m.view(ptgs::jint(attrs.get("WEIGHTS_0"), -1), 0, wgt_bytes(attrs), "WEIGHTS_0");
    }
    // indices (or a sequential list for non-indexed primitives)
    std::vector<uint32_t> src_idx;
    int ia = ptgs::jint(prim.get("indices"), -1);
    if (ia >= 0) {
      const JVal* acc = arr_at(m.doc, "accessors", ia);
      int ct = acc ? ptgs::jint(acc->get("componentType"), 0) : 0;
      size_t es = ct == 5123 ? 2 : (ct == 5125 ? 4 : 1);
      Model::View iv = m.view(ia, es, es, "indices");
      src_idx.resize(iv.count);
      for (size_t i = 0; i < iv.count; ++i) {
        if (ct == 5123) src_idx[i] = ld_u16(iv.p + 2 * i);
        else if (ct == 5125) src_idx[i] = ld_u32(iv.p + 4 * i);
        else src_idx[i] = iv.p[i];
      }
    } else {
      src_idx.resize(pos.count);
      for (size_t i = 0; i < pos.count; ++i) src_idx[i] = (uint32_t)i;
    }
    const G::mat3 nmat = G::transpose(G::inverse(G::upper3(transform)));
    const G::mat3 tmat = G::upper3(transform);
    std::vector<uint32_t> local;
    local.reserve(src_idx.size());
    for (uint32_t idx : src_idx) {
      if (idx >= pos.count) fail("vertex index out of range");
      ptgs_vertex v;
      memset(&v, 0, sizeof(v));
      v.color[0] = v.color[1] = v.color[2] = 1.0f;
      memcpy(v.pos, pos.p + idx * pos.stride, 12);
      if (nrm.p) {
        if (idx >= nrm.count) fail("NORMAL index out of range");
        memcpy(v.normal, nrm.p + idx * nrm.stride, 12);
      } else {
        v.normal[1] = 1.0f;
      }
      if (tan.p) {
        if (idx >= tan.count) fail("TANGENT index out of range");
        memcpy(v.tangent, tan.p + idx * tan.stride, 16);
      } else {
        v.tangent[0] = 1.0f;
      }
      if (uv0.p) {
        if (idx >= uv0.count) fail("TEXCOORD_0 index out of range");
        memcpy(v.tex_coord, uv0.p + idx * uv0.stride, 8);
      }
      if (uv1.p) {
        if (idx >= uv1.count) fail("TEXCOORD_1 index out of range");
        memcpy(v.tex_coord_1, uv1.p + idx * uv1.stride, 8);
      } else {
        v.tex_coord_1[0] = v.tex_coord[0];
        v.tex_coord_1[1] = v.tex_coord[1];
      }
      G::vec3 p = G::v3(v.pos[0], v.pos[1], v.pos[2]);
      G::vec3 n = G::v3(v.normal[0], v.normal[1], v.normal[2]);
      G::vec3 t = G::v3(v.tangent[0], v.tangent[1], v.tangent[2]);
      if (has_skin) {
        if (idx >= jnt.count || idx >= wgt.count) fail("skin attribute index out of range");
        uint32_t j[4];
        const uint8_t* jp = jnt.p + idx * jnt.stride;
        for (int k = 0; k < 4; ++k) j[k] = jnt.ctype == 5123 ? ld_u16(jp + 2 * k) : jp[k];
        float w[4] = {1.0f, 0.0f, 0.0f, 0.0f};
        if (wgt.ctype == 5126) memcpy(w, wgt.p + idx * wgt.stride, 16);
        float sum = ((w[0] + w[1]) + w[2]) + w[3];
        if (sum > 0.0f) {
          for (float& x : w) x = x / sum;
        } else {
          w[0] = 1.0f; w[1] = w[2] = w[3] = 0.0f;
        }
        for (uint32_t k : j)
          if (k >= skin.size()) fail("joint index out of range");
        G::mat4 S = G::add(G::add(G::add(G::scale(skin[j[0]], w[0]), G::scale(skin[j[1]], w[1])),
                                  G::scale(skin[j[2]], w[2])),
                           G::scale(skin[j[3]], w[3]));
        p = G::xyz(G::mul(S, G::v4(p.x, p.y, p.z, 1.0f)));
        float inv[16], sm[16];
        for (int a = 0; a < 16; ++a) sm[a] = S.c[a / 4][a % 4];
        ptgs_mat4_inverse_glm(sm, inv);  // glm::inverse(mat4) (a singular blend yields inf/NaN, as GLM)
        G::mat4 I;
        for (int a = 0; a < 16; ++a) I.c[a / 4][a % 4] = inv[a];
        n = G::normalize(G::mul(G::upper3(G::transpose(I)), n));
        if (v.tangent[3] != 0.0f) t = G::normalize(G::mul(G::upper3(S), t));
      } else {
        p = G::xyz(G::mul(transform, G::v4(p.x, p.y, p.z, 1.0f)));
        n = G::normalize(G::mul(nmat, n));
        if (v.tangent[3] != 0.0f) t = G::normalize(G::mul(tmat, t));
      }
      v.pos[0] = p.x; v.pos[1] = p.y; v.pos[2] = p.z;
      v.normal[0] = n.x; v.normal[1] = n.y; v.normal[2] = n.z;
      v.tangent[0] = t.x; v.tangent[1] = t.y; v.tangent[2] = t.z;
      local.push_back(add_vertex(v));
    }
    ptgs_primitive pr;
    pr.material_index = material_index;
    pr.first_index = (uint32_t)obj.indices.size();
    pr.index_count = (uint32_t)src_idx.size();
    obj.indices.insert(obj.indices.end(), local.begin(), local.end());
    for (size_t k = 0; k + 2 < local.size(); k += 3) {
      uint32_t i0 = local[k], i1 = local[k + 1], i2 = local[k + 2];
      obj.indices.push_back(i0);
      obj.indices.push_back(i1);
      obj.indices.push_back(i2);
      if (is_emissive) {
        G::vec3 p0 = vpos(i0), p1 = vpos(i1), p2 = vpos(i2);
        float area = 0.5f * G::length(G::cross(p1 - p0, p2 - p0));
        if (area > 1e-6f) obj.etris.push_back({i0, i1, i2, (uint32_t)material_index, area});
      }
    }
    obj.prims.push_back(pr);
  }
  size_t wgt_bytes(const JVal& attrs) const {
    const JVal* acc = arr_at(m.doc, "accessors", ptgs::jint(attrs.get("WEIGHTS_0"), -1));
    int ct = acc ? ptgs::jint(acc->get("componentType"), 0) : 0;
    return ct == 5126 ? 16 : (ct == 5123 ? 8 : 4);
  }
  G::vec3 vpos(uint32_t i) const {
    const ptgs_vertex& v = obj.vertices[i];
    return G::v3(v.pos[0], v.pos[1], v.pos[2]);
  }

  // processNode (:529-545)
  void node(int ni, const G::mat4& parent, int depth) {
    const JVal* n = m.node(ni);
    if (!n) fail("node index out of range");
    if (depth > 1024) fail("node hierarchy too deep (cycle?)");
    G::mat4 local = G::mul(parent, node_local(*n));
    bool skinned = ptgs::jint(n->get("skin"), -1) >= 0;
    const G::mat4& mesh_t = skinned ? parent : local;
    int mesh = ptgs::jint(n->get("mesh"), -1);
    if (mesh >= 0) {
      const JVal* me = arr_at(m.doc, "meshes", mesh);
      if (!me) fail("mesh index out of range");
      const JVal* prims = me->get("primitives");
      for (size_t i = 0; prims && i < prims->size(); ++i) primitive(prims->arr[i], mesh_t);
    }
    const JVal* ch = n->get("children");
    for (size_t i = 0; ch && i < ch->size(); ++i) node(ptgs::jint(ch->at(i), -1), local, depth + 1);
  }
};

// Gameobject::loadModel (:198-273): one object with model-space geometry (before the scene bake)
void load_gltf(const std::string& path, uint32_t flags, ptgs_scene_builder::Object& obj) {
  Model m;
  load_model_file(path, m);
  std::vector<G::mat4> globals;
  global_transforms(m, globals);
  load_lights(m, globals, obj.lights);
  Loader L{m, obj, {}, {}};
  const JVal* skins = m.doc.get("skins");
  if (skins && skins->size() > 0) {
    const JVal& sk = skins->arr[0];
    const JVal* joints = sk.get("joints");
    size_t nj = joints ? joints->size() : 0;
    L.skin.assign(nj, G::identity4());
    int ibm = ptgs::jint(sk.get("inverseBindMatrices"), -1);
    if (ibm > -1) {
      Model::View v = m.view(ibm, 0, 64, "inverseBindMatrices");
      if (v.count < nj) fail("inverseBindMatrices shorter than the joint list");
      for (size_t i = 0; i < nj; ++i) {
        int jn = ptgs::jint(joints->at(i), -1);
        if (jn < 0 || (size_t)jn >= m.n_nodes) fail("joint node out of range");
        G::mat4 M;
        memcpy(M.c, v.p + i * v.stride, 64);
        L.skin[i] = G::mul(globals[(size_t)jn], M);
      }
    }
  }
  // textures: default white, then every image (loadTextures :344-368)
  std::map<int, uint32_t> fmt = texture_formats(m);
  obj.textures.clear();
  ptgs_scene_builder::Texture white;
  white.rgba = {255, 255, 255, 255};
  obj.textures.push_back(white);
  const JVal* imgs = m.doc.get("images");
  struct Job {
    std::vector<uint8_t> bytes;
    std::string uri, err;
    bool ok = false;
    ptgs::DecodedImage img;
  };
  std::vector<Job> jobs(m.n_images);
  for (size_t i = 0; i < m.n_images; ++i) {
    const JVal& im = imgs->arr[i];
    Job& jb = jobs[i];
    jb.uri = ptgs::jstr(im.get("uri"), "");
    if (!jb.uri.empty()) {
      jb.ok = load_uri(jb.uri, m.base, jb.bytes);
    } else {
      int bvi = ptgs::jint(im.get("bufferView"), -1);
      const JVal* bv = arr_at(m.doc, "bufferViews", bvi);
      if (bv) {
        int bi = ptgs::jint(bv->get("buffer"), -1);
        size_t off = (size_t)ptgs::jdouble(bv->get("byteOffset"), 0), len = (size_t)ptgs::jdouble(bv->get("byteLength"), 0);
        if (bi >= 0 && (size_t)bi < m.buffers.size() && off <= m.buffers[bi].size() && len <= m.buffers[bi].size() - off) {
          jb.bytes.assign(m.buffers[bi].begin() + off, m.buffers[bi].begin() + off + len);
          jb.ok = true;
        }
      }
    }
  }
  // decode in parallel (images are independent); errors are reported for the lowest index
  {
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t i; (i = next.fetch_add(1)) < jobs.size();) {
        Job& jb = jobs[i];
        // no exception may leave a worker thread (std::terminate would abort the host process)
        try {
          if (jb.ok) jb.ok = ptgs::decode_image_rgba8(jb.bytes.data(), jb.bytes.size(), jb.img, jb.err);
        } catch (const std::bad_alloc&) {
          jb.ok = false;
          jb.err = "out of memory decoding the image";
        } catch (const std::exception& ex) {
          jb.ok = false;
          jb.err = ex.what();
        } catch (...) {
          jb.ok = false;
          jb.err = "image decode failed";
        }
        std::vector<uint8_t>().swap(jb.bytes);
      }
    };
    unsigned nt = std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 16u);
    nt = (unsigned)std::min<size_t>(nt, jobs.size());
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
  }
  for (size_t i = 0; i < m.n_images; ++i) {
    Job& jb = jobs[i];
    ptgs_scene_builder::Texture t;
    auto it = fmt.find((int)i);
    t.srgb = it == fmt.end() ? 1u : it->second;
    if (!jb.ok) {
      if (!(flags & PTGS_INGEST_MISSING_IMAGES_WHITE))
        fail("failed to load texture image '" + jb.uri + "' of " + path + (jb.err.empty() ? "" : ": " + jb.err));
      t.rgba = {255, 255, 255, 255};
      t.w = t.h = 1;
    } else {
      t.rgba = std::move(jb.img.rgba);
      t.w = jb.img.w;
      t.h = jb.img.h;
    }
    obj.textures.push_back(std::move(t));
  }
  obj.num_textures = (uint32_t)obj.textures.size();
  load_materials(m, obj.materials);
  int si = scene_index(m);
  const JVal* roots = m.doc.get("scenes")->arr[(size_t)si].get("nodes");
  for (size_t i = 0; roots && i < roots->size(); ++i) L.node(ptgs::jint(roots->at(i), -1), G::identity4(), 0);
}

// Engine::loadScene STEP 1-3 (engine.cpp:1271-1331): bake T * R * S into the object
void bake(ptgs_scene_builder::Object& o, const G::vec3& pos, const G::vec3& rot_deg, const G::vec3& scl) {
  G::mat4 T = G::trs(pos, G::quat_from_euler(G::radians(rot_deg)), scl);
  G::mat3 nm = G::transpose(G::inverse(G::upper3(T)));
  G::mat3 t3 = G::upper3(T);
  for (ptgs_vertex& v : o.vertices) {
    G::vec3 p = G::xyz(G::mul(T, G::v4(v.pos[0], v.pos[1], v.pos[2], 1.0f)));
    G::vec3 n = G::normalize(G::mul(nm, G::v3(v.normal[0], v.normal[1], v.normal[2])));
    G::vec3 t = G::normalize(G::mul(t3, G::v3(v.tangent[0], v.tangent[1], v.tangent[2])));
    v.pos[0] = p.x; v.pos[1] = p.y; v.pos[2] = p.z;
    v.normal[0] = n.x; v.normal[1] = n.y; v.normal[2] = n.z;
    v.tangent[0] = t.x; v.tangent[1] = t.y; v.tangent[2] = t.z;
  }
  float sf = G::length(G::v3(T.c[0][0], T.c[0][1], T.c[0][2]));
  for (ptgs_punctual_light& l : o.lights) {
    G::vec3 p = G::xyz(G::mul(T, G::v4(l.position[0], l.position[1], l.position[2], 1.0f)));
    G::vec3 d = G::normalize(G::mul(nm, G::v3(l.direction[0], l.direction[1], l.direction[2])));
    l.position[0] = p.x; l.position[1] = p.y; l.position[2] = p.z;
    l.direction[0] = d.x; l.direction[1] = d.y; l.direction[2] = d.z;
    if (l.range > 0.0f) l.range *= sf;
    l.intensity *= (sf * sf);
  }
  for (auto& e : o.etris) {
    const ptgs_vertex &a = o.vertices[e.i0], &b = o.vertices[e.i1], &c = o.vertices[e.i2];
    G::vec3 p0 = G::v3(a.pos[0], a.pos[1], a.pos[2]), p1 = G::v3(b.pos[0], b.pos[1], b.pos[2]),
            p2 = G::v3(c.pos[0], c.pos[1], c.pos[2]);
    e.area = 0.5f * G::length(G::cross(p1 - p0, p2 - p0));
  }
}

int add_gltf_impl(ptgs_scene_builder* b, const std::string& path, const float* pos, const float* rot,
                  const float* scl, uint32_t flags) {
  try {
    ptgs_scene_builder::Object o;
    load_gltf(path, flags, o);
    bake(o, pos ? G::v3(pos[0], pos[1], pos[2]) : G::v3(0, 0, 0), rot ? G::v3(rot[0], rot[1], rot[2]) : G::v3(0, 0, 0),
         scl ? G::v3(scl[0], scl[1], scl[2]) : G::v3(1, 1, 1));
    b->objects.push_back(std::move(o));
    return PTGS_OK;
  } catch (const LoadError& e) {
    b->err = e.msg;
    return PTGS_EIO;
  } catch (const std::bad_alloc&) {
    b->err = "out of memory while loading " + path;
    return PTGS_ERANGE;
  }
}

}  // namespace

extern "C" {

int ptgs_image_decode_rgba8(const void* bytes, size_t size, uint8_t* rgba, size_t capacity, uint32_t* width,
                            uint32_t* height, uint32_t* comp) {
  if (!bytes) return PTGS_EINVAL;
  ptgs::DecodedImage d;
  std::string err;
  if (!ptgs::decode_image_rgba8((const uint8_t*)bytes, size, d, err, rgba == nullptr)) return PTGS_EIO;
  if (width) *width = d.w;
  if (height) *height = d.h;
  if (comp) *comp = d.comp;
  if (!rgba) return PTGS_OK;
  if (capacity < d.rgba.size()) return PTGS_ERANGE;
  memcpy(rgba, d.rgba.data(), d.rgba.size());
  return PTGS_OK;
}

int ptgs_builder_add_gltf(ptgs_scene_builder* b, const char* path, const float position[3], const float rotation_deg[3],
                          const float scale[3], uint32_t flags) {
  if (!b || !path) return PTGS_EINVAL;
  return add_gltf_impl(b, path, position, rotation_deg, scale, flags);
}

int ptgs_builder_add_punctual_light(ptgs_scene_builder* b, const ptgs_punctual_light* light) {
  if (!b || !light) return PTGS_EINVAL;
  b->global_lights.push_back(*light);
  return PTGS_OK;
}

int ptgs_builder_load_scene_json(ptgs_scene_builder* b, const char* path, const char* root_dir, uint32_t flags,
                                 ptgs_scene_settings* settings) {
  if (!b || !path) return PTGS_EINVAL;
  std::string root = root_dir ? root_dir : "";
  ptgs_scene_settings s;
  memset(&s, 0, sizeof(s));
  // Engine member defaults (engine.h:246-255, :316-317; GeneralHeaders.h:279-285)
  s.ambient_light[3] = 1.0f;
  s.render_torus = 1;
  s.render_pointcloud = 1;
  s.torus_major_radius = 16.0f; s.torus_minor_radius = 1.0f; s.torus_height = 8.0f;
  s.torus_major_segments = 500; s.torus_minor_segments = 500;
  s.num_rays = 1000000;
  s.use_lod = 0.0f; s.lod_factor = 1.0f;
  s.accumulation_steps = 512; s.total_positions = 336;
  s.min_beta = -45.0f; s.max_beta = 45.0f; s.image_divisor = 2.0f;
  s.capture_images = 1; s.capture_pointcloud = 1;
  std::vector<uint8_t> bytes;
  std::string p = join_path(root, path);
  if (!ptgs::read_file(p, bytes)) { b->err = "Failed to open scene file: " + p; return PTGS_EIO; }
  JVal doc;
  if (!ptgs::parse_json((const char*)bytes.data(), bytes.size(), doc) || doc.kind != JVal::OBJ) {
    b->err = "bad JSON in " + p;
    return PTGS_EIO;
  }
  // main_scene.json names the scene file to load (engine.cpp:1182-1186); a file that is itself a
  // scene (has "objects" / "settings") is accepted directly
  if (doc.get("scene") && !doc.has("objects") && !doc.has("settings")) {
    std::string q = join_path(root, ptgs::jstr(doc.get("scene"), ""));
    if (!ptgs::read_file(q, bytes)) { b->err = "Failed to open scene file: " + q; return PTGS_EIO; }
    if (!ptgs::parse_json((const char*)bytes.data(), bytes.size(), doc) || doc.kind != JVal::OBJ) {
      b->err = "bad JSON in " + q;
      return PTGS_EIO;
    }
  }
  std::string rtbox_path;
  bool use_rt_box = false;
  std::vector<ptgs_punctual_light> suns;
  if (const JVal* st = doc.get("settings")) {
    use_rt_box = ptgs::jbool(st->get("use_rt_box"), false);
    rtbox_path = ptgs::jstr(st->get("rt_box_file"), "");
    s.render_torus = ptgs::jbool(st->get("render_torus"), s.render_torus != 0);
    s.render_pointcloud = ptgs::jbool(st->get("render_pointcloud"), s.render_pointcloud != 0);
    if (const JVal* a = st->get("ambient_light")) {
      for (int k = 0; k < 4; ++k) s.ambient_light[k] = (float)ptgs::jdouble(a->at((size_t)k), 0);
    } else {
      s.ambient_light[0] = s.ambient_light[1] = s.ambient_light[2] = 0.0f;
      s.ambient_light[3] = 1.0f;
    }
    if (const JVal* t = st->get("torus_settings")) {
      s.torus_major_radius = ptgs::jnum(t->get("major_radius"), 16.0f);
      s.torus_minor_radius = ptgs::jnum(t->get("minor_radius"), 1.0f);
      s.torus_height = ptgs::jnum(t->get("height"), 8.0f);
      s.torus_major_segments = ptgs::jint(t->get("major_segments"), 500);
      s.torus_minor_segments = ptgs::jint(t->get("minor_segments"), 500);
      s.num_rays = (uint32_t)ptgs::jint(t->get("num_rays"), (int)s.num_rays);
    }
    if (const JVal* sun = st->get("sun")) {
      ptgs_punctual_light l;
      memset(&l, 0, sizeof(l));
      const JVal* c = sun->get("color");
      const JVal* d = sun->get("direction");
      for (int k = 0; k < 3; ++k) {
        l.color[k] = (float)ptgs::jdouble(c ? c->at((size_t)k) : nullptr, 0);
        l.direction[k] = (float)ptgs::jdouble(d ? d->at((size_t)k) : nullptr, 0);
      }
      l.intensity = ptgs::jnum(sun->get("intensity"), 1.0f);
      l.type = 1;
      suns.push_back(l);
    }
    s.use_lod = ptgs::jnum(st->get("use_lod"), s.use_lod);
    s.lod_factor = ptgs::jnum(st->get("lod_factor"), s.lod_factor);
    s.accumulation_steps = (uint32_t)ptgs::jint(st->get("accumulation_steps"), 512);
    s.total_positions = (uint32_t)ptgs::jint(st->get("total_positions"), 336);
    s.min_beta = ptgs::jnum(st->get("min_beta"), -45.0f);
    s.max_beta = ptgs::jnum(st->get("max_beta"), 45.0f);
    s.image_divisor = ptgs::jnum(st->get("image_divisor"), 2.0f);
    s.capture_images = ptgs::jbool(st->get("capture_images"), true);
    s.capture_pointcloud = ptgs::jbool(st->get("capture_pointcloud"), true);
  }
  b->global_lights = suns;  // global_punctual_lights.clear() + sun (engine.cpp:1193, :1225-1242)
  s.use_rt_box = use_rt_box ? 1 : 0;
  if (const JVal* objs = doc.get("objects")) {
    for (size_t i = 0; i < objs->size(); ++i) {
      const JVal& od = objs->arr[i];
      std::string model = ptgs::jstr(od.get("model"), "");
      if (model.empty()) { b->err = "scene object " + std::to_string(i) + " has no model"; return PTGS_EIO; }
      float pos[3] = {0, 0, 0}, rot[3] = {0, 0, 0}, scl[3] = {1, 1, 1};
      auto rd3 = [&](const char* key, float* dst) {
        if (const JVal* a = od.get(key))
          for (int k = 0; k < 3; ++k) dst[k] = (float)ptgs::jdouble(a->at((size_t)k), 0);
      };
      rd3("position", pos);
      rd3("scale", scl);
      rd3("rotation", rot);
      int rc = add_gltf_impl(b, join_path(root, model), pos, rot, scl, flags);
      if (rc) return rc;
      ++s.num_objects;
    }
  }
  if (use_rt_box && !rtbox_path.empty()) {
    int rc = ptgs_builder_add_rtbox_json(b, join_path(root, rtbox_path).c_str());
    if (rc) return rc;
  }
  if (settings) *settings = s;
  return PTGS_OK;
}

}  // extern "C"
