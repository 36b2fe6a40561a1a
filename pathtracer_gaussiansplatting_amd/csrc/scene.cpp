// scene.cpp — host mirror of the reference Engine's camera + scene flattening (include/ptgs/ptgs_host.h).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/ptgs/ptgs_host.h"
#include "hostmath.h"
#include "image_decode.h"
#include "json.h"
#include "scene_builder.h"

using ptgs::JVal;
using ptgs::jnum;

namespace {

// ---------------------------------------------------------------------------------------------
// glm-style float helpers (GLM 0.9.9 formulas: normalize = v * inversesqrt(dot(v,v)))
// ---------------------------------------------------------------------------------------------
struct f3 { float x, y, z; };
inline f3 sub(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline f3 add(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline f3 mul(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline f3 cross(f3 a, f3 b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
inline float length(f3 v) { return std::sqrt(dot(v, v)); }
inline f3 normalize(f3 v) { return mul(v, 1.0f / std::sqrt(dot(v, v))); }
inline float radians(float d) { return d * 0.01745329251994329576923690768489f; }
inline float gmod(float x, float y) { return x - y * std::floor(x / y); }

void lookat(f3 eye, f3 center, f3 up, float* m) {
  f3 f = normalize(sub(center, eye));
  f3 s = normalize(cross(f, up));
  f3 u = cross(s, f);
  for (int k = 0; k < 16; ++k) m[k] = (k % 5 == 0) ? 1.0f : 0.0f;
  m[0] = s.x; m[4] = s.y; m[8] = s.z;
  m[1] = u.x; m[5] = u.y; m[9] = u.z;
  m[2] = -f.x; m[6] = -f.y; m[10] = -f.z;
  m[12] = -dot(s, eye);
  m[13] = -dot(u, eye);
  m[14] = dot(f, eye);
}

void perspective_zo(float fovy, float aspect, float zn, float zf, float* m) {
  float t = std::tan(fovy / 2.0f);
  for (int k = 0; k < 16; ++k) m[k] = 0.0f;
  m[0] = 1.0f / (aspect * t);
  m[5] = 1.0f / t;
  m[10] = zf / (zn - zf);
  m[11] = -1.0f;
  m[14] = -(zf * zn) / (zf - zn);
  m[5] *= -1.0f;  // camera.cpp:95 / :187 / :227
}

// glm::rotate(mat4(1), angle, axis) applied to a direction (w = 0)
f3 rotate_dir(float angle, f3 axis_in, f3 v) {
  float c = std::cos(angle), s = std::sin(angle);
  f3 axis = normalize(axis_in);
  f3 temp = mul(axis, 1.0f - c);
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
  // (R * vec4(v, 0)).xyz, columns R[c]
  return {(R[0][0] * v.x + R[1][0] * v.y) + R[2][0] * v.z, (R[0][1] * v.x + R[1][1] * v.y) + R[2][1] * v.z,
          (R[0][2] * v.x + R[1][2] * v.y) + R[2][2] * v.z};
}

}  // namespace


ptgs_material ptgs_default_material() {
  ptgs_material m;
  std::memset(&m, 0, sizeof(m));
  // Material defaults, GeneralHeaders.h:202-235
  for (int k = 0; k < 4; ++k) m.base_color_factor[k] = 1.0f;
  for (int k = 0; k < 16; ++k) {
    m.uv_normal[k] = (k % 5 == 0) ? 1.0f : 0.0f;
    m.uv_emissive[k] = m.uv_normal[k];
    m.uv_albedo[k] = m.uv_normal[k];
  }
  m.metallic_factor = 1.0f;
  m.roughness_factor = 1.0f;
  m.occlusion_strength = 1.0f;
  m.specular_factor = 0.5f;
  for (int k = 0; k < 3; ++k) m.specular_color_factor[k] = 1.0f;
  m.sg_id = -1;
  return m;
}

extern "C" {

int ptgs_camera_lookat(const float eye[3], const float center[3], const float up[3], float view[16]) {
  if (!eye || !center || !up || !view) return PTGS_EINVAL;
  lookat({eye[0], eye[1], eye[2]}, {center[0], center[1], center[2]}, {up[0], up[1], up[2]}, view);
  return PTGS_OK;
}

int ptgs_camera_perspective(float fovy, float aspect, float zn, float zf, float proj[16]) {
  if (!proj || !(aspect > 0.0f) || zn == zf) return PTGS_EINVAL;
  perspective_zo(fovy, aspect, zn, zf, proj);
  return PTGS_OK;
}

int ptgs_mat4_inverse(const float m[16], float out[16]) {
  if (!m || !out) return PTGS_EINVAL;
  return ptgs::inverse4(m, out) ? PTGS_OK : PTGS_EINVAL;
}

int ptgs_camera_toroidal(float alpha_deg, float beta_deg, float radius, float height, float fov_deg, float aspect,
                         float zn, float zf, float view[16], float proj[16], float position[3]) {
  if (!view || !proj) return PTGS_EINVAL;
  float alpha = gmod(alpha_deg, 360.0f);
  if (alpha < 0.0f) alpha += 360.0f;
  float beta = gmod(beta_deg, 360.0f);
  if (beta < 0.0f) beta += 360.0f;
  float a = radians(alpha), b = radians(beta);
  // camera.cpp:205,208 call cos / sin unqualified on a float: with no float overload in the global
  // namespace that is the C library's double ::cos / ::sin, rounded to float by the vec3 constructor
  // (glm::rotate below uses the float std::cos / std::sin). With float cosf / sinf here pose 36 of
  // dataset/transforms_test.json came out 2 ulps off; with double all 64 golden poses are exact.
  const float ca = (float)std::cos((double)a), sa = (float)std::sin((double)a);
  f3 pos = add(mul(f3{ca, 0.0f, sa}, radius), f3{0.0f, height, 0.0f});
  f3 base_forward = normalize(f3{-ca, 0.0f, -sa});
  f3 base_up = {0.0f, 1.0f, 0.0f};
  f3 right = normalize(cross(base_forward, base_up));
  f3 new_forward = rotate_dir(b, right, base_forward);
  f3 new_up = rotate_dir(b, right, base_up);
  lookat(pos, add(pos, new_forward), new_up, view);
  perspective_zo(radians(fov_deg), aspect, zn, zf, proj);
  if (position) { position[0] = pos.x; position[1] = pos.y; position[2] = pos.z; }
  return PTGS_OK;
}

int ptgs_builder_create(ptgs_scene_builder** out) {
  if (!out) return PTGS_EINVAL;
  *out = new ptgs_scene_builder();
  return PTGS_OK;
}

void ptgs_builder_destroy(ptgs_scene_builder* b) { delete b; }

const char* ptgs_builder_last_error(const ptgs_scene_builder* b) { return b ? b->err.c_str() : "null builder"; }

// Engine::createRTBox, engine.cpp:181-335
int ptgs_builder_add_rtbox_json(ptgs_scene_builder* b, const char* path) {
  if (!b || !path) return PTGS_EINVAL;
  std::vector<uint8_t> bytes;
  if (!ptgs::read_file(path, bytes)) { b->err = std::string("cannot read ") + path; return PTGS_EIO; }
  const std::string text(bytes.begin(), bytes.end());
  JVal cfg;
  if (!ptgs::parse_json(text.data(), text.size(), cfg) || cfg.kind != JVal::OBJ) { b->err = std::string("bad JSON in ") + path; return PTGS_EIO; }
  const JVal* jpos = cfg.get("position");
  const JVal* jdim = cfg.get("dimensions");
  const JVal* jpanels = cfg.get("panels");
  if (!jpos || !jdim || !jpanels || jpos->arr.size() < 3 || jdim->arr.size() < 3) {
    b->err = "rt-box JSON needs position, dimensions and panels";
    return PTGS_EIO;
  }
  f3 pos = {(float)jpos->arr[0].num, (float)jpos->arr[1].num, (float)jpos->arr[2].num};
  f3 dim = {(float)jdim->arr[0].num, (float)jdim->arr[1].num, (float)jdim->arr[2].num};
  float w = dim.x / 2.0f, h = dim.y, d = dim.z / 2.0f;
  float yb = pos.y, yt = pos.y + h;
  ptgs_scene_builder::Object o;
  o.vertices.resize(24);
  const float P[24][3] = {
      {pos.x - w, yb, pos.z - d}, {pos.x + w, yb, pos.z - d}, {pos.x + w, yb, pos.z + d}, {pos.x - w, yb, pos.z + d},
      {pos.x - w, yt, pos.z - d}, {pos.x + w, yt, pos.z - d}, {pos.x + w, yt, pos.z + d}, {pos.x - w, yt, pos.z + d},
      {pos.x - w, yb, pos.z - d}, {pos.x + w, yb, pos.z - d}, {pos.x + w, yt, pos.z - d}, {pos.x - w, yt, pos.z - d},
      {pos.x - w, yb, pos.z + d}, {pos.x - w, yb, pos.z - d}, {pos.x - w, yt, pos.z - d}, {pos.x - w, yt, pos.z + d},
      {pos.x + w, yb, pos.z - d}, {pos.x + w, yb, pos.z + d}, {pos.x + w, yt, pos.z + d}, {pos.x + w, yt, pos.z - d},
      {pos.x - w, yb, pos.z + d}, {pos.x + w, yb, pos.z + d}, {pos.x + w, yt, pos.z + d}, {pos.x - w, yt, pos.z + d}};
  const float N[6][3] = {{0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {1, 0, 0}, {-1, 0, 0}, {0, 0, -1}};
  for (int i = 0; i < 24; ++i) {
    ptgs_vertex& vx = o.vertices[i];
    std::memset(&vx, 0, sizeof(vx));
    for (int k = 0; k < 3; ++k) {
      vx.pos[k] = P[i][k];
      vx.normal[k] = N[i / 4][k];
      vx.color[k] = 1.0f;
    }
    vx.tangent[0] = 1.0f;  // (1,0,0,0): w = 0 -> no normal map
  }
  o.indices = {0, 3, 2, 2, 1, 0, 4, 5, 6, 6, 7, 4, 8, 9, 10, 10, 11, 8,
               12, 13, 14, 14, 15, 12, 16, 17, 18, 18, 19, 16, 20, 21, 22, 22, 23, 20};
  const char* names[6] = {"floor", "ceiling", "back_wall", "left_wall", "right_wall", "front_wall"};
  for (int i = 0; i < 6; ++i) {
    const JVal* panel = jpanels->get(names[i]);
    const JVal* jm = panel ? panel->get("material") : nullptr;
    const JVal* bc = jm ? jm->get("base_color") : nullptr;
    if (!bc || bc->arr.size() < 3) { b->err = std::string("panel ") + names[i] + " lacks material.base_color"; return PTGS_EIO; }
    ptgs_material m = ptgs_default_material();
    float c0 = (float)bc->arr[0].num, c1 = (float)bc->arr[1].num, c2 = (float)bc->arr[2].num;
    m.base_color_factor[0] = c0; m.base_color_factor[1] = c1; m.base_color_factor[2] = c2; m.base_color_factor[3] = 1.0f;
    m.metallic_factor = jnum(jm->get("metallic"), 0.0f);
    m.roughness_factor = jnum(jm->get("roughness"), 1.0f);
    const JVal* jl = panel->get("light");
    float intensity = jl ? jnum(jl->get("intensity"), 0.0f) : 0.0f;
    m.emissive_factor_and_pad[0] = c0 * intensity;
    m.emissive_factor_and_pad[1] = c1 * intensity;
    m.emissive_factor_and_pad[2] = c2 * intensity;
    m.emissive_factor_and_pad[3] = 0.0f;
    m.occlusion_strength = 1.0f;
    m.albedo_texture_index = 0;
    m.pad = 0.0f;
    o.materials.push_back(m);
    o.prims.push_back({(uint32_t)(i * 6), 6u, i});
  }
  for (size_t k = 0; k < o.indices.size(); k += 3) {
    uint32_t mi = (uint32_t)(k / 6);
    const float* e = o.materials[mi].emissive_factor_and_pad;
    if (length(f3{e[0], e[1], e[2]}) < 0.00001f) continue;
    uint32_t i0 = o.indices[k], i1 = o.indices[k + 1], i2 = o.indices[k + 2];
    f3 p0 = {o.vertices[i0].pos[0], o.vertices[i0].pos[1], o.vertices[i0].pos[2]};
    f3 p1 = {o.vertices[i1].pos[0], o.vertices[i1].pos[1], o.vertices[i1].pos[2]};
    f3 p2 = {o.vertices[i2].pos[0], o.vertices[i2].pos[1], o.vertices[i2].pos[2]};
    o.etris.push_back({i0, i1, i2, mi, 0.5f * length(cross(sub(p1, p0), sub(p2, p0)))});
  }
  o.num_textures = 1;
  // the rt-box's only texture: a 1x1 (125, 125, 125, 255) sRGB default (engine.cpp:331-333)
  ptgs_scene_builder::Texture gray;
  gray.rgba = {125, 125, 125, 255};
  o.textures.push_back(gray);
  b->rtbox = o;
  b->has_rtbox = true;
  return PTGS_OK;
}

int ptgs_builder_add_object(ptgs_scene_builder* b, const ptgs_vertex* vertices, uint32_t nv, const uint32_t* indices,
                            uint32_t ni, const ptgs_primitive* prims, uint32_t np, const ptgs_material* materials,
                            uint32_t nm, const ptgs_punctual_light* lights, uint32_t nl, uint32_t num_textures) {
  if (!b || (nv && !vertices) || (ni && !indices) || (np && !prims) || (nm && !materials) || (nl && !lights))
    return PTGS_EINVAL;
  ptgs_scene_builder::Object o;
  o.vertices.assign(vertices, vertices + nv);
  o.indices.assign(indices, indices + ni);
  o.prims.assign(prims, prims + np);
  o.materials.assign(materials, materials + nm);
  o.lights.assign(lights, lights + nl);
  o.num_textures = num_textures;
  for (const ptgs_primitive& p : o.prims) {
    if (p.material_index < 0 || (uint32_t)p.material_index >= nm) { b->err = "primitive material out of range"; return PTGS_EINVAL; }
    if ((uint64_t)p.first_index + p.index_count > ni) { b->err = "primitive index range out of bounds"; return PTGS_EINVAL; }
    const float* e = o.materials[p.material_index].emissive_factor_and_pad;
    bool is_emissive = length(f3{e[0], e[1], e[2]}) > 0.001f;  // gameobject.cpp:567
    if (!is_emissive) continue;
    for (uint32_t k = 0; k + 2 < p.index_count; k += 3) {
      uint32_t i0 = o.indices[p.first_index + k], i1 = o.indices[p.first_index + k + 1], i2 = o.indices[p.first_index + k + 2];
      if (i0 >= nv || i1 >= nv || i2 >= nv) { b->err = "index out of range"; return PTGS_EINVAL; }
      f3 p0 = {o.vertices[i0].pos[0], o.vertices[i0].pos[1], o.vertices[i0].pos[2]};
      f3 p1 = {o.vertices[i1].pos[0], o.vertices[i1].pos[1], o.vertices[i1].pos[2]};
      f3 p2 = {o.vertices[i2].pos[0], o.vertices[i2].pos[1], o.vertices[i2].pos[2]};
      float area = 0.5f * length(cross(sub(p1, p0), sub(p2, p0)));
      if (area > 1e-6f) o.etris.push_back({i0, i1, i2, (uint32_t)p.material_index, area});  // :779-790
    }
  }
  b->objects.push_back(std::move(o));
  return PTGS_OK;
}

// Engine::createGlobalBindlessBuffers, engine.cpp:1658-1860
int ptgs_builder_finalize(ptgs_scene_builder* b, ptgs_scene_desc* desc, ptgs_ubo* ubo) {
  if (!b || !desc || !ubo) return PTGS_EINVAL;
  b->v.clear(); b->idx.clear(); b->meshes.clear(); b->mesh_count.clear(); b->mats.clear();
  b->ltris.clear(); b->lcdf.clear(); b->plights.clear(); b->pcdf.clear(); b->tex.clear();
  std::vector<float> tri_flux;
  // Texture pixels are emitted (desc->textures) once any object carries decoded images (glTF
  // ingest); objects added without pixel data then contribute 1x1 white placeholders.
  bool emit_tex = false;
  for (const auto& o : b->objects) emit_tex |= !o.textures.empty();
  static const uint8_t white[4] = {255, 255, 255, 255};
  // loadScene pushes the scene "sun" before any object light (engine.cpp:1193, :1225-1242)
  b->plights = b->global_lights;
  int tex_offset = 0;
  auto aggregate = [&](const ptgs_scene_builder::Object& o) {
    if (o.vertices.empty()) return;
    uint32_t voff = (uint32_t)b->v.size(), ioff = (uint32_t)b->idx.size(), moff = (uint32_t)b->mats.size();
    b->v.insert(b->v.end(), o.vertices.begin(), o.vertices.end());
    b->idx.insert(b->idx.end(), o.indices.begin(), o.indices.end());
    for (const ptgs_material& m0 : o.materials) {
      ptgs_material m = m0;
      m.albedo_texture_index += tex_offset;
      m.normal_texture_index += tex_offset;
      m.metallic_roughness_texture_index += tex_offset;
      m.emissive_texture_index += tex_offset;
      m.occlusion_texture_index += tex_offset;
      m.clearcoat_texture_index += tex_offset;
      m.clearcoat_roughness_texture_index += tex_offset;
      m.sg_id += tex_offset;
      b->mats.push_back(m);
    }
    for (const ptgs_primitive& p : o.prims) {
      b->meshes.push_back({moff + (uint32_t)p.material_index, voff, ioff + p.first_index, 0u});
      b->mesh_count.push_back(p.index_count);
    }
    for (const auto& t : o.etris) {
      b->ltris.push_back({voff + t.i0, voff + t.i1, voff + t.i2, moff + t.mat});
      const float* e = o.materials[t.mat].emissive_factor_and_pad;
      float strength = length(f3{e[0], e[1], e[2]});
      tri_flux.push_back(t.area * strength);
    }
    for (const ptgs_punctual_light& l : o.lights)
      if (l.intensity > 0.0f) b->plights.push_back(l);
    if (emit_tex) {
      for (uint32_t t = 0; t < o.num_textures; ++t) {
        ptgs_texture d{};
        if (t < o.textures.size()) {
          d.rgba8 = o.textures[t].rgba.data(); d.width = o.textures[t].w; d.height = o.textures[t].h;
          d.srgb = o.textures[t].srgb;
        } else {
          d.rgba8 = white; d.width = 1; d.height = 1; d.srgb = 1;
        }
        b->tex.push_back(d);
      }
    }
    tex_offset += (int)o.num_textures;
  };
  for (const auto& o : b->objects) aggregate(o);
  if (b->has_rtbox) aggregate(b->rtbox);

  uint32_t nlt = (uint32_t)b->ltris.size();
  float emissive_flux = 0.0f;
  if (nlt > 0) {
    for (float f : tri_flux) emissive_flux += f;
    float running = 0.0f;
    for (uint32_t i = 0; i < nlt; ++i) {
      running += tri_flux[i];
      ptgs_light_cdf e{};
      e.cumulative_probability = (emissive_flux > 0.0f) ? (running / emissive_flux) : 0.0f;
      e.triangle_index = i;
      b->lcdf.push_back(e);
    }
    b->lcdf.back().cumulative_probability = 1.0f;
  } else {
    b->ltris.push_back({0, 0, 0, 0});
    ptgs_light_cdf e{};
    e.cumulative_probability = 1.0f;
    b->lcdf.push_back(e);
  }
  float punctual_flux = 0.0f;
  if (!b->plights.empty()) {
    std::vector<float> pf;
    for (const auto& l : b->plights) {
      pf.push_back(l.type == 1 ? l.intensity * 400.0f : l.intensity * 12.566f);
      punctual_flux += pf.back();
    }
    float running = 0.0f;
    for (size_t i = 0; i < pf.size(); ++i) {
      running += pf[i];
      ptgs_punctual_cdf e{};
      e.cumulative_probability = (punctual_flux > 0.0f) ? (running / punctual_flux) : 0.0f;
      e.light_index = (uint32_t)i;
      b->pcdf.push_back(e);
    }
  } else {
    ptgs_punctual_light z{};
    b->plights.push_back(z);
    ptgs_punctual_cdf e{};
    e.cumulative_probability = 1.0f;
    b->pcdf.push_back(e);
  }
  ubo->emissive_flux = emissive_flux;
  ubo->punctual_flux = punctual_flux;
  ubo->total_flux = emissive_flux + punctual_flux;
  if (emissive_flux > 0.0f && punctual_flux > 0.0f) {
    float p = emissive_flux / ubo->total_flux;
    ubo->p_emissive = p < 0.1f ? 0.1f : (p > 0.9f ? 0.9f : p);
  }
  std::memset(desc, 0, sizeof(*desc));
  desc->vertices = b->v.data();
  desc->num_vertices = (uint32_t)b->v.size();
  desc->indices = b->idx.data();
  desc->num_indices = (uint32_t)b->idx.size();
  desc->meshes = b->meshes.data();
  desc->mesh_index_count = b->mesh_count.data();
  desc->num_meshes = (uint32_t)b->meshes.size();
  desc->materials = b->mats.data();
  desc->num_materials = (uint32_t)b->mats.size();
  desc->light_triangles = b->ltris.data();
  desc->num_light_triangles = (uint32_t)b->ltris.size();
  desc->light_cdf = b->lcdf.data();
  desc->num_light_cdf = (uint32_t)b->lcdf.size();
  desc->punctual_lights = b->plights.data();
  desc->num_punctual_lights = (uint32_t)b->plights.size();
  desc->punctual_cdf = b->pcdf.data();
  desc->num_punctual_cdf = (uint32_t)b->pcdf.size();
  desc->textures = b->tex.empty() ? nullptr : b->tex.data();
  desc->num_textures = (uint32_t)b->tex.size();
  return PTGS_OK;
}

}  // extern "C"
