// pt_shade.h — closest-hit shading, restating shaders/rt_render/closesthit.rchit:324-621
// (WITH_HITPOS = the rt_datacollect variant, which also writes payload.hit_pos / normal,
// shaders/rt_datacollect/closesthit.rchit:443-447). Textures: texture.h (sampleTexture :39-42,
// computeLOD :21-37).
#pragma once

#include "pt_device.h"

namespace ptgs {

// closesthit.rchit:21-37 computeLOD (the ray origin argument is unused there)
__device__ __forceinline__ float compute_lod(const CamParams& cp, const DevTextures& tx, v3 dir, float dist, v3 normal,
                                             int tex_id) {
  const float spread = (2.0f * tanx(cp.fov * 0.5f)) / cp.win_height;
  float footprint = dist * spread;
  const float ndv = absx(dot3(normal, -dir));
  footprint = footprint / fmaxx(ndv, 0.25f);
  float dim = 2048.0f;
  if (tex_id >= 0) dim = (float)texture_max_dim(tx, tex_id);
  const float raw = log2x(footprint * dim);
  const float bias = (dim > 2048.0f) ? 0.0f : -0.5f;
  return fmaxx(raw * 0.7f + bias, 0.0f);
}

// The NEE shadow ray is not traced here: it is returned in q (q.flags == 0: none) and traced by the
// caller after shading (resolve_shadow, pt_device.h), which adds its contribution to p.color.
template <bool WITH_HITPOS, bool TEX>
__device__ void closest_hit(const ShadeCtx& c, Payload& p, const Ray& ray, const Hit& hit, ShadowQuery& q) {
  const DevScene& sc = *c.sc;
  const CamParams& cp = *c.cp;

  // one 16-B fetch by gid replaces the triangle record -> MeshInfo -> indices chain (three dependent
  // round trips): the same vertex / material indices, precomputed at upload
  const uint4 hr = sc.hitrec[hit.gid];
  const ptgs_material& mat = sc.materials[hr.w];
  const ptgs_vertex& v0 = sc.vertices[hr.x];
  const ptgs_vertex& v1 = sc.vertices[hr.y];
  const ptgs_vertex& v2 = sc.vertices[hr.z];

  // :336-346
  float bx = (1.0f - hit.u) - hit.v, by = hit.u, bz = hit.v;
  v3 hit_pos = ray.o + ray.d * hit.t;
  const float tc_u = (v0.tex_coord[0] * bx + v1.tex_coord[0] * by) + v2.tex_coord[0] * bz;
  const float tc_v = (v0.tex_coord[1] * bx + v1.tex_coord[1] * by) + v2.tex_coord[1] * bz;
  v3 vcol = (ld3(v0.color) * bx + ld3(v1.color) * by) + ld3(v2.color) * bz;
  v3 nobj = (ld3(v0.normal) * bx + ld3(v1.normal) * by) + ld3(v2.normal) * bz;
  v3 tobj = (ld3(v0.tangent) * bx + ld3(v1.tangent) * by) + ld3(v2.tangent) * bz;
  float tw = (v0.tangent[3] * bx + v1.tangent[3] * by) + v2.tangent[3] * bz;
  // instance transforms are identity (transforms are baked into vertices, engine.cpp:1294-1338)
  v3 n_geo = safe_normalize(nobj);
  v3 t_geo = safe_normalize(tobj);
  t_geo = safe_normalize(t_geo - n_geo * dot3(t_geo, n_geo));

  v3 V = -ray.d;
  v3 n_geo_orig = n_geo;
  if (dot3(n_geo, V) < 0.0f) n_geo = -n_geo;
  v3 N = n_geo;
  v3 T = t_geo;
  bool tangent_valid = (absx(tw) > 0.001f) && (length3(T) > 0.001f);
  if (!tangent_valid) {
    v3 up = sel3(absx(N.y) < 0.999f, mk3(0.f, 1.f, 0.f), mk3(1.f, 0.f, 0.f));
    T = safe_normalize(cross3(up, N));
  }
  // :358-385 tangent frame + normal map
  if (TEX && absx(tw) > 0.0001f && mat.normal_texture_index > 0) {
    const float handed = (tw < 0.0f) ? -1.0f : 1.0f;
    const v3 B = safe_normalize(cross3(N, T)) * handed;
    float tex_lod = 0.0f;
    if (cp.use_lod > 0.0f) {
      if (p.last_pdf <= 0.0f) {
        if (mat.albedo_texture_index > 0)
          tex_lod = compute_lod(cp, sc.tex, ray.d, hit.t, n_geo, mat.albedo_texture_index);
      } else {
        tex_lod = clampf(mat.roughness_factor * 5.0f + log2x(hit.t * 0.1f + 1.0f), 0.0f, 8.0f);
      }
    }
    const float* un = mat.uv_normal;  // (uv_normal * vec4(tc, 0, 1)).xy
    const float nu = ((un[0] * tc_u + un[4] * tc_v) + un[8] * 0.0f) + un[12];
    const float nv = ((un[1] * tc_u + un[5] * tc_v) + un[9] * 0.0f) + un[13];
    const v4 mv = sample_texture(sc.tex, mat.normal_texture_index, nu, nv, tex_lod);
    v3 nm = mk3(mv.x * 2.0f - 1.0f, mv.y * 2.0f - 1.0f, mv.z * 2.0f - 1.0f);
    nm.x = nm.x * cp.lod_factor;
    nm.y = nm.y * cp.lod_factor;
    nm = normalize3(nm);
    N = safe_normalize((T * nm.x + B * nm.y) + N * nm.z);
  }

  v3 albedo, f0;
  float roughness, metallic;
  int32_t sg_bits;
  {
    union { float f; int32_t i; } pun; pun.f = mat.use_specular_glossiness_workflow;
    sg_bits = pun.i;  // float stored, int read
  }
  v3 bcs = mk3(1.0f);  // :393-394 base colour sample
  if (TEX && mat.albedo_texture_index > 0) {
    const v4 b4 = sample_texture(sc.tex, mat.albedo_texture_index, tc_u, tc_v, 0.0f);
    bcs = mk3(b4.x, b4.y, b4.z);
  }
  v3 bcf = mk3(mat.base_color_factor[0], mat.base_color_factor[1], mat.base_color_factor[2]);
  if ((float)sg_bits > 0.5f) {
    albedo = (bcf * vcol) * bcs;
    v3 spec_col = ld3(mat.specular_color_factor);
    float gloss = mat.roughness_factor;
    if (TEX && mat.sg_id > 0) {
      const v4 sg4 = sample_texture(sc.tex, mat.sg_id, tc_u, tc_v, 0.0f);
      spec_col = spec_col * mk3(sg4.x, sg4.y, sg4.z);
      gloss = gloss * sg4.w;
    }
    f0 = spec_col;
    roughness = sqrtx(fmaxx(1.0f - gloss, 0.04f));
    metallic = 0.0f;
  } else {
    albedo = (bcf * vcol) * bcs;
    metallic = mat.metallic_factor;
    roughness = mat.roughness_factor;
    if (TEX && mat.metallic_roughness_texture_index > 0) {
      const v4 mr = sample_texture(sc.tex, mat.metallic_roughness_texture_index, tc_u, tc_v, 0.0f);
      metallic = metallic * mr.z;
      roughness = roughness * mr.y;
    }
    f0 = mix3(mk3(0.04f), albedo, metallic);
    albedo = albedo * (1.0f - metallic);
  }
  float clearcoat = mat.clearcoat_factor;
  float cc_rough = mat.clearcoat_roughness_factor;
  if (TEX && clearcoat > 0.0f && mat.clearcoat_texture_index > 0)
    clearcoat = clearcoat * sample_texture(sc.tex, mat.clearcoat_texture_index, tc_u, tc_v, 0.0f).x;
  if (TEX && clearcoat > 0.0f && mat.clearcoat_roughness_texture_index > 0)
    cc_rough = cc_rough * sample_texture(sc.tex, mat.clearcoat_roughness_texture_index, tc_u, tc_v, 0.0f).x;
  // (:432-434 occlusion is fetched but never used by the reference: not restated)
  v3 emissive = ld3(mat.emissive_factor_and_pad);
  if (TEX && length3(emissive) > 0.0f && mat.emissive_texture_index > 0) {  // :437-440
    const float* ue = mat.uv_emissive;
    const float eu = ((ue[0] * tc_u + ue[4] * tc_v) + ue[8] * 0.0f) + ue[12];
    const float ev = ((ue[1] * tc_u + ue[5] * tc_v) + ue[9] * 0.0f) + ue[13];
    const v4 e4 = sample_texture(sc.tex, mat.emissive_texture_index, eu, ev, 0.0f);
    emissive = emissive * mk3(e4.x, e4.y, e4.z);
  }
  float transmission = mat.transmission_factor;

  if (WITH_HITPOS) {
    p.hit_pos = hit_pos;
    p.normal = N;
  }

  // :444-468
  v3 lo = mk3(0.0f);
  v3 le = emissive;
  float es = length3(emissive);
  bool use_nee = (transmission == 0.0f) && (roughness > 0.001f);
  if (p.hit_flag > 3.0f) use_nee = false;
  if (es > 0.0f) {
    if (p.last_pdf <= 0.0f || !use_nee) {
      lo = lo + le;
    } else if (es < 0.001f) {
      p.color = mk3(0.0f);
      return;
    } else {
      float pdf_bsdf = p.last_pdf;
      float es_cpu = length3(ld3(mat.emissive_factor_and_pad));
      v3 l_to_cam = -ray.d;
      float ldn = absx(dot3(N, l_to_cam));
      float dist_sq = hit.t * hit.t;
      float pdf_nee = 0.0f;
      if (cp.emissive_flux > 0.0f) pdf_nee = (es_cpu / cp.emissive_flux) * (dist_sq / fmaxx(ldn, 0.001f));
      float prob_nee = (cp.punctual_flux > 0.0f) ? cp.p_emissive : 1.0f;
      pdf_nee = pdf_nee * prob_nee;
      float mis = (pdf_bsdf * pdf_bsdf) / (pdf_bsdf * pdf_bsdf + pdf_nee * pdf_nee);
      lo = lo + le * mis;
    }
  }

  // :470-494 (with both light kinds: lc = (0 + contribution) * (1 / p_select), lo += lc)
  bool has_emissive = cp.emissive_flux > 0.0f;
  bool has_punctual = cp.punctual_flux > 0.0f;
  bool sg = (float)sg_bits > 0.0f;
  if (has_emissive && has_punctual) {
    float p_punctual = 1.0f - cp.p_emissive;
    if (blue_noise_dim(p, 10) < cp.p_emissive) {
      if (use_nee) {
        sample_emissive(c, p, sg, hit_pos, N, n_geo, V, albedo, roughness, metallic, f0, transmission, q);
        q.scale = 1.0f / cp.p_emissive;
        q.flags |= SQ_MIXED;
      }
    } else {
      sample_punctual(c, p, hit_pos, N, n_geo, V, albedo, roughness, f0, transmission, q);
      q.scale = 1.0f / p_punctual;
      q.flags |= SQ_MIXED;
    }
  } else if (has_emissive && use_nee) {
    sample_emissive(c, p, sg, hit_pos, N, n_geo, V, albedo, roughness, metallic, f0, transmission, q);
  } else if (has_punctual) {
    sample_punctual(c, p, hit_pos, N, n_geo, V, albedo, roughness, f0, transmission, q);
  }
  p.color = lo;

  // :503-531 glass
  if (transmission > 0.0f) {
    p.hit_flag = 2.0f;
    bool entering = dot3(n_geo_orig, V) > 0.0f;
    v3 n_refr = sel3(entering, n_geo_orig, -n_geo_orig);
    p.next_o = hit_pos - n_refr * 0.001f;
    v3 fv = f_schlick(absx(dot3(n_geo_orig, V)), f0);
    float prob_reflect = fmaxx(fmaxx(fv.x, fv.y), fv.z);
    if (blue_noise_dim(p, 11) < prob_reflect) {
      p.next_o = hit_pos + n_refr * 0.001f;
      p.next_d = reflect3(-V, n_refr);
      p.weight = mk3(1.0f);
    } else {
      const float ior = 1.01f;
      float eta = entering ? (1.0f / ior) : ior;
      v3 rd = refract3(-V, n_refr, eta);
      if (length3(rd) > 0.0f) {
        p.next_d = rd;
        p.weight = albedo;
      } else {
        p.next_o = hit_pos + n_geo * 0.001f;
        p.next_d = reflect3(-V, N);
        p.weight = mk3(1.0f);
      }
    }
    p.last_pdf = 0.0f;
    return;
  }

  // :534-620 opaque
  p.hit_flag = 1.0f;
  p.next_o = hit_pos + n_geo * 0.001f;
  float ndv = fmaxx(dot3(N, V), 0.0f);
  float cc_prob = 0.0f;
  v3 f_cc_view = mk3(0.0f);
  if (clearcoat > 0.0f) {
    f_cc_view = f_schlick(ndv, mk3(0.04f)) * clearcoat;
    cc_prob = clampf(fmaxx(f_cc_view.x, fmaxx(f_cc_view.y, f_cc_view.z)), 0.0f, 1.0f);
  }
  if (clearcoat > 0.0f && blue_noise_dim(p, 12) < cc_prob) {
    v3 hcc = sample_ggx(p, N, cc_rough);
    v3 lcc = reflect3(-V, hcc);
    float ndl = fmaxx(dot3(N, lcc), 0.0f);
    float ndh = fmaxx(dot3(N, hcc), 0.0f);
    float vdh = fmaxx(dot3(V, hcc), 0.0f);
    if (dot3(lcc, n_geo) <= 0.0f) {
      p.weight = mk3(0.0f);
      p.last_pdf = 0.0f;
    } else {
      p.next_d = lcc;
      v3 f = f_schlick(vdh, mk3(0.04f)) * clearcoat;
      float vis = v_smith(ndv, ndl, cc_rough);
      v3 sw = ((f * vis) * 4.0f) * ndl * (vdh / fmaxx(ndh, 0.0001f));
      float pdf_cc = pdf_ggx(N, V, lcc, cc_rough);
      float psb = mixf(0.04f, 1.0f, metallic);
      psb = mixf(psb, 1.0f, pow5(1.0f - ndv));
      psb = clampf(psb, 0.05f, 0.95f);
      float pdb = 1.0f - psb;
      float pdf_sb = pdf_ggx(N, V, lcc, roughness);
      float pdf_db = pdf_lambert(N, lcc);
      float pdf_base = pdf_sb * psb + pdf_db * pdb;
      p.last_pdf = pdf_cc * cc_prob + pdf_base * (1.0f - cc_prob);
      p.weight = sw * (1.0f / cc_prob);
    }
  } else {
    v3 tf = mk3(1.0f) - f_cc_view;
    float selw = 1.0f / (1.0f - cc_prob);
    v3 ea = tf * selw;
    float ps = mixf(0.04f, 1.0f, metallic);
    ps = mixf(ps, 1.0f, pow5(1.0f - ndv));
    ps = clampf(ps, 0.05f, 0.95f);
    float pd = 1.0f - ps;
    if (blue_noise_dim(p, 13) < ps) {
      v3 h = sample_ggx(p, N, roughness);
      v3 l = reflect3(-V, h);
      float ndl = fmaxx(dot3(N, l), 0.0f);
      float ndh = fmaxx(dot3(N, h), 0.0f);
      float vdh = fmaxx(dot3(V, h), 0.0f);
      if (dot3(l, n_geo) <= 0.0f) {
        p.weight = mk3(0.0f);
        p.last_pdf = 0.0f;
      } else {
        p.next_d = l;
        v3 f = f_schlick(fmaxx(dot3(h, V), 0.0f), f0);
        float vis = v_smith(ndv, ndl, roughness);
        v3 sw = ((f * vis) * 4.0f) * ndl * (vdh / fmaxx(ndh, 0.0001f));
        float pdf_s = pdf_ggx(N, V, l, roughness);
        float pdf_d = pdf_lambert(N, l);
        p.last_pdf = (pdf_s * ps + pdf_d * pd) * (1.0f - cc_prob);
        p.weight = (sw * (1.0f / ps)) * ea;
      }
    } else {
      v3 l = sample_cosine(p, N);
      if (dot3(l, n_geo) <= 0.0f) {
        p.weight = mk3(0.0f);
        p.last_pdf = 0.0f;
      } else {
        p.next_d = l;
        p.weight = (albedo * (1.0f / (1.0f - ps))) * ea;
        float pdf_s = pdf_ggx(N, V, l, roughness);
        float pdf_d = pdf_lambert(N, l);
        p.last_pdf = (pdf_s * ps + pdf_d * pd) * (1.0f - cc_prob);
      }
    }
  }
}

// miss.rmiss:9-14 (rt_datacollect/miss.rmiss also resets hit_pos / normal)
template <bool WITH_HITPOS>
__device__ __forceinline__ void miss(const CamParams& cp, Payload& p) {
  p.hit_flag = -1.0f;
  p.color = mk3(cp.ambient[0], cp.ambient[1], cp.ambient[2]) * 2.0f;
  p.weight = mk3(1.0f);
  if (WITH_HITPOS) {
    p.hit_pos = mk3(0.0f);
    p.normal = mk3(0.0f, 1.0f, 0.0f);
  }
}

}  // namespace ptgs
