// texture.h — global_textures[] (raytracing.glsl:138) for the kernels: the reference's
// textureLod(sampler2D, uv, lod) with the sampler of Image::createTextureSampler (image.cpp:124-138):
// linear mag/min filtering, linear mip blending, repeat addressing, LOD clamped to the chain.
//
// Layout (built by textures.cpp): every level of every texture packed RGBA8 (r | g<<8 | b<<16 |
// a<<24) in one texel pool; per texture GS_TEX_INFO words [w0, h0, levels, srgb, off_0..off_15];
// 512 floats of decode tables: [0..255] UNORM c/255, [256..511] sRGB -> linear (alpha is always
// UNORM). Filtering is in linear space after the per-texel decode, as Vulkan specifies for sRGB.
// The same arithmetic, in the same order, is restated in oracle/ptgs_oracle.c (or_tex_sample).
#pragma once

#include <hip/hip_runtime.h>

#include "detmath.h"
#include "textures.h"

namespace ptgs {

struct DevTextures {
  const uint32_t* texels;
  const uint32_t* info;
  const float* lut;
  uint32_t count;
};

__device__ __forceinline__ int tex_wrap(int i, int n) {
  int r = i % n;
  return r < 0 ? r + n : r;
}

__device__ __forceinline__ v4 tex_texel(const DevTextures& tx, uint32_t idx, uint32_t srgb) {
  const uint32_t p = tx.texels[idx];
  const float* rgb = tx.lut + (srgb ? 256 : 0);
  return mk4(rgb[p & 255u], rgb[(p >> 8) & 255u], rgb[(p >> 16) & 255u], tx.lut[p >> 24]);
}

// bilinear at one level, repeat addressing on the integer texel coordinates
__device__ __forceinline__ v4 tex_bilinear(const DevTextures& tx, uint32_t base, int w, int h, uint32_t srgb,
                                           float u, float v) {
  const float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
  const float fx = floorx(x), fy = floorx(y);
  const float a = x - fx, b = y - fy;
  const int ix = (int)fx, iy = (int)fy;
  const int x0 = tex_wrap(ix, w), x1 = tex_wrap(ix + 1, w);
  const int y0 = tex_wrap(iy, h), y1 = tex_wrap(iy + 1, h);
  const v4 t00 = tex_texel(tx, base + (uint32_t)(y0 * w + x0), srgb);
  const v4 t10 = tex_texel(tx, base + (uint32_t)(y0 * w + x1), srgb);
  const v4 t01 = tex_texel(tx, base + (uint32_t)(y1 * w + x0), srgb);
  const v4 t11 = tex_texel(tx, base + (uint32_t)(y1 * w + x1), srgb);
  const float ia = 1.0f - a, ib = 1.0f - b;
  return mk4((t00.x * ia + t10.x * a) * ib + (t01.x * ia + t11.x * a) * b,
             (t00.y * ia + t10.y * a) * ib + (t01.y * ia + t11.y * a) * b,
             (t00.z * ia + t10.z * a) * ib + (t01.z * ia + t11.z * a) * b,
             (t00.w * ia + t10.w * a) * ib + (t01.w * ia + t11.w * a) * b);
}

// closesthit.rchit:39-42 sampleTexture(): id < 0 (or past the table) -> vec4(1)
// Inlined (an out-of-line call measured 2456 vs 3057 Mrays/s on C3: the call ABI spills the kernel's
// live registers); the path-tracer kernels are instantiated without the texture branches for
// scenes that reference no texture (DevScene::uses_textures).
__device__ __forceinline__ v4 sample_texture(const DevTextures& tx, int id, float u, float v, float lod) {
  if (id < 0 || (uint32_t)id >= tx.count) return mk4(1.0f, 1.0f, 1.0f, 1.0f);
  const uint32_t* ti = tx.info + (uint32_t)id * PTGS_TEX_INFO;
  const uint32_t w0 = ti[0], h0 = ti[1], levels = ti[2], srgb = ti[3];
  const float lam = fmaxx(lod, 0.0f);
  const float fl = floorx(lam), delta = lam - fl;
  const uint32_t dl = (uint32_t)fminx(fl, (float)(levels - 1u));
  const uint32_t dh = dl + 1u < levels ? dl + 1u : dl;
  const int wl = (int)max(1u, w0 >> dl), hl = (int)max(1u, h0 >> dl);
  const v4 a = tex_bilinear(tx, ti[4 + dl], wl, hl, srgb, u, v);
  if (delta == 0.0f || dh == dl) return a;
  const int wh = (int)max(1u, w0 >> dh), hh = (int)max(1u, h0 >> dh);
  const v4 b = tex_bilinear(tx, ti[4 + dh], wh, hh, srgb, u, v);
  const float id_ = 1.0f - delta;
  return mk4(a.x * id_ + b.x * delta, a.y * id_ + b.y * delta, a.z * id_ + b.z * delta, a.w * id_ + b.w * delta);
}

// textureSize(global_textures[id], 0)
__device__ __forceinline__ uint32_t texture_max_dim(const DevTextures& tx, int id) {
  if (id < 0 || (uint32_t)id >= tx.count) return 1u;
  const uint32_t* ti = tx.info + (uint32_t)id * PTGS_TEX_INFO;
  return ti[0] > ti[1] ? ti[0] : ti[1];
}

}  // namespace ptgs
