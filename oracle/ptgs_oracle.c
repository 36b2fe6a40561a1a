/*
 * ptgs_oracle.c — CPU ORACLE (test infrastructure only; never linked into the product).
 *
 * A plain-C restatement of the reference's hot path, used by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker. Nothing in pathtracer_gaussiansplatting_amd/ may
 * import or call it.
 *
 * Reference files restated (all paths relative to /root/reference):
 *   ray-gen          shaders/rt_render/raygen_camera.rgen:11-88            -> or_trace_pixel()
 *   closest hit      shaders/rt_render/closesthit.rchit:16-621             -> or_closest_hit()
 *   miss / shadow    shaders/rt_render/miss.rmiss:9-14, shadow.rmiss:9-11  -> or_miss(), or_any_hit()
 *   any hit          shaders/rt_render/alpha.rahit:14-61                    -> or_anyhit_accept()
 *   RNG              shaders/rt_render/raytracing.glsl:141-146              -> or_rnd()
 *   torus ray-gen    shaders/rt_datacollect/raygen.rgen:31-141             -> or_trace_torus()
 *   point raster     shaders/pointcloud/pointcloud.vert:44-89, .frag:1-11  -> oracle_splat_points()
 *   camera           Vulkan_Engine/camera.cpp:195-228 (glm 0.9.9 formulas) -> oracle_camera_toroidal()
 *   3DGS forward     Kerbl et al. 2023 (absent from the reference: parity unpinned)
 *
 * Pinning: the camera restatement is checked against the reference's only golden vectors,
 * dataset/transforms_{train,test}.json (tests/test_oracle_golden.py). The path tracer and the
 * rasterizers have no golden outputs in the reference (no image/PLY goldens; the Vulkan path
 * cannot be built here) — see DESIGN.md "parity".
 *
 * Arithmetic contract (shared with the HIP kernels, restated independently here): IEEE f32
 * add/sub/mul/div/sqrt, no FMA contraction (-ffp-contract=off), fixed evaluation order of the GLSL
 * built-ins, and the polynomial sin/cos/exp2/log2 below. Ray/triangle intersection is
 * Moller-Trumbore with the closest-hit tie broken towards the lower triangle id, which makes the
 * hit independent of the acceleration structure (this file uses its own SAH BVH2).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ptgs/ptgs.h"

#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------ */
/* math                                                                                        */
/* ------------------------------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;
static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 S(float s) { return V(s, s, s); }
static inline v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mulv(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 mul(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 divs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static inline v3 divv(v3 a, v3 b) { return V(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline v3 neg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline v3 rsub(float s, v3 a) { return V(s - a.x, s - a.y, s - a.z); }
static inline float mn(float a, float b) { return b < a ? b : a; }
static inline float mx(float a, float b) { return a < b ? b : a; }
static inline float clampf_(float x, float lo, float hi) { return mn(mx(x, lo), hi); }
static inline float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) { return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static inline float len(v3 v) { return sqrtf(dot(v, v)); }
static inline v3 nrm(v3 v) { return divs(v, len(v)); }
static inline float fract_(float x) { return x - floorf(x); }
static inline float mixf_(float x, float y, float a) { return x * (1.0f - a) + y * a; }
static inline v3 mix3_(v3 x, v3 y, float a) { return V(mixf_(x.x, y.x, a), mixf_(x.y, y.y, a), mixf_(x.z, y.z, a)); }
static inline float p5(float x) { float x2 = x * x; return (x2 * x2) * x; }
static inline float p4(float x) { float x2 = x * x; return x2 * x2; }
static inline v3 ld3(const float* p) { return V(p[0], p[1], p[2]); }
static inline v3 reflect_(v3 i, v3 n) { float d = 2.0f * dot(n, i); return sub(i, mul(n, d)); }
static inline v3 refract_(v3 i, v3 n, float eta) {
    float ni = dot(n, i);
    float k = 1.0f - eta * eta * (1.0f - ni * ni);
    if (k < 0.0f) return S(0.0f);
    return sub(mul(i, eta), mul(n, eta * ni + sqrtf(k)));
}

static inline float p2i(int n) { union { uint32_t u; float f; } c; c.u = (uint32_t)(n + 127) << 23; return c.f; }

/* sin/cos: Cody-Waite by pi/2 + Cephes sinf/cosf polynomials */
static void or_sincos(float x, float* s, float* c) {
    float k = floorf(x * 0.636619772367581343f + 0.5f);
    int q = (int)k;
    float r = x - k * 1.5703125f;
    r = r - k * 4.837512969970703125e-4f;
    r = r - k * 7.54978995489188216e-8f;
    float z = r * r;
    float sp = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
    float cp = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z
               - 0.5f * z + 1.0f;
    switch (q & 3) {
        case 0: *s = sp; *c = cp; break;
        case 1: *s = cp; *c = -sp; break;
        case 2: *s = -sp; *c = -cp; break;
        default: *s = -cp; *c = sp; break;
    }
}

static float or_exp2(float x) {
    if (x < -126.0f) return 0.0f;
    if (x > 127.99f) x = 127.99f;
    float n = floorf(x + 0.5f);
    float f = x - n;
    float p = 1.535336188319500e-4f;
    p = p * f + 1.339887440266574e-3f;
    p = p * f + 9.618437357674640e-3f;
    p = p * f + 5.550332471162809e-2f;
    p = p * f + 2.402264791363012e-1f;
    p = p * f + 6.931472028550421e-1f;
    p = p * f + 1.0f;
    int ni = (int)n;
    if (ni > 127) { p = p * 2.0f; ni -= 1; }
    return p * p2i(ni);
}
static float or_exp(float x) { return or_exp2(x * 1.44269504088896341f); }

static float or_log2(float x) {
    if (!(x > 0.0f)) return -1.0e30f;
    union { float f; uint32_t u; } c; c.f = x;
    int e = (int)((c.u >> 23) & 0xffu) - 127;
    if (e == -127) { c.f = x * 8388608.0f; e = (int)((c.u >> 23) & 0xffu) - 127 - 23; }
    c.u = (c.u & 0x007fffffu) | 0x3f800000u;
    float m = c.f;
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
    float s = (m - 1.0f) / (m + 1.0f);
    float s2 = s * s;
    float p = 0.2222222222f;
    p = p * s2 + 0.2857142857f;
    p = p * s2 + 0.4f;
    p = p * s2 + 0.6666666667f;
    p = p * s2 + 2.0f;
    float ln = s * p;
    return (float)e + ln * 1.44269504088896341f;
}
static float or_pow(float x, float y) { return or_exp2(y * or_log2(x)); }

/* column-major mat4 * vec4, GLSL order */
static void mv(const float* m, const float* v, float* o) {
    for (int r = 0; r < 4; ++r) o[r] = ((m[r] * v[0] + m[4 + r] * v[1]) + m[8 + r] * v[2]) + m[12 + r] * v[3];
}
static void mm(const float* a, const float* b, float* o) {
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            o[c * 4 + r] = ((a[r] * b[c * 4] + a[4 + r] * b[c * 4 + 1]) + a[8 + r] * b[c * 4 + 2]) + a[12 + r] * b[c * 4 + 3];
}

/* inverse in double, Gauss-Jordan with partial pivoting, rounded once */
int oracle_mat4_inverse(const float* m, float* out) {
    double a[4][8];
    for (int r = 0; r < 4; ++r) {
        for (int c = 0; c < 4; ++c) a[r][c] = (double)m[c * 4 + r];
        for (int c = 0; c < 4; ++c) a[r][4 + c] = (r == c) ? 1.0 : 0.0;
    }
    for (int col = 0; col < 4; ++col) {
        int piv = col;
        double best = fabs(a[col][col]);
        for (int r = col + 1; r < 4; ++r) { double v = fabs(a[r][col]); if (v > best) { best = v; piv = r; } }
        if (best == 0.0) return -1;
        if (piv != col) for (int c = 0; c < 8; ++c) { double t = a[col][c]; a[col][c] = a[piv][c]; a[piv][c] = t; }
        double inv = 1.0 / a[col][col];
        for (int c = 0; c < 8; ++c) a[col][c] *= inv;
        for (int r = 0; r < 4; ++r) {
            if (r == col) continue;
            double f = a[r][col];
            if (f == 0.0) continue;
            for (int c = 0; c < 8; ++c) a[r][c] -= f * a[col][c];
        }
    }
    for (int r = 0; r < 4; ++r) for (int c = 0; c < 4; ++c) out[c * 4 + r] = (float)a[r][4 + c];
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* camera (camera.cpp:195-228; glm 0.9.9: normalize = v * (1/sqrt(dot)), perspective RH_ZO)     */
/* ------------------------------------------------------------------------------------------ */
static v3 g_norm(v3 v) { return mul(v, 1.0f / sqrtf(dot(v, v))); }
static v3 g_cross(v3 a, v3 b) { return V(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }

static void g_lookat(v3 eye, v3 center, v3 up, float* m) {
    v3 f = g_norm(sub(center, eye));
    v3 s = g_norm(g_cross(f, up));
    v3 u = g_cross(s, f);
    for (int k = 0; k < 16; ++k) m[k] = (k % 5 == 0) ? 1.0f : 0.0f;
    m[0] = s.x; m[4] = s.y; m[8] = s.z;
    m[1] = u.x; m[5] = u.y; m[9] = u.z;
    m[2] = -f.x; m[6] = -f.y; m[10] = -f.z;
    m[12] = -dot(s, eye); m[13] = -dot(u, eye); m[14] = dot(f, eye);
}

static v3 g_rotate(float angle, v3 axis_in, v3 v) {
    float c = cosf(angle), s = sinf(angle);
    v3 a = g_norm(axis_in);
    v3 t = mul(a, 1.0f - c);
    float R00 = c + t.x * a.x, R01 = t.x * a.y + s * a.z, R02 = t.x * a.z - s * a.y;
    float R10 = t.y * a.x - s * a.z, R11 = c + t.y * a.y, R12 = t.y * a.z + s * a.x;
    float R20 = t.z * a.x + s * a.y, R21 = t.z * a.y - s * a.x, R22 = c + t.z * a.z;
    return V((R00 * v.x + R10 * v.y) + R20 * v.z, (R01 * v.x + R11 * v.y) + R21 * v.z, (R02 * v.x + R12 * v.y) + R22 * v.z);
}

void oracle_camera_toroidal(float alpha_deg, float beta_deg, float radius, float height, float fov_deg,
                            float aspect, float zn, float zf, float* view, float* proj, float* pos_out) {
    float al = alpha_deg - 360.0f * floorf(alpha_deg / 360.0f);
    if (al < 0.0f) al += 360.0f;
    float be = beta_deg - 360.0f * floorf(beta_deg / 360.0f);
    if (be < 0.0f) be += 360.0f;
    const float D2R = 0.01745329251994329576923690768489f;
    float a = al * D2R, b = be * D2R;
    /* camera.cpp:205,208: unqualified cos / sin of a float resolve to the double ::cos / ::sin */
    const float ca = (float)cos((double)a), sa = (float)sin((double)a);
    v3 pos = add(mul(V(ca, 0.0f, sa), radius), V(0.0f, height, 0.0f));
    v3 fwd = g_norm(V(-ca, 0.0f, -sa));
    v3 up = V(0.0f, 1.0f, 0.0f);
    v3 right = g_norm(g_cross(fwd, up));
    v3 nf = g_rotate(b, right, fwd);
    v3 nu = g_rotate(b, right, up);
    g_lookat(pos, add(pos, nf), nu, view);
    float t = tanf((fov_deg * D2R) / 2.0f);
    for (int k = 0; k < 16; ++k) proj[k] = 0.0f;
    proj[0] = 1.0f / (aspect * t);
    proj[5] = -(1.0f / t);
    proj[10] = zf / (zn - zf);
    proj[11] = -1.0f;
    proj[14] = -(zf * zn) / (zf - zn);
    if (pos_out) { pos_out[0] = pos.x; pos_out[1] = pos.y; pos_out[2] = pos.z; }
}

/* ------------------------------------------------------------------------------------------ */
/* scene + BVH (oracle's own: binned SAH, median split on degenerate centroids, leaves <= 4)      */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    float lo[3], hi[3];
    int left, right;   /* children (node indices) or -1 */
    int first, count;  /* leaf range in tri order */
} ONode;

typedef struct {
    v3 v0, e1, e2;
    uint32_t mesh, prim, gid, flags;
} OTri;

typedef struct {
    const ptgs_scene_desc* d;
    OTri* tris;
    uint32_t ntris;
    ONode* nodes;
    int nnodes, cap;
    int has_transparent;
    const float* bn;
    int bn_size;
    /* global_textures[]: all levels packed RGBA8 (r | g<<8 | b<<16 | a<<24); 20 info words per texture
     * (w0, h0, levels, srgb, level offsets); decode tables [0..255] UNORM, [256..511] sRGB */
    uint32_t* tex_texels;
    uint32_t* tex_info;
    float tex_lut[512];
    uint32_t num_tex;
} OScene;

/* ------------------------------------------------------------------------------------------ */
/* textures: Image::createTextureImage/generateMipmaps (image.cpp:35, :203-290) and the sampler of */
/* image.cpp:124-138 (linear/linear/linear-mip, repeat), closesthit.rchit:39-42 sampleTexture      */
/* ------------------------------------------------------------------------------------------ */
#define OR_TEX_INFO 20
#define OR_TEX_MAX_LEVELS 16

static float or_srgb_dec(float c) { return c <= 0.04045f ? c / 12.92f : powf((c + 0.055f) / 1.055f, 2.4f); }
static float or_srgb_enc(float c) { return c <= 0.0031308f ? c * 12.92f : 1.055f * powf(c, 1.0f / 2.4f) - 0.055f; }
static uint32_t or_u8(float c) {
    float v = floorf(c * 255.0f + 0.5f);
    if (!(v > 0.0f)) return 0u;
    if (v > 255.0f) return 255u;
    return (uint32_t)v;
}
static int or_clampi(int i, int lo, int hi) { return i < lo ? lo : (i > hi ? hi : i); }

/* mip level l = linear blit of level l-1 onto max(1, w/2) x max(1, h/2): bilinear, clamp-to-edge,
 * in linear space (sRGB decoded, filtered, re-encoded and rounded; alpha linear) */
static int or_build_textures(OScene* s, const ptgs_texture* tex, uint32_t count) {
    for (int i = 0; i < 256; ++i) {
        s->tex_lut[i] = (float)i / 255.0f;
        s->tex_lut[256 + i] = or_srgb_dec((float)i / 255.0f);
    }
    s->num_tex = count;
    s->tex_info = (uint32_t*)calloc((size_t)(count ? count : 1) * OR_TEX_INFO, 4);
    size_t total = 0;
    for (uint32_t t = 0; t < count; ++t) {
        uint32_t w = tex[t].width, h = tex[t].height;
        uint32_t big = w > h ? w : h, levels = 1;
        while ((big >> levels) > 0u) ++levels;
        if (levels > OR_TEX_MAX_LEVELS) levels = OR_TEX_MAX_LEVELS;
        for (uint32_t l = 0; l < levels; ++l) {
            total += (size_t)w * h;
            w = w > 1 ? w / 2 : 1;
            h = h > 1 ? h / 2 : 1;
        }
    }
    s->tex_texels = (uint32_t*)malloc((total ? total : 1) * 4);
    size_t at = 0;
    for (uint32_t t = 0; t < count; ++t) {
        const ptgs_texture* T = &tex[t];
        uint32_t* info = s->tex_info + (size_t)t * OR_TEX_INFO;
        uint32_t big = T->width > T->height ? T->width : T->height, levels = 1;
        while ((big >> levels) > 0u) ++levels;
        if (levels > OR_TEX_MAX_LEVELS) levels = OR_TEX_MAX_LEVELS;
        info[0] = T->width; info[1] = T->height; info[2] = levels; info[3] = T->srgb ? 1u : 0u;
        info[4] = (uint32_t)at;
        memcpy(s->tex_texels + at, T->rgba8, (size_t)T->width * T->height * 4);
        at += (size_t)T->width * T->height;
        const float* dec = s->tex_lut + (T->srgb ? 256 : 0);
        uint32_t sw = T->width, sh = T->height;
        for (uint32_t l = 1; l < levels; ++l) {
            uint32_t dw = sw > 1 ? sw / 2 : 1, dh = sh > 1 ? sh / 2 : 1;
            const uint32_t* src = s->tex_texels + info[4 + l - 1];
            uint32_t* dst = s->tex_texels + at;
            info[4 + l] = (uint32_t)at;
            at += (size_t)dw * dh;
            float sxs = (float)sw / (float)dw, sys = (float)sh / (float)dh;
            for (uint32_t y = 0; y < dh; ++y) {
                float fy = ((float)y + 0.5f) * sys - 0.5f, fy0 = floorf(fy), b = fy - fy0;
                int iy = (int)fy0;
                int y0 = or_clampi(iy, 0, (int)sh - 1), y1 = or_clampi(iy + 1, 0, (int)sh - 1);
                for (uint32_t x = 0; x < dw; ++x) {
                    float fx = ((float)x + 0.5f) * sxs - 0.5f, fx0 = floorf(fx), a = fx - fx0;
                    int ix = (int)fx0;
                    int x0 = or_clampi(ix, 0, (int)sw - 1), x1 = or_clampi(ix + 1, 0, (int)sw - 1);
                    uint32_t q00 = src[y0 * sw + x0], q10 = src[y0 * sw + x1];
                    uint32_t q01 = src[y1 * sw + x0], q11 = src[y1 * sw + x1];
                    uint32_t out = 0;
                    for (int ch = 0; ch < 4; ++ch) {
                        const float* dd = ch == 3 ? s->tex_lut : dec;
                        int sh8 = 8 * ch;
                        float c00 = dd[(q00 >> sh8) & 255u], c10 = dd[(q10 >> sh8) & 255u];
                        float c01 = dd[(q01 >> sh8) & 255u], c11 = dd[(q11 >> sh8) & 255u];
                        float cf = (c00 * (1.0f - a) + c10 * a) * (1.0f - b) + (c01 * (1.0f - a) + c11 * a) * b;
                        float e = (T->srgb && ch < 3) ? or_srgb_enc(cf) : cf;
                        out |= or_u8(e) << sh8;
                    }
                    dst[y * dw + x] = out;
                }
            }
            sw = dw; sh = dh;
        }
    }
    return 0;
}

static int or_wrap(int i, int n) { int r = i % n; return r < 0 ? r + n : r; }

static void or_texel(const OScene* s, uint32_t idx, uint32_t srgb, float* o) {
    uint32_t q = s->tex_texels[idx];
    const float* rgb = s->tex_lut + (srgb ? 256 : 0);
    o[0] = rgb[q & 255u]; o[1] = rgb[(q >> 8) & 255u]; o[2] = rgb[(q >> 16) & 255u]; o[3] = s->tex_lut[q >> 24];
}

static void or_bilinear(const OScene* s, uint32_t base, int w, int h, uint32_t srgb, float u, float v, float* o) {
    float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    float fx = floorf(x), fy = floorf(y), a = x - fx, b = y - fy;
    int ix = (int)fx, iy = (int)fy;
    int x0 = or_wrap(ix, w), x1 = or_wrap(ix + 1, w), y0 = or_wrap(iy, h), y1 = or_wrap(iy + 1, h);
    float t00[4], t10[4], t01[4], t11[4];
    or_texel(s, base + (uint32_t)(y0 * w + x0), srgb, t00);
    or_texel(s, base + (uint32_t)(y0 * w + x1), srgb, t10);
    or_texel(s, base + (uint32_t)(y1 * w + x0), srgb, t01);
    or_texel(s, base + (uint32_t)(y1 * w + x1), srgb, t11);
    float ia = 1.0f - a, ib = 1.0f - b;
    for (int k = 0; k < 4; ++k) o[k] = (t00[k] * ia + t10[k] * a) * ib + (t01[k] * ia + t11[k] * a) * b;
}

/* textureLod(global_textures[id], uv, lod); id < 0 (or past the table) -> vec4(1) */
static void or_tex_sample(const OScene* s, int id, float u, float v, float lod, float* o) {
    if (id < 0 || (uint32_t)id >= s->num_tex) { o[0] = o[1] = o[2] = o[3] = 1.0f; return; }
    const uint32_t* ti = s->tex_info + (uint32_t)id * OR_TEX_INFO;
    uint32_t w0 = ti[0], h0 = ti[1], levels = ti[2], srgb = ti[3];
    float lam = mx(lod, 0.0f), fl = floorf(lam), delta = lam - fl;
    uint32_t dl = (uint32_t)mn(fl, (float)(levels - 1u));
    uint32_t dh = dl + 1u < levels ? dl + 1u : dl;
    uint32_t wl = w0 >> dl, hl = h0 >> dl;
    or_bilinear(s, ti[4 + dl], (int)(wl ? wl : 1), (int)(hl ? hl : 1), srgb, u, v, o);
    if (delta == 0.0f || dh == dl) return;
    float b4[4];
    uint32_t wh = w0 >> dh, hh = h0 >> dh;
    or_bilinear(s, ti[4 + dh], (int)(wh ? wh : 1), (int)(hh ? hh : 1), srgb, u, v, b4);
    float id_ = 1.0f - delta;
    for (int k = 0; k < 4; ++k) o[k] = o[k] * id_ + b4[k] * delta;
}

static uint32_t or_tex_max_dim(const OScene* s, int id) {
    if (id < 0 || (uint32_t)id >= s->num_tex) return 1u;
    const uint32_t* ti = s->tex_info + (uint32_t)id * OR_TEX_INFO;
    return ti[0] > ti[1] ? ti[0] : ti[1];
}

static float g_pad_abs;

static void tri_bounds(const OTri* t, float* lo, float* hi) {
    v3 p1 = add(t->v0, t->e1), p2 = add(t->v0, t->e2);
    lo[0] = mn(t->v0.x, mn(p1.x, p2.x)); hi[0] = mx(t->v0.x, mx(p1.x, p2.x));
    lo[1] = mn(t->v0.y, mn(p1.y, p2.y)); hi[1] = mx(t->v0.y, mx(p1.y, p2.y));
    lo[2] = mn(t->v0.z, mn(p1.z, p2.z)); hi[2] = mx(t->v0.z, mx(p1.z, p2.z));
}

/* sort key for median split */
static int g_axis;

static int cmp_tri(const void* a, const void* b) {
    const OTri* x = (const OTri*)a;
    const OTri* y = (const OTri*)b;
    float lx[3], hx[3], ly[3], hy[3];
    tri_bounds(x, lx, hx);
    tri_bounds(y, ly, hy);
    float cx = lx[g_axis] + hx[g_axis], cy = ly[g_axis] + hy[g_axis];
    if (cx < cy) return -1;
    if (cx > cy) return 1;
    return (x->gid < y->gid) ? -1 : (x->gid > y->gid);
}

/* Binned SAH split of tris[first, first + count) (16 bins on the centroid axis of largest extent...
 * all three axes tried); returns the left count, or 0 when no bin boundary separates the centroids.
 * The oracle's tree only decides which boxes are tested: the closest hit is the minimum over
 * (t, gid) of every candidate and any-hit is a boolean, so any valid tree gives the same image; a
 * SAH tree with nearest-child-first traversal keeps the CPU baseline honest (bench.py). */
#define OR_SAH_BINS 16
static int sah_partition(OScene* s, int first, int count) {
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = first; i < first + count; ++i) {
        float lo[3], hi[3];
        tri_bounds(&s->tris[i], lo, hi);
        for (int a = 0; a < 3; ++a) { float c = lo[a] + hi[a]; clo[a] = mn(clo[a], c); chi[a] = mx(chi[a], c); }
    }
    float best = INFINITY;
    int best_axis = -1, best_bin = -1;
    for (int a = 0; a < 3; ++a) {
        float ext = chi[a] - clo[a];
        if (!(ext > 0.0f)) continue;
        float blo[OR_SAH_BINS][3], bhi[OR_SAH_BINS][3];
        int cnt[OR_SAH_BINS];
        for (int k = 0; k < OR_SAH_BINS; ++k) {
            cnt[k] = 0;
            for (int q = 0; q < 3; ++q) { blo[k][q] = INFINITY; bhi[k][q] = -INFINITY; }
        }
        float scale = (float)OR_SAH_BINS / ext;
        for (int i = first; i < first + count; ++i) {
            float lo[3], hi[3];
            tri_bounds(&s->tris[i], lo, hi);
            int k = (int)((lo[a] + hi[a] - clo[a]) * scale);
            k = k < 0 ? 0 : (k >= OR_SAH_BINS ? OR_SAH_BINS - 1 : k);
            cnt[k]++;
            for (int q = 0; q < 3; ++q) { blo[k][q] = mn(blo[k][q], lo[q]); bhi[k][q] = mx(bhi[k][q], hi[q]); }
        }
        float rarea[OR_SAH_BINS];
        int rcnt[OR_SAH_BINS];
        float alo[3] = {INFINITY, INFINITY, INFINITY}, ahi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int c = 0;
        for (int k = OR_SAH_BINS - 1; k > 0; --k) {
            for (int q = 0; q < 3; ++q) { alo[q] = mn(alo[q], blo[k][q]); ahi[q] = mx(ahi[q], bhi[k][q]); }
            c += cnt[k];
            float dx = ahi[0] - alo[0], dy = ahi[1] - alo[1], dz = ahi[2] - alo[2];
            rarea[k] = c ? dx * dy + dy * dz + dz * dx : 0.0f;
            rcnt[k] = c;
        }
        for (int q = 0; q < 3; ++q) { alo[q] = INFINITY; ahi[q] = -INFINITY; }
        c = 0;
        for (int k = 0; k < OR_SAH_BINS - 1; ++k) {
            for (int q = 0; q < 3; ++q) { alo[q] = mn(alo[q], blo[k][q]); ahi[q] = mx(ahi[q], bhi[k][q]); }
            c += cnt[k];
            if (c == 0 || rcnt[k + 1] == 0) continue;
            float dx = ahi[0] - alo[0], dy = ahi[1] - alo[1], dz = ahi[2] - alo[2];
            float cost = (dx * dy + dy * dz + dz * dx) * (float)c + rarea[k + 1] * (float)rcnt[k + 1];
            if (cost < best) { best = cost; best_axis = a; best_bin = k; }
        }
    }
    if (best_axis < 0) return 0;
    /* stable partition (deterministic tree) */
    OTri* tmp = (OTri*)malloc(sizeof(OTri) * (size_t)count);
    float scale = (float)OR_SAH_BINS / (chi[best_axis] - clo[best_axis]);
    int nl = 0, nr = 0;
    for (int pass = 0; pass < 2; ++pass)
        for (int i = first; i < first + count; ++i) {
            float lo[3], hi[3];
            tri_bounds(&s->tris[i], lo, hi);
            int k = (int)((lo[best_axis] + hi[best_axis] - clo[best_axis]) * scale);
            k = k < 0 ? 0 : (k >= OR_SAH_BINS ? OR_SAH_BINS - 1 : k);
            if ((k <= best_bin) == (pass == 0)) tmp[pass == 0 ? nl++ : count - 1 - nr++] = s->tris[i];
        }
    for (int i = 0; i < nr / 2; ++i) {  /* the right part was filled from the end: restore its order */
        OTri t = tmp[nl + i]; tmp[nl + i] = tmp[count - 1 - i]; tmp[count - 1 - i] = t;
    }
    memcpy(s->tris + first, tmp, sizeof(OTri) * (size_t)count);
    free(tmp);
    return (nl > 0 && nr > 0) ? nl : 0;
}

static int build_node(OScene* s, int first, int count) {
    if (s->nnodes == s->cap) { s->cap = s->cap * 2 + 16; s->nodes = (ONode*)realloc(s->nodes, sizeof(ONode) * s->cap); }
    int idx = s->nnodes++;
    ONode n;
    for (int a = 0; a < 3; ++a) { n.lo[a] = INFINITY; n.hi[a] = -INFINITY; }
    for (int i = first; i < first + count; ++i) {
        float lo[3], hi[3];
        tri_bounds(&s->tris[i], lo, hi);
        for (int a = 0; a < 3; ++a) { n.lo[a] = mn(n.lo[a], lo[a]); n.hi[a] = mx(n.hi[a], hi[a]); }
    }
    float ext = mx(n.hi[0] - n.lo[0], mx(n.hi[1] - n.lo[1], n.hi[2] - n.lo[2]));
    float pad = ext * 1e-5f + g_pad_abs;
    for (int a = 0; a < 3; ++a) { n.lo[a] -= pad; n.hi[a] += pad; }
    n.left = n.right = -1;
    n.first = first;
    n.count = count;
    if (count > 4) {
        int half = sah_partition(s, first, count);
        if (half == 0) {  /* degenerate centroids: median split along the widest axis */
            int axis = 0;
            float e0 = n.hi[0] - n.lo[0], e1 = n.hi[1] - n.lo[1], e2 = n.hi[2] - n.lo[2];
            if (e1 > e0 && e1 >= e2) axis = 1;
            else if (e2 > e0 && e2 > e1) axis = 2;
            g_axis = axis;
            qsort(s->tris + first, (size_t)count, sizeof(OTri), cmp_tri);
            half = count / 2;
        }
        int l = build_node(s, first, half);
        int r = build_node(s, first + half, count - half);
        n.left = l;
        n.right = r;
        n.count = 0;
    }
    s->nodes[idx] = n;
    return idx;
}

static int scene_init(OScene* s, const ptgs_scene_desc* d) {
    memset(s, 0, sizeof(*s));
    s->d = d;
    uint32_t total = 0;
    for (uint32_t m = 0; m < d->num_meshes; ++m) if (d->mesh_index_count[m] >= 3) total += d->mesh_index_count[m] / 3;
    s->tris = (OTri*)malloc(sizeof(OTri) * (total ? total : 1));
    float maxabs = 0.0f;
    uint32_t g = 0;
    for (uint32_t m = 0; m < d->num_meshes; ++m) {
        uint32_t cnt = d->mesh_index_count[m];
        if (cnt < 3) continue;
        const ptgs_mesh_info* mi = &d->meshes[m];
        int transparent = d->materials[mi->material_index].pad > 0.5f;
        s->has_transparent |= transparent;
        for (uint32_t p = 0; p < cnt / 3; ++p) {
            v3 q[3];
            for (int k = 0; k < 3; ++k) {
                uint32_t vi = d->indices[mi->index_offset + 3 * p + k] + mi->vertex_offset;
                q[k] = ld3(d->vertices[vi].pos);
                maxabs = mx(maxabs, mx(fabsf(q[k].x), mx(fabsf(q[k].y), fabsf(q[k].z))));
            }
            OTri* t = &s->tris[g];
            t->v0 = q[0];
            t->e1 = sub(q[1], q[0]);
            t->e2 = sub(q[2], q[0]);
            t->mesh = m; t->prim = p; t->gid = g; t->flags = transparent ? 1u : 0u;
            g++;
        }
    }
    s->ntris = g;
    g_pad_abs = maxabs * 4e-7f + 1e-30f;
    if (g > 0) build_node(s, 0, (int)g);
    s->bn = d->blue_noise_rgba32f;
    s->bn_size = (int)d->blue_noise_size;
    or_build_textures(s, d->textures, d->num_textures);
    return 0;
}

static void scene_free(OScene* s) { free(s->tris); free(s->nodes); free(s->tex_texels); free(s->tex_info); }

/* ------------------------------------------------------------------------------------------ */
/* traversal                                                                                   */
/* ------------------------------------------------------------------------------------------ */
typedef struct { v3 o, d; float tmin, tmax; v3 inv; } ORay;
typedef struct { float t, u, v; uint32_t gid; const OTri* tri; } OHit;

static float safe_inv_(float d) {
    const float eps = 1e-20f;
    float a = fabsf(d) < eps ? (d < 0.0f ? -eps : eps) : d;
    return 1.0f / a;
}
static ORay mkray(v3 o, v3 d, float tmin, float tmax) {
    ORay r; r.o = o; r.d = d; r.tmin = tmin; r.tmax = tmax;
    r.inv = V(safe_inv_(d.x), safe_inv_(d.y), safe_inv_(d.z));
    return r;
}

static int box_hit(const ORay* r, const ONode* n, float tcap) {
    float tn = r->tmin, tf = tcap;
    float o[3] = {r->o.x, r->o.y, r->o.z}, iv[3] = {r->inv.x, r->inv.y, r->inv.z};
    for (int a = 0; a < 3; ++a) {
        float t0 = (n->lo[a] - o[a]) * iv[a], t1 = (n->hi[a] - o[a]) * iv[a];
        float lo = mn(t0, t1), hi = mx(t0, t1);
        tn = mx(tn, lo);
        tf = mn(tf, hi);
    }
    return tn <= tf * 1.0000004f;
}

/* Moller-Trumbore — same operation order as the HIP kernel (parity contract) */
static int tri_intersect(const ORay* r, const OTri* t, float* tt, float* uu, float* vv) {
    v3 pvec = cross(r->d, t->e2);
    float det = dot(t->e1, pvec);
    if (det == 0.0f) return 0;
    float inv_det = 1.0f / det;
    v3 tvec = sub(r->o, t->v0);
    float u = dot(tvec, pvec) * inv_det;
    if (u < 0.0f || u > 1.0f) return 0;
    v3 qvec = cross(tvec, t->e1);
    float v = dot(r->d, qvec) * inv_det;
    if (v < 0.0f || u + v > 1.0f) return 0;
    *tt = dot(t->e2, qvec) * inv_det;
    *uu = u;
    *vv = v;
    return 1;
}

static float or_rnd(uint32_t* state) {
    uint32_t prev = *state;
    *state = prev * 747796405u + 2891336453u;
    uint32_t s = *state;
    uint32_t word = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (float)((word >> 22u) ^ word) / 4294967296.0f;
}

/* alpha.rahit:14-61; BLEND uses a stateless (seed, triangle) hash */
static int or_anyhit_accept(const OScene* s, const OTri* t, float u, float v, uint32_t seed) {
    const ptgs_mesh_info* info = &s->d->meshes[t->mesh];
    const ptgs_material* m = &s->d->materials[info->material_index];
    float cutoff = m->alpha_cutoff;
    int blend = m->pad > 0.5f;
    if (cutoff == 0.0f && !blend) return 1;
    float alpha = m->base_color_factor[3];
    if (m->albedo_texture_index > 0) {
        const ptgs_vertex* vs = s->d->vertices + info->vertex_offset;
        const uint32_t* ix = s->d->indices + info->index_offset + t->prim * 3u;
        const ptgs_vertex *v0 = &vs[ix[0]], *v1 = &vs[ix[1]], *v2 = &vs[ix[2]];
        float bx = (1.0f - u) - v;
        float tu = (v0->tex_coord[0] * bx + v1->tex_coord[0] * u) + v2->tex_coord[0] * v;
        float tv = (v0->tex_coord[1] * bx + v1->tex_coord[1] * u) + v2->tex_coord[1] * v;
        float o[4];
        or_tex_sample(s, m->albedo_texture_index, tu, tv, 0.0f, o);
        alpha = alpha * o[3];
    }
    if (cutoff > 0.0f) return !(alpha < cutoff);
    uint32_t h = seed ^ (t->gid * 0x9E3779B9u);
    return !(or_rnd(&h) > alpha);
}

/* entry distance of the ray into n's box within [tmin, tcap], or +inf (box_hit's test) */
static float box_enter(const ORay* r, const ONode* n, float tcap) {
    float tn = r->tmin, tf = tcap;
    float o[3] = {r->o.x, r->o.y, r->o.z}, iv[3] = {r->inv.x, r->inv.y, r->inv.z};
    for (int a = 0; a < 3; ++a) {
        float t0 = (n->lo[a] - o[a]) * iv[a], t1 = (n->hi[a] - o[a]) * iv[a];
        tn = mx(tn, mn(t0, t1));
        tf = mn(tf, mx(t0, t1));
    }
    return tn <= tf * 1.0000004f ? tn : INFINITY;
}

/* n's box is hit; children nearest first, the farther one re-tested against the shortened h->t */
static void closest(const OScene* s, const ONode* n, const ORay* r, OHit* h, uint32_t seed, uint64_t* nodes_visited) {
    (*nodes_visited)++;
    if (n->left < 0) {
        for (int i = n->first; i < n->first + n->count; ++i) {
            const OTri* t = &s->tris[i];
            float tt, u, v;
            if (!tri_intersect(r, t, &tt, &u, &v)) continue;
            if (!(tt >= r->tmin && tt <= h->t)) continue;
            if (tt == h->t && t->gid >= h->gid) continue;
            if (s->has_transparent && (t->flags & 1u) && !or_anyhit_accept(s, t, u, v, seed)) continue;
            h->t = tt; h->u = u; h->v = v; h->gid = t->gid; h->tri = t;
        }
        return;
    }
    const ONode *a = &s->nodes[n->left], *b = &s->nodes[n->right];
    float ta = box_enter(r, a, h->t), tb = box_enter(r, b, h->t);
    if (tb < ta) { const ONode* x = a; a = b; b = x; float y = ta; ta = tb; tb = y; }
    if (ta != INFINITY) closest(s, a, r, h, seed, nodes_visited);
    if (tb != INFINITY && box_hit(r, b, h->t)) closest(s, b, r, h, seed, nodes_visited);
}

static int anyhit(const OScene* s, const ONode* n, const ORay* r, uint32_t seed) {
    if (!box_hit(r, n, r->tmax)) return 0;
    if (n->left < 0) {
        for (int i = n->first; i < n->first + n->count; ++i) {
            const OTri* t = &s->tris[i];
            float tt, u, v;
            if (!tri_intersect(r, t, &tt, &u, &v)) continue;
            if (!(tt >= r->tmin && tt <= r->tmax)) continue;
            if (s->has_transparent && (t->flags & 1u) && !or_anyhit_accept(s, t, u, v, seed)) continue;
            return 1;
        }
        return 0;
    }
    return anyhit(s, &s->nodes[n->left], r, seed) || anyhit(s, &s->nodes[n->right], r, seed);
}

static OHit trace_closest(const OScene* s, const ORay* r, uint32_t seed) {
    OHit h; h.t = r->tmax; h.u = 0; h.v = 0; h.gid = 0xffffffffu; h.tri = NULL;
    uint64_t dummy = 0;
    if (s->ntris && box_hit(r, &s->nodes[0], h.t)) closest(s, &s->nodes[0], r, &h, seed, &dummy);
    return h;
}

/* ------------------------------------------------------------------------------------------ */
/* shading                                                                                     */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    v3 color, next_o, next_d;
    float hit_flag;
    v3 weight;
    uint32_t seed;
    float last_pdf;
    float blue_x, blue_y;
    int depth;
    v3 hit_pos, normal;
} OPayload;

typedef struct {
    float inv_view[16], inv_proj[16];
    float ambient[4];
    float emissive_flux, punctual_flux, p_emissive;
    float lod_factor, fov, win_height, use_lod;
} OCam;

typedef struct {
    const OScene* s;
    const OCam* cam;
    uint64_t shadow_rays;
} OCtx;

#define OPI 3.14159265359f
#define OPHI 1.61803398875f

static float bnd(const OPayload* p, int dim) {
    float base = (dim % 2 == 0) ? p->blue_x : p->blue_y;
    return fract_((base + ((float)p->depth * OPHI)) + ((float)dim * 0.754877f));
}
static v3 safe_nrm(v3 v) { float l = len(v); return (l < 1e-6f) ? V(0.0f, 1.0f, 0.0f) : divs(v, l); }
static v3 f_schlick(float c, v3 f0) { float p = p5(clampf_(1.0f - c, 0.0f, 1.0f)); return add(f0, mul(rsub(1.0f, f0), p)); }
static void basis(v3 n, v3* t, v3* b) {
    v3 up = fabsf(n.z) < 0.999f ? V(0, 0, 1) : V(1, 0, 0);
    *t = safe_nrm(cross(up, n));
    *b = cross(n, *t);
}
static v3 sample_cos(const OPayload* p, v3 n) {
    float r1 = bnd(p, 0), r2 = bnd(p, 1);
    float phi = (2.0f * OPI) * r1;
    float sq = sqrtf(r2);
    float sn, cs; or_sincos(phi, &sn, &cs);
    v3 l = V(cs * sq, sn * sq, sqrtf(1.0f - r2));
    v3 t, b; basis(n, &t, &b);
    return safe_nrm(add(add(mul(t, l.x), mul(b, l.y)), mul(n, l.z)));
}
static float d_ggx(v3 n, v3 h, float rough) {
    float a = rough * rough, a2 = a * a;
    float ndh = mx(dot(n, h), 0.0f), ndh2 = ndh * ndh;
    float den = ndh2 * (a2 - 1.0f) + 1.0f;
    return a2 / (((OPI * den) * den) + 0.0001f);
}
static float v_smith(float ndv, float ndl, float rough) {
    float a = rough * rough;
    float gv = ndl * (ndv * (1.0f - a) + a);
    float gl = ndv * (ndl * (1.0f - a) + a);
    return 0.5f / mx(gv + gl, 0.0001f);
}
static v3 sample_ggx(const OPayload* p, v3 n, float rough) {
    float r1 = bnd(p, 2), r2 = bnd(p, 3);
    float a = rough * rough;
    float phi = (2.0f * OPI) * r1;
    float den = 1.0f + (a * a - 1.0f) * r2;
    float ct = sqrtf((1.0f - r2) / mx(den, 0.0001f));
    float st = sqrtf(1.0f - ct * ct);
    float sn, cs; or_sincos(phi, &sn, &cs);
    v3 hl = V(st * cs, st * sn, ct);
    v3 t, b; basis(n, &t, &b);
    return safe_nrm(add(add(mul(t, hl.x), mul(b, hl.y)), mul(n, hl.z)));
}
static float pdf_ggx(v3 n, v3 v, v3 l, float rough) {
    v3 h = safe_nrm(add(v, l));
    float ndh = mx(dot(n, h), 0.0f), vdh = mx(dot(v, h), 0.0f);
    return (d_ggx(n, h, rough) * ndh) / (4.0f * vdh + 0.0001f);
}
static float pdf_lam(v3 n, v3 l) { return mx(dot(n, l), 0.0f) / OPI; }

static float shadow_dist(OCtx* c, v3 o, v3 d, float maxd, uint32_t seed) {
    c->shadow_rays++;
    ORay r = mkray(o, d, 0.001f, maxd);
    if (!c->s->ntris) return 1.0f;
    return anyhit(c->s, &c->s->nodes[0], &r, seed) ? 0.0f : 1.0f;
}
static float shadow_to(OCtx* c, v3 o, v3 lp, uint32_t seed) {
    v3 l = sub(lp, o);
    float dist = len(l);
    l = safe_nrm(l);
    return shadow_dist(c, o, l, dist - 0.005f, seed);
}

static uint32_t cdf_find_light(const ptgs_light_cdf* cdf, uint32_t n, float r) {
    uint32_t idx = 0, left = 0, right = n;
    while (left < right) { uint32_t mid = (left + right) >> 1; if (cdf[mid].cumulative_probability < r) left = mid + 1; else { idx = mid; right = mid; } }
    return idx;
}
static uint32_t cdf_find_punct(const ptgs_punctual_cdf* cdf, uint32_t n, float r) {
    uint32_t idx = 0, left = 0, right = n;
    while (left < right) { uint32_t mid = (left + right) >> 1; if (cdf[mid].cumulative_probability < r) left = mid + 1; else { idx = mid; right = mid; } }
    return idx;
}

/* closesthit.rchit:128-192 */
static void punctual(OCtx* c, const OPayload* p, v3 hp, v3 n, v3 ng, v3 v, v3 albedo, float rough, v3 f0, float tr, v3* lo) {
    const ptgs_scene_desc* d = c->s->d;
    uint32_t nl = d->num_punctual_lights;
    float rs = bnd(p, 4);
    uint32_t li = cdf_find_punct(d->punctual_cdf, nl, rs);
    const ptgs_punctual_light* L = &d->punctual_lights[li];
    v3 l;
    float att = 1.0f;
    v3 lpos = ld3(L->position), ldir = ld3(L->direction);
    if (L->type == 1) {
        l = nrm(neg(ldir));
        att = 1.0f;
    } else {
        v3 off = sub(lpos, hp);
        float dsq = dot(off, off);
        dsq = mx(dsq, 0.01f);
        float dist = sqrtf(dsq);
        l = divs(off, dist);
        att = 1.0f / dsq;
        if (L->range > 0.0f) {
            float ra = mx(mn(1.0f - p4(dist / L->range), 1.0f), 0.0f) / dsq;
            att = ra / dsq;
        }
        if (L->type == 2) {
            float cd = dot(neg(l), nrm(ldir));
            float ss = 1.0f / mx(L->inner_cone_cos - L->outer_cone_cos, 0.001f);
            float so = -L->outer_cone_cos * ss;
            float sa = clampf_(cd * ss + so, 0.0f, 1.0f);
            att = att * (sa * sa);
        }
    }
    v3 le = mul(mul(ld3(L->color), L->intensity), att);
    float ndl = mx(dot(n, l), 0.0f);
    if (ndl < 0.001f) return;
    if (ndl > 0.0f && len(le) > 0.0f) {
        v3 so = add(hp, mul(ng, 0.001f));
        float vis = (L->type == 1) ? shadow_dist(c, so, l, 10000.0f, p->seed) : shadow_to(c, so, lpos, p->seed);
        vis = mx(vis, tr);
        if (vis > 0.0f) {
            float w = (float)nl;
            v3 h = safe_nrm(add(v, l));
            float ndf = d_ggx(n, h, rough);
            float vt = v_smith(dot(n, v), ndl, rough);
            v3 f = f_schlick(dot(h, v), f0);
            v3 kd = mul(rsub(1.0f, f), 1.0f - tr);
            v3 spec = mul(f, ndf * vt);
            v3 diff = mul(divs(mulv(kd, albedo), OPI), 1.0f - tr);
            *lo = add(*lo, mul(mul(mul(mulv(add(diff, spec), le), ndl), vis), w));
        }
    }
}

/* closesthit.rchit:194-257 (sg) / :259-320 */
static void emissive_nee(OCtx* c, const OPayload* p, int sg, v3 hp, v3 n, v3 ng, v3 v, v3 albedo, float rough, float metal, v3 f0, float tr, v3* lo) {
    const ptgs_scene_desc* d = c->s->d;
    float rs = bnd(p, sg ? 4 : 7);
    uint32_t idx = cdf_find_light(d->light_cdf, d->num_light_cdf, rs);
    uint32_t ti = d->light_cdf[idx].triangle_index;
    ptgs_light_triangle tri = d->light_triangles[ti];
    v3 p0 = ld3(d->vertices[tri.v0].pos), p1 = ld3(d->vertices[tri.v1].pos), p2 = ld3(d->vertices[tri.v2].pos);
    float u = bnd(p, sg ? 5 : 8), w = bnd(p, sg ? 6 : 9);
    if (u + w > 1.0f) { u = 1.0f - u; w = 1.0f - w; }
    v3 lp = add(add(mul(p0, (1.0f - u) - w), mul(p1, u)), mul(p2, w));
    v3 cr = cross(sub(p1, p0), sub(p2, p0));
    v3 ln = sg ? nrm(cr) : safe_nrm(cr);
    v3 l = sub(lp, hp);
    float dsq = dot(l, l);
    dsq = mx(dsq, 0.0001f);
    float dist = sqrtf(dsq);
    l = divs(l, dist);
    float ndl = mx(dot(n, l), 0.0f);
    if (ndl < 0.001f) return;
    float ldn = fabsf(dot(neg(l), ln));
    if (ndl > 0.0f && ldn > 0.0f) {
        v3 so = add(hp, mul(ng, 0.001f));
        float vis = shadow_to(c, so, lp, p->seed);
        vis = mx(vis, tr);
        if (vis > 0.0f) {
            const ptgs_material* lm = &d->materials[tri.material_index];
            v3 le = ld3(lm->emissive_factor_and_pad);
            float es = mx(le.x, mx(le.y, le.z));
            float pdf_nee = (es / c->cam->emissive_flux) * (dsq / ldn);
            float ps, pdf_s, pdf_d;
            if (sg) {
                pdf_s = pdf_ggx(n, v, l, rough);
                pdf_d = pdf_lam(n, l);
                ps = clampf_(len(f0), 0.05f, 0.95f);
            } else {
                ps = mixf_(0.04f, 1.0f, metal);
                pdf_s = pdf_ggx(n, v, l, rough);
                pdf_d = pdf_lam(n, l);
            }
            float pd = 1.0f - ps;
            float pdf_b = pdf_s * ps + pdf_d * pd;
            float mis = (pdf_nee * pdf_nee) / (pdf_nee * pdf_nee + pdf_b * pdf_b);
            v3 h = safe_nrm(add(v, l));
            float ndf = d_ggx(n, h, rough);
            float vt = v_smith(dot(n, v), ndl, rough);
            v3 f = f_schlick(dot(h, v), f0);
            v3 kd = rsub(1.0f, f);
            v3 spec = mul(f, ndf * vt);
            v3 diff = mul(divs(mulv(kd, albedo), OPI), 1.0f - tr);
            v3 brdf = add(diff, spec);
            if (pdf_nee > 1e-10f)
                *lo = add(*lo, mul(mul(mul(mul(mul(mulv(brdf, le), ndl), 1.0f / pdf_nee), mis), vis), c->cam->ambient[3]));
        }
    }
}

/* closesthit.rchit:324-621 (with_hitpos: rt_datacollect variant) */
static void or_closest_hit(OCtx* c, OPayload* p, const ORay* ray, const OHit* hit, int with_hitpos) {
    const ptgs_scene_desc* d = c->s->d;
    const OCam* cp = c->cam;
    const OTri* tri = hit->tri;
    const ptgs_mesh_info* info = &d->meshes[tri->mesh];
    const ptgs_material* mat = &d->materials[info->material_index];
    uint32_t i0 = d->indices[info->index_offset + tri->prim * 3u + 0u];
    uint32_t i1 = d->indices[info->index_offset + tri->prim * 3u + 1u];
    uint32_t i2 = d->indices[info->index_offset + tri->prim * 3u + 2u];
    const ptgs_vertex* v0 = &d->vertices[info->vertex_offset + i0];
    const ptgs_vertex* v1 = &d->vertices[info->vertex_offset + i1];
    const ptgs_vertex* v2 = &d->vertices[info->vertex_offset + i2];
    float bx = (1.0f - hit->u) - hit->v, by = hit->u, bz = hit->v;
    v3 hp = add(ray->o, mul(ray->d, hit->t));
    v3 vcol = add(add(mul(ld3(v0->color), bx), mul(ld3(v1->color), by)), mul(ld3(v2->color), bz));
    v3 nobj = add(add(mul(ld3(v0->normal), bx), mul(ld3(v1->normal), by)), mul(ld3(v2->normal), bz));
    v3 tobj = add(add(mul(ld3(v0->tangent), bx), mul(ld3(v1->tangent), by)), mul(ld3(v2->tangent), bz));
    float tw = (v0->tangent[3] * bx + v1->tangent[3] * by) + v2->tangent[3] * bz;
    v3 ng = safe_nrm(nobj);
    v3 tg = safe_nrm(tobj);
    tg = safe_nrm(sub(tg, mul(ng, dot(tg, ng))));
    v3 vv = neg(ray->d);
    v3 ng_orig = ng;
    if (dot(ng, vv) < 0.0f) ng = neg(ng);
    v3 N = ng;
    const OScene* sc = c->s;
    float tcu = (v0->tex_coord[0] * bx + v1->tex_coord[0] * by) + v2->tex_coord[0] * bz;
    float tcv = (v0->tex_coord[1] * bx + v1->tex_coord[1] * by) + v2->tex_coord[1] * bz;
    v3 T = tg;
    int tvalid = (fabsf(tw) > 0.001f) && (len(T) > 0.001f);
    if (!tvalid) {
        v3 up = (fabsf(N.y) < 0.999f) ? V(0.0f, 1.0f, 0.0f) : V(1.0f, 0.0f, 0.0f);
        T = safe_nrm(cross(up, N));
    }
    /* :358-385 normal map */
    if (fabsf(tw) > 0.0001f && mat->normal_texture_index > 0) {
        float hand = (tw < 0.0f) ? -1.0f : 1.0f;
        v3 B = mul(safe_nrm(cross(N, T)), hand);
        float tex_lod = 0.0f;
        if (cp->use_lod > 0.0f) {
            if (p->last_pdf <= 0.0f) {
                if (mat->albedo_texture_index > 0) { /* computeLOD :21-37 */
                    float sn, cs;
                    or_sincos(cp->fov * 0.5f, &sn, &cs);
                    float spread = (2.0f * (sn / cs)) / cp->win_height;
                    float fp = hit->t * spread;
                    float ndv = fabsf(dot(ng, neg(ray->d)));
                    fp = fp / mx(ndv, 0.25f);
                    float dim = (float)or_tex_max_dim(sc, mat->albedo_texture_index);
                    float raw = or_log2(fp * dim);
                    float bias = (dim > 2048.0f) ? 0.0f : -0.5f;
                    tex_lod = mx(raw * 0.7f + bias, 0.0f);
                }
            } else {
                tex_lod = clampf_(mat->roughness_factor * 5.0f + or_log2(hit->t * 0.1f + 1.0f), 0.0f, 8.0f);
            }
        }
        const float* un = mat->uv_normal;
        float nu = ((un[0] * tcu + un[4] * tcv) + un[8] * 0.0f) + un[12];
        float nv = ((un[1] * tcu + un[5] * tcv) + un[9] * 0.0f) + un[13];
        float m4[4];
        or_tex_sample(sc, mat->normal_texture_index, nu, nv, tex_lod, m4);
        v3 nm = V(m4[0] * 2.0f - 1.0f, m4[1] * 2.0f - 1.0f, m4[2] * 2.0f - 1.0f);
        nm.x = nm.x * cp->lod_factor;
        nm.y = nm.y * cp->lod_factor;
        nm = nrm(nm);
        N = safe_nrm(add(add(mul(T, nm.x), mul(B, nm.y)), mul(N, nm.z)));
    }

    union { float f; int32_t i; } pun;
    pun.f = mat->use_specular_glossiness_workflow;
    int32_t sgb = pun.i;
    v3 bcf = ld3(mat->base_color_factor);
    v3 bcs = S(1.0f);
    if (mat->albedo_texture_index > 0) {
        float b4[4];
        or_tex_sample(sc, mat->albedo_texture_index, tcu, tcv, 0.0f, b4);
        bcs = V(b4[0], b4[1], b4[2]);
    }
    v3 albedo, f0;
    float rough, metal;
    if ((float)sgb > 0.5f) {
        albedo = mulv(mulv(bcf, vcol), bcs);
        v3 spec = ld3(mat->specular_color_factor);
        float gloss = mat->roughness_factor;
        if (mat->sg_id > 0) {
            float g4[4];
            or_tex_sample(sc, mat->sg_id, tcu, tcv, 0.0f, g4);
            spec = mulv(spec, V(g4[0], g4[1], g4[2]));
            gloss = gloss * g4[3];
        }
        f0 = spec;
        rough = sqrtf(mx(1.0f - gloss, 0.04f));
        metal = 0.0f;
    } else {
        albedo = mulv(mulv(bcf, vcol), bcs);
        metal = mat->metallic_factor;
        rough = mat->roughness_factor;
        if (mat->metallic_roughness_texture_index > 0) {
            float r4[4];
            or_tex_sample(sc, mat->metallic_roughness_texture_index, tcu, tcv, 0.0f, r4);
            metal = metal * r4[2];
            rough = rough * r4[1];
        }
        f0 = mix3_(S(0.04f), albedo, metal);
        albedo = mul(albedo, 1.0f - metal);
    }
    float cc = mat->clearcoat_factor, ccr = mat->clearcoat_roughness_factor;
    if (cc > 0.0f && mat->clearcoat_texture_index > 0) {
        float q[4];
        or_tex_sample(sc, mat->clearcoat_texture_index, tcu, tcv, 0.0f, q);
        cc = cc * q[0];
    }
    if (cc > 0.0f && mat->clearcoat_roughness_texture_index > 0) {
        float q[4];
        or_tex_sample(sc, mat->clearcoat_roughness_texture_index, tcu, tcv, 0.0f, q);
        ccr = ccr * q[0];
    }
    v3 em = ld3(mat->emissive_factor_and_pad);
    if (len(em) > 0.0f && mat->emissive_texture_index > 0) {
        const float* ue = mat->uv_emissive;
        float eu = ((ue[0] * tcu + ue[4] * tcv) + ue[8] * 0.0f) + ue[12];
        float ev = ((ue[1] * tcu + ue[5] * tcv) + ue[9] * 0.0f) + ue[13];
        float q[4];
        or_tex_sample(sc, mat->emissive_texture_index, eu, ev, 0.0f, q);
        em = mulv(em, V(q[0], q[1], q[2]));
    }
    float tr = mat->transmission_factor;
    if (with_hitpos) { p->hit_pos = hp; p->normal = N; }

    v3 lo = S(0.0f);
    float es = len(em);
    int use_nee = (tr == 0.0f) && (rough > 0.001f);
    if (p->hit_flag > 3.0f) use_nee = 0;
    if (es > 0.0f) {
        if (p->last_pdf <= 0.0f || !use_nee) {
            lo = add(lo, em);
        } else if (es < 0.001f) {
            p->color = S(0.0f);
            return;
        } else {
            float pb = p->last_pdf;
            float esc = len(ld3(mat->emissive_factor_and_pad));
            float ldn = fabsf(dot(N, neg(ray->d)));
            float dsq = hit->t * hit->t;
            float pn = 0.0f;
            if (cp->emissive_flux > 0.0f) pn = (esc / cp->emissive_flux) * (dsq / mx(ldn, 0.001f));
            float pr = (cp->punctual_flux > 0.0f) ? cp->p_emissive : 1.0f;
            pn = pn * pr;
            float mis = (pb * pb) / (pb * pb + pn * pn);
            lo = add(lo, mul(em, mis));
        }
    }
    int has_e = cp->emissive_flux > 0.0f, has_p = cp->punctual_flux > 0.0f;
    int sg = (float)sgb > 0.0f;
    if (has_e && has_p) {
        v3 lc = S(0.0f);
        float pp = 1.0f - cp->p_emissive;
        if (bnd(p, 10) < cp->p_emissive) {
            if (use_nee) {
                emissive_nee(c, p, sg, hp, N, ng, vv, albedo, rough, metal, f0, tr, &lc);
                lc = mul(lc, 1.0f / cp->p_emissive);
            }
        } else {
            punctual(c, p, hp, N, ng, vv, albedo, rough, f0, tr, &lc);
            lc = mul(lc, 1.0f / pp);
        }
        lo = add(lo, lc);
    } else if (has_e && use_nee) {
        emissive_nee(c, p, sg, hp, N, ng, vv, albedo, rough, metal, f0, tr, &lo);
    } else if (has_p) {
        punctual(c, p, hp, N, ng, vv, albedo, rough, f0, tr, &lo);
    }
    p->color = lo;

    if (tr > 0.0f) {
        p->hit_flag = 2.0f;
        int entering = dot(ng_orig, vv) > 0.0f;
        v3 nr = entering ? ng_orig : neg(ng_orig);
        p->next_o = sub(hp, mul(nr, 0.001f));
        v3 fv = f_schlick(fabsf(dot(ng_orig, vv)), f0);
        float prf = mx(mx(fv.x, fv.y), fv.z);
        if (bnd(p, 11) < prf) {
            p->next_o = add(hp, mul(nr, 0.001f));
            p->next_d = reflect_(neg(vv), nr);
            p->weight = S(1.0f);
        } else {
            float eta = entering ? (1.0f / 1.01f) : 1.01f;
            v3 rd = refract_(neg(vv), nr, eta);
            if (len(rd) > 0.0f) {
                p->next_d = rd;
                p->weight = albedo;
            } else {
                p->next_o = add(hp, mul(ng, 0.001f));
                p->next_d = reflect_(neg(vv), N);
                p->weight = S(1.0f);
            }
        }
        p->last_pdf = 0.0f;
        return;
    }
    p->hit_flag = 1.0f;
    p->next_o = add(hp, mul(ng, 0.001f));
    float ndv = mx(dot(N, vv), 0.0f);
    float ccp = 0.0f;
    v3 fcc = S(0.0f);
    if (cc > 0.0f) {
        fcc = mul(f_schlick(ndv, S(0.04f)), cc);
        ccp = clampf_(mx(fcc.x, mx(fcc.y, fcc.z)), 0.0f, 1.0f);
    }
    if (cc > 0.0f && bnd(p, 12) < ccp) {
        v3 hc = sample_ggx(p, N, ccr);
        v3 lc = reflect_(neg(vv), hc);
        float ndl = mx(dot(N, lc), 0.0f), ndh = mx(dot(N, hc), 0.0f), vdh = mx(dot(vv, hc), 0.0f);
        if (dot(lc, ng) <= 0.0f) {
            p->weight = S(0.0f);
            p->last_pdf = 0.0f;
        } else {
            p->next_d = lc;
            v3 f = mul(f_schlick(vdh, S(0.04f)), cc);
            float vis = v_smith(ndv, ndl, ccr);
            v3 sw = mul(mul(mul(mul(f, vis), 4.0f), ndl), vdh / mx(ndh, 0.0001f));
            float pcc = pdf_ggx(N, vv, lc, ccr);
            float psb = mixf_(0.04f, 1.0f, metal);
            psb = mixf_(psb, 1.0f, p5(1.0f - ndv));
            psb = clampf_(psb, 0.05f, 0.95f);
            float pdb = 1.0f - psb;
            float pbase = pdf_ggx(N, vv, lc, rough) * psb + pdf_lam(N, lc) * pdb;
            p->last_pdf = pcc * ccp + pbase * (1.0f - ccp);
            p->weight = mul(sw, 1.0f / ccp);
        }
    } else {
        v3 tf = rsub(1.0f, fcc);
        float selw = 1.0f / (1.0f - ccp);
        v3 ea = mul(tf, selw);
        float ps = mixf_(0.04f, 1.0f, metal);
        ps = mixf_(ps, 1.0f, p5(1.0f - ndv));
        ps = clampf_(ps, 0.05f, 0.95f);
        float pd = 1.0f - ps;
        if (bnd(p, 13) < ps) {
            v3 h = sample_ggx(p, N, rough);
            v3 l = reflect_(neg(vv), h);
            float ndl = mx(dot(N, l), 0.0f), ndh = mx(dot(N, h), 0.0f), vdh = mx(dot(vv, h), 0.0f);
            if (dot(l, ng) <= 0.0f) {
                p->weight = S(0.0f);
                p->last_pdf = 0.0f;
            } else {
                p->next_d = l;
                v3 f = f_schlick(mx(dot(h, vv), 0.0f), f0);
                float vis = v_smith(ndv, ndl, rough);
                v3 sw = mul(mul(mul(mul(f, vis), 4.0f), ndl), vdh / mx(ndh, 0.0001f));
                float pdf_s = pdf_ggx(N, vv, l, rough), pdf_d = pdf_lam(N, l);
                p->last_pdf = (pdf_s * ps + pdf_d * pd) * (1.0f - ccp);
                p->weight = mulv(mul(sw, 1.0f / ps), ea);
            }
        } else {
            v3 l = sample_cos(p, N);
            if (dot(l, ng) <= 0.0f) {
                p->weight = S(0.0f);
                p->last_pdf = 0.0f;
            } else {
                p->next_d = l;
                p->weight = mulv(mul(albedo, 1.0f / (1.0f - ps)), ea);
                float pdf_s = pdf_ggx(N, vv, l, rough), pdf_d = pdf_lam(N, l);
                p->last_pdf = (pdf_s * ps + pdf_d * pd) * (1.0f - ccp);
            }
        }
    }
}

static void or_miss(const OCam* cp, OPayload* p, int with_hitpos) {
    p->hit_flag = -1.0f;
    p->color = mul(V(cp->ambient[0], cp->ambient[1], cp->ambient[2]), 2.0f);
    p->weight = S(1.0f);
    if (with_hitpos) { p->hit_pos = S(0.0f); p->normal = V(0.0f, 1.0f, 0.0f); }
}

static const float* bn_texel(const OScene* s, uint32_t lx, uint32_t ly, uint32_t frame) {
    const float a1 = 0.75487766624669276f, a2 = 0.56984029099805327f;
    float rx = fract_((float)frame * a1), ry = fract_((float)frame * a2);
    int ox = (int)(rx * (float)s->bn_size), oy = (int)(ry * (float)s->bn_size);
    int px = ((int)lx + ox) & (s->bn_size - 1), py = ((int)ly + oy) & (s->bn_size - 1);
    return s->bn + 4 * ((size_t)py * s->bn_size + px);
}

/* raygen_camera.rgen:17-78 — returns the clamped accumulated radiance of one sample */
static v3 or_trace_pixel(OCtx* c, uint32_t x, uint32_t y, uint32_t W, uint32_t H, uint32_t frame, uint64_t* ext) {
    const OCam* cp = c->cam;
    const float* blue = bn_texel(c->s, x, y, frame);
    uint32_t index = y * W + x;
    uint32_t seed = index + frame * 719393u;
    float pcx = (float)x + blue[0], pcy = (float)y + blue[1];
    float ux = pcx / (float)W, uy = pcy / (float)H;
    float dx = ux * 2.0f - 1.0f, dy = uy * 2.0f - 1.0f;
    float o4[4], t4[4], d4[4];
    float e0[4] = {0.f, 0.f, 0.f, 1.f};
    mv(cp->inv_view, e0, o4);
    float tv[4] = {dx, dy, 1.f, 1.f};
    mv(cp->inv_proj, tv, t4);
    v3 dc = nrm(divs(V(t4[0], t4[1], t4[2]), t4[3]));
    float dv[4] = {dc.x, dc.y, dc.z, 0.f};
    mv(cp->inv_view, dv, d4);
    v3 ro = V(o4[0], o4[1], o4[2]);
    v3 rd = nrm(V(d4[0], d4[1], d4[2]));
    v3 acc = S(0.0f), thr = S(1.0f);
    OPayload p;
    memset(&p, 0, sizeof(p));
    p.seed = seed;
    p.blue_x = blue[2];
    p.blue_y = blue[3];
    p.last_pdf = 0.0f;
    p.hit_flag = 0.0f;
    p.weight = S(1.0f);
    p.next_o = ro;
    p.next_d = rd;
    int max_depth = 12;
    for (int depth = 0; depth < max_depth; ++depth) {
        p.depth = depth;
        ORay ray = mkray(ro, rd, 0.001f, 10000.0f);
        (*ext)++;
        OHit h = trace_closest(c->s, &ray, p.seed);
        if (h.gid == 0xffffffffu) or_miss(cp, &p, 0);
        else or_closest_hit(c, &p, &ray, &h, 0);
        acc = add(acc, mulv(p.color, thr));
        acc = V(mn(acc.x, 5.0f), mn(acc.y, 5.0f), mn(acc.z, 5.0f));
        if (p.hit_flag < 0.0f) break;
        if (depth == 0 && p.hit_flag < 1.5f) max_depth = 4;
        thr = mulv(thr, p.weight);
        ro = p.next_o;
        rd = p.next_d;
        float mt = mx(mx(thr.x, thr.y), thr.z);
        if (mt < 0.001f) break;
        if (depth >= 4) {
            float pr = clampf_(mt, 0.05f, 0.95f);
            if (or_rnd(&p.seed) > pr) break;
            thr = divs(thr, pr);
        }
    }
    return acc;
}

static void fill_cam(OCam* c, const ptgs_ubo* ubo) {
    oracle_mat4_inverse(ubo->view, c->inv_view);
    oracle_mat4_inverse(ubo->proj, c->inv_proj);
    for (int k = 0; k < 4; ++k) c->ambient[k] = ubo->ambient_light[k];
    c->emissive_flux = ubo->emissive_flux;
    c->punctual_flux = ubo->punctual_flux;
    c->p_emissive = ubo->p_emissive;
    c->lod_factor = ubo->lod_factor;
    c->fov = ubo->fov;
    c->win_height = ubo->height;
    c->use_lod = ubo->use_lod;
}

/* ------------------------------------------------------------------------------------------ */
/* public oracle API                                                                           */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    uint64_t extension_rays, shadow_rays, samples;
} oracle_stats;

/* Render `spp` samples for rows [row0,row1) (pixel_stride: every k-th row only, for bounded
 * CPU-baseline samples; 1 = all). accum: W*H RGBA32F, same semantics as ptgs_trace_camera. */
int oracle_trace_camera(const ptgs_scene_desc* d, const ptgs_ubo* ubo, uint32_t W, uint32_t H, uint32_t row0,
                        uint32_t row1, uint32_t row_stride, float* accum, uint32_t spp, uint32_t frame_stride,
                        uint32_t mode, int threads, oracle_stats* st) {
    OScene s;
    scene_init(&s, d);
    OCam cam;
    fill_cam(&cam, ubo);
    if (row1 > H) row1 = H;
    if (row_stride == 0) row_stride = 1;
    uint64_t ext = 0, shadow = 0, samples = 0;
    uint32_t nrows = row1 > row0 ? (row1 - row0 + row_stride - 1) / row_stride : 0;
    long long total = (long long)nrows * W;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : ext, shadow, samples)
#endif
    for (long long k = 0; k < total; ++k) {
        uint32_t y = row0 + (uint32_t)(k / W) * row_stride, x = (uint32_t)(k % W);
        OCtx c;
        c.s = &s;
        c.cam = &cam;
        c.shadow_rays = 0;
        float* px = accum + 4 * ((size_t)y * W + x);
        v3 state = S(0.0f);
        float sa = 0.0f;
        uint32_t f0 = ubo->frame_count;
        if (mode == PTGS_ACCUM_SUM || f0 > 0) { state = V(px[0], px[1], px[2]); sa = px[3]; }
        uint64_t e = 0;
        for (uint32_t smp = 0; smp < spp; ++smp) {
            uint32_t frame = f0 + smp * frame_stride;
            v3 a = or_trace_pixel(&c, x, y, W, H, frame, &e);
            if (mode == PTGS_ACCUM_SUM) { state = add(state, a); sa = sa + 1.0f; }
            else if (frame > 0) { float bl = 1.0f / (float)(frame + 1u); state = mix3_(state, a, bl); }
            else state = a;
        }
        px[0] = state.x; px[1] = state.y; px[2] = state.z;
        px[3] = (mode == PTGS_ACCUM_SUM) ? sa : 1.0f;
        ext += e;
        shadow += c.shadow_rays;
        samples += spp;
    }
    if (st) { st->extension_rays = ext; st->shadow_rays = shadow; st->samples = samples; }
    scene_free(&s);
    return 0;
}

/* rt_datacollect/raygen.rgen:31-141 */
int oracle_trace_torus(const ptgs_scene_desc* d, const ptgs_ubo* ubo, const ptgs_ray_push* push,
                       const ptgs_ray_sample* samples, uint32_t n, ptgs_hitdata* hits, int threads, oracle_stats* st) {
    OScene s;
    scene_init(&s, d);
    OCam cam;
    fill_cam(&cam, ubo);
    uint32_t side = (uint32_t)ceil(sqrt((double)n));
    while ((uint64_t)side * side < n) side++;
    uint64_t ext = 0, shadow = 0;
    uint32_t frame = ubo->frame_count;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : ext, shadow)
#endif
    for (long long ii = 0; ii < (long long)n; ++ii) {
        uint32_t index = (uint32_t)ii;
        OCtx c;
        c.s = &s;
        c.cam = &cam;
        c.shadow_rays = 0;
        uint32_t lx = index % side, ly = index / side;
        float u = (samples[index].uv[0] * 2.0f) * OPI, v = (samples[index].uv[1] * 2.0f) * OPI;
        float R = push->major_radius, r = push->minor_radius, hh = push->height;
        float su, cu, sv, cv;
        or_sincos(u, &su, &cu);
        or_sincos(v, &sv, &cv);
        float lp[4] = {(R + r * cv) * cu, r * sv + hh, (R + r * cv) * su, 1.0f};
        float ln[4] = {cv * cu, sv, cv * su, 0.0f};
        float wo[4], wn[4];
        mv(push->model, lp, wo);
        mv(push->model, ln, wn);
        v3 rd = nrm(V(wn[0], wn[1], wn[2]));
        v3 so = add(V(wo[0], wo[1], wo[2]), mul(rd, 0.05f));
        const float* blue = bn_texel(&s, lx, ly, frame);
        v3 acc = S(0.0f), thr = S(1.0f);
        OPayload p;
        memset(&p, 0, sizeof(p));
        p.seed = index + frame * 719393u;
        p.last_pdf = 0.0f;
        p.blue_x = blue[2];
        p.blue_y = blue[3];
        p.depth = 0;
        p.hit_flag = 0.0f;
        p.weight = S(1.0f);
        p.next_o = so;
        p.next_d = rd;
        p.normal = V(0.0f, 1.0f, 0.0f);
        uint64_t e = 0;
        ORay ray = mkray(so, rd, 0.0f, 10000.0f);
        e++;
        OHit h = trace_closest(&s, &ray, p.seed);
        if (h.gid == 0xffffffffu) or_miss(&cam, &p, 1);
        else or_closest_hit(&c, &p, &ray, &h, 1);
        v3 fpos = p.hit_pos, fnorm = p.normal;
        float fflag = p.hit_flag;
        if (p.hit_flag > 0.5f) {
            acc = add(acc, mulv(p.color, thr));
            for (int depth = 1; depth < 12; ++depth) {
                p.depth = depth;
                thr = mulv(thr, p.weight);
                float mt = mx(mx(thr.x, thr.y), thr.z);
                if (mt < 0.001f) break;
                if (depth >= 4) {
                    float pr = clampf_(mt, 0.05f, 0.95f);
                    if (or_rnd(&p.seed) > pr) break;
                    thr = divs(thr, pr);
                }
                ORay r2 = mkray(p.next_o, p.next_d, 0.001f, 10000.0f);
                e++;
                OHit h2 = trace_closest(&s, &r2, p.seed);
                if (h2.gid == 0xffffffffu) or_miss(&cam, &p, 1);
                else or_closest_hit(&c, &p, &r2, &h2, 1);
                acc = add(acc, mulv(p.color, thr));
                acc = V(mn(acc.x, 5.0f), mn(acc.y, 5.0f), mn(acc.z, 5.0f));
                if (p.hit_flag < 1.5f) break;
            }
        }
        ptgs_hitdata* hd = &hits[index];
        v3 cur = acc;
        if (frame > 0) {
            float bf = 1.0f / (float)(frame + 1u);
            cur = mix3_(V(hd->color[0], hd->color[1], hd->color[2]), cur, bf);
        }
        hd->pos[0] = fpos.x; hd->pos[1] = fpos.y; hd->pos[2] = fpos.z;
        hd->flag = fflag;
        hd->normal[0] = fnorm.x; hd->normal[1] = fnorm.y; hd->normal[2] = fnorm.z;
        hd->color[0] = cur.x; hd->color[1] = cur.y; hd->color[2] = cur.z; hd->color[3] = 1.0f;
        ext += e;
        shadow += c.shadow_rays;
    }
    if (st) { st->extension_rays = ext; st->shadow_rays = shadow; st->samples = n; }
    scene_free(&s);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* sRGB encode + point raster                                                                  */
/* ------------------------------------------------------------------------------------------ */
static uint32_t or_srgb8(float c) {
    c = clampf_(c, 0.0f, 1.0f);
    float s = (c <= 0.0031308f) ? c * 12.92f : 1.055f * or_pow(c, 0.41666666666666667f) - 0.055f;
    return (uint32_t)(s * 255.0f + 0.5f);
}

void oracle_encode_srgb8(const float* rgba, uint32_t n, uint32_t* out) {
    for (uint32_t i = 0; i < n; ++i)
        out[i] = or_srgb8(rgba[4 * i]) | (or_srgb8(rgba[4 * i + 1]) << 8) | (or_srgb8(rgba[4 * i + 2]) << 16) | (255u << 24);
}

/* pointcloud.vert:44-89 / .frag:1-11, sequential draw order, depth LESS */
void oracle_splat_points(const ptgs_ubo* ubo, const ptgs_ray_push* push, const ptgs_hitdata* hits,
                         const ptgs_ray_sample* samples, uint32_t n, uint32_t W, uint32_t H, uint32_t* rgba8,
                         float* depth) {
    float mvp[16];
    mm(ubo->proj, ubo->view, mvp);
    for (uint32_t i = 0; i < n; ++i) {
        const ptgs_hitdata* hd = &hits[i];
        if (!(hd->flag > 0.0f)) continue;
        float fp[4];
        if (push->mode == 1) {
            float u = (samples[i].uv[0] * 2.0f) * OPI, v = (samples[i].uv[1] * 2.0f) * OPI;
            float su, cu, sv, cv;
            or_sincos(u, &su, &cu);
            or_sincos(v, &sv, &cv);
            float R = push->major_radius, r = push->minor_radius, h = push->height;
            v3 lp = V((R + r * cv) * cu, r * sv + h, (R + r * cv) * su);
            v3 ln = V(cv * cu, sv, cv * su);
            lp = add(lp, mul(ln, 0.01f));
            float l4[4] = {lp.x, lp.y, lp.z, 1.0f};
            mv(push->model, l4, fp);
            fp[3] = 1.0f;
        } else {
            fp[0] = hd->pos[0]; fp[1] = hd->pos[1]; fp[2] = hd->pos[2]; fp[3] = 1.0f;
        }
        float clip[4];
        mv(mvp, fp, clip);
        if (!(clip[3] > 0.0f)) continue;
        if (clip[0] < -clip[3] || clip[0] > clip[3] || clip[1] < -clip[3] || clip[1] > clip[3]) continue;
        if (clip[2] < 0.0f || clip[2] > clip[3]) continue;
        float nx = clip[0] / clip[3], ny = clip[1] / clip[3], nz = clip[2] / clip[3];
        float xw = nx * ((float)W * 0.5f) + (float)W * 0.5f;
        float yw = ny * ((float)H * 0.5f) + (float)H * 0.5f;
        for (int py = 0; py < (int)H; ++py) {
            float cy = (float)py + 0.5f;
            if (!(cy >= yw - 1.0f && cy < yw + 1.0f)) continue;
            for (int px = 0; px < (int)W; ++px) {
                float cx = (float)px + 0.5f;
                if (!(cx >= xw - 1.0f && cx < xw + 1.0f)) continue;
                size_t pix = (size_t)py * W + px;
                if (!(nz < depth[pix])) continue;
                depth[pix] = nz;
                rgba8[pix] = or_srgb8(hd->color[0]) | (or_srgb8(hd->color[1]) << 8) | (or_srgb8(hd->color[2]) << 16) | (255u << 24);
            }
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* 3D Gaussian splatting forward (Kerbl et al. 2023) in the reference camera conventions       */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    uint64_t key;
    uint32_t val;
} OPair;

static int cmp_pair(const void* a, const void* b) {
    const OPair* x = (const OPair*)a;
    const OPair* y = (const OPair*)b;
    if (x->key < y->key) return -1;
    if (x->key > y->key) return 1;
    return (x->val < y->val) ? -1 : (x->val > y->val);
}

static int ndc_rect(float v, int r, int blk, int grid, int hi) {
    float f = hi ? (v + (float)r + (float)(blk - 1)) / (float)blk : (v - (float)r) / (float)blk;
    int i = (int)f;
    if (i < 0) i = 0;
    if (i > grid) i = grid;
    return i;
}

/* Outputs (caller-allocated): radii[N], touched[N], means2d[2N], depths[N], conic[4N]. Returns K and
 * allocates keys_out / vals_out (malloc; caller frees) sorted by (key, gaussian); ranges[tiles*2]; image. */
/* primary-hit view depth (the product's ptgs_trace_depth): pixel-centre camera ray of
 * raygen_camera.rgen:25-41, closest hit with the frame's any-hit seed, -(view * hit).z, +inf on a miss */
int oracle_trace_depth(const ptgs_scene_desc* d, const ptgs_ubo* ubo, uint32_t W, uint32_t H, float* depth,
                       int threads) {
    OScene s;
    scene_init(&s, d);
    OCam cam;
    fill_cam(&cam, ubo);
    long long total = (long long)W * H;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 256)
#endif
    for (long long k = 0; k < total; ++k) {
        uint32_t x = (uint32_t)(k % W), y = (uint32_t)(k / W);
        uint32_t seed = y * W + x + ubo->frame_count * 719393u;
        float ux = ((float)x + 0.5f) / (float)W, uy = ((float)y + 0.5f) / (float)H;
        float dx = ux * 2.0f - 1.0f, dy = uy * 2.0f - 1.0f;
        float o4[4], t4[4], d4[4];
        float e0[4] = {0.f, 0.f, 0.f, 1.f};
        mv(cam.inv_view, e0, o4);
        float tv[4] = {dx, dy, 1.f, 1.f};
        mv(cam.inv_proj, tv, t4);
        v3 dc = nrm(divs(V(t4[0], t4[1], t4[2]), t4[3]));
        float dv[4] = {dc.x, dc.y, dc.z, 0.f};
        mv(cam.inv_view, dv, d4);
        v3 ro = V(o4[0], o4[1], o4[2]);
        v3 rd = nrm(V(d4[0], d4[1], d4[2]));
        ORay r = mkray(ro, rd, 0.001f, 10000.0f);
        OHit h = trace_closest(&s, &r, seed);
        float out = INFINITY;
        if (h.tri) {
            v3 hp = add(ro, mul(rd, h.t));
            float hv[4] = {hp.x, hp.y, hp.z, 1.0f}, pv[4];
            mv(ubo->view, hv, pv);
            out = -pv[2];
        }
        depth[k] = out;
    }
    scene_free(&s);
    return 0;
}

/* depth / under (both NULL, or W*H arrays): the hybrid composite of ptgs_splat_gaussians_over — a
 * pixel stops at the first Gaussian with depth >= depth[pixel]; out = C + T * under.
 * tight = 0: each Gaussian is binned to its 3-sigma tile rectangle (Kerbl et al. 2023's getRect: the
 * published / stats frames of the product). tight = 1: the rectangle is further clipped to the tiles its
 * alpha >= 1/255 box overlaps — the binning of the product's stream-ordered (timed) frames, restated from
 * pathtracer_gaussiansplatting_amd/csrc/splat.hip gs_preprocess_one (the SplatCam::tight branch): the half
 * extents ex = sqrt(-2 s a) * 1.01 + 0.01, ey = sqrt(-2 s c) * 1.01 + 0.01 with s = -ln(255 o) - 0.001
 * (log2 of the shared polynomial, times ln 2), tiles [ceil((x - ex - 15) / 16), floor((x + ex) / 16) + 1);
 * no pairs when s >= 0 (o <= 1/255). Pixels the clip removes have alpha < 1/255 for that Gaussian: the
 * image is the same in both modes. */
static int splat_gaussians_mode(const float* means, const float* scales, const float* rots, const float* opac,
                                const float* colors, uint32_t n, const ptgs_ubo* ubo, uint32_t W, uint32_t H,
                                const float* bg, const float* depth_lim, const float* under, uint32_t trow0,
                                uint32_t trow1, int tight, int32_t* radii, uint32_t* touched, float* means2d,
                                float* depths, float* conic, uint64_t** keys_out, uint32_t** vals_out,
                                uint32_t* ranges, float* image) {
    const int BX = 16, BY = 16;
    float mvp[16];
    mm(ubo->proj, ubo->view, mvp);
    const float* Vm = ubo->view;
    float p00 = ubo->proj[0], p11 = ubo->proj[5];
    float fx = p00 * (float)W * 0.5f, fy = p11 * (float)H * 0.5f;
    float tfx = 1.0f / p00, tfy = 1.0f / (p11 < 0.0f ? -p11 : p11);
    int gx = (int)((W + BX - 1) / BX), gy = (int)((H + BY - 1) / BY);
    if (trow0 > (uint32_t)gy) trow0 = (uint32_t)gy;
    if (trow1 > (uint32_t)gy) trow1 = (uint32_t)gy;
    if (trow1 < trow0) trow1 = trow0;
    uint64_t K = 0;
    int32_t* rect = (int32_t*)malloc(sizeof(int32_t) * 4 * ((size_t)n + 1));  /* the binned tile rect */
    /* per-Gaussian preprocess: independent iterations (OpenMP; K is a sum) */
#pragma omp parallel for schedule(static, 4096) reduction(+ : K)
    for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
        const uint32_t i = (uint32_t)ii;
        radii[i] = 0;
        touched[i] = 0;
        float m4[4] = {means[3 * i], means[3 * i + 1], means[3 * i + 2], 1.0f}, pv[4], ph[4];
        mv(Vm, m4, pv);
        float d = -pv[2];
        if (d <= 0.2f) continue;
        mv(mvp, m4, ph);
        float pw = 1.0f / (ph[3] + 0.0000001f);
        float px = ph[0] * pw, py = ph[1] * pw;
        float qr = rots[4 * i], qx = rots[4 * i + 1], qy = rots[4 * i + 2], qz = rots[4 * i + 3];
        float qn = sqrtf(((qr * qr + qx * qx) + qy * qy) + qz * qz);
        qr = qr / qn; qx = qx / qn; qy = qy / qn; qz = qz / qn;
        float sx = scales[3 * i], sy = scales[3 * i + 1], sz = scales[3 * i + 2];
        float R[3][3] = {{1.0f - 2.0f * (qy * qy + qz * qz), 2.0f * (qx * qy - qr * qz), 2.0f * (qx * qz + qr * qy)},
                         {2.0f * (qx * qy + qr * qz), 1.0f - 2.0f * (qx * qx + qz * qz), 2.0f * (qy * qz - qr * qx)},
                         {2.0f * (qx * qz - qr * qy), 2.0f * (qy * qz + qr * qx), 1.0f - 2.0f * (qx * qx + qy * qy)}};
        float M[3][3];
        for (int r = 0; r < 3; ++r) { M[r][0] = R[r][0] * sx; M[r][1] = R[r][1] * sy; M[r][2] = R[r][2] * sz; }
        float Sg[3][3];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) Sg[a][b] = (M[a][0] * M[b][0] + M[a][1] * M[b][1]) + M[a][2] * M[b][2];
        float limx = 1.3f * tfx, limy = 1.3f * tfy;
        float txtz = pv[0] / d, tytz = pv[1] / d;
        float tx = mn(limx, mx(-limx, txtz)) * d, ty = mn(limy, mx(-limy, tytz)) * d;
        float J00 = fx / d, J02 = (fx * tx) / (d * d), J11 = fy / d, J12 = (fy * ty) / (d * d);
        float T0[3] = {J00 * Vm[0] + J02 * Vm[2], J00 * Vm[4] + J02 * Vm[6], J00 * Vm[8] + J02 * Vm[10]};
        float T1[3] = {J11 * Vm[1] + J12 * Vm[2], J11 * Vm[5] + J12 * Vm[6], J11 * Vm[9] + J12 * Vm[10]};
        float U0[3], U1[3];
        for (int b = 0; b < 3; ++b) {
            U0[b] = (T0[0] * Sg[0][b] + T0[1] * Sg[1][b]) + T0[2] * Sg[2][b];
            U1[b] = (T1[0] * Sg[0][b] + T1[1] * Sg[1][b]) + T1[2] * Sg[2][b];
        }
        float ca = ((U0[0] * T0[0] + U0[1] * T0[1]) + U0[2] * T0[2]) + 0.3f;
        float cb = (U0[0] * T1[0] + U0[1] * T1[1]) + U0[2] * T1[2];
        float cc = ((U1[0] * T1[0] + U1[1] * T1[1]) + U1[2] * T1[2]) + 0.3f;
        float det = ca * cc - cb * cb;
        if (det == 0.0f) continue;
        float di = 1.0f / det;
        float mid = 0.5f * (ca + cc);
        float disc = sqrtf(mx(0.1f, mid * mid - det));
        float l1 = mid + disc, l2 = mid - disc;
        float rad = ceilf(3.0f * sqrtf(mx(l1, l2)));
        float ix = ((px + 1.0f) * (float)W - 1.0f) * 0.5f, iy = ((py + 1.0f) * (float)H - 1.0f) * 0.5f;
        int r = (int)rad;
        int x0 = ndc_rect(ix, r, BX, gx, 0), y0 = ndc_rect(iy, r, BY, gy, 0);
        int x1 = ndc_rect(ix, r, BX, gx, 1), y1 = ndc_rect(iy, r, BY, gy, 1);
        if (y0 < (int)trow0) y0 = (int)trow0;
        if (y1 > (int)trow1) y1 = (int)trow1;
        if (tight) {
            const float skip = -(or_log2(255.0f * opac[i]) * 0.69314718055994531f) - 0.001f;
            const float sq = -2.0f * skip;
            if (!(sq > 0.0f)) continue;
            const float ex = sqrtf(sq * ca) * 1.01f + 0.01f, ey = sqrtf(sq * cc) * 1.01f + 0.01f;
            const int tx0 = (int)ceilf((ix - ex - (float)(BX - 1)) * (1.0f / (float)BX));
            const int tx1 = (int)floorf((ix + ex) * (1.0f / (float)BX)) + 1;
            const int ty0 = (int)ceilf((iy - ey - (float)(BY - 1)) * (1.0f / (float)BY));
            const int ty1 = (int)floorf((iy + ey) * (1.0f / (float)BY)) + 1;
            if (x0 < tx0) x0 = tx0;
            if (x1 > tx1) x1 = tx1;
            if (y0 < ty0) y0 = ty0;
            if (y1 > ty1) y1 = ty1;
        }
        if (x1 <= x0 || y1 <= y0) continue;
        rect[4 * i] = x0;
        rect[4 * i + 1] = y0;
        rect[4 * i + 2] = x1;
        rect[4 * i + 3] = y1;
        radii[i] = r;
        touched[i] = (uint32_t)((x1 - x0) * (y1 - y0));
        means2d[2 * i] = ix;
        means2d[2 * i + 1] = iy;
        depths[i] = d;
        conic[4 * i] = cc * di;
        conic[4 * i + 1] = -cb * di;
        conic[4 * i + 2] = ca * di;
        conic[4 * i + 3] = opac[i];
        K += touched[i];
    }
    OPair* pairs = (OPair*)malloc(sizeof(OPair) * (K ? K : 1));
    /* duplicate with keys: each Gaussian's pairs at the prefix of the counts (the order before the
     * total-order qsort below does not matter) */
    uint64_t* first = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)n + 1));
    first[0] = 0;
    for (uint32_t i = 0; i < n; ++i) first[i + 1] = first[i] + (radii[i] > 0 ? touched[i] : 0);
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
        const uint32_t i = (uint32_t)ii;
        uint64_t k = first[i];
        if (radii[i] <= 0) continue;
        const int x0 = rect[4 * i], y0 = rect[4 * i + 1], x1 = rect[4 * i + 2], y1 = rect[4 * i + 3];
        union { float f; uint32_t u; } db; db.f = depths[i];
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) {
                pairs[k].key = ((uint64_t)(uint32_t)(y * gx + x) << 32) | db.u;
                pairs[k].val = i;
                k++;
            }
    }
    free(first);
    free(rect);
    {   /* the total order of cmp_pair, tile by tile: bucket the pairs by tile (the key's high word),
         * then sort every tile's bucket with the same comparator in parallel (same result as one
         * qsort over all K pairs) */
        const uint32_t nt = (uint32_t)(gx * gy);
        uint64_t* start = (uint64_t*)calloc((size_t)nt + 1, sizeof(uint64_t));
        for (uint64_t j = 0; j < K; ++j) start[(uint32_t)(pairs[j].key >> 32) + 1]++;
        for (uint32_t t = 0; t < nt; ++t) start[t + 1] += start[t];
        uint64_t* cur = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)nt + 1));
        memcpy(cur, start, sizeof(uint64_t) * ((size_t)nt + 1));
        OPair* bucketed = (OPair*)malloc(sizeof(OPair) * (K ? K : 1));
        for (uint64_t j = 0; j < K; ++j) bucketed[cur[(uint32_t)(pairs[j].key >> 32)]++] = pairs[j];
        free(cur);
        free(pairs);
        pairs = bucketed;
#pragma omp parallel for schedule(dynamic, 16)
        for (int64_t t = 0; t < (int64_t)nt; ++t)
            if (start[t + 1] - start[t] > 1) qsort(pairs + start[t], (size_t)(start[t + 1] - start[t]), sizeof(OPair), cmp_pair);
        free(start);
    }
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (K ? K : 1));
    uint32_t* vals = (uint32_t*)malloc(sizeof(uint32_t) * (K ? K : 1));
    for (uint64_t j = 0; j < K; ++j) { keys[j] = pairs[j].key; vals[j] = pairs[j].val; }
    free(pairs);
    uint32_t tiles = (uint32_t)(gx * gy);
    memset(ranges, 0, sizeof(uint32_t) * 2 * tiles);
    for (uint64_t j = 0; j < K; ++j) {
        uint32_t t = (uint32_t)(keys[j] >> 32);
        if (j == 0 || (uint32_t)(keys[j - 1] >> 32) != t) ranges[2 * t] = (uint32_t)j;
        if (j == K - 1 || (uint32_t)(keys[j + 1] >> 32) != t) ranges[2 * t + 1] = (uint32_t)(j + 1);
    }
    /* blend: tiles are independent (OpenMP over the tiles of the rendered rows) */
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t tt = (int64_t)trow0 * gx; tt < (int64_t)trow1 * gx; ++tt) {
        {
            const uint32_t t = (uint32_t)tt, ty = t / (uint32_t)gx, tx = t % (uint32_t)gx;
            uint32_t s0 = ranges[2 * t], s1 = ranges[2 * t + 1];
            for (uint32_t ly = 0; ly < (uint32_t)BY; ++ly)
                for (uint32_t lx = 0; lx < (uint32_t)BX; ++lx) {
                    uint32_t px = tx * BX + lx, py = ty * BY + ly;
                    if (px >= W || py >= H) continue;
                    float T = 1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
                    size_t pix = (size_t)py * W + px;
                    for (uint32_t j = s0; j < s1; ++j) {
                        uint32_t g = vals[j];
                        if (depth_lim && !(depths[g] < depth_lim[pix])) break;
                        float dx = means2d[2 * g] - (float)px, dy = means2d[2 * g + 1] - (float)py;
                        const float* co = conic + 4 * g;
                        float power = -0.5f * ((co[0] * dx) * dx + (co[2] * dy) * dy) - (co[1] * dx) * dy;
                        if (power > 0.0f) continue;
                        float alpha = mn(0.99f, co[3] * or_exp(power));
                        if (alpha < 1.0f / 255.0f) continue;
                        float test_T = T * (1.0f - alpha);
                        if (test_T < 0.0001f) break;
                        C0 = C0 + (colors[3 * g] * alpha) * T;
                        C1 = C1 + (colors[3 * g + 1] * alpha) * T;
                        C2 = C2 + (colors[3 * g + 2] * alpha) * T;
                        T = test_T;
                    }
                    float* o = image + 4 * pix;
                    if (under) {
                        const float* u = under + 4 * pix;
                        o[0] = C0 + T * u[0];
                        o[1] = C1 + T * u[1];
                        o[2] = C2 + T * u[2];
                        o[3] = (1.0f - T) + T * u[3];
                    } else {
                        o[0] = C0 + T * bg[0];
                        o[1] = C1 + T * bg[1];
                        o[2] = C2 + T * bg[2];
                        o[3] = 1.0f - T;
                    }
                }
        }
    }
    *keys_out = keys;
    *vals_out = vals;
    return (int)K;
}

int oracle_splat_gaussians(const float* means, const float* scales, const float* rots, const float* opac,
                           const float* colors, uint32_t n, const ptgs_ubo* ubo, uint32_t W, uint32_t H,
                           const float* bg, const float* depth_lim, const float* under, uint32_t trow0, uint32_t trow1,
                           int32_t* radii, uint32_t* touched, float* means2d, float* depths, float* conic,
                           uint64_t** keys_out, uint32_t** vals_out, uint32_t* ranges, float* image) {
    return splat_gaussians_mode(means, scales, rots, opac, colors, n, ubo, W, H, bg, depth_lim, under, trow0, trow1, 0,
                                radii, touched, means2d, depths, conic, keys_out, vals_out, ranges, image);
}

int oracle_splat_gaussians_tight(const float* means, const float* scales, const float* rots, const float* opac,
                                 const float* colors, uint32_t n, const ptgs_ubo* ubo, uint32_t W, uint32_t H,
                                 const float* bg, const float* depth_lim, const float* under, uint32_t trow0,
                                 uint32_t trow1, int32_t* radii, uint32_t* touched, float* means2d, float* depths,
                                 float* conic, uint64_t** keys_out, uint32_t** vals_out, uint32_t* ranges, float* image) {
    return splat_gaussians_mode(means, scales, rots, opac, colors, n, ubo, W, H, bg, depth_lim, under, trow0, trow1, 1,
                                radii, touched, means2d, depths, conic, keys_out, vals_out, ranges, image);
}

/* ---------------------------------------------------------------------------------------------
 * 3DGS initialisation (Kerbl et al. 2023 create_from_pcd; the distCUDA2 3-NN term): brute force
 * over all pairs, O(N^2) — the checker for ptgs_knn3_mean_dist2 at small N. Same f32 expressions:
 * d = (dx*dx + dy*dy) + dz*dz, mean = ((b0 + b1) + b2) / 3; < 3 other points: mean of those; none: 0.
 * --------------------------------------------------------------------------------------------- */
void oracle_knn3_mean_dist2(const float* xyz, uint32_t n, float* dist2) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    float b0 = INFINITY, b1 = INFINITY, b2 = INFINITY;
    const float qx = xyz[3 * i], qy = xyz[3 * i + 1], qz = xyz[3 * i + 2];
    for (uint32_t j = 0; j < n; ++j) {
      if ((int64_t)j == i) continue;
      const float dx = xyz[3 * j] - qx, dy = xyz[3 * j + 1] - qy, dz = xyz[3 * j + 2] - qz;
      const float d = (dx * dx + dy * dy) + dz * dz;
      if (d < b2) {
        if (d < b1) {
          b2 = b1;
          if (d < b0) { b1 = b0; b0 = d; } else b1 = d;
        } else {
          b2 = d;
        }
      }
    }
    const uint32_t k = n - 1 < 3 ? n - 1 : 3;
    dist2[i] = k == 3 ? ((b0 + b1) + b2) / 3.0f : k == 2 ? (b0 + b1) / 2.0f : k == 1 ? b0 : 0.0f;
  }
}

void oracle_free(void* p) { free(p); }

/* exposes the math primitives for unit tests */
void oracle_sincos(float x, float* s, float* c) { or_sincos(x, s, c); }
float oracle_exp2(float x) { return or_exp2(x); }
float oracle_log2(float x) { return or_log2(x); }
