// PNG / JPEG -> RGBA8 decode for texture ingest (host side of the scene loader).
//
// Output semantics follow stbi_load(..., STBI_rgb_alpha) as the reference uses it for every glTF
// texture (Vulkan_Engine/image.cpp:12, stb_image v2.30):
//   PNG : 16-bit samples reduced by >> 8; sub-byte grey scaled by 0xff/0x55/0x11; grey/RGB tRNS
//         keys compared at the file's bit depth (8-bit keys use the low byte); palette alpha from
//         tRNS; Adam7 de-interlaced; grey -> (g, g, g, a).
//   JPEG: baseline + progressive Huffman; the jidctint-style integer IDCT with 12-bit constants
//         (pass 1 keeps 2 extra bits, pass 2 rounds at bit 17 with the +128 level shift folded in);
//         fixed-point YCbCr->RGB on 20 fractional bits with the green Cb term truncated to 16 bits;
//         "fancy" triangle-filter chroma upsampling for 2x1 / 1x2 / 2x2 and nearest otherwise,
//         with stb's row-phase state machine; Adobe APP14 transform 0 -> CMYK (x*k/255 "blinn"),
//         2 -> YCCK, component ids 'R','G','B' (or no JFIF and transform 0) -> RGB stored directly.
// The parsers (chunks, markers, Huffman / progressive scans, Adam7) are written from the format
// specifications (PNG ISO/IEC 15948, JPEG ITU T.81). The arithmetic that decides pixel values
// follows stb_image (the reference's vendored Helpers/stb_image.h, public domain) because the texels
// must equal stbi_load's: the integer IDCT (idct8x8 restates stbi__idct_block, stb_image.h:2426-2520:
// same constants, biases and output order), the fixed-point YCbCr->RGB and the chroma resamplers.
// Inflate is zlib's.
#include "image_decode.h"

#include <zlib.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstring>
#include <sys/stat.h>

namespace ptgs {

// regular files only (a directory opens as a stream and then throws from its first read); no
// exceptions (callers are behind the C-ABI)
bool read_file(const std::string& path, std::vector<uint8_t>& bytes) {
  bytes.clear();
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  struct stat st;
  bool ok = fstat(fileno(f), &st) == 0 && S_ISREG(st.st_mode) && st.st_size >= 0;
  if (ok) {
    try {
      bytes.resize((size_t)st.st_size);
    } catch (...) {
      ok = false;
    }
  }
  if (ok && !bytes.empty()) ok = fread(bytes.data(), 1, bytes.size(), f) == bytes.size();
  fclose(f);
  if (!ok) bytes.clear();
  return ok;
}

namespace {

inline uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | (uint32_t)p[3];
}
inline uint32_t be16(const uint8_t* p) { return (uint32_t)p[0] << 8 | (uint32_t)p[1]; }

// =============================================================================================
// PNG
// =============================================================================================
struct PngHeader {
  uint32_t w = 0, h = 0;
  int depth = 0, color = 0, interlace = 0;
  int channels = 0;  // samples per pixel in the file
};

int png_channels(int color) {
  switch (color) {
    case 0: return 1;
    case 2: return 3;
    case 3: return 1;
    case 4: return 2;
    case 6: return 4;
    default: return 0;
  }
}

bool png_depth_ok(int color, int depth) {
  switch (color) {
    case 0: return depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16;
    case 3: return depth == 1 || depth == 2 || depth == 4 || depth == 8;
    case 2: case 4: case 6: return depth == 8 || depth == 16;
    default: return false;
  }
}

inline size_t png_row_bytes(uint32_t w, const PngHeader& h) {
  return ((size_t)w * h.channels * h.depth + 7) / 8;
}

inline int paeth(int a, int b, int c) {
  int p = a + b - c;
  int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

// Undo the per-row filters in place. raw holds rows of (1 + rb) bytes; out gets rows of rb bytes.
bool png_unfilter(const uint8_t* raw, uint32_t rows, size_t rb, int bpp, std::vector<uint8_t>& out, std::string& err) {
  out.assign((size_t)rows * rb, 0);
  for (uint32_t y = 0; y < rows; ++y) {
    const uint8_t* src = raw + (size_t)y * (rb + 1);
    int f = src[0];
    ++src;
    uint8_t* cur = out.data() + (size_t)y * rb;
    const uint8_t* prev = y ? cur - rb : nullptr;
    const size_t k = std::min((size_t)bpp, rb);
    switch (f) {  // one loop per filter; the first bpp bytes have no left neighbour
      case 0: memcpy(cur, src, rb); break;
      case 1:
        memcpy(cur, src, k);
        for (size_t i = k; i < rb; ++i) cur[i] = (uint8_t)(src[i] + cur[i - bpp]);
        break;
      case 2:
        if (prev) for (size_t i = 0; i < rb; ++i) cur[i] = (uint8_t)(src[i] + prev[i]);
        else memcpy(cur, src, rb);
        break;
      case 3:
        if (prev) {
          for (size_t i = 0; i < k; ++i) cur[i] = (uint8_t)(src[i] + (prev[i] >> 1));
          for (size_t i = k; i < rb; ++i) cur[i] = (uint8_t)(src[i] + ((cur[i - bpp] + prev[i]) >> 1));
        } else {
          memcpy(cur, src, k);
          for (size_t i = k; i < rb; ++i) cur[i] = (uint8_t)(src[i] + (cur[i - bpp] >> 1));
        }
        break;
      case 4:
        if (prev) {
          for (size_t i = 0; i < k; ++i) cur[i] = (uint8_t)(src[i] + prev[i]);  // paeth(0, b, 0) = b
          for (size_t i = k; i < rb; ++i) cur[i] = (uint8_t)(src[i] + paeth(cur[i - bpp], prev[i], prev[i - bpp]));
        } else {  // paeth(a, 0, 0) = a
          memcpy(cur, src, k);
          for (size_t i = k; i < rb; ++i) cur[i] = (uint8_t)(src[i] + cur[i - bpp]);
        }
        break;
      default: err = "PNG: invalid filter type"; return false;
    }
  }
  return true;
}

bool decode_png(const uint8_t* d, size_t n, DecodedImage& out, std::string& err, bool header_only) {
  PngHeader H;
  bool have_ihdr = false, have_trns = false;
  uint8_t pal[256][4];
  for (auto& e : pal) { e[0] = e[1] = e[2] = 0; e[3] = 255; }
  uint32_t pal_len = 0;
  uint32_t trns_key[3] = {0, 0, 0};
  std::vector<uint8_t> idat;
  size_t pos = 8;
  bool iend = false;
  while (!iend) {
    if (pos + 8 > n) { err = "PNG: truncated chunk"; return false; }
    uint32_t len = be32(d + pos);
    const uint8_t* type = d + pos + 4;
    const uint8_t* body = d + pos + 8;
    if ((size_t)len > n - pos - 8) { err = "PNG: chunk overruns the file"; return false; }
    if (!memcmp(type, "IHDR", 4)) {
      if (len != 13) { err = "PNG: bad IHDR"; return false; }
      H.w = be32(body);
      H.h = be32(body + 4);
      H.depth = body[8];
      H.color = body[9];
      if (body[10] != 0 || body[11] != 0) { err = "PNG: bad compression/filter method"; return false; }
      H.interlace = body[12];
      if (H.interlace > 1) { err = "PNG: bad interlace method"; return false; }
      if (!H.w || !H.h || H.w > (1u << 24) || H.h > (1u << 24)) { err = "PNG: bad dimensions"; return false; }
      if (!png_depth_ok(H.color, H.depth)) { err = "PNG: unsupported colour type / bit depth"; return false; }
      H.channels = png_channels(H.color);
      have_ihdr = true;
      if (header_only) {
        out.w = H.w; out.h = H.h;
        out.comp = H.color == 3 ? 3 : (uint32_t)H.channels;  // refined by tRNS below when present
      }
    } else if (!memcmp(type, "PLTE", 4)) {
      if (len % 3 || len / 3 > 256 || len == 0) { err = "PNG: bad PLTE"; return false; }
      pal_len = len / 3;
      for (uint32_t i = 0; i < pal_len; ++i) {
        pal[i][0] = body[3 * i]; pal[i][1] = body[3 * i + 1]; pal[i][2] = body[3 * i + 2]; pal[i][3] = 255;
      }
    } else if (!memcmp(type, "tRNS", 4)) {
      if (!have_ihdr) { err = "PNG: tRNS before IHDR"; return false; }
      if (H.color == 3) {
        if (len > pal_len) { err = "PNG: bad tRNS length"; return false; }
        for (uint32_t i = 0; i < len; ++i) pal[i][3] = body[i];
      } else if (H.color == 0 || H.color == 2) {
        if (len != (uint32_t)H.channels * 2) { err = "PNG: bad tRNS length"; return false; }
        for (int k = 0; k < H.channels; ++k) trns_key[k] = be16(body + 2 * k);
      } else {
        err = "PNG: tRNS with an alpha channel";
        return false;
      }
      have_trns = true;
    } else if (!memcmp(type, "IDAT", 4)) {
      if (!have_ihdr) { err = "PNG: IDAT before IHDR"; return false; }
      if (header_only) break;
      idat.insert(idat.end(), body, body + len);
    } else if (!memcmp(type, "IEND", 4)) {
      iend = true;
    } else if (!(type[0] & 0x20)) {
      err = std::string("PNG: unsupported critical chunk ") + std::string((const char*)type, 4);
      return false;
    }
    pos += 12 + (size_t)len;
  }
  if (!have_ihdr) { err = "PNG: missing IHDR"; return false; }
  if (header_only) {
    if (have_trns) out.comp = H.color == 3 ? 4 : (uint32_t)H.channels + 1;
    return true;
  }
  if (H.color == 3 && pal_len == 0) { err = "PNG: palette image without PLTE"; return false; }

  // pass geometry (Adam7 or a single pass)
  static const int ax0[7] = {0, 4, 0, 2, 0, 1, 0}, ay0[7] = {0, 0, 4, 0, 2, 0, 1};
  static const int adx[7] = {8, 8, 4, 4, 2, 2, 1}, ady[7] = {8, 8, 8, 4, 4, 2, 2};
  int passes = H.interlace ? 7 : 1;
  uint32_t pw[7], ph[7];
  size_t need = 0;
  for (int p = 0; p < passes; ++p) {
    int x0 = H.interlace ? ax0[p] : 0, y0 = H.interlace ? ay0[p] : 0;
    int dx = H.interlace ? adx[p] : 1, dy = H.interlace ? ady[p] : 1;
    pw[p] = H.w > (uint32_t)x0 ? (H.w - x0 + dx - 1) / dx : 0;
    ph[p] = H.h > (uint32_t)y0 ? (H.h - y0 + dy - 1) / dy : 0;
    if (pw[p] && ph[p]) need += (size_t)ph[p] * (png_row_bytes(pw[p], H) + 1);
  }
  // bound the allocations by what the file can hold before making them: at most 2^28 pixels (as the
  // JPEG path), and deflate expands at most ~1032:1, so a short IDAT cannot describe a huge image
  if ((uint64_t)H.w * H.h > (1ull << 28)) { err = "PNG: image too large"; return false; }
  if (need > idat.size() * (size_t)1040 + 4096) { err = "PNG: not enough pixel data"; return false; }
  std::vector<uint8_t> raw(need);
  {
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) { err = "PNG: inflateInit failed"; return false; }
    zs.next_in = idat.data();
    zs.avail_in = (uInt)idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    int rc = inflate(&zs, Z_FINISH);
    size_t got = raw.size() - zs.avail_out;
    inflateEnd(&zs);
    // surplus data after the last row is ignored, as is a bad Adler-32 trailer (stb checks neither)
    if (rc == Z_STREAM_ERROR || rc == Z_MEM_ERROR) { err = "PNG: zlib failure"; return false; }
    if (got < need) { err = "PNG: not enough pixel data (corrupt zlib stream?)"; return false; }
  }

  out.w = H.w;
  out.h = H.h;
  out.comp = H.color == 3 ? (have_trns ? 4 : 3) : (uint32_t)H.channels + (have_trns ? 1 : 0);
  out.rgba.assign((size_t)H.w * H.h * 4, 0);
  const int scale = H.depth == 1 ? 0xff : H.depth == 2 ? 0x55 : H.depth == 4 ? 0x11 : 1;
  const int bpp = (H.channels * H.depth + 7) / 8;  // filter unit in bytes (>= 1)
  // 8-bit keys: low byte of the 16-bit field times the grey scale, truncated to a byte
  uint32_t key8[3];
  for (int k = 0; k < 3; ++k) key8[k] = (uint8_t)((trns_key[k] & 255) * scale);

  size_t off = 0;
  std::vector<uint8_t> rows;
  for (int p = 0; p < passes; ++p) {
    if (!pw[p] || !ph[p]) continue;
    size_t rb = png_row_bytes(pw[p], H);
    if (!png_unfilter(raw.data() + off, ph[p], rb, bpp, rows, err)) return false;
    off += (size_t)ph[p] * (rb + 1);
    int x0 = H.interlace ? ax0[p] : 0, y0 = H.interlace ? ay0[p] : 0;
    int dx = H.interlace ? adx[p] : 1, dy = H.interlace ? ady[p] : 1;
    for (uint32_t j = 0; j < ph[p]; ++j) {
      const uint8_t* row = rows.data() + (size_t)j * rb;
      if (H.depth == 8 && !H.interlace && (!have_trns || H.color == 3)) {  // common layouts, no key test
        uint8_t* o = out.rgba.data() + (size_t)j * H.w * 4;
        const uint8_t* q = row;
        switch (H.color) {
          case 2: for (uint32_t i = 0; i < H.w; ++i, o += 4, q += 3) { o[0] = q[0]; o[1] = q[1]; o[2] = q[2]; o[3] = 255; } break;
          case 6: memcpy(o, q, (size_t)H.w * 4); break;
          case 0: for (uint32_t i = 0; i < H.w; ++i, o += 4) { o[0] = o[1] = o[2] = q[i]; o[3] = 255; } break;
          case 4: for (uint32_t i = 0; i < H.w; ++i, o += 4, q += 2) { o[0] = o[1] = o[2] = q[0]; o[3] = q[1]; } break;
          default: for (uint32_t i = 0; i < H.w; ++i, o += 4) memcpy(o, pal[q[i]], 4);
        }
        continue;
      }
      auto sample = [&](size_t idx) -> uint32_t {
        if (H.depth == 16) return be16(row + 2 * idx);
        if (H.depth == 8) return row[idx];
        size_t bit = idx * H.depth;
        return (row[bit >> 3] >> (8 - H.depth - (int)(bit & 7))) & ((1u << H.depth) - 1);
      };
      for (uint32_t i = 0; i < pw[p]; ++i) {
        uint8_t* o = out.rgba.data() + (((size_t)(y0 + j * dy)) * H.w + (x0 + i * dx)) * 4;
        size_t s0 = (size_t)i * H.channels;
        switch (H.color) {
          case 3: {
            uint32_t ix = sample(s0);
            memcpy(o, pal[ix & 255], 4);
            break;
          }
          case 0: {
            uint32_t g = sample(s0);
            uint8_t g8 = H.depth == 16 ? (uint8_t)(g >> 8) : (uint8_t)(g * scale);
            bool clear = have_trns && (H.depth == 16 ? g == trns_key[0] : g8 == key8[0]);
            o[0] = o[1] = o[2] = g8;
            o[3] = clear ? 0 : 255;
            break;
          }
          case 2: {
            uint32_t r = sample(s0), g = sample(s0 + 1), b = sample(s0 + 2);
            uint8_t c[3];
            bool clear;
            if (H.depth == 16) {
              c[0] = (uint8_t)(r >> 8); c[1] = (uint8_t)(g >> 8); c[2] = (uint8_t)(b >> 8);
              clear = have_trns && r == trns_key[0] && g == trns_key[1] && b == trns_key[2];
            } else {
              c[0] = (uint8_t)r; c[1] = (uint8_t)g; c[2] = (uint8_t)b;
              clear = have_trns && c[0] == key8[0] && c[1] == key8[1] && c[2] == key8[2];
            }
            o[0] = c[0]; o[1] = c[1]; o[2] = c[2];
            o[3] = clear ? 0 : 255;
            break;
          }
          case 4: {
            uint32_t g = sample(s0), a = sample(s0 + 1);
            uint8_t g8 = H.depth == 16 ? (uint8_t)(g >> 8) : (uint8_t)g;
            o[0] = o[1] = o[2] = g8;
            o[3] = H.depth == 16 ? (uint8_t)(a >> 8) : (uint8_t)a;
            break;
          }
          default: {  // 6
            for (int k = 0; k < 4; ++k) {
              uint32_t v = sample(s0 + k);
              o[k] = H.depth == 16 ? (uint8_t)(v >> 8) : (uint8_t)v;
            }
          }
        }
      }
    }
  }
  return true;
}

// =============================================================================================
// JPEG
// =============================================================================================
// natural-order position of zig-zag index k; indices past 63 (corrupt run lengths) land on 63
const uint8_t kZigzag[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct HuffTable {
  bool defined = false;
  uint8_t vals[256];
  int32_t maxcode[18];  // largest code of each length (+1 sentinel), -1 if none
  int32_t valoff[17];   // vals index of the first code of each length minus that code
  uint16_t look[1 << 9];  // (length << 8) | value for codes up to 9 bits, 0 = slow path
};

bool build_huff(HuffTable& t, const uint8_t counts[16], const uint8_t* vals, int nvals) {
  memcpy(t.vals, vals, nvals);
  memset(t.look, 0, sizeof(t.look));
  int code = 0, k = 0;
  for (int len = 1; len <= 16; ++len) {
    t.valoff[len] = k - code;
    int c = counts[len - 1];
    if (c) {
      for (int i = 0; i < c; ++i, ++k, ++code) {
        if (code >= (1 << len) || k >= nvals) return false;  // over-subscribed lengths (corrupt DHT)
        if (len <= 9) {
          int shift = 9 - len;
          for (int f = 0; f < (1 << shift); ++f) t.look[(code << shift) | f] = (uint16_t)(len << 8 | t.vals[k]);
        }
      }
      t.maxcode[len] = code - 1;
      if (code - 1 >= (1 << len)) return false;
    } else {
      t.maxcode[len] = -1;
    }
    code <<= 1;
  }
  t.maxcode[17] = INT32_MAX;
  t.defined = true;
  return true;
}

struct Component {
  int id = 0, h = 1, v = 1, tq = 0;
  int td = 0, ta = 0;
  int dc_pred = 0;
  int x = 0, y = 0;    // samples covered by this component
  int w2 = 0, h2 = 0;  // padded plane size (whole MCUs)
  std::vector<uint8_t> plane;
  std::vector<int16_t> coef;  // progressive: (w2/8) * (h2/8) blocks of 64 natural-order coefficients
};

class JpegDecoder {
 public:
  JpegDecoder(const uint8_t* d, size_t n) : p_(d), end_(d + n) {}
  bool decode(DecodedImage& out, std::string& err, bool header_only);

 private:
  const uint8_t* p_;
  const uint8_t* end_;
  // entropy-coded segment reader
  uint32_t bits_ = 0;
  int nbits_ = 0;
  int marker_ = -1;  // marker met inside entropy data (-1: none)
  bool nomore_ = false;

  uint16_t q_[4][64];
  HuffTable hdc_[4], hac_[4];
  Component comp_[4];
  int ncomp_ = 0;
  int W_ = 0, H_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
  bool progressive_ = false, have_frame_ = false;
  int restart_ = 0;
  bool jfif_ = false;
  int app14_ = -1;
  int rgb_ids_ = 0;
  // current scan
  int sn_ = 0, sorder_[4];
  int ss_ = 0, se_ = 63, ah_ = 0, al_ = 0;
  int eobrun_ = 0;
  int todo_ = 0;
  std::string* err_ = nullptr;

  bool fail(const char* m) { *err_ = std::string("JPEG: ") + m; return false; }
  int byte() { return p_ < end_ ? *p_++ : -1; }

  void fill() {
    while (nbits_ <= 24) {
      uint32_t b = 0;
      if (!nomore_) {
        int c = byte();
        if (c < 0) { nomore_ = true; c = 0; }
        else if (c == 0xFF) {
          int m = byte();
          while (m == 0xFF) m = byte();
          if (m != 0) {
            marker_ = m < 0 ? -1 : m;
            nomore_ = true;
            c = 0;
          }
        }
        b = (uint32_t)c;
      }
      bits_ |= b << (24 - nbits_);
      nbits_ += 8;
    }
  }
  int getbits(int n) {  // n <= 16
    if (nbits_ < n) fill();
    uint32_t v = bits_ >> (32 - n);
    bits_ <<= n;
    nbits_ -= n;
    return (int)v;
  }
  int getbit() { return getbits(1); }
  int extend(int s) {  // receive s magnitude bits and sign-extend (T.81 F.2.2.1)
    if (s == 0) return 0;
    int v = getbits(s);
    return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v;
  }
  int huff(const HuffTable& t) {
    if (nbits_ < 16) fill();
    uint32_t top = bits_ >> (32 - 9);
    uint16_t e = t.look[top];
    if (e) {
      int len = e >> 8;
      bits_ <<= len;
      nbits_ -= len;
      return e & 255;
    }
    uint32_t code16 = bits_ >> 16;
    for (int len = 10; len <= 16; ++len) {
      int32_t c = (int32_t)(code16 >> (16 - len));
      if (c <= t.maxcode[len]) {
        bits_ <<= len;
        nbits_ -= len;
        int idx = t.valoff[len] + c;
        return (idx >= 0 && idx < 256) ? t.vals[idx] : -1;
      }
    }
    return -1;
  }
  void reset_entropy() {
    bits_ = 0; nbits_ = 0; nomore_ = false; marker_ = -1;
    for (int i = 0; i < ncomp_; ++i) comp_[i].dc_pred = 0;
    eobrun_ = 0;
    todo_ = restart_ ? restart_ : INT_MAX;
  }

  bool read_segment(std::vector<uint8_t>& seg) {
    if (end_ - p_ < 2) return fail("truncated segment");
    int L = (int)be16(p_);
    if (L < 2 || end_ - p_ < L) return fail("bad segment length");
    seg.assign(p_ + 2, p_ + L);
    p_ += L;
    return true;
  }
  bool frame(const std::vector<uint8_t>& s);
  bool scan_header(const std::vector<uint8_t>& s);
  bool scan();
  bool block_baseline(Component& c, int16_t* data);
  bool block_dc_prog(Component& c, int16_t* data);
  bool block_ac_prog(Component& c, int16_t* data);
  void finish_progressive();
  void output(DecodedImage& out);
};

// jidctint-style 8x8 integer IDCT on dequantised coefficients (stb_image.h stbi__idct_block:
// same constants, biases and output order); writes 8 bytes per row. 64-bit intermediates: a corrupt
// stream can carry coefficients whose 32-bit products overflow (valid data never does, so the
// results equal the 32-bit ones)
inline int64_t fx(float x) { return (int64_t)(x * 4096 + 0.5); }
#define PTGS_IDCT_1D(s0, s1, s2, s3, s4, s5, s6, s7)                                        \
  int64_t e2 = s2, e6 = s6;                                                                    \
  int64_t z1 = (e2 + e6) * fx(0.5411961f);                                                     \
  int64_t ev2 = z1 + e6 * fx(-1.847759065f);                                                   \
  int64_t ev3 = z1 + e2 * fx(0.765366865f);                                                    \
  int64_t ev0 = (s0 + s4) * 4096, ev1 = (s0 - s4) * 4096;                                      \
  int64_t a0 = ev0 + ev3, a3 = ev0 - ev3, a1 = ev1 + ev2, a2 = ev1 - ev2;                      \
  int64_t o7 = s7, o5 = s5, o3 = s3, o1 = s1;                                                  \
  int64_t q3 = o7 + o3, q4 = o5 + o1, q1 = o7 + o1, q2 = o5 + o3;                              \
  int64_t q5 = (q3 + q4) * fx(1.175875602f);                                                   \
  o7 = o7 * fx(0.298631336f);                                                              \
  o5 = o5 * fx(2.053119869f);                                                              \
  o3 = o3 * fx(3.072711026f);                                                              \
  o1 = o1 * fx(1.501321110f);                                                              \
  q1 = q5 + q1 * fx(-0.899976223f);                                                        \
  q2 = q5 + q2 * fx(-2.562915447f);                                                        \
  q3 = q3 * fx(-1.961570560f);                                                             \
  q4 = q4 * fx(-0.390180644f);                                                             \
  o1 += q1 + q4;                                                                           \
  o3 += q2 + q3;                                                                           \
  o5 += q2 + q4;                                                                           \
  o7 += q1 + q3;

inline uint8_t clamp255(int64_t x) { return (uint8_t)(x < 0 ? 0 : (x > 255 ? 255 : x)); }

void idct8x8(uint8_t* out, int stride, const int16_t* d) {
  int64_t tmp[64];
  for (int c = 0; c < 8; ++c) {
    const int16_t* col = d + c;
    PTGS_IDCT_1D(col[0], col[8], col[16], col[24], col[32], col[40], col[48], col[56])
    a0 += 512; a1 += 512; a2 += 512; a3 += 512;
    tmp[c] = (a0 + o1) >> 10;
    tmp[c + 56] = (a0 - o1) >> 10;
    tmp[c + 8] = (a1 + o3) >> 10;
    tmp[c + 48] = (a1 - o3) >> 10;
    tmp[c + 16] = (a2 + o5) >> 10;
    tmp[c + 40] = (a2 - o5) >> 10;
    tmp[c + 24] = (a3 + o7) >> 10;
    tmp[c + 32] = (a3 - o7) >> 10;
  }
  for (int r = 0; r < 8; ++r) {
    const int64_t* t = tmp + 8 * r;
    uint8_t* o = out + (size_t)r * stride;
    PTGS_IDCT_1D(t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7])
    const int64_t bias = 65536 + (128 << 17);
    a0 += bias; a1 += bias; a2 += bias; a3 += bias;
    o[0] = clamp255((a0 + o1) >> 17);
    o[7] = clamp255((a0 - o1) >> 17);
    o[1] = clamp255((a1 + o3) >> 17);
    o[6] = clamp255((a1 - o3) >> 17);
    o[2] = clamp255((a2 + o5) >> 17);
    o[5] = clamp255((a2 - o5) >> 17);
    o[3] = clamp255((a3 + o7) >> 17);
    o[4] = clamp255((a3 - o7) >> 17);
  }
}
#undef PTGS_IDCT_1D

bool JpegDecoder::frame(const std::vector<uint8_t>& s) {
  if (have_frame_) return fail("multiple frames");
  if (s.size() < 6) return fail("bad SOF");
  if (s[0] != 8) return fail("only 8-bit samples are supported");
  H_ = (int)be16(&s[1]);
  W_ = (int)be16(&s[3]);
  ncomp_ = s[5];
  if (!H_ || !W_) return fail("zero-sized frame (DNL unsupported)");
  if (ncomp_ != 1 && ncomp_ != 3 && ncomp_ != 4) return fail("unsupported component count");
  if (s.size() < 6 + 3 * (size_t)ncomp_) return fail("bad SOF length");
  rgb_ids_ = 0;
  hmax_ = vmax_ = 1;
  for (int i = 0; i < ncomp_; ++i) {
    Component& c = comp_[i];
    c.id = s[6 + 3 * i];
    if (ncomp_ == 3 && c.id == "RGB"[i]) ++rgb_ids_;
    c.h = s[7 + 3 * i] >> 4;
    c.v = s[7 + 3 * i] & 15;
    c.tq = s[8 + 3 * i];
    if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4) return fail("bad sampling factors");
    if (c.tq > 3) return fail("bad quantisation table id");
    hmax_ = std::max(hmax_, c.h);
    vmax_ = std::max(vmax_, c.v);
  }
  for (int i = 0; i < ncomp_; ++i)
    if (hmax_ % comp_[i].h || vmax_ % comp_[i].v) return fail("non-integer subsampling ratio");
  if ((int64_t)W_ * H_ > (int64_t)1 << 28) return fail("image too large");
  mcux_ = (W_ + 8 * hmax_ - 1) / (8 * hmax_);
  mcuy_ = (H_ + 8 * vmax_ - 1) / (8 * vmax_);
  for (int i = 0; i < ncomp_; ++i) {
    Component& c = comp_[i];
    c.x = (W_ * c.h + hmax_ - 1) / hmax_;
    c.y = (H_ * c.v + vmax_ - 1) / vmax_;
    c.w2 = mcux_ * c.h * 8;
    c.h2 = mcuy_ * c.v * 8;
    c.plane.assign((size_t)c.w2 * c.h2, 0);
    if (progressive_) c.coef.assign((size_t)c.w2 * c.h2, 0);
  }
  have_frame_ = true;
  return true;
}

bool JpegDecoder::scan_header(const std::vector<uint8_t>& s) {
  if (!have_frame_) return fail("scan before frame");
  if (s.empty()) return fail("bad SOS");
  sn_ = s[0];
  if (sn_ < 1 || sn_ > 4 || sn_ > ncomp_ || s.size() != 4 + 2 * (size_t)sn_) return fail("bad SOS");
  for (int i = 0; i < sn_; ++i) {
    int id = s[1 + 2 * i], t = s[2 + 2 * i];
    int k = -1;
    for (int j = 0; j < ncomp_; ++j)
      if (comp_[j].id == id) k = j;
    if (k < 0) return fail("scan references an unknown component");
    comp_[k].td = t >> 4;
    comp_[k].ta = t & 15;
    if (comp_[k].td > 3 || comp_[k].ta > 3) return fail("bad Huffman table id");
    sorder_[i] = k;
  }
  ss_ = s[1 + 2 * sn_];
  se_ = s[2 + 2 * sn_];
  ah_ = s[3 + 2 * sn_] >> 4;
  al_ = s[3 + 2 * sn_] & 15;
  if (progressive_) {
    if (ss_ > 63 || se_ > 63 || ss_ > se_ || ah_ > 13 || al_ > 13) return fail("bad progressive scan parameters");
  } else {
    if (ss_ != 0 || ah_ != 0 || al_ != 0) return fail("bad baseline scan parameters");
    se_ = 63;
  }
  return true;
}

bool JpegDecoder::block_baseline(Component& c, int16_t* data) {
  const HuffTable& dc = hdc_[c.td];
  const HuffTable& ac = hac_[c.ta];
  if (!dc.defined || !ac.defined) return fail("missing Huffman table");
  int t = huff(dc);
  if (t < 0 || t > 15) return fail("bad Huffman code");
  memset(data, 0, 64 * sizeof(int16_t));
  int diff = extend(t);
  c.dc_pred += diff;
  const uint16_t* q = q_[c.tq];
  int dcq = c.dc_pred * (int)q[0];
  if (dcq < -32768 || dcq > 32767) return fail("DC coefficient overflow");
  data[0] = (int16_t)dcq;
  int k = 1;
  do {
    int rs = huff(ac);
    if (rs < 0) return fail("bad Huffman code");
    int s = rs & 15, r = rs >> 4;
    if (s == 0) {
      if (rs != 0xF0) break;
      k += 16;
    } else {
      k += r;
      int z = kZigzag[k++];
      data[z] = (int16_t)(extend(s) * (int)q[z]);
    }
  } while (k < 64);
  return true;
}

bool JpegDecoder::block_dc_prog(Component& c, int16_t* data) {
  if (se_ != 0) return fail("progressive scan mixes DC and AC");
  if (ah_ == 0) {
    const HuffTable& dc = hdc_[c.td];
    if (!dc.defined) return fail("missing Huffman table");
    memset(data, 0, 64 * sizeof(int16_t));
    int t = huff(dc);
    if (t < 0 || t > 15) return fail("bad Huffman code");
    c.dc_pred += extend(t);
    data[0] = (int16_t)(c.dc_pred * (1 << al_));
  } else if (getbit()) {
    data[0] = (int16_t)(data[0] + (1 << al_));
  }
  return true;
}

bool JpegDecoder::block_ac_prog(Component& c, int16_t* data) {
  if (ss_ == 0) return fail("progressive scan mixes DC and AC");
  const HuffTable& ac = hac_[c.ta];
  if (!ac.defined) return fail("missing Huffman table");
  if (ah_ == 0) {  // first pass over this band (T.81 G.1.2.2)
    if (eobrun_) { --eobrun_; return true; }
    int k = ss_;
    do {
      int rs = huff(ac);
      if (rs < 0) return fail("bad Huffman code");
      int s = rs & 15, r = rs >> 4;
      if (s == 0) {
        if (r < 15) {
          eobrun_ = (1 << r);
          if (r) eobrun_ += getbits(r);
          --eobrun_;
          break;
        }
        k += 16;
      } else {
        k += r;
        data[kZigzag[k++]] = (int16_t)(extend(s) * (1 << al_));
      }
    } while (k <= se_);
    return true;
  }
  // refinement (T.81 G.1.2.3): correction bits for non-zero coefficients, new +-1 coefficients
  const int16_t bit = (int16_t)(1 << al_);
  auto refine = [&](int16_t* q) {
    if (getbit() && (*q & bit) == 0) *q = (int16_t)(*q > 0 ? *q + bit : *q - bit);
  };
  int k = ss_;
  if (eobrun_) {
    --eobrun_;
    for (; k <= se_; ++k) {
      int16_t* q = &data[kZigzag[k]];
      if (*q) refine(q);
    }
    return true;
  }
  do {
    int rs = huff(ac);
    if (rs < 0) return fail("bad Huffman code");
    int s = rs & 15, r = rs >> 4;
    int val = 0;
    if (s == 0) {
      if (r < 15) {
        eobrun_ = (1 << r) - 1;
        if (r) eobrun_ += getbits(r);
        r = 64;  // the rest of the band only gets correction bits
      }
    } else {
      if (s != 1) return fail("bad refinement code");
      val = getbit() ? bit : -bit;
    }
    while (k <= se_) {
      int16_t* q = &data[kZigzag[k++]];
      if (*q) {
        refine(q);
      } else {
        if (r == 0) { *q = (int16_t)val; break; }
        --r;
      }
    }
  } while (k <= se_);
  return true;
}

bool JpegDecoder::scan() {
  reset_entropy();
  int16_t blk[64];
  auto restart_check = [&]() -> int {  // 1 continue, 0 end of scan
    if (--todo_ <= 0) {
      if (nbits_ < 24) fill();
      if (!(marker_ >= 0xD0 && marker_ <= 0xD7)) return 0;
      reset_entropy();
    }
    return 1;
  };
  if (sn_ == 1) {
    Component& c = comp_[sorder_[0]];
    int bw = (c.x + 7) >> 3, bh = (c.y + 7) >> 3;
    for (int j = 0; j < bh; ++j)
      for (int i = 0; i < bw; ++i) {
        if (!progressive_) {
          if (!block_baseline(c, blk)) return false;
          idct8x8(c.plane.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, blk);
        } else {
          int16_t* d = c.coef.data() + 64 * ((size_t)i + (size_t)j * (c.w2 / 8));
          if (!(ss_ == 0 ? block_dc_prog(c, d) : block_ac_prog(c, d))) return false;
        }
        if (!restart_check()) return true;
      }
    return true;
  }
  for (int j = 0; j < mcuy_; ++j)
    for (int i = 0; i < mcux_; ++i) {
      for (int k = 0; k < sn_; ++k) {
        Component& c = comp_[sorder_[k]];
        for (int y = 0; y < c.v; ++y)
          for (int x = 0; x < c.h; ++x) {
            int bx = i * c.h + x, by = j * c.v + y;
            if (!progressive_) {
              if (!block_baseline(c, blk)) return false;
              idct8x8(c.plane.data() + (size_t)c.w2 * by * 8 + bx * 8, c.w2, blk);
            } else {
              if (ss_ != 0) return fail("interleaved AC scan");
              int16_t* d = c.coef.data() + 64 * ((size_t)bx + (size_t)by * (c.w2 / 8));
              if (!block_dc_prog(c, d)) return false;
            }
          }
      }
      if (!restart_check()) return true;
    }
  return true;
}

void JpegDecoder::finish_progressive() {
  int16_t blk[64];
  for (int n = 0; n < ncomp_; ++n) {
    Component& c = comp_[n];
    int bw = (c.x + 7) >> 3, bh = (c.y + 7) >> 3;
    const uint16_t* q = q_[c.tq];
    for (int j = 0; j < bh; ++j)
      for (int i = 0; i < bw; ++i) {
        const int16_t* d = c.coef.data() + 64 * ((size_t)i + (size_t)j * (c.w2 / 8));
        for (int k = 0; k < 64; ++k) blk[k] = (int16_t)(d[k] * (int)q[k]);
        idct8x8(c.plane.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, blk);
      }
  }
}

inline uint8_t blinn(int x, int y) {  // x * y / 255, rounded
  unsigned t = (unsigned)(x * y + 128);
  return (uint8_t)((t + (t >> 8)) >> 8);
}

void JpegDecoder::output(DecodedImage& out) {
  out.w = (uint32_t)W_;
  out.h = (uint32_t)H_;
  out.comp = (uint32_t)ncomp_;
  out.rgba.assign((size_t)W_ * H_ * 4, 0);
  const bool is_rgb = ncomp_ == 3 && (rgb_ids_ == 3 || (app14_ == 0 && !jfif_));
  struct Phase {
    int hs, vs, ystep, ypos, wlo;
    const uint8_t *l0, *l1;
    std::vector<uint8_t> buf;
  } ph[4];
  for (int k = 0; k < ncomp_; ++k) {
    Phase& r = ph[k];
    r.hs = hmax_ / comp_[k].h;
    r.vs = vmax_ / comp_[k].v;
    r.ystep = r.vs >> 1;
    r.wlo = (W_ + r.hs - 1) / r.hs;
    r.ypos = 0;
    r.l0 = r.l1 = comp_[k].plane.data();
    r.buf.assign((size_t)W_ + 3 + 8, 0);
  }
  auto resample = [](Phase& r, const uint8_t* nr, const uint8_t* fr) -> const uint8_t* {
    uint8_t* o = r.buf.data();
    const int w = r.wlo;
    if (r.hs == 1 && r.vs == 1) return nr;
    if (r.hs == 1 && r.vs == 2) {
      for (int i = 0; i < w; ++i) o[i] = (uint8_t)((3 * nr[i] + fr[i] + 2) >> 2);
      return o;
    }
    if (r.hs == 2 && r.vs == 1) {
      if (w == 1) { o[0] = o[1] = nr[0]; return o; }
      o[0] = nr[0];
      o[1] = (uint8_t)((nr[0] * 3 + nr[1] + 2) >> 2);
      int i = 1;
      for (; i < w - 1; ++i) {
        int n3 = 3 * nr[i] + 2;
        o[2 * i] = (uint8_t)((n3 + nr[i - 1]) >> 2);
        o[2 * i + 1] = (uint8_t)((n3 + nr[i + 1]) >> 2);
      }
      o[2 * i] = (uint8_t)((nr[w - 2] * 3 + nr[w - 1] + 2) >> 2);
      o[2 * i + 1] = nr[w - 1];
      return o;
    }
    if (r.hs == 2 && r.vs == 2) {
      if (w == 1) { o[0] = o[1] = (uint8_t)((3 * nr[0] + fr[0] + 2) >> 2); return o; }
      int t1 = 3 * nr[0] + fr[0];
      o[0] = (uint8_t)((t1 + 2) >> 2);
      for (int i = 1; i < w; ++i) {
        int t0 = t1;
        t1 = 3 * nr[i] + fr[i];
        o[2 * i - 1] = (uint8_t)((3 * t0 + t1 + 8) >> 4);
        o[2 * i] = (uint8_t)((3 * t1 + t0 + 8) >> 4);
      }
      o[2 * w - 1] = (uint8_t)((t1 + 2) >> 2);
      return o;
    }
    for (int i = 0; i < w; ++i)
      for (int j = 0; j < r.hs; ++j) o[i * r.hs + j] = nr[i];
    return o;
  };
  const uint8_t* row[4];
  for (int y = 0; y < H_; ++y) {
    for (int k = 0; k < ncomp_; ++k) {
      Phase& r = ph[k];
      bool bot = r.ystep >= (r.vs >> 1);
      row[k] = resample(r, bot ? r.l1 : r.l0, bot ? r.l0 : r.l1);
      if (++r.ystep >= r.vs) {
        r.ystep = 0;
        r.l0 = r.l1;
        if (++r.ypos < comp_[k].y) r.l1 += comp_[k].w2;
      }
    }
    uint8_t* o = out.rgba.data() + (size_t)y * W_ * 4;
    auto ycc = [&](int i, uint8_t* px) {
      // 20-bit fixed point; the Cb contribution to green is truncated to its top 16 bits
      const int kr = ((int)(1.40200f * 4096.0f + 0.5f)) << 8, kgr = ((int)(0.71414f * 4096.0f + 0.5f)) << 8;
      const int kgb = ((int)(0.34414f * 4096.0f + 0.5f)) << 8, kb = ((int)(1.77200f * 4096.0f + 0.5f)) << 8;
      int yf = (row[0][i] << 20) + (1 << 19);
      int cr = row[2][i] - 128, cb = row[1][i] - 128;
      int R = (yf + cr * kr) >> 20;
      int G = (yf + cr * -kgr + (int)((unsigned)(cb * -kgb) & 0xffff0000u)) >> 20;
      int B = (yf + cb * kb) >> 20;
      px[0] = clamp255(R); px[1] = clamp255(G); px[2] = clamp255(B);
    };
    for (int i = 0; i < W_; ++i, o += 4) {
      if (ncomp_ == 3) {
        if (is_rgb) { o[0] = row[0][i]; o[1] = row[1][i]; o[2] = row[2][i]; }
        else ycc(i, o);
      } else if (ncomp_ == 4) {
        if (app14_ == 0) {
          int m = row[3][i];
          o[0] = blinn(row[0][i], m); o[1] = blinn(row[1][i], m); o[2] = blinn(row[2][i], m);
        } else if (app14_ == 2) {
          ycc(i, o);
          int m = row[3][i];
          o[0] = blinn(255 - o[0], m); o[1] = blinn(255 - o[1], m); o[2] = blinn(255 - o[2], m);
        } else {
          ycc(i, o);
        }
      } else {
        o[0] = o[1] = o[2] = row[0][i];
      }
      o[3] = 255;
    }
  }
}

bool JpegDecoder::decode(DecodedImage& out, std::string& err, bool header_only) {
  err_ = &err;
  if (end_ - p_ < 2 || p_[0] != 0xFF || p_[1] != 0xD8) return fail("missing SOI");
  p_ += 2;
  std::vector<uint8_t> seg;
  int m = -1;
  auto next_marker = [&]() -> int {
    if (marker_ >= 0) { int r = marker_; marker_ = -1; return r; }
    int c = byte();
    while (c >= 0 && c != 0xFF) c = byte();  // tolerate fill / stray bytes between segments
    while (c == 0xFF) c = byte();
    return c;
  };
  bool scanned = false;
  for (;;) {
    m = next_marker();
    if (m < 0) {
      if (scanned && have_frame_) break;  // missing EOI: keep what was decoded
      return fail("unexpected end of data");
    }
    if (m == 0xD9) break;
    if (m == 0xC0 || m == 0xC1 || m == 0xC2) {
      progressive_ = (m == 0xC2);
      if (!read_segment(seg) || !frame(seg)) return false;
      if (header_only) {
        out.w = (uint32_t)W_; out.h = (uint32_t)H_; out.comp = (uint32_t)ncomp_;
        return true;
      }
    } else if ((m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC)) {
      return fail("unsupported JPEG process (lossless / hierarchical / arithmetic)");
    } else if (m == 0xCC) {
      return fail("arithmetic coding is not supported");
    } else if (m == 0xC4) {
      if (!read_segment(seg)) return false;
      size_t q = 0;
      while (q < seg.size()) {
        if (seg.size() - q < 17) return fail("bad DHT");
        int tc = seg[q] >> 4, th = seg[q] & 15;
        if (tc > 1 || th > 3) return fail("bad DHT table id");
        int total = 0;
        for (int i = 0; i < 16; ++i) total += seg[q + 1 + i];
        if (total > 256 || seg.size() - q - 17 < (size_t)total) return fail("bad DHT length");
        if (!build_huff(tc ? hac_[th] : hdc_[th], &seg[q + 1], &seg[q + 17], total)) return fail("bad Huffman table");
        q += 17 + (size_t)total;
      }
    } else if (m == 0xDB) {
      if (!read_segment(seg)) return false;
      size_t q = 0;
      while (q < seg.size()) {
        int pq = seg[q] >> 4, tq = seg[q] & 15;
        if (pq > 1 || tq > 3) return fail("bad DQT");
        size_t need = 1 + 64 * (pq ? 2 : 1);
        if (seg.size() - q < need) return fail("bad DQT length");
        for (int i = 0; i < 64; ++i)
          q_[tq][kZigzag[i]] = (uint16_t)(pq ? be16(&seg[q + 1 + 2 * i]) : seg[q + 1 + i]);
        q += need;
      }
    } else if (m == 0xDD) {
      if (!read_segment(seg)) return false;
      if (seg.size() != 2) return fail("bad DRI");
      restart_ = (int)be16(seg.data());
    } else if (m == 0xDA) {
      if (!read_segment(seg) || !scan_header(seg)) return false;
      if (!scan()) return false;
      scanned = true;
      if (marker_ < 0) {  // entropy data ended without the reader meeting the next marker
        while (p_ < end_) {
          if (*p_++ == 0xFF && p_ < end_) { marker_ = *p_++; break; }
        }
      }
    } else if (m >= 0xD0 && m <= 0xD7) {
      // stray restart marker between segments: nothing to read
    } else if (m == 0xD8) {
      return fail("nested SOI");
    } else {
      if (!read_segment(seg)) return false;
      if (m == 0xE0 && seg.size() >= 5 && !memcmp(seg.data(), "JFIF\0", 5)) jfif_ = true;
      if (m == 0xEE && seg.size() >= 12 && !memcmp(seg.data(), "Adobe\0", 6)) app14_ = seg[11];
    }
  }
  if (!have_frame_) return fail("no frame");
  if (progressive_) finish_progressive();
  output(out);
  return true;
}

}  // namespace

bool decode_image_rgba8(const uint8_t* data, size_t size, DecodedImage& out, std::string& err, bool header_only) {
  out = DecodedImage();
  static const uint8_t png_sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (!data || size < 4) { err = "image: empty input"; return false; }
  if (size >= 8 && !memcmp(data, png_sig, 8)) return decode_png(data, size, out, err, header_only);
  if (data[0] == 0xFF && data[1] == 0xD8) {
    JpegDecoder j(data, size);
    return j.decode(out, err, header_only);
  }
  err = "image: unknown format (PNG and JPEG are supported)";
  return false;
}

}  // namespace ptgs
