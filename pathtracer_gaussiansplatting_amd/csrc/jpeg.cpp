// jpeg.cpp — baseline JFIF encoder for the capture pipeline (the reference writes dataset images
// with stbi_write_jpg, quality 90, Helpers/GeneralHeaders.cpp:178-190). Written from ITU T.81:
// YCbCr (JFIF), 4:2:0 chroma subsampling at quality <= 90 (4:4:4 above, the same switch as stb's
// writer), Annex K example tables scaled with the IJG quality formula, float DCT, Annex K Huffman
// tables. Output bytes are a valid baseline JPEG; they are not byte-identical to stb's.
#include "jpeg.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

namespace ptgs {
namespace {

const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// T.81 Annex K.1 (natural order)
const uint8_t kLumQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                           14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                           18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                           49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const uint8_t kChrQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99,
                           99, 99, 47, 66, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                           99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

// T.81 Annex K.3 Huffman tables: code counts per length 1..16, then symbols
const uint8_t kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcLumVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kDcChrBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcChrVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kAcLumBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcLumVal[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChrBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcChrVal[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

struct Huff {
  uint16_t code[256];
  uint8_t len[256];
};

// T.81 Annex C: canonical codes from the counts per length
void build_huff(const uint8_t* bits, const uint8_t* val, Huff& h) {
  std::memset(&h, 0, sizeof(h));
  uint16_t code = 0;
  int k = 0;
  for (int l = 1; l <= 16; ++l) {
    for (int i = 0; i < bits[l - 1]; ++i, ++k) {
      h.code[val[k]] = code++;
      h.len[val[k]] = (uint8_t)l;
    }
    code <<= 1;
  }
}

struct BitWriter {
  std::vector<uint8_t>& out;
  uint32_t acc = 0;
  int nbits = 0;
  explicit BitWriter(std::vector<uint8_t>& o) : out(o) {}
  void put(uint32_t bits, int n) {
    for (int i = n - 1; i >= 0; --i) {
      acc = (acc << 1) | ((bits >> i) & 1u);
      if (++nbits == 8) {
        out.push_back((uint8_t)acc);
        if ((uint8_t)acc == 0xFF) out.push_back(0x00);  // byte stuffing
        acc = 0;
        nbits = 0;
      }
    }
  }
  void flush() {
    while (nbits) put(1, 1);  // pad with 1-bits
  }
};

void scaled_table(const uint8_t* base, int quality, uint8_t* out) {
  if (quality < 1) quality = 1;
  if (quality > 100) quality = 100;
  const int scale = quality < 50 ? 5000 / quality : 200 - quality * 2;
  for (int i = 0; i < 64; ++i) {
    int q = (base[i] * scale + 50) / 100;
    out[i] = (uint8_t)(q < 1 ? 1 : (q > 255 ? 255 : q));
  }
}

// separable float DCT-II of one 8x8 block (level-shifted samples), result in natural order
void fdct8x8(const float* in, float* out) {
  static float c[8][8];
  static bool init = false;
  if (!init) {
    for (int u = 0; u < 8; ++u)
      for (int x = 0; x < 8; ++x)
        c[u][x] = (u == 0 ? std::sqrt(0.125f) : 0.5f) * std::cos((2 * x + 1) * u * 3.14159265358979f / 16.0f);
    init = true;
  }
  float tmp[64];
  for (int y = 0; y < 8; ++y)
    for (int u = 0; u < 8; ++u) {
      float s = 0.0f;
      for (int x = 0; x < 8; ++x) s += c[u][x] * in[y * 8 + x];
      tmp[y * 8 + u] = s;
    }
  for (int v = 0; v < 8; ++v)
    for (int u = 0; u < 8; ++u) {
      float s = 0.0f;
      for (int y = 0; y < 8; ++y) s += c[v][y] * tmp[y * 8 + u];
      out[v * 8 + u] = s;
    }
}

int category(int v) {
  int a = v < 0 ? -v : v, n = 0;
  while (a) {
    a >>= 1;
    ++n;
  }
  return n;
}

void encode_block(BitWriter& bw, const float* samples, const uint8_t* q, const Huff& dc, const Huff& ac, int& pred) {
  float coef[64];
  fdct8x8(samples, coef);
  int zz[64];
  for (int i = 0; i < 64; ++i) {
    const int n = kZigzag[i];
    zz[i] = (int)std::lround(coef[n] / (float)q[n]);
  }
  const int diff = zz[0] - pred;
  pred = zz[0];
  int cat = category(diff);
  bw.put(dc.code[cat], dc.len[cat]);
  if (cat) bw.put((uint32_t)(diff < 0 ? diff + (1 << cat) - 1 : diff), cat);
  int run = 0;
  for (int i = 1; i < 64; ++i) {
    if (zz[i] == 0) {
      ++run;
      continue;
    }
    while (run > 15) {
      bw.put(ac.code[0xF0], ac.len[0xF0]);  // ZRL
      run -= 16;
    }
    cat = category(zz[i]);
    const int sym = (run << 4) | cat;
    bw.put(ac.code[sym], ac.len[sym]);
    bw.put((uint32_t)(zz[i] < 0 ? zz[i] + (1 << cat) - 1 : zz[i]), cat);
    run = 0;
  }
  if (run) bw.put(ac.code[0x00], ac.len[0x00]);  // EOB
}

void put16(std::vector<uint8_t>& o, int v) {
  o.push_back((uint8_t)(v >> 8));
  o.push_back((uint8_t)v);
}

void put_dht(std::vector<uint8_t>& o, int cls_id, const uint8_t* bits, const uint8_t* val) {
  int n = 0;
  for (int i = 0; i < 16; ++i) n += bits[i];
  o.push_back(0xFF);
  o.push_back(0xC4);
  put16(o, 2 + 1 + 16 + n);
  o.push_back((uint8_t)cls_id);
  o.insert(o.end(), bits, bits + 16);
  o.insert(o.end(), val, val + n);
}

}  // namespace

bool encode_jpeg(const uint8_t* pixels, uint32_t w, uint32_t h, uint32_t comp, int quality, std::vector<uint8_t>& o) {
  if (!pixels || w == 0 || h == 0 || w > 65535 || h > 65535 || comp < 1 || comp > 4) return false;
  const bool sub = quality <= 90;  // 4:2:0 as stb's writer does at quality <= 90
  uint8_t ql[64], qc[64];
  scaled_table(kLumQ, quality, ql);
  scaled_table(kChrQ, quality, qc);
  Huff dcl, dcc, acl, acc;
  build_huff(kDcLumBits, kDcLumVal, dcl);
  build_huff(kDcChrBits, kDcChrVal, dcc);
  build_huff(kAcLumBits, kAcLumVal, acl);
  build_huff(kAcChrBits, kAcChrVal, acc);
  o.clear();
  const uint8_t soi_app0[] = {0xFF, 0xD8, 0xFF, 0xE0, 0, 16, 'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0};
  o.insert(o.end(), soi_app0, soi_app0 + sizeof(soi_app0));
  o.push_back(0xFF);
  o.push_back(0xDB);
  put16(o, 2 + 2 * 65);
  o.push_back(0);
  for (int i = 0; i < 64; ++i) o.push_back(ql[kZigzag[i]]);
  o.push_back(1);
  for (int i = 0; i < 64; ++i) o.push_back(qc[kZigzag[i]]);
  o.push_back(0xFF);
  o.push_back(0xC0);  // SOF0
  put16(o, 8 + 3 * 3);
  o.push_back(8);
  put16(o, (int)h);
  put16(o, (int)w);
  o.push_back(3);
  const uint8_t ysamp = sub ? 0x22 : 0x11;
  const uint8_t sof_comps[] = {1, ysamp, 0, 2, 0x11, 1, 3, 0x11, 1};
  o.insert(o.end(), sof_comps, sof_comps + 9);
  put_dht(o, 0x00, kDcLumBits, kDcLumVal);
  put_dht(o, 0x10, kAcLumBits, kAcLumVal);
  put_dht(o, 0x01, kDcChrBits, kDcChrVal);
  put_dht(o, 0x11, kAcChrBits, kAcChrVal);
  const uint8_t sos[] = {0xFF, 0xDA, 0, 12, 3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0};
  o.insert(o.end(), sos, sos + sizeof(sos));

  // YCbCr planes (JFIF), edge-replicated to whole MCUs
  const uint32_t mcu = sub ? 16 : 8;
  const uint32_t W = (w + mcu - 1) / mcu * mcu, H = (h + mcu - 1) / mcu * mcu;
  std::vector<float> Y((size_t)W * H), Cb((size_t)W * H), Cr((size_t)W * H);
  for (uint32_t y = 0; y < H; ++y)
    for (uint32_t x = 0; x < W; ++x) {
      const uint8_t* p = pixels + ((size_t)(y < h ? y : h - 1) * w + (x < w ? x : w - 1)) * comp;
      const float r = p[0], g = comp >= 3 ? p[1] : p[0], b = comp >= 3 ? p[2] : p[0];
      const size_t k = (size_t)y * W + x;
      Y[k] = 0.299f * r + 0.587f * g + 0.114f * b - 128.0f;
      Cb[k] = -0.168736f * r - 0.331264f * g + 0.5f * b;
      Cr[k] = 0.5f * r - 0.418688f * g - 0.081312f * b;
    }
  BitWriter bw(o);
  int py = 0, pb = 0, pr = 0;
  float blk[64];
  for (uint32_t my = 0; my < H; my += mcu)
    for (uint32_t mx = 0; mx < W; mx += mcu) {
      for (uint32_t by = 0; by < mcu; by += 8)
        for (uint32_t bx = 0; bx < mcu; bx += 8) {
          for (int i = 0; i < 64; ++i) blk[i] = Y[(size_t)(my + by + i / 8) * W + mx + bx + i % 8];
          encode_block(bw, blk, ql, dcl, acl, py);
        }
      for (int c = 0; c < 2; ++c) {
        const std::vector<float>& P = c == 0 ? Cb : Cr;
        for (int i = 0; i < 64; ++i) {
          const uint32_t yy = i / 8, xx = i % 8;
          if (sub) {  // 2x2 average
            const size_t k = (size_t)(my + 2 * yy) * W + mx + 2 * xx;
            blk[i] = 0.25f * (P[k] + P[k + 1] + P[k + W] + P[k + W + 1]);
          } else {
            blk[i] = P[(size_t)(my + yy) * W + mx + xx];
          }
        }
        encode_block(bw, blk, qc, dcc, acc, c == 0 ? pb : pr);
      }
    }
  bw.flush();
  o.push_back(0xFF);
  o.push_back(0xD9);  // EOI
  return true;
}

}  // namespace ptgs
