// ply.cpp — PLY point-cloud reader for the 3DGS initialisation. Reads the vertex
// element of what Engine::savePly writes (ASCII, "x y z nx ny nz red green blue" with float / uchar
// properties, engine.cpp:2849-2895) and the binary little / big endian variants other tools write.
// Properties are matched by name: x y z (required), nx ny nz, red green blue (uchar, or float in
// [0, 1] scaled by 255 and rounded); a trained-3DGS file without rgb gives colours from its SH DC
// term f_dc_0..2 (0.5 + C0 * f_dc, clamped). Elements before "vertex" must have fixed-size rows in
// binary files (list properties are only skippable in ASCII).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/ptgs/ptgs_host.h"
#include "image_decode.h"

namespace {

struct Prop {
  std::string name, type;
  bool list = false;
  int size = 0;
};
struct Elem {
  std::string name;
  uint64_t count = 0;
  std::vector<Prop> props;
};

int type_size(const std::string& t) {
  if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
  if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
  if (t == "int" || t == "uint" || t == "int32" || t == "uint32" || t == "float" || t == "float32") return 4;
  if (t == "double" || t == "float64") return 8;
  return 0;
}

double read_bin(const uint8_t* p, const std::string& t, bool big) {
  uint8_t b[8];
  int n = type_size(t);
  for (int i = 0; i < n; ++i) b[i] = big ? p[n - 1 - i] : p[i];
  if (t == "char" || t == "int8") return (int8_t)b[0];
  if (t == "uchar" || t == "uint8") return b[0];
  if (t == "short" || t == "int16") { int16_t v; memcpy(&v, b, 2); return v; }
  if (t == "ushort" || t == "uint16") { uint16_t v; memcpy(&v, b, 2); return v; }
  if (t == "int" || t == "int32") { int32_t v; memcpy(&v, b, 4); return v; }
  if (t == "uint" || t == "uint32") { uint32_t v; memcpy(&v, b, 4); return v; }
  if (t == "float" || t == "float32") { float v; memcpy(&v, b, 4); return v; }
  double v;
  memcpy(&v, b, 8);
  return v;
}

bool is_float_type(const std::string& t) { return t == "float" || t == "float32" || t == "double" || t == "float64"; }

uint8_t to_u8(double v, bool is_float) {
  if (is_float) v = std::floor(v * 255.0 + 0.5);
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

}  // namespace

extern "C" int ptgs_read_ply(const char* path, float* xyz, float* normals, uint8_t* rgb, uint32_t capacity,
                             uint32_t* count) {
  if (!path || !count) return PTGS_EINVAL;
  std::vector<uint8_t> bytes;
  if (!ptgs::read_file(path, bytes)) return PTGS_EIO;
  // header
  size_t hdr_end = 0;
  {
    const char* tag = "end_header";
    const char* s = (const char*)bytes.data();
    size_t n = bytes.size();
    for (size_t i = 0; i + 10 <= n; ++i)
      if (!memcmp(s + i, tag, 10)) {
        size_t j = i + 10;
        while (j < n && s[j] != '\n') ++j;
        hdr_end = std::min(j + 1, n);  // (a header that ends the file without a newline)
        break;
      }
  }
  if (!hdr_end || bytes.size() < 4 || memcmp(bytes.data(), "ply", 3)) return PTGS_EIO;
  std::istringstream hs(std::string((const char*)bytes.data(), hdr_end));
  std::string line, fmt;
  std::vector<Elem> elems;
  while (std::getline(hs, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    std::istringstream ls(line);
    std::string kw;
    ls >> kw;
    if (kw == "format") {
      ls >> fmt;
    } else if (kw == "element") {
      Elem e;
      ls >> e.name >> e.count;
      elems.push_back(e);
    } else if (kw == "property") {
      if (elems.empty()) return PTGS_EIO;
      Prop p;
      std::string t;
      ls >> t;
      if (t == "list") {  // "list <count type> <item type> <name>": ASCII only
        std::string ct, it;
        ls >> ct >> it >> p.name;
        p.list = true;
        p.type = it;
      } else {
        p.type = t;
        ls >> p.name;
        p.size = type_size(t);
        if (!p.size) return PTGS_EIO;
      }
      elems.back().props.push_back(p);
    }
  }
  const bool ascii = fmt == "ascii", big = fmt == "binary_big_endian";
  if (!ascii && fmt != "binary_little_endian" && !big) return PTGS_EIO;
  int vi = -1;
  for (size_t i = 0; i < elems.size(); ++i)
    if (elems[i].name == "vertex") { vi = (int)i; break; }
  if (vi < 0) return PTGS_EIO;
  const Elem& V = elems[vi];
  if (V.count > 0xFFFFFFFFull) return PTGS_ERANGE;
  if (V.props.empty()) return PTGS_EIO;  // (rows of no bytes: the count would be unbounded)
  // header counts must fit the body (checked before the count query returns, so a caller never
  // sizes buffers from an impossible count): ASCII rows take at least one byte each, binary rows
  // exactly their size (elements before "vertex" must have fixed-size rows)
  const uint64_t body = bytes.size() - std::min(hdr_end, bytes.size());
  size_t vert_off = hdr_end, vert_rs = 0;
  if (ascii) {
    for (int e = 0; e <= vi; ++e)
      if (elems[e].count > body) return PTGS_EIO;
  } else {
    for (int e = 0; e <= vi; ++e) {
      size_t rs = 0;
      for (const Prop& pr : elems[e].props) {
        if (pr.list) return PTGS_EIO;  // variable-size rows: unsupported in binary
        rs += (size_t)pr.size;
      }
      const size_t left = bytes.size() - std::min(vert_off, bytes.size());
      if (rs && elems[e].count > left / rs) return PTGS_EIO;  // (overflow-free)
      if (e == vi) vert_rs = rs;
      else vert_off += rs * elems[e].count;
    }
  }
  *count = (uint32_t)V.count;
  if (!xyz && !normals && !rgb) return PTGS_OK;
  if (capacity < V.count) return PTGS_ERANGE;
  int ix[3] = {-1, -1, -1}, in[3] = {-1, -1, -1}, ic[3] = {-1, -1, -1}, idc[3] = {-1, -1, -1};
  const char* names[4][3] = {{"x", "y", "z"}, {"nx", "ny", "nz"}, {"red", "green", "blue"}, {"f_dc_0", "f_dc_1", "f_dc_2"}};
  int* slots[4] = {ix, in, ic, idc};
  for (size_t p = 0; p < V.props.size(); ++p)
    for (int g = 0; g < 4; ++g)
      for (int a = 0; a < 3; ++a)
        if (V.props[p].name == names[g][a] && !V.props[p].list) slots[g][a] = (int)p;
  if (ix[0] < 0 || ix[1] < 0 || ix[2] < 0) return PTGS_EIO;
  const bool have_n = in[0] >= 0 && in[1] >= 0 && in[2] >= 0;
  const bool have_c = ic[0] >= 0 && ic[1] >= 0 && ic[2] >= 0;
  const bool have_dc = idc[0] >= 0 && idc[1] >= 0 && idc[2] >= 0;
  std::vector<double> row(V.props.size());
  auto emit = [&](uint64_t i) {
    for (int a = 0; a < 3; ++a) {
      if (xyz) xyz[3 * i + a] = (float)row[ix[a]];
      if (normals) normals[3 * i + a] = have_n ? (float)row[in[a]] : 0.0f;
      if (rgb) {
        uint8_t c = 0;
        if (have_c) c = to_u8(row[ic[a]], is_float_type(V.props[ic[a]].type));
        else if (have_dc) c = to_u8(0.5 + 0.28209479177387814 * row[idc[a]], true);
        rgb[3 * i + a] = c;
      }
    }
  };
  if (ascii) {
    // strtod / strtol stop at the terminating NUL, never past the buffer
    bytes.push_back('\0');
    const char* p = (const char*)bytes.data() + hdr_end;
    const char* end = (const char*)bytes.data() + bytes.size() - 1;
    auto next_line = [&]() {
      while (p < end && *p != '\n') ++p;
      if (p < end) ++p;
    };
    for (int e = 0; e < vi; ++e)
      for (uint64_t r = 0; r < elems[e].count && p < end; ++r) next_line();
    for (uint64_t i = 0; i < V.count; ++i) {
      if (p >= end) return PTGS_EIO;  // fewer rows than the header's vertex count
      for (size_t k = 0; k < V.props.size(); ++k) {
        char* q = nullptr;
        if (V.props[k].list) {  // count then items
          long cnt = strtol(p, &q, 10);
          if (q == p || cnt < 0) return PTGS_EIO;
          p = q;
          for (long t = 0; t < cnt; ++t) { strtod(p, &q); if (q == p) return PTGS_EIO; p = q; }
          row[k] = 0;
          continue;
        }
        row[k] = strtod(p, &q);
        if (q == p) return PTGS_EIO;
        p = q;
      }
      emit(i);
      next_line();
    }
    return PTGS_OK;
  }
  const size_t off = vert_off, rs = vert_rs;
  for (uint64_t i = 0; i < V.count; ++i) {
    const uint8_t* q = bytes.data() + off + i * rs;
    for (size_t k = 0; k < V.props.size(); ++k) {
      row[k] = read_bin(q, V.props[k].type, big);
      q += V.props[k].size;
    }
    emit(i);
  }
  return PTGS_OK;
}
