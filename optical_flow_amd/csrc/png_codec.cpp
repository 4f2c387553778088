// PNG codec on the host (zlib inflate/deflate + the PNG row filters), for the KITTI data path
// (SURVEY.md §8 f row 1: cv2.imread at data_reader.py:53-54) and the offline flow pictures
// (row 4: drawing.py).  Decoding follows the PNG specification (ISO/IEC 15948): chunk
// stream, zlib stream of filtered scanlines (Adam7 passes when interlaced), filter types
// 0-4, then the conversion cv2.imread(path) applies with IMREAD_COLOR: 8-bit BGR, gray
// replicated, palette expanded, alpha dropped, 16-bit samples reduced to their high byte,
// 1/2/4-bit gray scaled to 0..255.
#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "image_io.h"

namespace oflow {
namespace png {

static const uint8_t kSig[8] = {137, 80, 78, 71, 13, 10, 26, 10};

static uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
static void put32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back(x >> 24);
  v.push_back(x >> 16);
  v.push_back(x >> 8);
  v.push_back(x);
}

static bool valid_depth(int ctype, int depth) {
  switch (ctype) {
    case 0: return depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16;
    case 3: return depth == 1 || depth == 2 || depth == 4 || depth == 8;
    case 2: case 4: case 6: return depth == 8 || depth == 16;
    default: return false;
  }
}

bool parse_info(const uint8_t* d, size_t n, Info& info, std::string& err) {
  if (n < 33 || memcmp(d, kSig, 8) != 0) { err = "not a PNG file"; return false; }
  if (be32(d + 8) != 13 || memcmp(d + 12, "IHDR", 4) != 0) { err = "PNG: IHDR missing"; return false; }
  const uint8_t* h = d + 16;
  info.w = (int)be32(h);
  info.h = (int)be32(h + 4);
  info.depth = h[8];
  info.ctype = h[9];
  info.interlace = h[12];
  if (info.w <= 0 || info.h <= 0 || info.w > (1 << 15) || info.h > (1 << 15)) {
    err = "PNG: unsupported dimensions";
    return false;
  }
  if (!valid_depth(info.ctype, info.depth) || h[10] != 0 || h[11] != 0 || info.interlace > 1) {
    err = "PNG: invalid IHDR (colour type / bit depth / method)";
    return false;
  }
  if (be32(d + 29) != (uint32_t)crc32(0, d + 12, 17)) { err = "PNG: IHDR CRC mismatch"; return false; }
  return true;
}

bool read_file(const char* path, std::vector<uint8_t>& buf, std::string& err) {
  FILE* f = fopen(path, "rb");
  if (!f) { err = std::string("cannot open ") + path; return false; }
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  if (sz < 0) { fclose(f); err = std::string("cannot size ") + path; return false; }
  buf.resize((size_t)sz);
  size_t got = sz ? fread(buf.data(), 1, (size_t)sz, f) : 0;
  fclose(f);
  if (got != (size_t)sz) { err = std::string("short read ") + path; return false; }
  return true;
}

bool file_info(const char* path, Info& info, std::string& err) {
  uint8_t head[33];
  FILE* f = fopen(path, "rb");
  if (!f) { err = std::string("cannot open ") + path; return false; }
  size_t got = fread(head, 1, sizeof head, f);
  fclose(f);
  if (!parse_info(head, got, info, err)) { err += std::string(": ") + path; return false; }
  return true;
}

static inline int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
  return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// Undo one scanline's filter in place; prev = the unfiltered previous row of the same pass
// (nullptr for the first row), bpp = bytes per complete pixel (>= 1).
static bool unfilter(uint8_t* row, const uint8_t* prev, size_t len, int bpp, int type) {
  switch (type) {
    case 0: return true;
    case 1:
      for (size_t i = bpp; i < len; ++i) row[i] += row[i - bpp];
      return true;
    case 2:
      if (prev) for (size_t i = 0; i < len; ++i) row[i] += prev[i];
      return true;
    case 3:
      for (size_t i = 0; i < len; ++i) {
        const int a = i >= (size_t)bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
        row[i] += (uint8_t)((a + b) >> 1);
      }
      return true;
    case 4:
      for (size_t i = 0; i < len; ++i) {
        const int a = i >= (size_t)bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
        const int c = (prev && i >= (size_t)bpp) ? prev[i - bpp] : 0;
        row[i] += (uint8_t)paeth(a, b, c);
      }
      return true;
    default: return false;
  }
}

static inline size_t row_bytes(int w, const Info& in) {
  return ((size_t)w * in.channels() * in.depth + 7) / 8;
}

// Sample k (of channel-interleaved samples) of an unfiltered row, reduced to 8 bits the way
// IMREAD_COLOR does: 16-bit -> high byte; sub-byte gray -> scaled to 0..255; palette indices
// are returned raw.
static inline int sample8(const uint8_t* row, size_t k, const Info& in) {
  switch (in.depth) {
    case 8: return row[k];
    case 16: return row[2 * k];
    default: {
      const size_t bit = k * in.depth;
      const int v = (row[bit >> 3] >> (8 - in.depth - (int)(bit & 7))) & ((1 << in.depth) - 1);
      return in.ctype == 3 ? v : v * (255 / ((1 << in.depth) - 1));
    }
  }
}

static bool put_pixel(const uint8_t* row, int x, const Info& in, const uint8_t* plte, int nplte,
                      uint8_t* dst, std::string& err) {
  const size_t s = (size_t)x * in.channels();
  int r, g, b;
  switch (in.ctype) {
    case 0: case 4: r = g = b = sample8(row, s, in); break;
    case 2: case 6: r = sample8(row, s, in); g = sample8(row, s + 1, in); b = sample8(row, s + 2, in); break;
    default: {  // palette
      const int i = sample8(row, s, in);
      if (i >= nplte) { err = "PNG: palette index out of range"; return false; }
      r = plte[3 * i]; g = plte[3 * i + 1]; b = plte[3 * i + 2];
    }
  }
  dst[0] = (uint8_t)b; dst[1] = (uint8_t)g; dst[2] = (uint8_t)r;
  return true;
}

bool decode_bgr(const uint8_t* d, size_t n, uint8_t* out, size_t cap, Info& in, std::string& err) {
  if (!parse_info(d, n, in, err)) return false;
  if (cap < (size_t)in.w * in.h * 3) { err = "PNG: output buffer too small"; return false; }
  // ---- chunk walk: PLTE + concatenated IDAT ----
  uint8_t plte[256 * 3];
  int nplte = 0;
  std::vector<uint8_t> idat;
  size_t pos = 8;
  bool end = false;
  while (pos + 12 <= n) {
    const uint32_t len = be32(d + pos);
    const uint8_t* type = d + pos + 4;
    if (len > n - pos - 12) { err = "PNG: truncated chunk"; return false; }
    const uint8_t* body = d + pos + 8;
    if (be32(body + len) != (uint32_t)crc32(0, type, len + 4)) {
      err = std::string("PNG: CRC mismatch in ") + std::string((const char*)type, 4);
      return false;
    }
    if (!memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), body, body + len);
    } else if (!memcmp(type, "PLTE", 4)) {
      if (len % 3 || len > 768) { err = "PNG: bad PLTE"; return false; }
      nplte = (int)len / 3;
      memcpy(plte, body, len);
    } else if (!memcmp(type, "IEND", 4)) {
      end = true;
      break;
    } else if (!(type[0] & 0x20) && memcmp(type, "IHDR", 4)) {
      err = std::string("PNG: unknown critical chunk ") + std::string((const char*)type, 4);
      return false;
    }
    pos += 12 + len;
  }
  if (!end) { err = "PNG: IEND missing (truncated file)"; return false; }
  if (in.ctype == 3 && nplte == 0) { err = "PNG: palette image without PLTE"; return false; }
  // ---- inflate: exactly the filtered scanlines of every pass ----
  static const int ax0[7] = {0, 4, 0, 2, 0, 1, 0}, ay0[7] = {0, 0, 4, 0, 2, 0, 1};
  static const int adx[7] = {8, 8, 4, 4, 2, 2, 1}, ady[7] = {8, 8, 8, 4, 4, 2, 2};
  const int npass = in.interlace ? 7 : 1;
  int pw[7], ph[7];
  size_t raw = 0;
  for (int p = 0; p < npass; ++p) {
    pw[p] = in.interlace ? (in.w - ax0[p] + adx[p] - 1) / adx[p] : in.w;
    ph[p] = in.interlace ? (in.h - ay0[p] + ady[p] - 1) / ady[p] : in.h;
    if (pw[p] > 0 && ph[p] > 0) raw += (size_t)ph[p] * (1 + row_bytes(pw[p], in));
  }
  std::vector<uint8_t> buf(raw);
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (inflateInit(&zs) != Z_OK) { err = "PNG: inflateInit failed"; return false; }
  zs.next_in = idat.data();
  zs.avail_in = (uInt)idat.size();
  zs.next_out = buf.data();
  zs.avail_out = (uInt)raw;
  const int zr = inflate(&zs, Z_FINISH);
  const size_t produced = raw - zs.avail_out;
  inflateEnd(&zs);
  if ((zr != Z_STREAM_END && zr != Z_BUF_ERROR && zr != Z_OK) || produced != raw) {
    err = "PNG: corrupt or short image data";
    return false;
  }
  // ---- unfilter + convert ----
  const int bpp = std::max(1, in.channels() * in.depth / 8);
  uint8_t* p_row = buf.data();
  for (int p = 0; p < npass; ++p) {
    if (pw[p] <= 0 || ph[p] <= 0) continue;
    const size_t rb = row_bytes(pw[p], in);
    const uint8_t* prev = nullptr;
    for (int y = 0; y < ph[p]; ++y) {
      const int ft = p_row[0];
      uint8_t* row = p_row + 1;
      if (!unfilter(row, prev, rb, bpp, ft)) { err = "PNG: invalid filter type"; return false; }
      const int oy = in.interlace ? ay0[p] + y * ady[p] : y;
      for (int x = 0; x < pw[p]; ++x) {
        const int ox = in.interlace ? ax0[p] + x * adx[p] : x;
        if (!put_pixel(row, x, in, plte, nplte, out + ((size_t)oy * in.w + ox) * 3, err))
          return false;
      }
      prev = row;
      p_row += 1 + rb;
    }
  }
  return true;
}

static void chunk(std::vector<uint8_t>& out, const char* type, const uint8_t* body, size_t len) {
  put32(out, (uint32_t)len);
  const size_t at = out.size();
  out.insert(out.end(), type, type + 4);
  if (len) out.insert(out.end(), body, body + len);
  put32(out, (uint32_t)crc32(0, out.data() + at, (uInt)(len + 4)));
}

bool encode(const uint8_t* img, int h, int w, int c, int filter, int level,
            std::vector<uint8_t>& out, std::string& err) {
  if (h <= 0 || w <= 0 || !(c == 1 || c == 3 || c == 4) || filter < 0 || filter > 6 ||
      level < 0 || level > 9) {
    err = "png encode: bad arguments";
    return false;
  }
  const size_t rb = (size_t)w * c;
  std::vector<uint8_t> raw((size_t)h * (rb + 1));
  std::vector<uint8_t> cur(rb), prev(rb, 0), cand(rb);
  for (int y = 0; y < h; ++y) {
    const uint8_t* src = img + (size_t)y * rb;
    for (int x = 0; x < w; ++x) {   // BGR(A) -> RGB(A)
      for (int k = 0; k < c; ++k) cur[(size_t)x * c + k] = src[(size_t)x * c + k];
      if (c >= 3) std::swap(cur[(size_t)x * c], cur[(size_t)x * c + 2]);
    }
    auto apply = [&](int t, uint8_t* dst) {
      for (size_t i = 0; i < rb; ++i) {
        const int a = i >= (size_t)c ? cur[i - c] : 0, b = y ? prev[i] : 0;
        const int cc = (y && i >= (size_t)c) ? prev[i - c] : 0;
        const int pred = t == 0 ? 0 : t == 1 ? a : t == 2 ? b : t == 3 ? (a + b) >> 1 : paeth(a, b, cc);
        dst[i] = (uint8_t)(cur[i] - pred);
      }
    };
    int t = filter;
    if (filter == 6) t = y % 5;
    if (filter == 5) {
      long best = -1;
      for (int k = 0; k < 5; ++k) {
        apply(k, cand.data());
        long s = 0;
        for (size_t i = 0; i < rb; ++i) s += abs((int)(int8_t)cand[i]);
        if (best < 0 || s < best) { best = s; t = k; }
      }
    }
    uint8_t* dst = raw.data() + (size_t)y * (rb + 1);
    dst[0] = (uint8_t)t;
    apply(t, dst + 1);
    prev.swap(cur);
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), level) != Z_OK) {
    err = "png encode: deflate failed";
    return false;
  }
  out.assign(kSig, kSig + 8);
  uint8_t ihdr[13];
  const uint32_t W = (uint32_t)w, H = (uint32_t)h;
  const uint8_t wh[8] = {(uint8_t)(W >> 24), (uint8_t)(W >> 16), (uint8_t)(W >> 8), (uint8_t)W,
                         (uint8_t)(H >> 24), (uint8_t)(H >> 16), (uint8_t)(H >> 8), (uint8_t)H};
  memcpy(ihdr, wh, 8);
  ihdr[8] = 8;
  ihdr[9] = c == 1 ? 0 : c == 3 ? 2 : 6;
  ihdr[10] = ihdr[11] = ihdr[12] = 0;
  chunk(out, "IHDR", ihdr, 13);
  chunk(out, "IDAT", z.data(), zlen);
  chunk(out, "IEND", nullptr, 0);
  return true;
}

}  // namespace png
}  // namespace oflow

using namespace oflow;

extern "C" {

int of_png_info(const char* path, int* h, int* w, int* channels, int* depth) {
  OF_CHECK_ARG(path && h && w, "png_info: null argument");
  png::Info in;
  std::string err;
  if (!png::file_info(path, in, err)) return fail(OF_EINVAL, err);
  *h = in.h;
  *w = in.w;
  if (channels) *channels = in.channels();
  if (depth) *depth = in.depth;
  return OF_OK;
}

int of_png_read_bgr(const char* path, uint8_t* out, int64_t cap, int* h, int* w) {
  OF_CHECK_ARG(path && out && h && w && cap >= 0, "png_read_bgr: null argument");
  std::vector<uint8_t> file;
  std::string err;
  png::Info in;
  if (!png::read_file(path, file, err)) return fail(OF_EINVAL, err);
  if (!png::decode_bgr(file.data(), file.size(), out, (size_t)cap, in, err))
    return fail(OF_EINVAL, err + ": " + path);
  *h = in.h;
  *w = in.w;
  return OF_OK;
}

int of_png_write(const char* path, const uint8_t* img, int h, int w, int c, int flags) {
  OF_CHECK_ARG(path && img, "png_write: null argument");
  // flags: filter (bits 0-7) | (zlib level + 1) << 8; level bits 0 -> level 6
  const int filter = flags & 0xff, lbits = (flags >> 8) & 0xf;
  std::vector<uint8_t> out;
  std::string err;
  if (!png::encode(img, h, w, c, filter, lbits ? lbits - 1 : 6, out, err)) return fail(OF_EINVAL, err);
  FILE* f = fopen(path, "wb");
  if (!f) return fail(OF_EINVAL, std::string("png_write: cannot create ") + path);
  const size_t put = fwrite(out.data(), 1, out.size(), f);
  const int cl = fclose(f);
  if (put != out.size() || cl != 0) return fail(OF_EINVAL, std::string("png_write: short write ") + path);
  return OF_OK;
}

}  // extern "C"

// ---- CRC32C (Castagnoli), for the TensorFlow checkpoint bundle (SURVEY.md §8 f row 2) ----
// Slicing-by-8 over the reflected polynomial 0x82F63B78; `crc` is the running (unmasked)
// value, 0 to start.
namespace {
struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};
const Crc32cTables& crc_tables() {
  static const Crc32cTables tabs;
  return tabs;
}
}  // namespace

extern "C" uint32_t of_crc32c(const void* data, int64_t n, uint32_t crc) {
  const auto& T = crc_tables().t;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = ~crc;
  for (; n >= 8; n -= 8, p += 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = T[7][lo & 0xff] ^ T[6][(lo >> 8) & 0xff] ^ T[5][(lo >> 16) & 0xff] ^ T[4][lo >> 24] ^
        T[3][hi & 0xff] ^ T[2][(hi >> 8) & 0xff] ^ T[1][(hi >> 16) & 0xff] ^ T[0][hi >> 24];
  }
  for (; n > 0; --n, ++p) c = (c >> 8) ^ T[0][(c ^ *p) & 0xff];
  return ~c;
}
