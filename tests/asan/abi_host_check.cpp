// Host-side checks of the C-ABI (include/vtd.h) for the AddressSanitizer build of the
// library's host code (`make -C vision_transformer_detector_amd/csrc asan`, SURVEY §5
// "sanitizers"): the calls test_host_cpu.py makes through ctypes -- ABI version, shape
// derivation and workspace sizing of every preset, argument validation of every compute
// entry point (rejected before any device call), the profiling state -- re-expressed in
// C++ so the instrumented code runs without preloading the sanitizer runtime into Python.
// No GPU is touched: every compute call below fails argument validation first.
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <string>
#include <vector>

#include "vtd.h"

static int failures = 0;
#define CHECK(c)                                                           \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::printf("FAIL %s:%d %s (last error: %s)\n", __FILE__, __LINE__, #c, \
                  vtd_last_error());                                       \
      ++failures;                                                          \
    }                                                                      \
  } while (0)

static vtd_config preset(int b, int hw, int p, int d, int heads, int kd, int q, int rep,
                         int last, int layers, int mish, int dtype) {
  vtd_config c{};
  c.batch = b; c.image_h = hw; c.image_w = hw; c.channels = 3; c.patch_size = p;
  c.embedding_dim = d; c.num_heads = heads; c.key_dim = kd; c.mlp_quantities = q;
  c.repeat_times = rep; c.head_last_units = last; c.head_layers = layers; c.head_repeats = 1;
  c.use_mish = mish; c.dtype = dtype;
  return c;
}

// 11x9 4:2:0 baseline JPEG with a restart marker per MCU row (Pillow, quality 70)
static const uint8_t kJpeg[] = {
    255,216,255,224,0,16,74,70,73,70,0,1,1,0,0,1,0,1,0,0,255,219,0,67,0,10,7,7,8,7,6,10,8,8,8,11,10,
    10,11,14,24,16,14,13,13,14,29,21,22,17,24,35,31,37,36,34,31,34,33,38,43,55,47,38,41,52,41,33,34,
    48,65,49,52,57,59,62,62,62,37,46,68,73,67,60,72,55,61,62,59,255,219,0,67,1,10,11,11,14,13,14,28,
    16,16,28,59,40,34,40,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,
    59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,255,192,0,17,8,0,9,0,
    11,3,1,34,0,2,17,1,3,17,1,255,196,0,31,0,0,1,5,1,1,1,1,1,1,0,0,0,0,0,0,0,0,1,2,3,4,5,6,7,8,9,10,
    11,255,196,0,181,16,0,2,1,3,3,2,4,3,5,5,4,4,0,0,1,125,1,2,3,0,4,17,5,18,33,49,65,6,19,81,97,7,
    34,113,20,50,129,145,161,8,35,66,177,193,21,82,209,240,36,51,98,114,130,9,10,22,23,24,25,26,37,
    38,39,40,41,42,52,53,54,55,56,57,58,67,68,69,70,71,72,73,74,83,84,85,86,87,88,89,90,99,100,101,
    102,103,104,105,106,115,116,117,118,119,120,121,122,131,132,133,134,135,136,137,138,146,147,148,
    149,150,151,152,153,154,162,163,164,165,166,167,168,169,170,178,179,180,181,182,183,184,185,186,
    194,195,196,197,198,199,200,201,202,210,211,212,213,214,215,216,217,218,225,226,227,228,229,230,
    231,232,233,234,241,242,243,244,245,246,247,248,249,250,255,196,0,31,1,0,3,1,1,1,1,1,1,1,1,1,0,
    0,0,0,0,0,1,2,3,4,5,6,7,8,9,10,11,255,196,0,181,17,0,2,1,2,4,4,3,4,7,5,4,4,0,1,2,119,0,1,2,3,17,
    4,5,33,49,6,18,65,81,7,97,113,19,34,50,129,8,20,66,145,161,177,193,9,35,51,82,240,21,98,114,209,
    10,22,36,52,225,37,241,23,24,25,26,38,39,40,41,42,53,54,55,56,57,58,67,68,69,70,71,72,73,74,83,
    84,85,86,87,88,89,90,99,100,101,102,103,104,105,106,115,116,117,118,119,120,121,122,130,131,132,
    133,134,135,136,137,138,146,147,148,149,150,151,152,153,154,162,163,164,165,166,167,168,169,170,
    178,179,180,181,182,183,184,185,186,194,195,196,197,198,199,200,201,202,210,211,212,213,214,215,
    216,217,218,226,227,228,229,230,231,232,233,234,242,243,244,245,246,247,248,249,250,255,221,0,4,
    0,1,255,218,0,12,3,1,0,2,17,3,17,0,63,0,98,249,254,96,158,230,105,110,74,225,90,99,188,182,240,
    221,0,7,104,201,10,121,227,228,192,60,102,157,107,13,147,91,169,26,108,243,0,72,14,176,121,128,
    128,72,24,96,192,17,142,42,150,173,255,0,30,86,191,245,210,111,253,1,171,182,111,245,211,127,
    215,105,63,244,35,90,58,50,115,81,82,105,187,187,166,214,214,236,250,223,240,243,211,151,25,82,
    157,40,65,168,104,210,118,245,87,234,158,218,253,231,255,217,
};

// 11x9 4:2:0 progressive JPEG (SOF2, libjpeg's simple progression script: 10 scans; Pillow,
// quality 70, random pixels)
static const uint8_t kJpegProg[] = {
    255,216,255,224,0,16,74,70,73,70,0,1,1,0,0,1,0,1,0,0,255,219,0,67,0,10,7,7,8,7,6,10,8,8,8,11,10,
    10,11,14,24,16,14,13,13,14,29,21,22,17,24,35,31,37,36,34,31,34,33,38,43,55,47,38,41,52,41,33,34,
    48,65,49,52,57,59,62,62,62,37,46,68,73,67,60,72,55,61,62,59,255,219,0,67,1,10,11,11,14,13,14,28,
    16,16,28,59,40,34,40,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,
    59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,59,255,194,0,17,8,0,9,0,
    11,3,1,34,0,2,17,1,3,17,1,255,196,0,23,0,0,3,1,0,0,0,0,0,0,0,0,0,0,0,0,0,1,2,3,4,255,196,0,21,1,
    1,1,0,0,0,0,0,0,0,0,0,0,0,0,0,0,2,3,255,218,0,12,3,1,0,2,16,3,16,0,0,1,121,12,130,95,255,196,0,
    25,16,1,1,0,3,1,0,0,0,0,0,0,0,0,0,0,0,1,2,3,4,50,52,255,218,0,8,1,1,0,1,5,2,100,36,207,112,87,
    59,126,175,255,196,0,23,17,0,3,1,0,0,0,0,0,0,0,0,0,0,0,0,0,0,1,66,97,255,218,0,8,1,3,1,1,63,1,
    149,167,255,196,0,23,17,0,3,1,0,0,0,0,0,0,0,0,0,0,0,0,0,0,2,17,1,255,218,0,8,1,2,1,1,63,1,93,
    175,15,255,196,0,31,16,0,2,1,2,7,0,0,0,0,0,0,0,0,0,0,0,0,2,17,1,3,18,81,113,114,129,130,193,255,
    218,0,8,1,1,0,6,63,2,196,171,57,82,57,33,109,214,55,157,95,194,230,167,255,196,0,29,16,0,2,2,1,
    5,0,0,0,0,0,0,0,0,0,0,0,1,17,0,49,81,16,33,65,97,129,255,218,0,8,1,1,0,1,63,33,4,160,6,166,27,
    140,46,123,129,135,213,132,66,253,148,233,3,255,218,0,12,3,1,0,2,0,3,0,0,0,16,15,255,196,0,25,
    17,1,0,2,3,0,0,0,0,0,0,0,0,0,0,0,0,1,0,33,49,97,193,255,218,0,8,1,3,1,1,63,16,80,100,26,56,208,
    246,231,255,196,0,27,17,0,1,4,3,0,0,0,0,0,0,0,0,0,0,0,0,1,0,17,65,113,33,49,81,255,218,0,8,1,2,
    1,1,63,16,118,111,78,204,22,130,44,230,105,127,255,196,0,28,16,1,0,3,0,2,3,0,0,0,0,0,0,0,0,0,0,
    1,0,17,33,97,240,49,65,81,255,218,0,8,1,1,0,1,63,16,101,25,7,133,75,116,52,182,202,226,172,97,
    253,129,3,246,115,147,58,111,145,213,224,159,255,217,
};

// ---- PNG / BMP files built here (the parsers' inputs are untrusted file bytes)
typedef std::vector<uint8_t> Bytes;
static void put_be32(Bytes& b, uint32_t v) {
  for (int s = 24; s >= 0; s -= 8) b.push_back((uint8_t)(v >> s));
}
static void put_le(Bytes& b, uint32_t v, int n) {
  for (int i = 0; i < n; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}
static Bytes png_chunk(const char* type, const Bytes& body, bool good_crc = true) {
  Bytes c;
  put_be32(c, (uint32_t)body.size());
  c.insert(c.end(), type, type + 4);
  c.insert(c.end(), body.begin(), body.end());
  uLong crc = crc32(0L, Z_NULL, 0);
  crc = crc32(crc, c.data() + 4, (uInt)(4 + body.size()));
  put_be32(c, good_crc ? (uint32_t)crc : (uint32_t)crc ^ 1u);
  return c;
}
static Bytes png_ihdr(uint32_t w, uint32_t h, int depth, int ctype, int interlace) {
  Bytes b;
  put_be32(b, w);
  put_be32(b, h);
  b.push_back((uint8_t)depth); b.push_back((uint8_t)ctype);
  b.push_back(0); b.push_back(0); b.push_back((uint8_t)interlace);
  return b;
}
static Bytes zcompress(const Bytes& raw) {
  uLongf n = compressBound((uLong)raw.size());
  Bytes out(n);
  compress(out.data(), &n, raw.data(), (uLong)raw.size());
  out.resize(n);
  return out;
}
// an RGB8 w x h PNG whose rows carry filter types 0..4 in turn; extra: chunks before IDAT
static Bytes make_png(int w, int h, const Bytes& extra = Bytes(), int bad_filter_row = -1) {
  Bytes raw;
  for (int r = 0; r < h; ++r) {
    raw.push_back((uint8_t)(r == bad_filter_row ? 9 : r % 5));
    for (int i = 0; i < 3 * w; ++i) raw.push_back((uint8_t)(r * 31 + i * 7));
  }
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
  Bytes f(sig, sig + 8);
  const Bytes ihdr = png_chunk("IHDR", png_ihdr(w, h, 8, 2, 0));
  f.insert(f.end(), ihdr.begin(), ihdr.end());
  f.insert(f.end(), extra.begin(), extra.end());
  const Bytes idat = png_chunk("IDAT", zcompress(raw));
  f.insert(f.end(), idat.begin(), idat.end());
  const Bytes iend = png_chunk("IEND", Bytes());
  f.insert(f.end(), iend.begin(), iend.end());
  return f;
}
// PNG with an arbitrary IHDR and IDAT payload
static Bytes png_raw(const Bytes& ihdr_body, const Bytes& idat_body, const Bytes& extra = Bytes()) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
  Bytes f(sig, sig + 8);
  for (const Bytes& c : {png_chunk("IHDR", ihdr_body), extra, png_chunk("IDAT", idat_body),
                         png_chunk("IEND", Bytes())})
    f.insert(f.end(), c.begin(), c.end());
  return f;
}
// host decode path of one file: info, workspace planning, inflate into an exactly sized buffer
static int png_host(const Bytes& f) {
  int h = 0, w = 0, c = 0;
  const int rc = vtd_png_info(f.data(), f.size(), &h, &w, &c);
  const uint8_t* pp[1] = {f.data()};
  size_t pl[1] = {f.size()};
  int32_t pd[2];
  size_t pb = 0, need = 0;
  (void)vtd_png_workspace_bytes(pp, pl, 1, pd, &pb);
  if (vtd_png_inflate(f.data(), f.size(), nullptr, 0, &need) != VTD_OK) return rc ? rc : -100;
  if (need > ((size_t)1 << 26)) return rc;        // plan only (no 2^28-pixel buffers here)
  Bytes out(need);
  const int ri = vtd_png_inflate(f.data(), f.size(), out.data(), out.size(), &need);
  return rc ? rc : ri;
}
static Bytes make_bmp(int32_t w, int32_t h, int bpp, uint32_t pix_off = 0, int32_t comp = 0,
                      int pixel_bytes = -1) {
  const int ncol = bpp == 8 ? 256 : 0;
  const uint32_t off = pix_off ? pix_off : 54 + 4 * ncol;
  const int64_t rows = h < 0 ? -(int64_t)h : h;
  const int64_t row = ((int64_t)bpp * (w > 0 ? w : 0) + 31) / 32 * 4;
  const int64_t pix = pixel_bytes >= 0 ? pixel_bytes : row * rows;
  Bytes b;
  b.push_back('B'); b.push_back('M');
  put_le(b, (uint32_t)(54 + 4 * ncol + pix), 4);
  put_le(b, 0, 4);
  put_le(b, off, 4);
  put_le(b, 40, 4);
  put_le(b, (uint32_t)w, 4);
  put_le(b, (uint32_t)h, 4);
  put_le(b, 1, 2);
  put_le(b, (uint32_t)bpp, 2);
  put_le(b, (uint32_t)comp, 4);
  for (int i = 0; i < 5; ++i) put_le(b, 0, 4);
  for (int i = 0; i < 4 * ncol; ++i) b.push_back((uint8_t)i);
  for (int64_t i = 0; i < pix; ++i) b.push_back((uint8_t)(i * 13));
  return b;
}
static int bmp_host(const Bytes& f) {
  int h = 0, w = 0, c = 0;
  const int rc = vtd_bmp_info(f.data(), f.size(), &h, &w, &c);
  const uint8_t* pp[1] = {f.data()};
  size_t pl[1] = {f.size()};
  int32_t pd[2];
  size_t pb = 0;
  const int rw = vtd_bmp_workspace_bytes(pp, pl, 1, pd, &pb);
  CHECK((rc == VTD_OK) == (rw == VTD_OK));
  return rc;
}

int main() {
  CHECK(vtd_abi_version() == VTD_ABI_VERSION);
  // presets (presets.py): C1 reference default, C2 / C3 ViT-B/16, C5 ViT-L/16
  struct { vtd_config c; int tokens; } cases[] = {
      {preset(1, 608, 17, 28, 8, 40, 8, 8, 136, 7, 1, VTD_F32), 1296},
      {preset(256, 224, 16, 768, 12, 64, 3, 12, 136, 7, 0, VTD_BF16), 196},
      {preset(32, 640, 16, 768, 12, 64, 3, 12, 136, 7, 0, VTD_BF16), 1600},
      {preset(128, 384, 16, 1024, 16, 64, 3, 24, 136, 7, 0, VTD_FP8), 576},
  };
  for (auto& t : cases) {
    vtd_dims d;
    std::memset(&d, 0xAB, sizeof d);
    CHECK(vtd_derive_dims(&t.c, &d) == VTD_OK);
    CHECK(d.tokens == t.tokens);
    CHECK(d.rows == (int64_t)t.c.batch * t.tokens);
    CHECK(d.head_rows == (int64_t)t.c.batch * VTD_MAX_DETECT);
    CHECK(d.d_p % VTD_KALIGN == 0 && d.d_p >= d.d);
    CHECK(d.key_dim_p == 32 || d.key_dim_p == 64 || d.key_dim_p == 128);
    size_t prev = 0;
    for (int b : {1, 2, 3, 17, 64, 256}) {
      vtd_config c = t.c;
      c.batch = b;
      size_t bytes = 0;
      CHECK(vtd_workspace_bytes(&c, &bytes) == VTD_OK);
      CHECK(bytes > 0 && bytes % 256 == 0);
      if (b > 1) CHECK(bytes >= prev);
      prev = bytes;
    }
  }
  // invalid configurations: rejected with a message
  vtd_config bad = cases[1].c;
  vtd_dims d;
  bad.batch = 0;
  CHECK(vtd_derive_dims(&bad, &d) == VTD_ERR_INVALID_ARG);
  CHECK(std::strlen(vtd_last_error()) > 0);
  bad = cases[1].c;
  bad.key_dim = 200;
  CHECK(vtd_derive_dims(&bad, &d) == VTD_ERR_INVALID_ARG);
  bad = cases[1].c;
  bad.mlp_quantities = VTD_MAX_MLP + 1;
  CHECK(vtd_derive_dims(&bad, &d) == VTD_ERR_INVALID_ARG);
  bad = cases[1].c;
  bad.dtype = 7;
  CHECK(vtd_derive_dims(&bad, &d) == VTD_ERR_INVALID_ARG);
  CHECK(vtd_derive_dims(nullptr, &d) == VTD_ERR_INVALID_ARG);
  CHECK(vtd_workspace_bytes(&cases[1].c, nullptr) == VTD_ERR_INVALID_ARG);
  // compute entry points: argument validation before any device call
  vtd_epilogue e{};
  CHECK(vtd_gemm(0, 64, 64, nullptr, 64, nullptr, 64, VTD_BF16, &e, nullptr) == VTD_ERR_INVALID_ARG);
  CHECK(vtd_gemm(64, 64, 60, nullptr, 64, nullptr, 64, VTD_BF16, &e, nullptr) == VTD_ERR_INVALID_ARG);
  CHECK(vtd_gemm(64, 64, 64, nullptr, 64, nullptr, 64, VTD_BF16, nullptr, nullptr) ==
        VTD_ERR_INVALID_ARG);
  CHECK(vtd_attention(nullptr, 1, 196, 12, 64, 2304, 0.125f, nullptr, 768, VTD_BF16, nullptr) ==
        VTD_ERR_INVALID_ARG);
  int dummy = 0;
  CHECK(vtd_attention(&dummy, 1, 196, 12, 48, 2304, 0.125f, &dummy, 768, VTD_BF16, nullptr) ==
        VTD_ERR_INVALID_ARG);
  CHECK(vtd_forward(&cases[1].c, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr) ==
        VTD_ERR_INVALID_ARG);
  CHECK(vtd_decode(nullptr, 17, nullptr, nullptr) == VTD_ERR_INVALID_ARG);
  // JPEG host side: header walk, planning, every truncation and a corrupted copy (host only)
  {
    int h = 0, w = 0, c = 0;
    CHECK(vtd_jpeg_info(kJpeg, sizeof(kJpeg), &h, &w, &c) == VTD_OK);
    CHECK(h == 9 && w == 11 && c == 3);
    const uint8_t* ptrs[2] = {kJpeg, kJpeg};
    size_t lens[2] = {sizeof(kJpeg), sizeof(kJpeg)};
    int32_t dims[4] = {0, 0, 0, 0};
    size_t bytes = 0;
    CHECK(vtd_jpeg_workspace_bytes(ptrs, lens, 2, dims, &bytes) == VTD_OK);
    CHECK(dims[0] == 9 && dims[1] == 11 && dims[2] == 9 && dims[3] == 11 && bytes > 0);
    for (size_t cut = 0; cut < sizeof(kJpeg); ++cut) {
      std::vector<uint8_t> part(kJpeg, kJpeg + cut);
      (void)vtd_jpeg_info(part.data(), part.size(), &h, &w, &c);
    }
    std::vector<uint8_t> bad(kJpeg, kJpeg + sizeof(kJpeg));
    for (size_t i = 2; i < bad.size(); i += 3) bad[i] ^= 0x5A;
    (void)vtd_jpeg_info(bad.data(), bad.size(), &h, &w, &c);
    CHECK(vtd_jpeg_info(nullptr, 10, &h, &w, &c) == VTD_ERR_INVALID_ARG);
    // a DRI / SOS segment with no payload that ends the buffer (exactly sized copies, so any
    // read of a payload byte is a heap overflow ASan reports)
    size_t sos = 0;
    for (size_t i = 0; i + 1 < sizeof(kJpeg); ++i)
      if (kJpeg[i] == 0xFF && kJpeg[i + 1] == 0xDA) { sos = i; break; }
    CHECK(sos > 0);
    for (uint8_t mk : {uint8_t(0xDD), uint8_t(0xDA)}) {
      std::vector<uint8_t> f(kJpeg, kJpeg + sos);
      const uint8_t seg[4] = {0xFF, mk, 0x00, 0x02};
      f.insert(f.end(), seg, seg + 4);
      std::vector<uint8_t> exact(f.begin(), f.end());
      CHECK(vtd_jpeg_info(exact.data(), exact.size(), &h, &w, &c) != VTD_OK);
    }
  }
  // progressive JPEG host side: per-scan table walk, planning of the scan / segment tables,
  // every truncation (exactly sized copies) through both entry points, and a corrupted copy
  {
    int h = 0, w = 0, c = 0;
    CHECK(vtd_jpeg_info(kJpegProg, sizeof(kJpegProg), &h, &w, &c) == VTD_OK);
    CHECK(h == 9 && w == 11 && c == 3);
    const uint8_t* ptrs[3] = {kJpegProg, kJpeg, kJpegProg};
    size_t lens[3] = {sizeof(kJpegProg), sizeof(kJpeg), sizeof(kJpegProg)};
    int32_t dims[6] = {0, 0, 0, 0, 0, 0};
    size_t bytes = 0;
    CHECK(vtd_jpeg_workspace_bytes(ptrs, lens, 3, dims, &bytes) == VTD_OK);
    CHECK(dims[4] == 9 && dims[5] == 11 && bytes > 0);
    for (size_t cut = 0; cut < sizeof(kJpegProg); ++cut) {
      std::vector<uint8_t> part(kJpegProg, kJpegProg + cut);
      (void)vtd_jpeg_info(part.data(), part.size(), &h, &w, &c);
      const uint8_t* pp[1] = {part.data()};
      size_t pl[1] = {part.size()};
      int32_t pd[2];
      size_t pb = 0;
      (void)vtd_jpeg_workspace_bytes(pp, pl, 1, pd, &pb);
    }
    for (int stride : {3, 7, 13}) {
      std::vector<uint8_t> bad(kJpegProg, kJpegProg + sizeof(kJpegProg));
      for (size_t i = 2; i < bad.size(); i += stride) bad[i] ^= 0x5A;
      (void)vtd_jpeg_info(bad.data(), bad.size(), &h, &w, &c);
      const uint8_t* pp[1] = {bad.data()};
      size_t pl[1] = {bad.size()};
      int32_t pd[2];
      size_t pb = 0;
      (void)vtd_jpeg_workspace_bytes(pp, pl, 1, pd, &pb);
    }
  }
  // PNG host side: every truncation, bad CRCs, IHDR size edges, short and
  // garbage zlib streams, long PLTE, bad filter bytes (exactly sized copies throughout)
  {
    const Bytes good = make_png(13, 9);
    CHECK(png_host(good) == VTD_OK);
    for (size_t cut = 0; cut < good.size(); ++cut) {
      Bytes part(good.begin(), good.begin() + cut);
      CHECK(png_host(part) != VTD_OK);
    }
    for (size_t i = 8; i < good.size(); ++i) {            // every byte flipped: CRC / structure
      Bytes bad = good;
      bad[i] ^= 0x41;
      (void)png_host(bad);
    }
    Bytes badcrc = make_png(13, 9, png_chunk("PLTE", Bytes(30, 7), false));
    CHECK(png_host(badcrc) != VTD_OK);
    // IHDR sizes: 2^28 pixels accepted (planned only), one more refused; 32-bit products and
    // widths >= 2^31 refused
    Bytes one(1, 0);
    int h = 0, w = 0, c = 0;
    const Bytes edge = png_raw(png_ihdr(1u << 14, 1u << 14, 8, 2, 0), zcompress(one));
    CHECK(vtd_png_info(edge.data(), edge.size(), &h, &w, &c) == VTD_OK);
    for (uint32_t ww : {(1u << 14) + 1u, 1u << 16, 0x80000000u, 0xFFFFFFFFu}) {
      const Bytes f = png_raw(png_ihdr(ww, ww == (1u << 14) + 1 ? 1u << 14 : ww, 8, 2, 0),
                              zcompress(one));
      CHECK(vtd_png_info(f.data(), f.size(), &h, &w, &c) != VTD_OK);
    }
    const Bytes ovf = png_raw(png_ihdr(0x10000u, 0x10000u, 16, 6, 1), zcompress(one));
    CHECK(vtd_png_info(ovf.data(), ovf.size(), &h, &w, &c) != VTD_OK);
    const Bytes zero = png_raw(png_ihdr(0, 5, 8, 2, 0), zcompress(one));
    CHECK(vtd_png_info(zero.data(), zero.size(), &h, &w, &c) != VTD_OK);
    // zlib: garbage, every prefix of a valid stream, a valid stream that is too short
    Bytes raw;
    for (int r = 0; r < 6; ++r) {
      raw.push_back(1);
      for (int i = 0; i < 15; ++i) raw.push_back((uint8_t)(i * r));
    }
    const Bytes z = zcompress(raw);
    CHECK(png_host(png_raw(png_ihdr(5, 6, 8, 2, 0), z)) == VTD_OK);
    // (a stream cut inside its trailing Adler-32, or just before the final block's
    // end-of-block code, has delivered every image byte: accepted, the image data is complete;
    // every shorter prefix is refused)
    for (size_t cut = 0; cut < z.size(); ++cut) {
      const int rc = png_host(png_raw(png_ihdr(5, 6, 8, 2, 0), Bytes(z.begin(), z.begin() + cut)));
      if (cut + 5 < z.size()) CHECK(rc != VTD_OK);
    }
    Bytes garbage(64);
    for (size_t i = 0; i < garbage.size(); ++i) garbage[i] = (uint8_t)(i * 97 + 13);
    CHECK(png_host(png_raw(png_ihdr(5, 6, 8, 2, 0), garbage)) != VTD_OK);
    CHECK(png_host(png_raw(png_ihdr(5, 7, 8, 2, 0), z)) != VTD_OK);   // one row short
    // PLTE: longer than 768 bytes, not a multiple of 3, empty
    for (size_t n : {size_t(771), size_t(769), size_t(0), size_t(768)}) {
      const Bytes f = make_png(4, 4, png_chunk("PLTE", Bytes(n, 9)));
      if (n == 768) CHECK(png_host(f) == VTD_OK);
      else CHECK(png_host(f) != VTD_OK);
    }
    // a filter-type byte above 4
    const Bytes bf = make_png(6, 5, Bytes(), 3);
    CHECK(png_host(bf) != VTD_OK);
    CHECK(std::string(vtd_last_error()).find("filter") != std::string::npos);
    size_t need = 0;
    CHECK(vtd_png_inflate(good.data(), good.size(), nullptr, 0, &need) == VTD_OK && need > 0);
    Bytes small(need - 1);
    CHECK(vtd_png_inflate(good.data(), good.size(), small.data(), small.size(), &need) ==
          VTD_ERR_WORKSPACE);
  }
  // BMP host side: 8 / 24 / 32-bit, negative (top-down) heights, zero heights, bad offsets,
  // RLE, every truncation
  {
    for (int bpp : {8, 24, 32}) {
      CHECK(bmp_host(make_bmp(7, 5, bpp)) == VTD_OK);
      CHECK(bmp_host(make_bmp(7, -5, bpp)) == VTD_OK);
      CHECK(bmp_host(make_bmp(7, 0, bpp)) != VTD_OK);
      CHECK(bmp_host(make_bmp(0, 5, bpp)) != VTD_OK);
      CHECK(bmp_host(make_bmp(-7, 5, bpp)) != VTD_OK);
      CHECK(bmp_host(make_bmp(7, INT32_MIN, bpp, 0, 0, 0)) != VTD_OK);
      CHECK(bmp_host(make_bmp(7, 5, bpp, 20)) != VTD_OK);                // offset inside the header
      CHECK(bmp_host(make_bmp(7, 5, bpp, 0x7FFFFFF0u)) != VTD_OK);       // offset past the file
      CHECK(bmp_host(make_bmp(7, 5, bpp, 0xFFFFFFF0u)) != VTD_OK);       // negative offset
      CHECK(bmp_host(make_bmp(7, 5, bpp, 0, 0, 10)) != VTD_OK);          // short pixel array
      CHECK(bmp_host(make_bmp(1 << 15, 1 << 14, bpp, 0, 0, 0)) != VTD_OK);   // 2^29 pixels
      CHECK(bmp_host(make_bmp(0x7FFFFFFF, 2, bpp, 0, 0, 0)) != VTD_OK);
      const Bytes f = make_bmp(9, -3, bpp);
      for (size_t cut = 0; cut < f.size(); ++cut)
        CHECK(bmp_host(Bytes(f.begin(), f.begin() + cut)) != VTD_OK);
    }
    CHECK(bmp_host(make_bmp(7, 5, 8, 0, 1)) != VTD_OK);                  // RLE8
    CHECK(bmp_host(make_bmp(7, 5, 16)) != VTD_OK);
    CHECK(bmp_host(make_bmp(7, 5, 32, 0, 3)) == VTD_OK);                 // BI_BITFIELDS
  }
  // profiling state (host only)
  CHECK(vtd_profile_reset() == VTD_OK);
  double ms[8];
  int64_t n[8];
  double fl[8];
  CHECK(vtd_profile_read(ms, n, fl, 8) == VTD_OK || vtd_profile_read(ms, n, fl, 5) == VTD_OK);
  std::printf("%s: %d failure(s)\n", failures ? "FAILED" : "ok", failures);
  return failures ? 1 : 0;
}
