// PNG decode for the input pipeline: `tf.image.decode_image(file, channels=3)`
// (vision_transformer_utilities.py:431) on PNG files.  TF decodes PNG with libpng
// (tensorflow/core/lib/png/png_io.cc) asking for 3 channels of 8 bits: palette -> RGB,
// gray 1 / 2 / 4-bit expanded to 8 (value * 255 / (2^depth - 1)), gray -> RGB replicated,
// alpha (and tRNS) stripped, 16-bit samples reduced by png_set_strip_16 (the high byte), no
// gamma or colour-space handling; Adam7-interlaced files are de-interlaced.
//
// Split of work: the chunk walk (CRC-checked for the critical chunks, as libpng errors on
// them) and the zlib inflate of the IDAT stream are serial per file and run on the host, over
// a few threads across the batch; the filtered scanlines go to the device in one copy, where
// png_unfilter_kernel (one workgroup per image, rows in order with the previous row in LDS)
// undoes the per-row filters (None / Sub / Up / Average / Paeth, PNG spec 9.2) and writes the
// RGB8 rows straight to the caller's packed output.  Parity: bit-exact vs Pillow's PNG
// decoder (its own zlib + unfilter; libpng's pixel arithmetic is the spec's) in
// tests/test_gpu_png.py; TF itself is not importable.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "vtd_common.h"

namespace vtd {
namespace {

// filtered bytes per row staged through LDS (e.g. 4096 RGBA-8 / 2048 RGBA-16 px); wider rows
// are unfiltered in place in the workspace (no width limit beyond the 2^28-pixel cap)
constexpr int kPngMaxRow = 16384;
constexpr int kPngThreads = 256;

struct PngDesc {
  int w, h, depth, ctype, interlace;
  int channels;              // samples per pixel (1 gray, 2 gray+alpha, 3 RGB, 4 RGBA; 1 palette)
  int bpp;                   // filter unit: bytes per complete pixel, at least 1
  int npal;
  int64_t data_off;          // filtered scanlines (all passes) in the data region
  int64_t out_off;           // RGB8 output (h * w * 3 bytes)
  uint8_t pal[256 * 3];
};

// Adam7 pass geometry (PNG spec 8.2): first column / row and steps
__constant__ int kA7X0[7] = {0, 4, 0, 2, 0, 1, 0}, kA7Y0[7] = {0, 0, 4, 0, 2, 0, 1};
__constant__ int kA7DX[7] = {8, 8, 4, 4, 2, 2, 1}, kA7DY[7] = {8, 8, 8, 4, 4, 2, 2};
const int kA7X0h[7] = {0, 4, 0, 2, 0, 1, 0}, kA7Y0h[7] = {0, 0, 4, 0, 2, 0, 1};
const int kA7DXh[7] = {8, 8, 4, 4, 2, 2, 1}, kA7DYh[7] = {8, 8, 8, 4, 4, 2, 2};

__host__ __device__ inline int64_t row_bytes(int pw, int channels, int depth) {
  return ((int64_t)pw * channels * depth + 7) / 8;
}

__device__ __forceinline__ int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
  return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// Undo one row's filter (PNG spec 9.2) in c, u = the unfiltered row above (all zero for a
// pass's first row); c / u are LDS rows or, for rows wider than kPngMaxRow, the rows in place
// in the workspace.  Up runs in parallel, Sub / Average / Paeth serially per byte lane.
template <typename P, typename Q>
__device__ __forceinline__ void png_unfilter_row(P c, Q u, bool has_u, int ft, int rb, int bpp,
                                                 int t) {
  if (ft == 2) {                                   // Up
    if (has_u)
      for (int i = t; i < rb; i += kPngThreads) c[i] = (uint8_t)(c[i] + u[i]);
  } else if (ft == 1 || ft == 3 || ft == 4) {      // Sub / Average / Paeth
    if (t < bpp) {
      int a = 0, cc = 0;                           // left and upper-left of this byte lane
      for (int i = t; i < rb; i += bpp) {
        const int b = has_u ? u[i] : 0;
        const int pred = ft == 1 ? a : ft == 3 ? (a + b) >> 1 : paeth(a, b, cc);
        a = (uint8_t)(c[i] + pred);
        c[i] = (uint8_t)a;
        cc = b;
      }
    }
  }
}

// One workgroup per image.  Rows of at most kPngMaxRow filtered bytes are staged through
// LDS (two row buffers); wider rows are unfiltered in place in the workspace (the row above
// is then the already-unfiltered previous row of the same pass, ordered by the barrier).
__global__ __launch_bounds__(kPngThreads) void png_unfilter_kernel(const PngDesc* __restrict__ descs,
                                                                   uint8_t* __restrict__ data,
                                                                   uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t rows[2][kPngMaxRow + 16];
  __shared__ uint8_t pal[256 * 3];
  const PngDesc& d = descs[blockIdx.x];
  const int t = threadIdx.x;
  for (int i = t; i < 256 * 3; i += kPngThreads) pal[i] = d.pal[i];
  uint8_t* src = data + d.data_off;
  uint8_t* dst = out + d.out_off;
  const int npass = d.interlace ? 7 : 1;
  const int bpp = d.bpp, depth = d.depth, ch = d.channels;
  for (int p = 0; p < npass; ++p) {
    const int x0 = d.interlace ? kA7X0[p] : 0, y0 = d.interlace ? kA7Y0[p] : 0;
    const int dx = d.interlace ? kA7DX[p] : 1, dy = d.interlace ? kA7DY[p] : 1;
    const int pw = d.w > x0 ? (d.w - x0 + dx - 1) / dx : 0;
    const int ph = d.h > y0 ? (d.h - y0 + dy - 1) / dy : 0;
    if (pw == 0 || ph == 0) continue;              // uniform: every thread skips
    const int rb = (int)row_bytes(pw, ch, depth);
    const bool wide = rb > kPngMaxRow;             // uniform
    int cur = 0;
    __syncthreads();
    for (int r = 0; r < ph; ++r, src += 1 + rb, cur ^= 1) {
      const int ft = src[0];
      const uint8_t* c;
      if (wide) {
        png_unfilter_row(src + 1, src - rb, r > 0, ft, rb, bpp, t);
        c = src + 1;
      } else {
        uint8_t* cl = rows[cur];
        for (int i = t; i < rb; i += kPngThreads) cl[i] = src[1 + i];
        __syncthreads();
        png_unfilter_row(cl, rows[cur ^ 1], r > 0, ft, rb, bpp, t);
        c = cl;
      }
      __syncthreads();
      // row -> RGB8 at output row y0 + r dy, columns x0 + px dx
      uint8_t* orow = dst + ((int64_t)(y0 + r * dy) * d.w + x0) * 3;
      for (int px = t; px < pw; px += kPngThreads) {
        int R, G, B;
        if (depth < 8) {                               // gray or palette, packed MSB first
          const int bit = px * depth;
          const int v = (c[bit >> 3] >> (8 - depth - (bit & 7))) & ((1 << depth) - 1);
          if (d.ctype == 3) {
            const bool ok = v < d.npal;
            R = ok ? pal[3 * v] : 0;
            G = ok ? pal[3 * v + 1] : 0;
            B = ok ? pal[3 * v + 2] : 0;
          } else {
            R = G = B = v * 255 / ((1 << depth) - 1);
          }
        } else {
          const int s = depth / 8;                      // bytes per sample (16-bit: high byte first)
          const uint8_t* q = c + (int64_t)px * ch * s;
          if (d.ctype == 3) {
            const int v = q[0];
            const bool ok = v < d.npal;
            R = ok ? pal[3 * v] : 0;
            G = ok ? pal[3 * v + 1] : 0;
            B = ok ? pal[3 * v + 2] : 0;
          } else if (ch >= 3) {
            R = q[0];
            G = q[s];
            B = q[2 * s];
          } else {
            R = G = B = q[0];
          }
        }
        uint8_t* o = orow + (int64_t)px * dx * 3;
        o[0] = (uint8_t)R;
        o[1] = (uint8_t)G;
        o[2] = (uint8_t)B;
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------ host
uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | p[1] << 16 | p[2] << 8 | p[3]; }
size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// Inflated size of the filtered scanlines (all passes)
int64_t filtered_bytes(const PngDesc& d) {
  int64_t total = 0;
  for (int p = 0; p < (d.interlace ? 7 : 1); ++p) {
    const int x0 = d.interlace ? kA7X0h[p] : 0, y0 = d.interlace ? kA7Y0h[p] : 0;
    const int dx = d.interlace ? kA7DXh[p] : 1, dy = d.interlace ? kA7DYh[p] : 1;
    const int64_t pw = d.w > x0 ? (d.w - x0 + dx - 1) / dx : 0;
    const int64_t ph = d.h > y0 ? (d.h - y0 + dy - 1) / dy : 0;
    if (pw && ph) total += ph * (1 + row_bytes((int)pw, d.channels, d.depth));
  }
  return total;
}

// Chunk walk (PNG spec 5): IHDR first, PLTE, IDAT runs, IEND.  idat: the IDAT payloads.
bool parse_png(const uint8_t* b, size_t n, PngDesc& d, std::vector<std::pair<size_t, size_t>>* idat,
               std::string& err) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
  memset(&d, 0, sizeof(d));
  if (n < 8 || memcmp(b, sig, 8) != 0) { err = "png: not a PNG file"; return false; }
  size_t pos = 8;
  bool ihdr = false, iend = false;
  while (pos + 12 <= n) {
    const uint32_t len = be32(b + pos);
    const uint8_t* type = b + pos + 4;
    if (len > n - pos - 12) { err = "png: truncated chunk"; return false; }
    const uint8_t* body = b + pos + 8;
    const bool critical = (type[0] & 0x20) == 0;
    if (critical) {                     // libpng: a critical chunk's CRC error is an error
      const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), type, 4 + len);
      if (crc != be32(body + len)) { err = "png: CRC error in a critical chunk"; return false; }
    }
    if (!memcmp(type, "IHDR", 4)) {
      if (len != 13 || ihdr) { err = "png: bad IHDR"; return false; }
      d.w = (int)be32(body);
      d.h = (int)be32(body + 4);
      d.depth = body[8];
      d.ctype = body[9];
      d.interlace = body[12];
      if ((int64_t)be32(body) * be32(body + 4) > ((int64_t)1 << 28)) {
        err = "png: image larger than 2^28 pixels";
        return false;
      }
      if (d.w <= 0 || d.h <= 0 || body[10] != 0 || body[11] != 0 || d.interlace > 1) {
        err = "png: bad IHDR (size, compression, filter or interlace method)";
        return false;
      }
      const int ct = d.ctype, bd = d.depth;
      const bool ok = (ct == 0 && (bd == 1 || bd == 2 || bd == 4 || bd == 8 || bd == 16)) ||
                      (ct == 3 && (bd == 1 || bd == 2 || bd == 4 || bd == 8)) ||
                      ((ct == 2 || ct == 4 || ct == 6) && (bd == 8 || bd == 16));
      if (!ok) { err = "png: invalid colour type / bit depth combination"; return false; }
      d.channels = ct == 0 ? 1 : ct == 2 ? 3 : ct == 3 ? 1 : ct == 4 ? 2 : 4;
      d.bpp = std::max(1, d.channels * d.depth / 8);
      // the widest pass (the full width) indexes its row with int in the unfilter kernel
      if (row_bytes(d.w, d.channels, d.depth) > (int64_t)INT32_MAX - kPngThreads - 1) {
        err = "png: row wider than 2^31 bytes";
        return false;
      }
      ihdr = true;
    } else if (!ihdr) {
      err = "png: first chunk is not IHDR";
      return false;
    } else if (!memcmp(type, "PLTE", 4)) {
      if (len % 3 || len == 0 || len > 768) { err = "png: bad PLTE"; return false; }
      d.npal = (int)(len / 3);
      memcpy(d.pal, body, len);
    } else if (!memcmp(type, "IDAT", 4)) {
      if (idat) idat->emplace_back(pos + 8, len);
    } else if (!memcmp(type, "IEND", 4)) {
      iend = true;
      break;
    } else if (critical) {
      err = std::string("png: unknown critical chunk ") + std::string((const char*)type, 4);
      return false;
    }
    pos += 12 + len;
  }
  if (!ihdr) { err = "png: no IHDR"; return false; }
  if (!iend) { err = "png: truncated file (no IEND)"; return false; }
  if (d.ctype == 3 && d.npal == 0) { err = "png: palette image without PLTE"; return false; }
  return true;
}

// zlib inflate of the IDAT stream into exactly `need` bytes (libpng: a short stream is an
// error, data past the image is ignored)
bool inflate_idat(const uint8_t* b, const std::vector<std::pair<size_t, size_t>>& idat, uint8_t* out,
                  size_t need, std::string& err) {
  z_stream z;
  memset(&z, 0, sizeof(z));
  if (inflateInit(&z) != Z_OK) { err = "png: zlib init failed"; return false; }
  z.next_out = out;
  z.avail_out = (uInt)need;
  int rc = Z_OK;
  for (size_t k = 0; k < idat.size() && rc == Z_OK && z.avail_out > 0; ++k) {
    z.next_in = const_cast<Bytef*>(b + idat[k].first);
    z.avail_in = (uInt)idat[k].second;
    while (z.avail_in > 0 && z.avail_out > 0 && rc == Z_OK) rc = inflate(&z, Z_NO_FLUSH);
  }
  const size_t got = need - z.avail_out;
  inflateEnd(&z);
  if (rc != Z_OK && rc != Z_STREAM_END && !(rc == Z_BUF_ERROR && got == need)) {
    err = "png: corrupt zlib stream";
    return false;
  }
  if (got != need) { err = "png: truncated image data"; return false; }
  return true;
}

// Every row's filter-type byte is 0..4 (libpng: "bad adaptive filter value" otherwise);
// rows = the inflated, still filtered scanlines of all passes
bool check_filters(const PngDesc& d, const uint8_t* rows, std::string& err) {
  int64_t pos = 0;
  for (int p = 0; p < (d.interlace ? 7 : 1); ++p) {
    const int x0 = d.interlace ? kA7X0h[p] : 0, y0 = d.interlace ? kA7Y0h[p] : 0;
    const int dx = d.interlace ? kA7DXh[p] : 1, dy = d.interlace ? kA7DYh[p] : 1;
    const int64_t pw = d.w > x0 ? (d.w - x0 + dx - 1) / dx : 0;
    const int64_t ph = d.h > y0 ? (d.h - y0 + dy - 1) / dy : 0;
    if (!pw || !ph) continue;
    const int64_t rb = row_bytes((int)pw, d.channels, d.depth);
    for (int64_t r = 0; r < ph; ++r, pos += 1 + rb)
      if (rows[pos] > 4) {
        err = "png: bad adaptive filter value " + std::to_string(rows[pos]) + " (pass " +
              std::to_string(p) + ", row " + std::to_string(r) + ")";
        return false;
      }
  }
  return true;
}

template <class F>
void png_parallel_for(int n, F&& f) {
  const int nt = std::max(1, std::min(8, n / 4));
  if (nt <= 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> pool;
  for (int k = 1; k < nt; ++k)
    pool.emplace_back(f, (int)((int64_t)n * k / nt), (int)((int64_t)n * (k + 1) / nt));
  f(0, n / nt);
  for (auto& th : pool) th.join();
}

struct PngStaging {
  std::mutex mu;
  uint8_t* host = nullptr;
  size_t cap = 0;
  hipEvent_t done = nullptr;
};
PngStaging& png_staging() {
  static PngStaging ring[2];
  static std::atomic<unsigned> next{0};
  return ring[next.fetch_add(1) & 1];
}

// descriptors + data layout; dims (h, w) per image when given
int png_plan(const uint8_t* const* files, const size_t* lens, int n, std::vector<PngDesc>& D,
             std::vector<std::vector<std::pair<size_t, size_t>>>* idat, int32_t* dims,
             size_t& data_off, size_t& total) {
  VTD_CHECK_ARG(files && lens && n > 0, "png: bad arguments");
  for (int i = 0; i < n; ++i) VTD_CHECK_ARG(files[i] && lens[i] > 0, "png: null / empty image");
  D.resize(n);
  if (idat) idat->assign(n, {});
  size_t data = 0;
  for (int i = 0; i < n; ++i) {
    std::string err;
    if (!parse_png(files[i], lens[i], D[i], idat ? &(*idat)[i] : nullptr, err))
      return fail(VTD_ERR_UNSUPPORTED, err + " (image " + std::to_string(i) + ")");
    D[i].data_off = (int64_t)data;
    data += align256((size_t)filtered_bytes(D[i]));
    if (dims) {
      dims[2 * i] = D[i].h;
      dims[2 * i + 1] = D[i].w;
    }
  }
  data_off = align256((size_t)n * sizeof(PngDesc));
  total = data_off + data;
  return VTD_OK;
}

}  // namespace
}  // namespace vtd

extern "C" int vtd_png_info(const uint8_t* png, size_t len, int* h, int* w, int* comps) {
  VTD_CHECK_ARG(png && len > 0 && h && w && comps, "png_info: bad arguments");
  vtd::PngDesc d;
  std::string err;
  if (!vtd::parse_png(png, len, d, nullptr, err)) return vtd::fail(VTD_ERR_UNSUPPORTED, err);
  *h = d.h;
  *w = d.w;
  *comps = d.channels;
  return VTD_OK;
}

// The host half of vtd_png_decode for one file: the chunk walk, the zlib inflate of the IDAT
// stream and the filter-byte check, into a caller host buffer (no device call)
extern "C" int vtd_png_inflate(const uint8_t* png, size_t len, uint8_t* out, size_t out_bytes,
                               size_t* need) {
  VTD_CHECK_ARG(png && len > 0 && need, "png_inflate: bad arguments");
  vtd::PngDesc d;
  std::vector<std::pair<size_t, size_t>> idat;
  std::string err;
  if (!vtd::parse_png(png, len, d, &idat, err)) return vtd::fail(VTD_ERR_UNSUPPORTED, err);
  *need = (size_t)vtd::filtered_bytes(d);
  if (!out) return VTD_OK;
  if (out_bytes < *need) return vtd::fail(VTD_ERR_WORKSPACE, "png_inflate: output buffer too small");
  if (!vtd::inflate_idat(png, idat, out, *need, err) || !vtd::check_filters(d, out, err))
    return vtd::fail(VTD_ERR_UNSUPPORTED, err);
  return VTD_OK;
}

extern "C" int vtd_png_workspace_bytes(const uint8_t* const* pngs, const size_t* lens, int n,
                                       int32_t* dims, size_t* bytes) {
  VTD_CHECK_ARG(bytes, "png_workspace_bytes: null bytes pointer");
  std::vector<vtd::PngDesc> D;
  size_t data_off = 0, total = 0;
  const int rc = vtd::png_plan(pngs, lens, n, D, nullptr, dims, data_off, total);
  if (rc != VTD_OK) return rc;
  *bytes = total;
  return VTD_OK;
}

extern "C" int vtd_png_decode(const uint8_t* const* pngs, const size_t* lens, int n,
                              uint8_t* out_dev, const int64_t* out_offsets, void* workspace_dev,
                              size_t workspace_bytes, void* stream) {
  using namespace vtd;
  VTD_CHECK_ARG(out_dev && out_offsets && workspace_dev, "png_decode: null pointer");
  VTD_CHECK_ARG(n <= 65535, "png_decode: at most 65535 images per call");
  std::vector<PngDesc> D;
  std::vector<std::vector<std::pair<size_t, size_t>>> idat;
  size_t data_off = 0, total = 0;
  int rc = png_plan(pngs, lens, n, D, &idat, nullptr, data_off, total);
  if (rc != VTD_OK) return rc;
  if (workspace_bytes < total) return fail(VTD_ERR_WORKSPACE, "png_decode: workspace too small");
  for (int i = 0; i < n; ++i) D[i].out_off = out_offsets[i];
  hipStream_t st = static_cast<hipStream_t>(stream);
  PngStaging& sg = png_staging();
  std::lock_guard<std::mutex> g(sg.mu);
  if (sg.done) {
    const hipError_t e = hipEventSynchronize(sg.done);
    if (e != hipSuccess) return fail(VTD_ERR_HIP, std::string("png: ") + hipGetErrorString(e));
  } else if (hipEventCreateWithFlags(&sg.done, hipEventDisableTiming) != hipSuccess) {
    return fail(VTD_ERR_HIP, "png: event create failed");
  }
  if (sg.cap < total) {
    if (sg.host) (void)hipHostFree(sg.host);
    sg.host = nullptr;
    sg.cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&sg.host), total) != hipSuccess)
      return fail(VTD_ERR_HIP, "png: pinned staging allocation failed");
    sg.cap = total;
  }
  std::vector<std::string> errs(n);
  std::vector<char> ok(n, 1);
  png_parallel_for(n, [&](int i0, int i1) {
    for (int i = i0; i < i1; ++i)
      ok[i] = inflate_idat(pngs[i], idat[i], sg.host + data_off + D[i].data_off,
                           (size_t)filtered_bytes(D[i]), errs[i]) &&
              check_filters(D[i], sg.host + data_off + D[i].data_off, errs[i]);
  });
  for (int i = 0; i < n; ++i)
    if (!ok[i]) return fail(VTD_ERR_UNSUPPORTED, errs[i] + " (image " + std::to_string(i) + ")");
  memcpy(sg.host, D.data(), n * sizeof(PngDesc));
  uint8_t* ws = static_cast<uint8_t*>(workspace_dev);
  hipError_t e = hipMemcpyAsync(ws, sg.host, total, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipEventRecord(sg.done, st);
  if (e != hipSuccess) return fail(VTD_ERR_HIP, std::string("png: ") + hipGetErrorString(e));
  ProfScope ps(st, PROF_OTHER, 0.0);
  hipLaunchKernelGGL(png_unfilter_kernel, dim3(n), dim3(kPngThreads), 0, st,
                     reinterpret_cast<const PngDesc*>(ws), ws + data_off, out_dev);
  VTD_LAUNCH_CHECK("png_unfilter");
  return VTD_OK;
}

// ------------------------------------------------------------------ BMP
// `tf.image.decode_image(file, channels=3)` on BMP files: TF 2.x's decode_image is the
// DecodeImageV2 op (tensorflow/core/kernels/image/decode_image_op.cc, DecodeBmpV2): it reads
// bits-per-pixel (byte 28) and the pixel-array offset (byte 10), takes the file's channels =
// bpp / 8 (1, 3 or 4; anything else is an error), row size (bpp * w + 31) / 32 * 4, bottom-up
// rows unless the height is negative, and converts to the 3 requested channels: 8-bit -> the
// byte replicated (the palette is NOT applied), 24-bit BGR -> RGB, 32-bit BGRA -> RGB (alpha
// dropped).  The compression field is not read by TF; here BI_RGB (0) and BI_BITFIELDS (3)
// files decode that way and every other value (RLE 1 / 2, BI_JPEG 4, BI_PNG 5, ...), whose
// bytes TF would misread as pixels, is refused.  TF is not importable here: parity against it is unpinned (restated from that
// source).  The host reads the header; the pixel array goes to the workspace in one copy and
// bmp_convert_kernel (one thread per output pixel) writes the RGB8 rows.
namespace vtd {
namespace {

struct BmpDesc {
  int w, h, top_down, row_size, in_ch;
  int64_t data_off, out_off;
};

__global__ __launch_bounds__(256) void bmp_convert_kernel(const BmpDesc* __restrict__ descs,
                                                          const uint8_t* __restrict__ data,
                                                          uint8_t* __restrict__ out) {
  const BmpDesc& d = descs[blockIdx.y];
  const int64_t npx = (int64_t)d.w * d.h;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < npx; i += (int64_t)gridDim.x * 256) {
    const int y = (int)(i / d.w), x = (int)(i - (int64_t)y * d.w);
    const int sy = d.top_down ? y : d.h - 1 - y;
    const uint8_t* s = data + d.data_off + (int64_t)sy * d.row_size + (int64_t)d.in_ch * x;
    uint8_t* o = out + d.out_off + 3 * i;
    if (d.in_ch == 1) {
      o[0] = o[1] = o[2] = s[0];
    } else {
      o[0] = s[2];
      o[1] = s[1];
      o[2] = s[0];
    }
  }
}

int32_t le32(const uint8_t* p) { return (int32_t)((uint32_t)p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24); }
int le16(const uint8_t* p) { return p[0] | p[1] << 8; }

bool parse_bmp(const uint8_t* b, size_t n, BmpDesc& d, int64_t& pix_off, std::string& err) {
  memset(&d, 0, sizeof(d));
  if (n < 54 || b[0] != 'B' || b[1] != 'M') { err = "bmp: not a BMP file"; return false; }
  pix_off = le32(b + 10);
  const int32_t w = le32(b + 18), h = le32(b + 22);
  const int bpp = le16(b + 28);
  const int32_t comp = le32(b + 30);
  if (bpp != 8 && bpp != 24 && bpp != 32) {
    err = "bmp: " + std::to_string(bpp) + "-bit file: TF's decoder takes 8-, 24- and 32-bit "
          "files (channels = bits-per-pixel / 8 in 1, 3, 4)";
    return false;
  }
  if (comp != 0 && comp != 3) {      // BI_RGB, BI_BITFIELDS (the default masks) only
    err = comp == 1 || comp == 2
              ? "bmp: RLE-compressed BMP files are not supported (TF's decoder reads every file "
                "as uncompressed rows)"
              : "bmp: compression " + std::to_string(comp) + " (BI_JPEG / BI_PNG / other) is not "
                "supported: only uncompressed rows (BI_RGB, BI_BITFIELDS) decode";
    return false;
  }
  if (w <= 0 || h == 0 || h == INT32_MIN) { err = "bmp: bad size"; return false; }
  if ((int64_t)w * (h < 0 ? -(int64_t)h : h) > ((int64_t)1 << 28)) {
    err = "bmp: image larger than 2^28 pixels";
    return false;
  }
  d.w = w;
  d.h = h < 0 ? -h : h;
  d.top_down = h < 0;
  d.in_ch = bpp / 8;
  d.row_size = (int)(((int64_t)bpp * w + 31) / 32 * 4);
  if (pix_off < 54 || (uint64_t)pix_off + (uint64_t)d.row_size * d.h > n) {
    err = "bmp: truncated pixel array";
    return false;
  }
  return true;
}

int bmp_plan(const uint8_t* const* files, const size_t* lens, int n, std::vector<BmpDesc>& D,
             std::vector<int64_t>& pix, int32_t* dims, size_t& data_off, size_t& total) {
  VTD_CHECK_ARG(files && lens && n > 0, "bmp: bad arguments");
  D.resize(n);
  pix.resize(n);
  size_t data = 0;
  for (int i = 0; i < n; ++i) {
    VTD_CHECK_ARG(files[i] && lens[i] > 0, "bmp: null / empty image");
    std::string err;
    if (!parse_bmp(files[i], lens[i], D[i], pix[i], err))
      return fail(VTD_ERR_UNSUPPORTED, err + " (image " + std::to_string(i) + ")");
    D[i].data_off = (int64_t)data;
    data += align256((size_t)D[i].row_size * D[i].h);
    if (dims) {
      dims[2 * i] = D[i].h;
      dims[2 * i + 1] = D[i].w;
    }
  }
  data_off = align256((size_t)n * sizeof(BmpDesc));
  total = data_off + data;
  return VTD_OK;
}

}  // namespace
}  // namespace vtd

extern "C" int vtd_bmp_info(const uint8_t* bmp, size_t len, int* h, int* w, int* comps) {
  VTD_CHECK_ARG(bmp && len > 0 && h && w && comps, "bmp_info: bad arguments");
  vtd::BmpDesc d;
  int64_t pix = 0;
  std::string err;
  if (!vtd::parse_bmp(bmp, len, d, pix, err)) return vtd::fail(VTD_ERR_UNSUPPORTED, err);
  *h = d.h;
  *w = d.w;
  *comps = 3;
  return VTD_OK;
}

extern "C" int vtd_bmp_workspace_bytes(const uint8_t* const* bmps, const size_t* lens, int n,
                                       int32_t* dims, size_t* bytes) {
  VTD_CHECK_ARG(bytes, "bmp_workspace_bytes: null bytes pointer");
  std::vector<vtd::BmpDesc> D;
  std::vector<int64_t> pix;
  size_t data_off = 0, total = 0;
  const int rc = vtd::bmp_plan(bmps, lens, n, D, pix, dims, data_off, total);
  if (rc != VTD_OK) return rc;
  *bytes = total;
  return VTD_OK;
}

extern "C" int vtd_bmp_decode(const uint8_t* const* bmps, const size_t* lens, int n,
                              uint8_t* out_dev, const int64_t* out_offsets, void* workspace_dev,
                              size_t workspace_bytes, void* stream) {
  using namespace vtd;
  VTD_CHECK_ARG(out_dev && out_offsets && workspace_dev, "bmp_decode: null pointer");
  VTD_CHECK_ARG(n <= 65535, "bmp_decode: at most 65535 images per call");
  std::vector<BmpDesc> D;
  std::vector<int64_t> pix;
  size_t data_off = 0, total = 0;
  int rc = bmp_plan(bmps, lens, n, D, pix, nullptr, data_off, total);
  if (rc != VTD_OK) return rc;
  if (workspace_bytes < total) return fail(VTD_ERR_WORKSPACE, "bmp_decode: workspace too small");
  int64_t maxpx = 0;
  for (int i = 0; i < n; ++i) {
    D[i].out_off = out_offsets[i];
    maxpx = std::max<int64_t>(maxpx, (int64_t)D[i].w * D[i].h);
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  PngStaging& sg = png_staging();
  std::lock_guard<std::mutex> g(sg.mu);
  if (sg.done) {
    const hipError_t e = hipEventSynchronize(sg.done);
    if (e != hipSuccess) return fail(VTD_ERR_HIP, std::string("bmp: ") + hipGetErrorString(e));
  } else if (hipEventCreateWithFlags(&sg.done, hipEventDisableTiming) != hipSuccess) {
    return fail(VTD_ERR_HIP, "bmp: event create failed");
  }
  if (sg.cap < total) {
    if (sg.host) (void)hipHostFree(sg.host);
    sg.host = nullptr;
    sg.cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&sg.host), total) != hipSuccess)
      return fail(VTD_ERR_HIP, "bmp: pinned staging allocation failed");
    sg.cap = total;
  }
  memcpy(sg.host, D.data(), n * sizeof(BmpDesc));
  for (int i = 0; i < n; ++i)
    memcpy(sg.host + data_off + D[i].data_off, bmps[i] + pix[i], (size_t)D[i].row_size * D[i].h);
  uint8_t* ws = static_cast<uint8_t*>(workspace_dev);
  hipError_t e = hipMemcpyAsync(ws, sg.host, total, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipEventRecord(sg.done, st);
  if (e != hipSuccess) return fail(VTD_ERR_HIP, std::string("bmp: ") + hipGetErrorString(e));
  ProfScope ps(st, PROF_OTHER, 0.0);
  const unsigned gx = (unsigned)std::min<int64_t>(1024, (maxpx + 255) / 256);
  hipLaunchKernelGGL(bmp_convert_kernel, dim3(gx, n), dim3(256), 0, st,
                     reinterpret_cast<const BmpDesc*>(ws), ws + data_off, out_dev);
  VTD_LAUNCH_CHECK("bmp_convert");
  return VTD_OK;
}
