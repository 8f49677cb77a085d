// Input pipeline image transform on the device:
// _get_image_tensor_coco (vision_transformer_utilities.py:418-449) after decode, i.e.
//   tf.image.resize_with_pad(image, 608, 608)   (bilinear, half_pixel_centers, no antialias)
//   -> tf.clip_by_value(0, 255) -> / 127.5 -> - 1
// for a batch of decoded uint8 HWC images of different sizes, written straight into the
// model's NHWC fp32 input batch.
//
// The upstream arithmetic (TF 2.9 image_ops_impl._resize_image_with_pad_common and the
// CPU ResizeBilinear kernel) is restated in oracle/preprocess.py; every float32 operation
// here happens in that order (this file is compiled with -ffp-contract=off, see the
// Makefile), so the output is bit-identical to the restatement.
//
// Shape of the work: HBM-bound byte work. Each output pixel reads <= 4 source pixels (L2
// resident: a decoded COCO image is <= 1 MB) and writes 12 B; a thread produces 4
// consecutive pixels of the flattened [TH*TW] plane = 48 contiguous bytes, stored as three
// 16-B vector stores, so a wave writes 3 KiB of contiguous output per instruction triple.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "vtd_common.h"

#pragma clang fp contract(off)

namespace vtd {
namespace {

// Per-image geometry, computed by every thread from (h, w) exactly as TF does in float32
// (_resize_image_with_pad_common): ratio = max(w / tw, h / th); resized = floor(side / ratio);
// pad_before = max(0, floor((target - side / ratio) / 2)); bilinear scale = side / resized.
struct Geom {
  int h, w, rh, rw, ph, pw;
  float sy, sx;
};

__device__ __forceinline__ Geom geometry(int h, int w, int th, int tw) {
  Geom g;
  g.h = h;
  g.w = w;
  const float fh = (float)h, fw = (float)w, fth = (float)th, ftw = (float)tw;
  const float ratio = fmaxf(fw / ftw, fh / fth);
  const float rhf = fh / ratio, rwf = fw / ratio;
  g.rh = (int)floorf(rhf);
  g.rw = (int)floorf(rwf);
  g.ph = max(0, (int)floorf((fth - rhf) / 2.f));
  g.pw = max(0, (int)floorf((ftw - rwf) / 2.f));
  // CalculateResizeScale(in, out, align_corners=false) = in / (float)out
  g.sy = g.rh > 0 ? fh / (float)g.rh : 0.f;
  g.sx = g.rw > 0 ? fw / (float)g.rw : 0.f;
  return g;
}

// One output pixel (3 channels) of the padded, normalised image.
// src points at source row ylo of the image (the whole image: ylo = 0; an LDS-staged band of
// rows: its first row).
__device__ __forceinline__ void pixel(const uint8_t* __restrict__ src, int ylo, const Geom& g,
                                      int y, int x, float* o) {
  const int ry = y - g.ph, rx = x - g.pw;
  if (ry < 0 || ry >= g.rh || rx < 0 || rx >= g.rw) {  // pad_to_bounding_box zeros
    o[0] = o[1] = o[2] = -1.f;                         // 0 / 127.5 - 1
    return;
  }
  // HalfPixelScaler: in = (i + 0.5) * scale - 0.5; lower = max(floor(in), 0),
  // upper = min(ceil(in), size - 1), lerp = in - floor(in)
  const float iny = ((float)ry + 0.5f) * g.sy - 0.5f;
  const float inx = ((float)rx + 0.5f) * g.sx - 0.5f;
  const float fy = floorf(iny), fx = floorf(inx);
  const int y0 = max((int)fy, 0), y1 = min((int)ceilf(iny), g.h - 1);
  const int x0 = max((int)fx, 0), x1 = min((int)ceilf(inx), g.w - 1);
  const float ly = iny - fy, lx = inx - fx;
  const uint8_t* r0 = src + (int64_t)(y0 - ylo) * g.w * 3;
  const uint8_t* r1 = src + (int64_t)(y1 - ylo) * g.w * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float tl = r0[x0 * 3 + c], tr = r0[x1 * 3 + c];
    const float bl = r1[x0 * 3 + c], br = r1[x1 * 3 + c];
    const float top = tl + (tr - tl) * lx;               // compute_lerp
    const float bottom = bl + (br - bl) * lx;
    float v = top + (bottom - top) * ly;
    v = fminf(fmaxf(v, 0.f), 255.f);                     // clip_by_value
    o[c] = v / 127.5f - 1.f;
  }
}

// grid (ceil(TH*TW / 4 / 256), B); 4 flattened pixels per thread.
__global__ __launch_bounds__(256) void resize_with_pad_kernel(
    const uint8_t* __restrict__ pixels, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ sizes, int th, int tw, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int64_t plane = (int64_t)th * tw;
  const int64_t p0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (p0 >= plane) return;
  const Geom g = geometry(sizes[2 * b], sizes[2 * b + 1], th, tw);
  const uint8_t* src = pixels + offsets[b];
  float* dst = out + ((int64_t)b * plane + p0) * 3;
  float v[12];
  const int n = (int)min<int64_t>(4, plane - p0);
  int y = (int)(p0 / tw), x = (int)(p0 - (int64_t)y * tw);
  for (int i = 0; i < n; ++i) {
    pixel(src, 0, g, y, x, v + 3 * i);
    if (++x == tw) { x = 0; ++y; }
  }
  if (n == 4 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    f32x4* d4 = reinterpret_cast<f32x4*>(dst);
    d4[0] = f32x4{v[0], v[1], v[2], v[3]};
    d4[1] = f32x4{v[4], v[5], v[6], v[7]};
    d4[2] = f32x4{v[8], v[9], v[10], v[11]};
  } else {
    for (int i = 0; i < 3 * n; ++i) dst[i] = v[i];
  }
}

// 4 output pixels starting at (y, x) of row-major plane position p -> dst (16-B stores when
// aligned and whole).
__device__ __forceinline__ void pixels4(const uint8_t* __restrict__ src, int ylo, const Geom& g,
                                        int y, int x, int tw, int n, float* __restrict__ dst) {
  float v[12];
  for (int i = 0; i < n; ++i) {
    pixel(src, ylo, g, y, x, v + 3 * i);
    if (++x == tw) { x = 0; ++y; }
  }
  if (n == 4 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    f32x4* d4 = reinterpret_cast<f32x4*>(dst);
    d4[0] = f32x4{v[0], v[1], v[2], v[3]};
    d4[1] = f32x4{v[4], v[5], v[6], v[7]};
    d4[2] = f32x4{v[8], v[9], v[10], v[11]};
  } else {
    for (int i = 0; i < 3 * n; ++i) dst[i] = v[i];
  }
}

// Band kernel (default): one workgroup = `rows` output rows of one image (rows * TW ~ 2048
// pixels, so that every thread of the block produces about two 4-pixel groups). The source rows
// those rows' taps touch are one contiguous byte range of the HWC image; the workgroup copies
// the 16-B blocks covering it into LDS with coalesced 16-B loads (a block holding at least one
// byte of the image lies in a mapped page, so the rounding never faults), then every tap is an
// LDS byte read instead of a global one. Bands whose rows need more than STAGE_BYTES (source
// images more than ~20x the target height's downscale) read global memory directly.
constexpr int STAGE_BYTES = 48 * 1024;

__global__ __launch_bounds__(256) void resize_with_pad_band_kernel(
    const uint8_t* __restrict__ pixels, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ sizes, int th, int tw, int rows, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE_BYTES];
  const int b = blockIdx.y;
  const int yb = blockIdx.x * rows, ye = min(yb + rows, th);
  const Geom g = geometry(sizes[2 * b], sizes[2 * b + 1], th, tw);
  const uint8_t* img = pixels + offsets[b];
  // resized rows [ra, rb) inside the band, their source rows [lo, hi]
  const int ra = max(yb - g.ph, 0), rb = min(ye - g.ph, g.rh);
  int lo = 0, hi = 0;
  if (ra < rb) {
    const float ina = ((float)ra + 0.5f) * g.sy - 0.5f;
    const float inb = ((float)(rb - 1) + 0.5f) * g.sy - 0.5f;
    lo = max((int)floorf(ina), 0);
    hi = min((int)ceilf(inb), g.h - 1);
  }
  const int64_t row_bytes = (int64_t)g.w * 3;
  const uintptr_t s0 = reinterpret_cast<uintptr_t>(img + lo * row_bytes);
  const uintptr_t s1 = reinterpret_cast<uintptr_t>(img + (hi + 1) * row_bytes);
  const uintptr_t a0 = s0 & ~(uintptr_t)15, a1 = (s1 + 15) & ~(uintptr_t)15;
  const bool staged = ra < rb && a1 - a0 <= (uintptr_t)STAGE_BYTES;   // uniform per block
  if (staged) {
    const int nblk = (int)((a1 - a0) >> 4);
    const i32x4* gsrc = reinterpret_cast<const i32x4*>(img + lo * row_bytes - (s0 - a0));
    for (int i = threadIdx.x; i < nblk; i += blockDim.x)
      reinterpret_cast<i32x4*>(stage)[i] = gsrc[i];
  }
  __syncthreads();
  const int nband = (ye - yb) * tw;
  float* dst0 = out + ((int64_t)b * th * tw + (int64_t)yb * tw) * 3;
  for (int q = threadIdx.x * 4; q < nband; q += blockDim.x * 4) {
    const int y = yb + q / tw, x = q - (q / tw) * tw, n = min(4, nband - q);
    if (staged)
      pixels4(stage + (s0 - a0), lo, g, y, x, tw, n, dst0 + (int64_t)q * 3);
    else
      pixels4(img, 0, g, y, x, tw, n, dst0 + (int64_t)q * 3);
  }
}

}  // namespace
}  // namespace vtd

extern "C" {

int vtd_resize_with_pad(const uint8_t* pixels_dev, const int64_t* offsets_dev,
                        const int32_t* sizes_dev, int B, int target_h, int target_w,
                        float* out_dev, void* stream) {
  VTD_CHECK_ARG(pixels_dev && offsets_dev && sizes_dev && out_dev, "resize_with_pad: null pointer");
  VTD_CHECK_ARG(B > 0 && B <= 65535 && target_h > 0 && target_w > 0,
                "resize_with_pad: bad batch / target size");
  const int64_t plane = (int64_t)target_h * target_w;
  const int64_t groups = (plane + 3) / 4;
  VTD_CHECK_ARG((groups + 255) / 256 < (1LL << 31), "resize_with_pad: target too large");
  hipStream_t st = static_cast<hipStream_t>(stream);
  vtd::ProfScope ps(st, vtd::PROF_OTHER, 0.0);
  static const int variant = [] {
    const char* v = getenv("VTD_RESIZE_VARIANT");
    return v ? atoi(v) : 1;
  }();
  if (variant == 0)   // one thread per 4 pixels, taps read from global memory
    hipLaunchKernelGGL(vtd::resize_with_pad_kernel, dim3((unsigned)((groups + 255) / 256), B),
                       dim3(256), 0, st, pixels_dev, offsets_dev, sizes_dev, target_h, target_w,
                       out_dev);
  else {
    const int rows = std::max(1, std::min(32, (2048 + target_w - 1) / target_w));
    hipLaunchKernelGGL(vtd::resize_with_pad_band_kernel,
                       dim3((unsigned)((target_h + rows - 1) / rows), B), dim3(256), 0, st,
                       pixels_dev, offsets_dev, sizes_dev, target_h, target_w, rows, out_dev);
  }
  VTD_LAUNCH_CHECK("resize_with_pad");
  return VTD_OK;
}

}  // extern "C"
