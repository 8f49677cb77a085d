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
// consecutive pixels of the flattened [TH*TW] plane = 48 contiguous bytes. A block's 12 KiB
// of output go through LDS and out as three coalesced 16-B stores per thread (lane i writes
// bytes [16 i, 16 i + 16) of each KiB): storing each thread's 48 B directly (three 16-B
// stores at a 48-B lane stride) ran 13% (608^2) to 16% (224^2) slower. Staging the source
// rows in LDS too (a band kernel, measured) did not pay: 2 workgroups per CU at 60 KiB.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

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
__device__ __forceinline__ void pixel(const uint8_t* __restrict__ src, const Geom& g, int y,
                                      int x, float* o) {
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
  const uint8_t* r0 = src + (int64_t)y0 * g.w * 3;
  const uint8_t* r1 = src + (int64_t)y1 * g.w * 3;
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
  __shared__ f32x4 stg[256 * 3];
  const int b = blockIdx.y;
  const int64_t plane = (int64_t)th * tw;
  const int64_t p0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  // whole block inside the plane and 16-B aligned: the block's 12 KiB of output go out as
  // 3 coalesced 16-B stores per thread (lane i writes bytes [16 i, 16 i + 16) of each KiB)
  // through LDS, instead of three 16-B stores at a 48-B lane stride
  float* blk = out + ((int64_t)b * plane + (int64_t)blockIdx.x * blockDim.x * 4) * 3;
  const bool coalesce = ((int64_t)blockIdx.x + 1) * blockDim.x * 4 <= plane &&
                        (reinterpret_cast<uintptr_t>(blk) & 15) == 0;
  if (coalesce) {
    const Geom g = geometry(sizes[2 * b], sizes[2 * b + 1], th, tw);
    const uint8_t* src = pixels + offsets[b];
    float v[12];
    int y = (int)(p0 / tw), x = (int)(p0 - (int64_t)y * tw);
    for (int i = 0; i < 4; ++i) {
      pixel(src, g, y, x, v + 3 * i);
      if (++x == tw) { x = 0; ++y; }
    }
    const int t = threadIdx.x;
    stg[3 * t] = f32x4{v[0], v[1], v[2], v[3]};
    stg[3 * t + 1] = f32x4{v[4], v[5], v[6], v[7]};
    stg[3 * t + 2] = f32x4{v[8], v[9], v[10], v[11]};
    __syncthreads();
    f32x4* d4 = reinterpret_cast<f32x4*>(blk);
#pragma unroll
    for (int k = 0; k < 3; ++k) d4[k * 256 + t] = stg[k * 256 + t];
    return;
  }
  if (p0 >= plane) return;
  const Geom g = geometry(sizes[2 * b], sizes[2 * b + 1], th, tw);
  const uint8_t* src = pixels + offsets[b];
  float* dst = out + ((int64_t)b * plane + p0) * 3;
  float v[12];
  const int n = (int)min<int64_t>(4, plane - p0);
  int y = (int)(p0 / tw), x = (int)(p0 - (int64_t)y * tw);
  for (int i = 0; i < n; ++i) {
    pixel(src, g, y, x, v + 3 * i);
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
  hipLaunchKernelGGL(vtd::resize_with_pad_kernel, dim3((unsigned)((groups + 255) / 256), B),
                     dim3(256), 0, st, pixels_dev, offsets_dev, sizes_dev, target_h, target_w,
                     out_dev);
  VTD_LAUNCH_CHECK("resize_with_pad");
  return VTD_OK;
}

}  // extern "C"
