// MX-fp8 operand quantization for the VTD_FP8 mode ("fp8 e4m3 weights
// on CDNA4 fp8 MFMA").  OCP MX format: elements OCP e4m3 (gfx950 v_cvt_pk_fp8_f32,
// round-to-nearest-even), one E8M0 scale (byte e = 2^(e - 127)) per 32 consecutive
// elements along K, consumed by v_mfma_scale_f32_16x16x128_f8f6f4 (vtd_gemm.hip).
//
// Block scale: the smallest power of two 2^E with amax <= 448 * 2^E (448 = e4m3 max),
// E clamped to [-126, 126]; amax = m * 2^ex (frexp, m in [0.5, 1)) gives
// E = ex - 9 + (m > 0.875), exact integer logic restated by oracle/mx8.py.
// Layout: q[row][ldq] bytes (columns [K, Kq) zero); scales s[k / 128][s_rows][4]: the four
// block scales of one 128-wide K-step of a row form one dword, so the GEMM stages a
// tile's scales for a K-step as one contiguous 1-KiB block.
#include <algorithm>

#include "vtd_common.h"

namespace vtd {

namespace {

// one thread per 32-element block; consecutive threads take consecutive blocks of a row
template <typename T>
__global__ __launch_bounds__(256) void quantize_mx8_kernel(
    const T* __restrict__ x, int64_t rows, int K, int ldx, int Kq, uint8_t* __restrict__ q,
    int ldq, uint8_t* __restrict__ s, int64_t s_rows) {
  const int nb = Kq >> 5;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * nb) return;
  const int64_t r = t / nb;
  const int blk = (int)(t - r * nb), k0 = blk * 32;
  float v[32];
  if constexpr (sizeof(T) == 2) {
    const bf16_t* p = reinterpret_cast<const bf16_t*>(x) + r * ldx + k0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      i32x4 w = k0 + 8 * c + 8 <= K ? *reinterpret_cast<const i32x4*>(p + 8 * c)
                                    : i32x4{0, 0, 0, 0};
      if (k0 + 8 * c < K && k0 + 8 * c + 8 > K) {    // ragged K (never with K % 8 == 0)
        for (int j = 0; j < 8; ++j) reinterpret_cast<bf16_t*>(&w)[j] = k0 + 8 * c + j < K ? p[8 * c + j] : 0;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t u = (uint32_t)w[j];
        v[8 * c + 2 * j] = __uint_as_float(u << 16);
        v[8 * c + 2 * j + 1] = __uint_as_float(u & 0xffff0000u);
      }
    }
  } else {
    const float* p = reinterpret_cast<const float*>(x) + r * ldx + k0;
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = k0 + j < K ? p[j] : 0.f;
  }
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
  const int E = mx8_exponent(amax);
  const float inv = __uint_as_float((uint32_t)(127 - E) << 23);     // 2^-E, exact
  i32x4 o[2];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* vv = v + 16 * c + 4 * j;
      int w = __builtin_amdgcn_cvt_pk_fp8_f32(vv[0] * inv, vv[1] * inv, 0, false);
      w = __builtin_amdgcn_cvt_pk_fp8_f32(vv[2] * inv, vv[3] * inv, w, true);
      o[c][j] = w;
    }
  uint8_t* qp = q + r * ldq + k0;
  *reinterpret_cast<i32x4*>(qp) = o[0];
  *reinterpret_cast<i32x4*>(qp + 16) = o[1];
  s[((int64_t)(k0 >> 7) * s_rows + r) * 4 + (blk & 3)] = (uint8_t)(E + 127);
}

}  // namespace

int quantize_mx8_launch(const void* x, int x_dtype, int64_t rows, int K, int ldx, int Kq,
                        uint8_t* q, int ldq, uint8_t* s, int64_t s_rows, hipStream_t st) {
  VTD_CHECK_ARG(x && q && s, "quantize_mx8: null pointer");
  VTD_CHECK_ARG(rows > 0 && K > 0 && ldx >= K && Kq >= K && Kq % 128 == 0 && ldq >= Kq &&
                    ldq % 16 == 0 && s_rows >= rows,
                "quantize_mx8: bad shape (Kq % 128, ldq % 16, ldq >= Kq >= K, s_rows >= rows)");
  VTD_CHECK_ARG(x_dtype == VTD_F32 || (x_dtype == VTD_BF16 && ldx % 8 == 0),
                "quantize_mx8: x dtype must be F32 or BF16 (ldx % 8)");
  ProfScope ps(st, PROF_OTHER, 0.0);
  const int64_t total = rows * (Kq / 32);
  const unsigned grid = (unsigned)((total + 255) / 256);
  if (x_dtype == VTD_BF16)
    hipLaunchKernelGGL(quantize_mx8_kernel<bf16_t>, dim3(grid), dim3(256), 0, st,
                       static_cast<const bf16_t*>(x), rows, K, ldx, Kq, q, ldq, s, s_rows);
  else
    hipLaunchKernelGGL(quantize_mx8_kernel<float>, dim3(grid), dim3(256), 0, st,
                       static_cast<const float*>(x), rows, K, ldx, Kq, q, ldq, s, s_rows);
  VTD_LAUNCH_CHECK("quantize_mx8");
  return VTD_OK;
}

}  // namespace vtd

extern "C" int vtd_quantize_mx8(const void* x_dev, int x_dtype, int64_t rows, int K, int ldx,
                                int Kq, uint8_t* q_dev, int ldq, uint8_t* s_dev,
                                int64_t s_rows, void* stream) {
  return vtd::quantize_mx8_launch(x_dev, x_dtype, rows, K, ldx, Kq, q_dev, ldq, s_dev, s_rows,
                                  static_cast<hipStream_t>(stream));
}
