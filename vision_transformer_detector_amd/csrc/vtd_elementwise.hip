// HBM-bound kernels of the forward path: LayerNorm (vtd.py:353-357, 375-379),
// ExtractImagePatches + flatten (vtd.py:177-206, 279-280), transform_predictions
// (vtd.py:586-647), and the one-time weight packing.
#include "vtd_common.h"

namespace vtd {

namespace {

// ------------------------------------------------------------------ LayerNorm
// One wave per token row; row held in registers as NV float4 per lane -> exact
// two-pass mean / biased variance, eps added to the variance (keras default 1e-3).
// 4 consecutive elements as f32 (16-B f32 / 8-B bf16 accesses)
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 ld4(const bf16_t* p) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
  return f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
               __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
}
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void st4(bf16_t* p, f32x4 v) {
  *reinterpret_cast<uint2*>(p) = uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
}

// split-bf16 output (VTD_BF16X3 A operand): [hi | lo] at p, p + P
__device__ __forceinline__ void st4x3(bf16_t* p, int P, f32x4 v) {
  const uint32_t h0 = pack_bf16x2(v[0], v[1]), h1 = pack_bf16x2(v[2], v[3]);
  const uint2 hi = {h0, h1}, lo = {pack_lo_bf16x2(v[0], v[1], h0), pack_lo_bf16x2(v[2], v[3], h1)};
  *reinterpret_cast<uint2*>(p) = hi;
  *reinterpret_cast<uint2*>(p + P) = lo;
}
// one element of a row of width ldy: plain, or split over two ldy / 2 wide pieces (X3)
template <bool X3, typename TO>
__device__ __forceinline__ void st1(TO* yr, int c, int P, float v) {
  if constexpr (X3) {
    const bf16_t h = f32_to_bf16(v);
    yr[c] = h;
    yr[P + c] = lo_bf16(v, h);
  } else {
    yr[c] = DT<TO>::from(v);
  }
}
template <bool X3, typename TO>
__device__ __forceinline__ void st4v(TO* p, int P, f32x4 v) {
  if constexpr (X3) st4x3(p, P, v);
  else st4(p, v);
}

// TI: the residual stream's dtype (f32, or bf16 in the bf16 / fp8 modes); TO: output.
// X3: TO = bf16_t and the output is the split-bf16 operand, two ldy / 2 wide pieces.
template <typename TI, typename TO, int NV, bool X3 = false>
__global__ __launch_bounds__(256) void layernorm_kernel(
    const TI* __restrict__ x, int64_t rows, int D, int ldx,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    TO* __restrict__ y, int ldy) {
  const int P = X3 ? ldy / 2 : ldy;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TI* xr = x + row * ldx;
  f32x4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    v[i] = c < D ? ld4(xr + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  s = wave_sum(s);
  const float mean = s / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
  }
  q = wave_sum(q);
  const float rstd = 1.f / sqrtf(q / D + eps);
  TO* yr = y + row * ldy;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      const f32x4 g = *reinterpret_cast<const f32x4*>(gamma + c);
      const f32x4 bb = *reinterpret_cast<const f32x4*>(beta + c);
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + bb[j];
      st4v<X3>(yr + c, P, o);
    }
  }
  for (int c = D + lane; c < P; c += 64) st1<X3>(yr, c, P, 0.f);
}

// generic fallback (unaligned, D % 4 != 0 or D > 4096): three passes over the row
template <typename TI, typename TO, bool X3 = false>
__global__ __launch_bounds__(256) void layernorm_generic_kernel(
    const TI* __restrict__ x, int64_t rows, int D, int ldx,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    TO* __restrict__ y, int ldy) {
  const int P = X3 ? ldy / 2 : ldy;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TI* xr = x + row * ldx;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += DT<TI>::load(xr + c);
  s = wave_sum(s);
  const float mean = s / D;
  float q = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float d = DT<TI>::load(xr + c) - mean;
    q += d * d;
  }
  q = wave_sum(q);
  const float rstd = 1.f / sqrtf(q / D + eps);
  TO* yr = y + row * ldy;
  for (int c = lane; c < P; c += 64)
    st1<X3>(yr, c, P, c < D ? (DT<TI>::load(xr + c) - mean) * rstd * gamma[c] + beta[c] : 0.f);
}

// ---- 16 columns per lane (D % 16 == 0): the wide LayerNorm pair.  layernorm16_kernel and
// layernorm16_mx8_kernel share the load and the statistics below (same lane layout, same
// reduction order: the MX-fp8 bytes equal layernorm16's bf16 output quantized), and move
// 16-B vectors per lane: 32 B of bf16 in, 16 B of e4m3 out (a 32-column MX block is a lane
// pair: one DPP step for its amax).  Lane l of chunk i owns columns 16 (64 i + l) .. + 15.
template <int NC>
struct Ln16Row {
  f32x4 v[NC][4];
};
__device__ __forceinline__ void ld16(const bf16_t* p, f32x4 (&v)[4]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint4 w = *reinterpret_cast<const uint4*>(p + 8 * h);
    v[2 * h] = f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                     __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
    v[2 * h + 1] = f32x4{__uint_as_float(w.z << 16), __uint_as_float(w.z & 0xffff0000u),
                         __uint_as_float(w.w << 16), __uint_as_float(w.w & 0xffff0000u)};
  }
}
__device__ __forceinline__ void ld16(const float* p, f32x4 (&v)[4]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) v[g] = *reinterpret_cast<const f32x4*>(p + 4 * g);
}
template <typename TI, int NC>
__device__ __forceinline__ void ln16_load(Ln16Row<NC>& r, const TI* xr, int D, int lane) {
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = (i * 64 + lane) * 16;
    if (c < D) {
      ld16(xr + c, r.v[i]);
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) r.v[i][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}
template <int NC>
__device__ __forceinline__ void ln16_stats(const Ln16Row<NC>& r, int D, int lane, float eps,
                                           float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) s += r.v[i][g][0] + r.v[i][g][1] + r.v[i][g][2] + r.v[i][g][3];
  mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    if ((i * 64 + lane) * 16 < D)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = r.v[i][g][j] - mean;
          q += d * d;
        }
  }
  rstd = 1.f / sqrtf(wave_sum(q) / D + eps);
}
// the normalized, affine-transformed 16 values of chunk i (bf16-rounded for the MX path)
template <int NC, bool ROUND>
__device__ __forceinline__ void ln16_out(const Ln16Row<NC>& r, int i, int c, float mean,
                                         float rstd, const float* gamma, const float* beta,
                                         f32x4 (&o)[4]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 ga = *reinterpret_cast<const f32x4*>(gamma + c + 4 * g);
    const f32x4 be = *reinterpret_cast<const f32x4*>(beta + c + 4 * g);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = (r.v[i][g][j] - mean) * rstd * ga[j] + be[j];
      o[g][j] = ROUND ? bf16_round(v) : v;
    }
  }
}

template <typename TI, typename TO, int NC, int RPW, bool X3 = false>
__global__ __launch_bounds__(256) void layernorm16_kernel(
    const TI* __restrict__ x, int64_t rows, int D, int ldx, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, TO* __restrict__ y, int ldy) {
  const int P = X3 ? ldy / 2 : ldy;
  const int lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= rows) return;
  Ln16Row<NC> r[RPW];
#pragma unroll
  for (int k = 0; k < RPW; ++k) ln16_load(r[k], x + min(row0 + k, rows - 1) * ldx, D, lane);
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int64_t row = row0 + k;
    if (row >= rows) break;
    float mean, rstd;
    ln16_stats(r[k], D, lane, eps, mean, rstd);
    TO* yr = y + row * ldy;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = (i * 64 + lane) * 16;
      if (c < D) {
        f32x4 o[4];
        ln16_out<NC, false>(r[k], i, c, mean, rstd, gamma, beta, o);
#pragma unroll
        for (int g = 0; g < 4; ++g) st4v<X3>(yr + c + 4 * g, P, o[g]);
      }
    }
    for (int c = D + lane; c < P; c += 64) st1<X3>(yr, c, P, 0.f);
  }
}

template <typename TI, int NC, int RPW>
__global__ __launch_bounds__(256) void layernorm16_mx8_kernel(
    const TI* __restrict__ x, int64_t rows, int D, int ldx, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, uint8_t* __restrict__ q, int ldq, int Kq,
    uint8_t* __restrict__ sc, int64_t s_rows) {
  const int lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= rows) return;
  Ln16Row<NC> r[RPW];
#pragma unroll
  for (int k = 0; k < RPW; ++k) ln16_load(r[k], x + min(row0 + k, rows - 1) * ldx, D, lane);
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int64_t row = row0 + k;
    if (row >= rows) break;
    float mean, rstd;
    ln16_stats(r[k], D, lane, eps, mean, rstd);
    uint8_t* qr = q + row * ldq;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = (i * 64 + lane) * 16;
      f32x4 o[4] = {};
      if (c < D) ln16_out<NC, true>(r[k], i, c, mean, rstd, gamma, beta, o);
      float am = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        am = fmaxf(am, fmaxf(fmaxf(fabsf(o[g][0]), fabsf(o[g][1])),
                             fmaxf(fabsf(o[g][2]), fabsf(o[g][3]))));
      am = fmaxf(am, dpp_get<0xB1>(am));               // the lane pair of the 32-block
      const int E = mx8_exponent(am);
      const float inv = __uint_as_float((uint32_t)(127 - E) << 23);
      if (c < Kq) {
        uint4 w;
        w.x = mx8_pack4(o[0][0], o[0][1], o[0][2], o[0][3], inv);
        w.y = mx8_pack4(o[1][0], o[1][1], o[1][2], o[1][3], inv);
        w.z = mx8_pack4(o[2][0], o[2][1], o[2][2], o[2][3], inv);
        w.w = mx8_pack4(o[3][0], o[3][1], o[3][2], o[3][3], inv);
        *reinterpret_cast<uint4*>(qr + c) = w;
        if ((lane & 1) == 0) {
          const int b = c >> 5;
          sc[((int64_t)(b >> 2) * s_rows + row) * 4 + (b & 3)] = (uint8_t)(E + 127);
        }
      }
    }
  }
}

// whether the 16-column LayerNorms apply (the plain and the MX-fp8 one decide alike, so the
// two give the same statistics for the same input)
bool ln16_ok(const void* x, int x_dtype, int D, int ldx, const float* g, const float* b) {
  auto al16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  return D % 16 == 0 && D <= 4096 && ldx % (x_dtype == VTD_BF16 ? 8 : 4) == 0 && al16(x) &&
         al16(g) && al16(b);
}

template <typename TI, typename TO, bool X3 = false>
int ln_dispatch(const void* xv, int64_t rows, int D, int ldx, const float* g,
                const float* b, float eps, void* y, int ldy, hipStream_t st) {
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  const TI* x = static_cast<const TI*>(xv);
  TO* yo = static_cast<TO*>(y);
  const bool vec = (D % 4 == 0) && (ldx % 4 == 0) && ((X3 ? ldy / 2 : ldy) % 4 == 0) &&
                   (reinterpret_cast<uintptr_t>(x) % (4 * sizeof(TI)) == 0) &&
                   (reinterpret_cast<uintptr_t>(y) % (4 * sizeof(TO)) == 0) &&
                   (reinterpret_cast<uintptr_t>(g) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(b) % 16 == 0);
  // the 16-column kernel for the bf16 residual stream only: with an f32 stream (the f32 and
  // split-bf16 parity modes) the 4-column kernel's fully coalesced 16-B loads win -- C2 B = 256
  // per LayerNorm 105 -> 62 us (split-bf16 out, forward +1.8 %), 76 -> 49 us (f32 out, +1.6 %),
  // profiles/r06_f32_stream_layernorm_ab.log
  if (vec && sizeof(TI) == 2 && ln16_ok(xv, VTD_BF16, D, ldx, g, b)) {
    constexpr int RPW = 2;
    const dim3 g16((unsigned)((rows + 4 * RPW - 1) / (4 * RPW)));
    const int nc = (D + 1023) / 1024;
#define VTD_LN16(NC) hipLaunchKernelGGL((layernorm16_kernel<TI, TO, NC, RPW, X3>), g16, block, 0, st, x, \
                                        rows, D, ldx, g, b, eps, yo, ldy)
    if (nc <= 1) VTD_LN16(1);
    else if (nc <= 2) VTD_LN16(2);
    else VTD_LN16(4);
#undef VTD_LN16
    VTD_LAUNCH_CHECK("layernorm");
    return VTD_OK;
  }
  const int nv = (D + 255) / 256;
#define VTD_LN(NV) hipLaunchKernelGGL((layernorm_kernel<TI, TO, NV, X3>), grid, block, 0, st, x, rows, \
                                      D, ldx, g, b, eps, yo, ldy)
  if (vec && nv <= 1) VTD_LN(1);
  else if (vec && nv <= 2) VTD_LN(2);
  else if (vec && nv <= 3) VTD_LN(3);
  else if (vec && nv <= 4) VTD_LN(4);
  else if (vec && nv <= 8) VTD_LN(8);
  else if (vec && nv <= 16) VTD_LN(16);
  else
    hipLaunchKernelGGL((layernorm_generic_kernel<TI, TO, X3>), grid, block, 0, st, x, rows, D,
                       ldx, g, b, eps, yo, ldy);
#undef VTD_LN
  VTD_LAUNCH_CHECK("layernorm");
  return VTD_OK;
}

// LayerNorm with the output quantized to MX-fp8 (VTD_FP8 mode: the next GEMM's A operand
// without a bf16 round trip through HBM).  Same statistics as layernorm_kernel (same lane
// layout and reduction order, so the same bits); each lane owns 4 consecutive columns, so a
// 32-column block is 8 consecutive lanes: block amax by DPP (quad xor 1, xor 2) + one
// lane ^ 4 exchange; values are bf16-rounded first so the bytes equal vtd_quantize_mx8 of
// layernorm_kernel's bf16 output.  NV covers Kq columns.  RPW rows per wave, all their loads
// issued before the first reduction (a read stream: the loads must be in flight together).
template <typename TI, int NV, int RPW>
__global__ __launch_bounds__(256) void layernorm_mx8_kernel(
    const TI* __restrict__ x, int64_t rows, int D, int ldx, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, uint8_t* __restrict__ q, int ldq, int Kq,
    uint8_t* __restrict__ sc, int64_t s_rows) {
  const int lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= rows) return;
  f32x4 v[RPW][NV];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const TI* xr = x + min(row0 + r, rows - 1) * ldx;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      v[r][i] = c < D ? ld4(xr + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int64_t row = row0 + r;
    if (row >= rows) break;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += v[r][i][0] + v[r][i][1] + v[r][i][2] + v[r][i][3];
    s = wave_sum(s);
    const float mean = s / D;
    float qv = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = v[r][i][j] - mean;
          qv += d * d;
        }
    }
    qv = wave_sum(qv);
    const float rstd = 1.f / sqrtf(qv / D + eps);
    uint8_t* qr = q + row * ldq;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      f32x4 o = {0.f, 0.f, 0.f, 0.f};
      if (c < D) {
        const f32x4 g = *reinterpret_cast<const f32x4*>(gamma + c);
        const f32x4 bb = *reinterpret_cast<const f32x4*>(beta + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = bf16_round((v[r][i][j] - mean) * rstd * g[j] + bb[j]);
      }
      float am = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3])));
      am = fmaxf(am, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(am), 0xB1, 0xF, 0xF, false)));
      am = fmaxf(am, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(am), 0x4E, 0xF, 0xF, false)));
      am = fmaxf(am, dpp_get<0x141>(am));   // row_half_mirror: the other quad
      const int E = mx8_exponent(am);
      const float inv = __uint_as_float((uint32_t)(127 - E) << 23);
      if (c < Kq) {
        *reinterpret_cast<uint32_t*>(qr + c) = mx8_pack4(o[0], o[1], o[2], o[3], inv);
        if ((lane & 7) == 0) {
          const int b = c >> 5;
          sc[((int64_t)(b >> 2) * s_rows + row) * 4 + (b & 3)] = (uint8_t)(E + 127);
        }
      }
    }
  }
}

// LayerNorm row statistics only (the fold path, vtd_epilogue.lnstat): one wave per RPW
// rows (all their loads issued before the first reduction: the pass is a pure read
// stream and needs the loads in flight), the same two-pass mean / variance as
// layernorm_kernel; stat[r] = (mean, rstd).
constexpr int LS_RPW = 2;
// 8 consecutive elements as two f32x4 (one 16-B bf16 load / two 16-B f32 loads)
__device__ __forceinline__ void ld8(const float* p, f32x4& a, f32x4& b) {
  a = *reinterpret_cast<const f32x4*>(p);
  b = *reinterpret_cast<const f32x4*>(p + 4);
}
__device__ __forceinline__ void ld8(const bf16_t* p, f32x4& a, f32x4& b) {
  const uint4 w = *reinterpret_cast<const uint4*>(p);
  a = f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
            __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
  b = f32x4{__uint_as_float(w.z << 16), __uint_as_float(w.z & 0xffff0000u),
            __uint_as_float(w.w << 16), __uint_as_float(w.w & 0xffff0000u)};
}
template <typename TI, int NV>      // NV = 8-element chunks per lane (D <= 512 NV)
__global__ __launch_bounds__(256) void ln_stats_kernel(const TI* __restrict__ x, int64_t rows,
                                                       int D, int ldx, float eps,
                                                       float2* __restrict__ stat) {
  const int lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * LS_RPW;
  if (row0 >= rows) return;
  f32x4 v[LS_RPW][NV][2];
#pragma unroll
  for (int r = 0; r < LS_RPW; ++r) {
    const TI* xr = x + min(row0 + r, rows - 1) * ldx;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (c < D) {
        ld8(xr + c, v[r][i][0], v[r][i][1]);
      } else {
        v[r][i][0] = v[r][i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
#pragma unroll
  for (int r = 0; r < LS_RPW; ++r) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) s += v[r][i][h][0] + v[r][i][h][1] + v[r][i][h][2] + v[r][i][h][3];
    s = wave_sum(s);
    const float mean = s / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (c < D)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = v[r][i][h][j] - mean;
            q += d * d;
          }
    }
    q = wave_sum(q);
    if (lane == 0 && row0 + r < rows) stat[row0 + r] = float2{mean, 1.f / sqrtf(q / D + eps)};
  }
}

template <typename TI>
__global__ __launch_bounds__(256) void ln_stats_generic_kernel(const TI* __restrict__ x,
                                                               int64_t rows, int D, int ldx,
                                                               float eps, float2* __restrict__ stat) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TI* xr = x + row * ldx;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += DT<TI>::load(xr + c);
  s = wave_sum(s);
  const float mean = s / D;
  float q = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float d = DT<TI>::load(xr + c) - mean;
    q += d * d;
  }
  q = wave_sum(q);
  if (lane == 0) stat[row] = float2{mean, 1.f / sqrtf(q / D + eps)};
}

template <typename TI>
void ln_stats_dispatch(const void* xv, int64_t rows, int D, int ldx, float eps, float2* stat,
                       hipStream_t st) {
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  const TI* x = static_cast<const TI*>(xv);
  const bool vec = (D % 8 == 0) && (ldx % 8 == 0) &&
                   (reinterpret_cast<uintptr_t>(x) % 16 == 0);
  const int nv = (D + 511) / 512;
  const dim3 gridv((unsigned)((rows + 4 * LS_RPW - 1) / (4 * LS_RPW)));
#define VTD_LS(NV) hipLaunchKernelGGL((ln_stats_kernel<TI, NV>), gridv, block, 0, st, x, rows, D, \
                                      ldx, eps, stat)
  if (vec && nv <= 1) VTD_LS(1);
  else if (vec && nv <= 2) VTD_LS(2);
  else if (vec && nv <= 4) VTD_LS(4);
  else
    hipLaunchKernelGGL((ln_stats_generic_kernel<TI>), grid, block, 0, st, x, rows, D, ldx, eps,
                       stat);
#undef VTD_LS
}

// (mean, rstd) per row from a producer GEMM's centred partials per 64-column block
// (block mean m_b, sum of squared deviations M2_b; every block holds 64 valid columns):
// Chan et al.'s pairwise merge for equal counts, mean = sum_b m_b / slots and
// M2 = sum_b M2_b + 64 sum_b (m_b - mean)^2, with the block means taken relative to the
// first one.  No large nearly-equal terms are subtracted, whatever |mean| / std is.
// One thread per row.
__global__ __launch_bounds__(256) void ln_stats_finalize_kernel(const float2* __restrict__ part,
                                                                int64_t rows, int slots, int D,
                                                                float eps,
                                                                float2* __restrict__ stat) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const float2* pr = part + r;                    // slot b at pr[b * rows]
  const float m0 = pr[0].x;
  float ds = 0.f, q = 0.f;
  for (int b = 0; b < slots; ++b) {
    const float2 t = pr[b * rows];
    ds += t.x - m0;
    q += t.y;
  }
  const float dmean = ds / slots;
  float between = 0.f;
  for (int b = 0; b < slots; ++b) {
    const float dv = (pr[b * rows].x - m0) - dmean;
    between += dv * dv;
  }
  const float var = (q + 64.f * between) / D;
  stat[r] = float2{m0 + dmean, 1.f / sqrtf(var + eps)};
}

// The same with the slot count known at compile time: the row's S partials are loaded as
// S / 2 16-B words before any arithmetic (one memory round trip instead of a dependent
// chain); same operations in the same order as ln_stats_finalize_kernel (identical results).
// Grid-stride over the rows (gridDim.x * blockDim.x threads): launched with few large
// workgroups in the two-stream forward, where every workgroup waits for a CU the other
// stream's GEMM tile vacates (knob VTD_KNOB_FIN_WGS).
template <int S>
__global__ __launch_bounds__(1024) void ln_stats_finalize_s_kernel(const float2* __restrict__ part,
                                                                   int64_t rows, int D, float eps,
                                                                   float2* __restrict__ stat) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    // slot-major planes: slot b of row r at part[b * rows + r] (a wave's loads are 512
    // contiguous bytes per slot)
    f32x4 v[S / 2];
#pragma unroll
    for (int b = 0; b < S / 2; ++b) {
      const float2 w0 = part[(2 * b) * rows + r], w1 = part[(2 * b + 1) * rows + r];
      v[b] = f32x4{w0.x, w0.y, w1.x, w1.y};
    }
    stat[r] = ln_merge_partials<S>(v, D, eps);
  }
}

// LayerNorm fold of one consumer Dense layer (one-time weight preparation): one wave per
// output row n; fp64 sums (bias' from the fp32 W, colsum from the rounded stored W').
template <typename TO>
__global__ __launch_bounds__(256) void fold_ln_kernel(const float* __restrict__ w, int N, int K,
                                                      int ldw, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta,
                                                      const float* __restrict__ bias_in,
                                                      TO* __restrict__ wo, int ldo,
                                                      float* __restrict__ bias_out,
                                                      float* __restrict__ colsum) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  double sb = 0.0, sc = 0.0;
  for (int k = lane; k < ldo; k += 64) {
    const float wk = k < K ? w[(int64_t)n * ldw + k] : 0.f;
    const TO q = DT<TO>::from(k < K ? wk * gamma[k] : 0.f);
    wo[(int64_t)n * ldo + k] = q;
    if (k < K) {
      sb += (double)wk * (double)beta[k];
      sc += (double)DT<TO>::load(&q);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    sb += __shfl_xor(sb, o);
    sc += __shfl_xor(sc, o);
  }
  if (lane == 0) {
    bias_out[n] = (float)((double)(bias_in ? bias_in[n] : 0.f) + sb);
    colsum[n] = (float)sc;
  }
}

// ------------------------------------------------------------------ patches
// tf.image.extract_patches(SAME, size = stride = p) + Reshape: output row m = b*N + t
// (t = gy*gw + gx), column k = (kh*p + kw)*C + c; outside the image -> 0.
// Each thread writes 8 consecutive output columns (one 16-B bf16 / 32-B f32 store).
// X3: TO = bf16_t, the split-bf16 operand (two ldo / 2 wide pieces)
template <typename TO, bool X3 = false>
__global__ __launch_bounds__(256) void patches_kernel(
    const float* __restrict__ img, int B, int H, int W, int C, int p, int gw, int N,
    int top, int left, int P, TO* __restrict__ out, int ldo) {
  const int pw = X3 ? ldo / 2 : ldo;          // width of one piece
  const int chunks = pw / 8;
  const int64_t total = (int64_t)B * N * chunks;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = g / chunks;
    const int k0 = (int)(g - m * chunks) * 8;
    const int b = (int)(m / N), t = (int)(m - (int64_t)b * N);
    const int gy = t / gw, gx = t - (t / gw) * gw;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + j;
      float val = 0.f;
      if (k < P) {
        const int kh = k / (p * C), r = k - kh * p * C;
        const int kw = r / C, c = r - kw * C;
        const int yy = gy * p + kh - top, xx = gx * p + kw - left;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W)
          val = img[(((int64_t)b * H + yy) * W + xx) * C + c];
      }
      v[j] = val;
    }
    TO* o = out + m * ldo + k0;
    if constexpr (X3) {
      uint4 hi, lo;
      hi.x = pack_bf16x2(v[0], v[1]); lo.x = pack_lo_bf16x2(v[0], v[1], hi.x);
      hi.y = pack_bf16x2(v[2], v[3]); lo.y = pack_lo_bf16x2(v[2], v[3], hi.y);
      hi.z = pack_bf16x2(v[4], v[5]); lo.z = pack_lo_bf16x2(v[4], v[5], hi.z);
      hi.w = pack_bf16x2(v[6], v[7]); lo.w = pack_lo_bf16x2(v[6], v[7], hi.w);
      *reinterpret_cast<uint4*>(o) = hi;
      *reinterpret_cast<uint4*>(o + pw) = lo;
    } else if constexpr (sizeof(TO) == 2) {
      bf16x8 w;
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = static_cast<short>(f32_to_bf16(v[j]));
      *reinterpret_cast<bf16x8*>(o) = w;
    } else {
      *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(o + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
  }
}

// Unpadded case (H, W multiples of p; p*C % 8 == 0), bf16 out with ld_out == P, or (X3) the
// split-bf16 operand with ld_out == 2 P: a patch row kh of token m is p*C consecutive floats
// of image row gy*p + kh, so each thread moves 8 consecutive floats (two 16-B loads) to one
// 16-B store per piece with no index arithmetic per element.  Same output as patches_kernel.
template <bool X3 = false>
__global__ __launch_bounds__(256) void patches_dense_kernel(
    const float* __restrict__ img, int64_t total, int H, int W, int C, int p, int gw, int N,
    bf16_t* __restrict__ out) {
  const int seg = p * C / 8;                 // 8-float chunks per patch row
  const int per_tok = p * seg;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = g / per_tok;
    const int r = (int)(g - m * per_tok);
    const int kh = r / seg, c8 = r - kh * seg;
    const int b = (int)(m / N), t = (int)(m - (int64_t)b * N);
    const int gy = t / gw, gx = t - gy * gw;
    const float* src = img + (((int64_t)b * H + gy * p + kh) * W + gx * p) * C + c8 * 8;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(src);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(src + 4);
    const uint4 o = {pack_bf16x2(v0[0], v0[1]), pack_bf16x2(v0[2], v0[3]),
                     pack_bf16x2(v1[0], v1[1]), pack_bf16x2(v1[2], v1[3])};
    const int P = p * p * C;
    bf16_t* const op = out + m * (int64_t)(X3 ? 2 * P : P) + kh * p * C + c8 * 8;
    *reinterpret_cast<uint4*>(op) = o;
    if constexpr (X3)
      *reinterpret_cast<uint4*>(op + P) =
          uint4{pack_lo_bf16x2(v0[0], v0[1], o.x), pack_lo_bf16x2(v0[2], v0[3], o.y),
                pack_lo_bf16x2(v1[0], v1[1], o.z), pack_lo_bf16x2(v1[2], v1[3], o.w)};
  }
}

// ------------------------------------------------------------------ split-bf16
// f32 x [rows][ldx] (K columns) -> split-bf16 y [rows][ldy]: role 0 [hi | lo] (A operand,
// P = ldy / 2), role 1 [hi | hi | lo] (B operand, P = ldy / 3); each thread 8 columns of one
// row (16-B stores; columns [K, P) zero).  VEC: K % 8 == 0, ldx % 4 == 0, 16-B bases.
template <bool VEC>
__global__ __launch_bounds__(256) void split_bf16x3_kernel(const float* __restrict__ x,
                                                           int64_t rows, int K, int ldx,
                                                           bf16_t* __restrict__ y, int ldy,
                                                           int role) {
  const int P = role ? ldy / 3 : ldy / 2, chunks = (P + 7) / 8;
  const int64_t total = rows * chunks;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = g / chunks;
    const int c0 = (int)(g - m * chunks) * 8;
    const float* xr = x + m * ldx;
    bf16_t* yr = y + m * ldy;
    bf16_t* const pc1 = yr + P;                      // second piece
    bf16_t* const pc2 = yr + 2 * P;                  // third piece (role 1)
    if (VEC && c0 + 8 <= P) {
      f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = a;
      if (c0 < K) {                                  // K % 8 == 0: all 8 or none
        a = *reinterpret_cast<const f32x4*>(xr + c0);
        b = *reinterpret_cast<const f32x4*>(xr + c0 + 4);
      }
      uint4 hi, lo;
      hi.x = pack_bf16x2(a[0], a[1]); lo.x = pack_lo_bf16x2(a[0], a[1], hi.x);
      hi.y = pack_bf16x2(a[2], a[3]); lo.y = pack_lo_bf16x2(a[2], a[3], hi.y);
      hi.z = pack_bf16x2(b[0], b[1]); lo.z = pack_lo_bf16x2(b[0], b[1], hi.z);
      hi.w = pack_bf16x2(b[2], b[3]); lo.w = pack_lo_bf16x2(b[2], b[3], hi.w);
      *reinterpret_cast<uint4*>(yr + c0) = hi;
      *reinterpret_cast<uint4*>(pc1 + c0) = role ? hi : lo;
      if (role) *reinterpret_cast<uint4*>(pc2 + c0) = lo;
    } else {
      for (int c = c0; c < min(c0 + 8, P); ++c) {
        const float v = c < K ? xr[c] : 0.f;
        const bf16_t h = f32_to_bf16(v), l = lo_bf16(v, h);
        yr[c] = h;
        pc1[c] = role ? h : l;
        if (role) pc2[c] = l;
      }
    }
  }
}

// ------------------------------------------------------------------ decode
// transform_predictions (vtd.py:586-647): sigmoid; clip last 4 to [0, 1];
// [conf, cls * (CLASSES-1), cx * W, cy * H, h * H, w * W] with W = H = 608 (constant
// Constants.MODEL_IMAGE_SIZE, not the input shape).
__global__ void decode_kernel(const float* __restrict__ logits, int64_t n,
                              float* __restrict__ dets) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * 6) return;
  dets[i] = decode_transform((int)(i % 6), logits[i]);
}

// transform_predictions + the thresholded detection test (vtd.py:1359-1384): one
// thread per detection slot.  tf.round is round-half-to-even -> rintf.
__global__ void decode_detections_kernel(const float* __restrict__ logits, int64_t n,
                                         float* __restrict__ dets, int32_t* __restrict__ cat,
                                         uint8_t* __restrict__ valid, float obj_thr,
                                         float cls_thr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float d[6];
#pragma unroll
  for (int f = 0; f < 6; ++f) {
    d[f] = decode_transform(f, logits[i * 6 + f]);
    if (dets) dets[i * 6 + f] = d[f];
  }
  const float c = rintf(d[1]);
  const float conf = (0.5f - fabsf(d[1] - c)) / 0.5f;
  if (cat) cat[i] = (int32_t)c;
  if (valid) valid[i] = (d[0] > obj_thr && conf > cls_thr) ? 1 : 0;
}

// ------------------------------------------------------------------ packing
template <typename TO>
__global__ void pack_dense_kernel(const float* __restrict__ src, int K, int N, int kg,
                                  int kgp, int ng, int ngp, TO* __restrict__ dst, int ld,
                                  int off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)K * N) return;
  const int k = (int)(i / N), n = (int)(i - (int64_t)k * N);
  const int kp = (k / kg) * kgp + k % kg;
  const int np = (n / ng) * ngp + n % ng;
  dst[(int64_t)(off + np) * ld + kp] = DT<TO>::from(src[i]);
}

__global__ void pack_vector_kernel(const float* __restrict__ src, int N, int ng, int ngp,
                                   float* __restrict__ dst, int off) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  dst[off + (n / ng) * ngp + n % ng] = src[n];
}

}  // namespace

int layernorm_launch(const void* x, int x_dtype, int64_t rows, int D, int ldx, const float* g,
                     const float* b, float eps, void* y, int ldy, int dtype,
                     hipStream_t st) {
  VTD_CHECK_ARG(x && g && b && y, "layernorm: null pointer");
  VTD_CHECK_ARG(rows > 0 && D > 0 && ldx >= D && ldy >= D, "layernorm: bad shape");
  VTD_CHECK_ARG(dtype == VTD_F32 || dtype == VTD_BF16 || dtype == VTD_BF16X3,
                "layernorm: bad dtype");
  VTD_CHECK_ARG(x_dtype == VTD_F32 || x_dtype == VTD_BF16, "layernorm: bad x dtype");
  VTD_CHECK_ARG(dtype != VTD_BF16X3 || (ldy % 2 == 0 && ldy / 2 >= D),
                "layernorm: a split-bf16 output needs ldy % 2 == 0 and ldy / 2 >= D");
  ProfScope ps(st, PROF_LN, 0.0);
  if (dtype == VTD_BF16X3)
    return x_dtype == VTD_BF16
               ? ln_dispatch<bf16_t, bf16_t, true>(x, rows, D, ldx, g, b, eps, y, ldy, st)
               : ln_dispatch<float, bf16_t, true>(x, rows, D, ldx, g, b, eps, y, ldy, st);
  if (x_dtype == VTD_BF16)
    return dtype == VTD_BF16 ? ln_dispatch<bf16_t, bf16_t>(x, rows, D, ldx, g, b, eps, y, ldy, st)
                             : ln_dispatch<bf16_t, float>(x, rows, D, ldx, g, b, eps, y, ldy, st);
  return dtype == VTD_BF16 ? ln_dispatch<float, bf16_t>(x, rows, D, ldx, g, b, eps, y, ldy, st)
                           : ln_dispatch<float, float>(x, rows, D, ldx, g, b, eps, y, ldy, st);
}

int layernorm_mx8_launch(const void* x, int x_dtype, int64_t rows, int D, int ldx,
                         const float* g, const float* b, float eps, uint8_t* q, int ldq, int Kq,
                         uint8_t* s, int64_t s_rows, hipStream_t st) {
  VTD_CHECK_ARG(x && g && b && q && s, "layernorm_mx8: null pointer");
  VTD_CHECK_ARG(rows > 0 && D > 0 && ldx >= D && Kq >= D && Kq % 128 == 0 && ldq >= Kq &&
                    ldq % 16 == 0 && s_rows >= rows && Kq <= 4096,
                "layernorm_mx8: bad shape (Kq % 128, D <= Kq <= 4096, ldq % 16, s_rows)");
  VTD_CHECK_ARG(x_dtype == VTD_F32 || x_dtype == VTD_BF16, "layernorm_mx8: bad x dtype");
  VTD_CHECK_ARG(D % 4 == 0 && ldx % 4 == 0 && reinterpret_cast<uintptr_t>(g) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(b) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(x) % (x_dtype == VTD_BF16 ? 8 : 16) == 0,
                "layernorm_mx8: D, ldx % 4 and 16-B aligned gamma / beta / x needed");
  ProfScope ps(st, PROF_LN, 0.0);
  // rows per wave: 2 (the loads of both rows in flight)
  constexpr int RPW = 2;
  if (ln16_ok(x, x_dtype, D, ldx, g, b)) {
    const dim3 g16((unsigned)((rows + 4 * RPW - 1) / (4 * RPW))), b16(256);
    const int nc = (Kq + 1023) / 1024;
#define VTD_LQ16(TI, NC) hipLaunchKernelGGL((layernorm16_mx8_kernel<TI, NC, RPW>), g16, b16, 0, st, \
                                            static_cast<const TI*>(x), rows, D, ldx, g, b, eps, q, \
                                            ldq, Kq, s, s_rows)
    if (x_dtype == VTD_BF16) {
      if (nc <= 1) VTD_LQ16(bf16_t, 1);
      else if (nc <= 2) VTD_LQ16(bf16_t, 2);
      else VTD_LQ16(bf16_t, 4);
    } else {
      if (nc <= 1) VTD_LQ16(float, 1);
      else if (nc <= 2) VTD_LQ16(float, 2);
      else VTD_LQ16(float, 4);
    }
#undef VTD_LQ16
    VTD_LAUNCH_CHECK("layernorm_mx8");
    return VTD_OK;
  }
  const dim3 grid((unsigned)((rows + 4 * RPW - 1) / (4 * RPW))), block(256);
  const int nv = (Kq + 255) / 256;
#define VTD_LQ(TI, NV) hipLaunchKernelGGL((layernorm_mx8_kernel<TI, NV, RPW>), grid, block, 0, st, \
                                          static_cast<const TI*>(x), rows, D, ldx, g, b, eps, q, \
                                          ldq, Kq, s, s_rows)
  if (x_dtype == VTD_BF16) {
    if (nv <= 2) VTD_LQ(bf16_t, 2);
    else if (nv <= 4) VTD_LQ(bf16_t, 4);
    else if (nv <= 8) VTD_LQ(bf16_t, 8);
    else VTD_LQ(bf16_t, 16);
  } else {
    if (nv <= 2) VTD_LQ(float, 2);
    else if (nv <= 4) VTD_LQ(float, 4);
    else if (nv <= 8) VTD_LQ(float, 8);
    else VTD_LQ(float, 16);
  }
#undef VTD_LQ
  VTD_LAUNCH_CHECK("layernorm_mx8");
  return VTD_OK;
}

int ln_stats_launch(const void* x, int x_dtype, int64_t rows, int D, int ldx, float eps,
                    float* stat, hipStream_t st) {
  VTD_CHECK_ARG(x && stat, "layernorm_stats: null pointer");
  VTD_CHECK_ARG(rows > 0 && D > 0 && ldx >= D, "layernorm_stats: bad shape");
  VTD_CHECK_ARG(x_dtype == VTD_F32 || x_dtype == VTD_BF16, "layernorm_stats: bad x dtype");
  VTD_CHECK_ARG(reinterpret_cast<uintptr_t>(stat) % 8 == 0, "layernorm_stats: stat alignment");
  ProfScope ps(st, PROF_LN, 0.0);
  float2* s2 = reinterpret_cast<float2*>(stat);
  if (x_dtype == VTD_BF16) ln_stats_dispatch<bf16_t>(x, rows, D, ldx, eps, s2, st);
  else ln_stats_dispatch<float>(x, rows, D, ldx, eps, s2, st);
  VTD_LAUNCH_CHECK("layernorm_stats");
  return VTD_OK;
}

int ln_stats_finalize_launch(const float* part, int64_t rows, int slots, int D, float eps,
                             float* stat, hipStream_t st) {
  VTD_CHECK_ARG(part && stat, "layernorm_stats_finalize: null pointer");
  VTD_CHECK_ARG(rows > 0 && slots > 0 && D == 64 * slots,
                "layernorm_stats_finalize: bad shape (D must be 64 * slots: every block full)");
  VTD_CHECK_ARG(reinterpret_cast<uintptr_t>(part) % 8 == 0 && reinterpret_cast<uintptr_t>(stat) % 8 == 0,
                "layernorm_stats_finalize: alignment");
  ProfScope ps(st, PROF_LN, 0.0);
  // the common widths: every partial loaded at once, one memory round trip
  if (slots == 12 || slots == 16) {
    {
      auto k = slots == 12 ? ln_stats_finalize_s_kernel<12> : ln_stats_finalize_s_kernel<16>;
      // knob VTD_KNOB_FIN_WGS = n > 0: n workgroups of 1024 threads (grid-stride)
      const int fw = knob(VTD_KNOB_FIN_WGS);
      const int64_t need = (rows + 1023) / 1024;
      if (fw > 0)
        hipLaunchKernelGGL(k, dim3((unsigned)std::min<int64_t>(fw, need)), dim3(1024), 0, st,
                           reinterpret_cast<const float2*>(part), rows, D, eps,
                           reinterpret_cast<float2*>(stat));
      else
        hipLaunchKernelGGL(k, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st,
                           reinterpret_cast<const float2*>(part), rows, D, eps,
                           reinterpret_cast<float2*>(stat));
      VTD_LAUNCH_CHECK("layernorm_stats_finalize");
      return VTD_OK;
    }
  }
  hipLaunchKernelGGL(ln_stats_finalize_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0,
                     st, reinterpret_cast<const float2*>(part), rows, slots, D, eps,
                     reinterpret_cast<float2*>(stat));
  VTD_LAUNCH_CHECK("layernorm_stats_finalize");
  return VTD_OK;
}

int fold_ln_launch(const float* w, int N, int K, int ldw, const float* gamma, const float* beta,
                   const float* bias_in, void* wo, int ldo, int dtype, float* bias_out,
                   float* colsum, hipStream_t st) {
  VTD_CHECK_ARG(w && gamma && beta && wo && bias_out && colsum, "fold_layernorm: null pointer");
  VTD_CHECK_ARG(N > 0 && K > 0 && ldw >= K && ldo >= K, "fold_layernorm: bad shape");
  VTD_CHECK_ARG(dtype == VTD_F32 || dtype == VTD_BF16, "fold_layernorm: bad dtype");
  const dim3 grid((unsigned)((N + 3) / 4)), block(256);
  if (dtype == VTD_BF16)
    hipLaunchKernelGGL(fold_ln_kernel<bf16_t>, grid, block, 0, st, w, N, K, ldw, gamma, beta,
                       bias_in, static_cast<bf16_t*>(wo), ldo, bias_out, colsum);
  else
    hipLaunchKernelGGL(fold_ln_kernel<float>, grid, block, 0, st, w, N, K, ldw, gamma, beta,
                       bias_in, static_cast<float*>(wo), ldo, bias_out, colsum);
  VTD_LAUNCH_CHECK("fold_layernorm");
  return VTD_OK;
}

int patches_launch(const float* img, int B, int H, int W, int C, int p, void* out,
                   int ldo, int dtype, hipStream_t st) {
  VTD_CHECK_ARG(img && out, "extract_patches: null pointer");
  VTD_CHECK_ARG(B > 0 && H > 0 && W > 0 && C > 0 && p > 0, "extract_patches: bad shape");
  const int gh = (H + p - 1) / p, gw = (W + p - 1) / p;
  const int P = p * p * C;
  VTD_CHECK_ARG(dtype == VTD_F32 || dtype == VTD_BF16 || dtype == VTD_BF16X3,
                "extract_patches: bad dtype");
  if (dtype == VTD_BF16X3)
    VTD_CHECK_ARG(ldo % 16 == 0 && ldo / 2 >= P,
                  "extract_patches: a split-bf16 output needs ld_out % 16 == 0, ld_out / 2 >= P");
  else
    VTD_CHECK_ARG(ldo >= P && ldo % 8 == 0, "extract_patches: ld_out must be >= P, % 8");
  const int pad_h = (gh - 1) * p + p - H, pad_w = (gw - 1) * p + p - W;
  const int N = gh * gw;
  const int64_t total = (int64_t)B * N * ((dtype == VTD_BF16X3 ? ldo / 2 : ldo) / 8);
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
  ProfScope ps(st, PROF_PATCH, 0.0);
  const bool dense = pad_h == 0 && pad_w == 0 && (p * C) % 8 == 0 && (W * C) % 4 == 0 &&
                     reinterpret_cast<uintptr_t>(img) % 16 == 0 &&
                     reinterpret_cast<uintptr_t>(out) % 16 == 0;
  if (dense && ((dtype == VTD_BF16 && ldo == P) || (dtype == VTD_BF16X3 && ldo == 2 * P))) {
    const int64_t tot = (int64_t)B * N * P / 8;
    const int gd = (int)std::min<int64_t>((tot + 255) / 256, 16384);
    if (dtype == VTD_BF16X3)
      hipLaunchKernelGGL(patches_dense_kernel<true>, dim3(gd), dim3(256), 0, st, img, tot, H, W,
                         C, p, gw, N, static_cast<bf16_t*>(out));
    else
      hipLaunchKernelGGL(patches_dense_kernel<false>, dim3(gd), dim3(256), 0, st, img, tot, H, W,
                         C, p, gw, N, static_cast<bf16_t*>(out));
  } else if (dtype == VTD_BF16X3)
    hipLaunchKernelGGL((patches_kernel<bf16_t, true>), dim3(grid), dim3(256), 0, st, img, B, H,
                       W, C, p, gw, N, pad_h / 2, pad_w / 2, P, static_cast<bf16_t*>(out), ldo);
  else if (dtype == VTD_BF16)
    hipLaunchKernelGGL(patches_kernel<bf16_t>, dim3(grid), dim3(256), 0, st, img, B, H, W,
                       C, p, gw, N, pad_h / 2, pad_w / 2, P, static_cast<bf16_t*>(out), ldo);
  else
    hipLaunchKernelGGL(patches_kernel<float>, dim3(grid), dim3(256), 0, st, img, B, H, W,
                       C, p, gw, N, pad_h / 2, pad_w / 2, P, static_cast<float*>(out), ldo);
  VTD_LAUNCH_CHECK("extract_patches");
  return VTD_OK;
}

int split_bf16x3_launch(const float* x, int64_t rows, int K, int ldx, void* y, int ldy, int role,
                        hipStream_t st) {
  VTD_CHECK_ARG(x && y && rows > 0 && K > 0 && ldx >= K, "split_bf16x3: bad arguments");
  VTD_CHECK_ARG(role == 0 || role == 1, "split_bf16x3: role 0 or 1");
  const int np = role ? 3 : 2;                       // pieces
  VTD_CHECK_ARG(ldy % np == 0 && ldy / np >= K,
                "split_bf16x3: ldy = 2 P (role 0) or 3 P (role 1) with P >= K");
  ProfScope ps(st, PROF_OTHER, 0.0);
  const int P = ldy / np;
  const int64_t total = rows * ((P + 7) / 8);
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 16384);
  const bool vec = K % 8 == 0 && ldx % 4 == 0 && P % 8 == 0 &&
                   reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(y) % 16 == 0;
  if (vec)
    hipLaunchKernelGGL(split_bf16x3_kernel<true>, dim3(grid), dim3(256), 0, st, x, rows, K, ldx,
                       static_cast<bf16_t*>(y), ldy, role);
  else
    hipLaunchKernelGGL(split_bf16x3_kernel<false>, dim3(grid), dim3(256), 0, st, x, rows, K, ldx,
                       static_cast<bf16_t*>(y), ldy, role);
  VTD_LAUNCH_CHECK("split_bf16x3");
  return VTD_OK;
}

int decode_launch(const float* logits, int64_t n, float* dets, hipStream_t st) {
  VTD_CHECK_ARG(logits && dets && n > 0, "decode: bad args");
  ProfScope ps(st, PROF_OTHER, 0.0);
  const int64_t total = n * 6;
  hipLaunchKernelGGL(decode_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     logits, n, dets);
  VTD_LAUNCH_CHECK("decode");
  return VTD_OK;
}

}  // namespace vtd

extern "C" {

int vtd_layernorm(const void* x_dev, int x_dtype, int64_t rows, int D, int ldx,
                  const float* gamma_dev, const float* beta_dev, float eps, void* y_dev, int ldy,
                  int dtype, void* stream) {
  return vtd::layernorm_launch(x_dev, x_dtype, rows, D, ldx, gamma_dev, beta_dev, eps, y_dev, ldy,
                               dtype, static_cast<hipStream_t>(stream));
}

int vtd_layernorm_mx8(const void* x_dev, int x_dtype, int64_t rows, int D, int ldx,
                      const float* gamma_dev, const float* beta_dev, float eps, uint8_t* q_dev,
                      int ldq, int Kq, uint8_t* s_dev, int64_t s_rows, void* stream) {
  return vtd::layernorm_mx8_launch(x_dev, x_dtype, rows, D, ldx, gamma_dev, beta_dev, eps, q_dev,
                                   ldq, Kq, s_dev, s_rows, static_cast<hipStream_t>(stream));
}

int vtd_layernorm_stats(const void* x_dev, int x_dtype, int64_t rows, int D, int ldx,
                        float eps, float* stat_dev, void* stream) {
  return vtd::ln_stats_launch(x_dev, x_dtype, rows, D, ldx, eps, stat_dev,
                              static_cast<hipStream_t>(stream));
}

int vtd_layernorm_stats_finalize(const float* partial_dev, int64_t rows, int slots, int D,
                                 float eps, float* stat_dev, void* stream) {
  return vtd::ln_stats_finalize_launch(partial_dev, rows, slots, D, eps, stat_dev,
                                       static_cast<hipStream_t>(stream));
}

int vtd_fold_layernorm(const float* w32_dev, int N, int K, int ldw, const float* gamma_dev,
                       const float* beta_dev, const float* bias_in_dev, void* w_out_dev,
                       int ldo, int dtype, float* bias_out_dev, float* colsum_dev,
                       void* stream) {
  return vtd::fold_ln_launch(w32_dev, N, K, ldw, gamma_dev, beta_dev, bias_in_dev, w_out_dev,
                             ldo, dtype, bias_out_dev, colsum_dev,
                             static_cast<hipStream_t>(stream));
}

int vtd_extract_patches(const float* images_dev, int B, int H, int W, int C, int p,
                        void* out_dev, int ld_out, int dtype, void* stream) {
  return vtd::patches_launch(images_dev, B, H, W, C, p, out_dev, ld_out, dtype,
                             static_cast<hipStream_t>(stream));
}

int vtd_split_bf16x3(const float* x_dev, int64_t rows, int K, int ldx, void* y_dev, int ldy,
                     int role, void* stream) {
  return vtd::split_bf16x3_launch(x_dev, rows, K, ldx, y_dev, ldy, role,
                                  static_cast<hipStream_t>(stream));
}

int vtd_decode(const float* logits_dev, int64_t n, float* dets_dev, void* stream) {
  return vtd::decode_launch(logits_dev, n, dets_dev, static_cast<hipStream_t>(stream));
}

int vtd_decode_detections(const float* logits_dev, int64_t n, float* dets_dev,
                          int32_t* category_dev, uint8_t* valid_dev, float obj_threshold,
                          float cls_threshold, void* stream) {
  VTD_CHECK_ARG(logits_dev && n > 0, "decode_detections: bad args");
  vtd::ProfScope ps(static_cast<hipStream_t>(stream), vtd::PROF_OTHER, 0.0);
  hipLaunchKernelGGL(vtd::decode_detections_kernel, dim3((unsigned)((n + 255) / 256)),
                     dim3(256), 0, static_cast<hipStream_t>(stream), logits_dev, n, dets_dev,
                     category_dev, valid_dev, obj_threshold, cls_threshold);
  VTD_LAUNCH_CHECK("decode_detections");
  return VTD_OK;
}

int vtd_pack_dense(const float* src_dev, int K, int N, int k_group, int k_group_p,
                   int n_group, int n_group_p, void* dst_dev, int ld_dst, int n_row_offset,
                   int dtype, void* stream) {
  VTD_CHECK_ARG(src_dev && dst_dev && K > 0 && N > 0, "pack_dense: bad args");
  VTD_CHECK_ARG(k_group > 0 && k_group_p >= k_group && n_group > 0 && n_group_p >= n_group,
                "pack_dense: bad groups");
  VTD_CHECK_ARG((K / k_group - 1) * k_group_p + k_group <= ld_dst,
                "pack_dense: ld_dst too small");
  const int64_t total = (int64_t)K * N;
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == VTD_BF16)
    hipLaunchKernelGGL(vtd::pack_dense_kernel<vtd::bf16_t>, grid, dim3(256), 0, st, src_dev,
                       K, N, k_group, k_group_p, n_group, n_group_p,
                       static_cast<vtd::bf16_t*>(dst_dev), ld_dst, n_row_offset);
  else if (dtype == VTD_F32)
    hipLaunchKernelGGL(vtd::pack_dense_kernel<float>, grid, dim3(256), 0, st, src_dev, K, N,
                       k_group, k_group_p, n_group, n_group_p, static_cast<float*>(dst_dev),
                       ld_dst, n_row_offset);
  else
    return vtd::fail(VTD_ERR_UNSUPPORTED, "pack_dense: bad dtype");
  VTD_LAUNCH_CHECK("pack_dense");
  return VTD_OK;
}

int vtd_pack_vector(const float* src_dev, int N, int n_group, int n_group_p, float* dst_dev,
                    int offset, void* stream) {
  VTD_CHECK_ARG(src_dev && dst_dev && N > 0 && n_group > 0 && n_group_p >= n_group,
                "pack_vector: bad args");
  hipLaunchKernelGGL(vtd::pack_vector_kernel, dim3((N + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), src_dev, N, n_group, n_group_p,
                     dst_dev, offset);
  VTD_LAUNCH_CHECK("pack_vector");
  return VTD_OK;
}

}  // extern "C"
