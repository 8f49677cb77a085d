// Shared helpers for the gfx950 kernels of libvtd.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <string>

#include "../../include/vtd.h"

namespace vtd {

// ----------------------------------------------------------------- errors (host)
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
#define VTD_CHECK_ARG(cond, msg)                                             \
  do {                                                                       \
    if (!(cond)) return ::vtd::fail(VTD_ERR_INVALID_ARG, std::string(msg));  \
  } while (0)
#define VTD_HIP(call)                                                        \
  do {                                                                       \
    hipError_t e_ = (call);                                                  \
    if (e_ != hipSuccess)                                                    \
      return ::vtd::fail(VTD_ERR_HIP, std::string(#call) + ": " +            \
                                          hipGetErrorString(e_));            \
  } while (0)
#define VTD_LAUNCH_CHECK(what)                                               \
  do {                                                                       \
    hipError_t e_ = hipGetLastError();                                       \
    if (e_ != hipSuccess)                                                    \
      return ::vtd::fail(VTD_ERR_HIP, std::string(what) + " launch: " +      \
                                          hipGetErrorString(e_));            \
  } while (0)

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Per-device lazily initialised launch state (kernel attributes, CU counts): one
// std::once_flag per device makes the first use on each device thread-safe, and the
// calls stay re-entrant across host threads.
constexpr int kMaxDevices = 64;
int current_device();              // hipGetDevice, clamped to [0, kMaxDevices)
int device_cu_count();             // compute units of the current device (cached)
template <class F>
void once_per_device(std::once_flag (&flags)[kMaxDevices], F&& fn) {
  std::call_once(flags[current_device()], fn);
}

// run-time A/B knob (vtd_set_knob): the environment's value read once per process, or the
// override; -1 = unset (vtd_runtime.hip)
int knob(int k);

// profiling hooks (vtd_profile.cpp); no-ops unless enabled
enum ProfClass { PROF_GEMM = 0, PROF_ATTN = 1, PROF_LN = 2, PROF_PATCH = 3, PROF_OTHER = 4 };
struct ProfScope {
  ProfScope(hipStream_t s, int cls, double flops);
  ~ProfScope();
  hipStream_t stream; int cls; int slot;
};

// ----------------------------------------------------------------- device types
typedef uint16_t bf16_t;  // raw bf16 bits
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) int i32x4;   // 16-B raw chunk

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}
// round-to-nearest-even via the hardware v_cvt_pk_bf16_f32 (a plain cast at -O3);
// NaN stays NaN.
typedef __bf16 bf16x2_hw __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(bf16_t, static_cast<__bf16>(f));
}
// two floats -> packed bf16 pair (lo = a), one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2_hw));
}

// split-bf16 (VTD_BF16X3, include/vtd.h "Split-bf16 operands"): hi = bf16(v) (RNE), lo =
// bf16(v - hi) -- v - hi is exact in f32.  For a pair packed as hi = pack_bf16x2(a, b):
__device__ __forceinline__ uint32_t pack_lo_bf16x2(float a, float b, uint32_t hi) {
  return pack_bf16x2(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xffff0000u));
}
__device__ __forceinline__ bf16_t lo_bf16(float v, bf16_t hi) {
  return f32_to_bf16(v - __uint_as_float((uint32_t)hi << 16));
}

template <typename T> struct DT;
template <> struct DT<float> {
  static constexpr int code = VTD_F32;
  __device__ static float load(const float* p) { return *p; }
  __device__ static float from(float v) { return v; }
};
template <> struct DT<bf16_t> {
  static constexpr int code = VTD_BF16;
  __device__ static float load(const bf16_t* p) { return bf16_to_f32(*p); }
  __device__ static bf16_t from(float v) { return f32_to_bf16(v); }
};

// ----------------------------------------------------------------- MX-fp8 (vtd_mx8.hip)
// E8M0 block exponent: the least E with amax <= 448 * 2^E (e4m3 max 448), clamped to
// [-126, 126]; amax = m 2^ex (m in [0.5, 1)) gives E = ex - 9 + (m > 0.875) (oracle/mx8.py).
__device__ __forceinline__ int mx8_exponent(float amax) {
  const uint32_t b = __float_as_uint(amax);
  const int e = (int)((b >> 23) & 0xff);
  if (e == 0) return -126;                           // zero / subnormal block
  const int E = e - 126 - 9 + ((b & 0x7fffff) > 0x600000 ? 1 : 0);
  return min(max(E, -126), 126);
}
// 4 values * inv (= 2^-E, exact) -> 4 e4m3 bytes (round to nearest even), little-endian
__device__ __forceinline__ uint32_t mx8_pack4(float a, float b, float c, float d, float inv) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a * inv, b * inv, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c * inv, d * inv, w, true);
  return (uint32_t)w;
}
// transform_predictions (vtd.py:586-647) of logit v in column f of the (.., 6) output:
// sigmoid; clip the last 4 to [0, 1]; [conf, cls * (CLASSES-1), cx * W, cy * H, h * H, w * W]
// with W = H = 608 (Constants.MODEL_IMAGE_SIZE, not the input shape).  Shared by
// decode_kernel and the fused GEMM epilogue so both give the same bits.
__device__ __forceinline__ float decode_transform(int f, float v) {
  float s = 1.f / (1.f + expf(-v));
  if (f >= 2) s = fminf(fmaxf(s, 0.f), 1.f);
  return s * (f == 0 ? 1.f : (f == 1 ? 79.f : 608.f));
}

// bf16 rounding of an f32 value, back in f32 (the fused quantizers quantize what the
// unfused path would have stored as bf16)
// Sum over the 64 lanes in the butterfly order s += s[l ^ o], o = 32, 16, 8, 4, 2, 1 (every
// lane ends with the total; the same bits as that __shfl_xor loop: each step adds the same
// two values) without the LDS round trips of ds_bpermute: the gfx950 lane swaps for 32 / 16,
// DPP for the rest.  After the xor-8 step lanes l and l ^ 8 agree, so row_ror:4 (lane
// (l + 4) mod 16) delivers the value of l ^ 4.
template <int CTRL>
__device__ __forceinline__ float dpp_get(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float s) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  s = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  s = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  s += dpp_get<0x128>(s);   // row_ror:8  (l ^ 8 within the 16-lane row)
  s += dpp_get<0x124>(s);   // row_ror:4  (l ^ 4, see above)
  s += dpp_get<0x4E>(s);    // quad_perm [2, 3, 0, 1]
  s += dpp_get<0xB1>(s);    // quad_perm [1, 0, 3, 2]
  return s;
}
__device__ __forceinline__ float bf16_round(float v) {
  return __uint_as_float((uint32_t)f32_to_bf16(v) << 16);
}
// bf16_round of four values through two paired conversions (v_cvt_pk_bf16_f32, the same
// rounding) and their unpacks: 6 VALU instead of 8
__device__ __forceinline__ void bf16_round4(f32x4& v) {
  const uint32_t p0 = pack_bf16x2(v[0], v[1]), p1 = pack_bf16x2(v[2], v[3]);
  v[0] = __uint_as_float(p0 << 16);
  v[1] = __uint_as_float(p0 & 0xffff0000u);
  v[2] = __uint_as_float(p1 << 16);
  v[3] = __uint_as_float(p1 & 0xffff0000u);
}

// ----------------------------------------------------------------- activations
// tfa.activations.mish = x * tanh(softplus(x)) (vtd.py:128-129).
// tanh(log(1+e^x)) = n / (n + 2) with n = e^x (e^x + 2): no cancellation for x << 0.
// v_exp_f32 / v_rcp_f32 (~1 ulp): 8 VALU, 2 of them transcendental.
__device__ __forceinline__ float act_mish(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 1.4426950408889634f);
  const float n = e * (e + 2.f);
  const float y = x * n * __builtin_amdgcn_rcpf(n + 2.f);
  return x > 20.f ? x : y;                     // tanh(softplus(x)) == 1 in fp32
}
// tfa GELU approximate=True: 0.5 x (1 + tanh(u)), u = sqrt(2/pi) (x + 0.044715 x^3)
// == x * sigmoid(2u) = x / (1 + 2^(x (c0 + c1 x^2))), c0 = -2 sqrt(2/pi) log2(e),
// c1 = 0.044715 c0: 7 VALU, 2 transcendental; saturates correctly (inf -> 0, 0 -> x).
__device__ __forceinline__ float act_gelu(float x) {
  constexpr float c0 = -2.f * 0.7978845608028654f * 1.4426950408889634f;
  constexpr float c1 = c0 * 0.044715f;
  const float e = __builtin_amdgcn_exp2f(x * __builtin_fmaf(c1, x * x, c0));
  return x * __builtin_amdgcn_rcpf(1.f + e);
}
// LayerNorm row statistics from a producer GEMM's S centred partials per 64-column block
// (block mean, sum of squared deviations), already in registers as S / 2 16-B words: Chan's
// pairwise merge for equal counts relative to the first block mean (ln_stats_finalize_s_kernel
// and the pp2 GEMM's fused finalize share this, so both give identical (mean, rstd)).
template <int S>
__device__ __forceinline__ float2 ln_merge_partials(const f32x4 (&v)[S / 2], int D, float eps) {
  // no FMA contraction: the same instructions wherever this is inlined
#pragma clang fp contract(off)
  float2 t[S];
#pragma unroll
  for (int b = 0; b < S / 2; ++b) {
    t[2 * b] = float2{v[b][0], v[b][1]};
    t[2 * b + 1] = float2{v[b][2], v[b][3]};
  }
  const float m0 = t[0].x;
  float ds = 0.f, q = 0.f;
#pragma unroll
  for (int b = 0; b < S; ++b) {
    ds += t[b].x - m0;
    q += t[b].y;
  }
  const float dmean = ds / S;
  float between = 0.f;
#pragma unroll
  for (int b = 0; b < S; ++b) {
    const float dv = (t[b].x - m0) - dmean;
    between += dv * dv;
  }
  const float var = (q + 64.f * between) / D;
  return float2{m0 + dmean, 1.f / sqrtf(var + eps)};
}

// Two values at once: the ordinary f32 arithmetic through the packed VALU
// (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32, one instruction per pair), the
// transcendentals one by one (there is no packed v_exp_f32 / v_rcp_f32).  Same operations,
// same order as the scalar forms above: identical results.  (GELU: 2.5 + 2 transcendental
// issue slots per value instead of 5 + 2; it is most of the activation layers' epilogue.)
__device__ __forceinline__ f32x2 act_gelu2(f32x2 x) {
  constexpr float c0 = -2.f * 0.7978845608028654f * 1.4426950408889634f;
  constexpr float c1 = c0 * 0.044715f;
  const f32x2 t = x * __builtin_elementwise_fma(f32x2{c1, c1}, x * x, f32x2{c0, c0});
  const f32x2 d = f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.f;
  return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
__device__ __forceinline__ f32x2 act_mish2(f32x2 x) {
  const f32x2 t = x * 1.4426950408889634f;
  const f32x2 e = f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  const f32x2 n = e * (e + 2.f);
  const f32x2 d = n + 2.f;
  const f32x2 y = x * n * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  return f32x2{x.x > 20.f ? x.x : y.x, x.y > 20.f ? x.y : y.y};
}
__device__ __forceinline__ float apply_act(int act, float x) {
  if (act == VTD_ACT_GELU_TANH) return act_gelu(x);
  if (act == VTD_ACT_MISH) return act_mish(x);
  return x;
}

}  // namespace vtd
