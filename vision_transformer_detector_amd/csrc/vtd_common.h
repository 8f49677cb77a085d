// Shared helpers for the gfx950 kernels of libvtd.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

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
__device__ __forceinline__ float apply_act(int act, float x) {
  if (act == VTD_ACT_GELU_TANH) return act_gelu(x);
  if (act == VTD_ACT_MISH) return act_mish(x);
  return x;
}

}  // namespace vtd
