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
// round-to-nearest-even; NaN stays NaN
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<bf16_t>((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<bf16_t>(u >> 16);
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
__device__ __forceinline__ float act_mish(float x) {
  if (x > 20.f) return x;                      // tanh(softplus(x)) == 1 in fp32
  float e = __expf(x);
  float n = e * (e + 2.f);
  return x * __fdividef(n, n + 2.f);
}
// tfa GELU approximate=True: 0.5 x (1 + tanh(u)), u = sqrt(2/pi) (x + 0.044715 x^3)
// == x * sigmoid(2u).
__device__ __forceinline__ float act_gelu(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  return __fdividef(x, 1.f + __expf(-2.f * u));
}
__device__ __forceinline__ float apply_act(int act, float x) {
  if (act == VTD_ACT_GELU_TANH) return act_gelu(x);
  if (act == VTD_ACT_MISH) return act_mish(x);
  return x;
}

}  // namespace vtd
