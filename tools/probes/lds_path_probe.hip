// Per-CU throughput of the two ways to stage a GEMM operand tile into LDS, 1 workgroup of
// 512 threads per CU (256 CUs), 64 KiB per step per CU (the 256x256x64 bf16 K-tile):
//   mode 0: buffer_load_dwordx4 ... lds (LDS-DMA, 8 per wave per step)
//   mode 1: global_load_dwordx4 -> VGPR, then ds_write_b128 (register staging)
//   mode 2: global_load_dwordx4 -> VGPR only (no LDS write; the data is consumed by a xor)
// Source: `span` bytes per CU-group read cyclically (small span = L2-resident, large = HBM).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512) void stage(const char* __restrict__ src, int64_t span,
                                             int steps, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t base = ((int64_t)blockIdx.x * 65536) % span;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src), 0, 0x7fffffff, 0x00020000);
  i32x4 acc = {0, 0, 0, 0};
  for (int s = 0; s < steps; ++s) {
    const int64_t off = (base + (int64_t)s * 65536) % span;
    if constexpr (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (lds_void_t*)(smem + (s & 1) * 65536 + (wave * 8 + j) * 1024), 16,
            (int)(off + (wave * 8 + j) * 1024 + lane * 16), 0, 0, 0);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      i32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = *reinterpret_cast<const i32x4*>(src + off + (wave * 8 + j) * 1024 + lane * 16);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (MODE == 1)
          *reinterpret_cast<i32x4*>(smem + (s & 1) * 65536 + (wave * 8 + j) * 1024 + lane * 16) = v[j];
        else
          acc ^= v[j];
      }
    }
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (MODE == 2 && acc[0] == 0x12345 && acc[1] == 7) sink[0] = acc[2];
  if (MODE != 2 && tid == 0 && smem[tid * 4] == 123 && smem[9] == 7) sink[1] = 1;
}

int main() {
  const int64_t big = (int64_t)4 << 30;
  char* src;
  int* sink;
  if (hipMalloc(&src, big) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  (void)hipMemset(src, 1, big);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int steps = 400;
  for (int64_t span : {(int64_t)1 << 20, (int64_t)64 << 20, big}) {
    for (int mode = 0; mode < 3; ++mode) {
      auto fn = mode == 0 ? stage<0> : mode == 1 ? stage<1> : stage<2>;
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(fn, dim3(256), dim3(512), 131072, 0, src, span, steps, sink);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double bytes = 256.0 * steps * 65536;
        if (rep == 1)
          printf("span %6lld MiB mode %d: %.1f us, %.2f TB/s total, %.1f GB/s per CU, %.2f us per 64 KiB step\n",
                 (long long)(span >> 20), mode, ms * 1e3, bytes / ms / 1e9, bytes / 256 / ms / 1e6,
                 ms * 1e3 / steps);
      }
    }
  }
  return 0;
}
