// Which XCD does each workgroup of a GEMM-sized grid land on, alone and with a second
// grid running concurrently on another stream?  Reports, per launch, the fraction of block
// pairs (b, b + 8) that share an XCD (the GEMM's tile remap assumes they do).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(int* xcc_out, int spin_us) {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) xcc_out[blockIdx.x] = x & 15;
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < (long long)spin_us * 100) {}   // 100 MHz wall clock
}

static double pair_share(const std::vector<int>& v) {
  int same = 0, n = 0;
  for (size_t b = 0; b + 8 < v.size(); ++b) { same += v[b] == v[b + 8]; ++n; }
  return n ? (double)same / n : 0.0;
}

int main() {
  const int nb = 588;
  int *d1, *d2;
  hipMalloc(&d1, nb * 4); hipMalloc(&d2, nb * 4);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  std::vector<int> h1(nb), h2(nb);
  for (int trial = 0; trial < 3; ++trial) {
    // alone, after an odd-sized grid
    hipLaunchKernelGGL(probe, dim3(13), dim3(512), 0, s1, d2, 5);
    hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 0, s1, d1, 20);
    hipStreamSynchronize(s1);
    hipMemcpy(h1.data(), d1, nb * 4, hipMemcpyDeviceToHost);
    printf("alone: pair share %.3f first xcc %d\n", pair_share(h1), h1[0]);
    // two grids concurrently
    hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 0, s1, d1, 20);
    hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 0, s2, d2, 20);
    hipDeviceSynchronize();
    hipMemcpy(h1.data(), d1, nb * 4, hipMemcpyDeviceToHost);
    hipMemcpy(h2.data(), d2, nb * 4, hipMemcpyDeviceToHost);
    printf("concurrent: pair share %.3f / %.3f\n", pair_share(h1), pair_share(h2));
  }
  int hist[16] = {0};
  for (int v : h2) hist[v & 15]++;
  printf("xcc histogram (second grid):");
  for (int i = 0; i < 8; ++i) printf(" %d", hist[i]);
  printf("\n");
  return 0;
}
