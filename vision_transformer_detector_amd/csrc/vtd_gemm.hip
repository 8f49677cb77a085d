// Dense layers of the detector (vtd.py:297, 389-403, 454-458, 472-483, 489-493) as one
// MFMA GEMM with a fused epilogue:  C = act(A Bt^T + bias + rowadd) + resid.
//
// Layout: A [M][lda] and Bt [N][ldb] are both K-contiguous ("TN"), so both MFMA operands
// are read the same way: each lane takes 16 contiguous bytes of one row.
// Tile: 128 x 128 outputs, K step = 128 bytes (64 bf16 / 32 f32), 256 threads = 4 waves
// in a 2x2 arrangement, 64 x 64 outputs per wave = 4 x 4 blocks of 16 x 16.
//   bf16: v_mfma_f32_16x16x32_bf16, one per (block, 32-k step)
//   f32 : v_mfma_f32_16x16x4_f32,   four per (block, 16-k step)  (exact f32 fma chain)
// Staging: global -> registers (issued before the MFMAs of the current tile) -> LDS
// (written after them), two LDS buffers, one barrier per K step.  LDS rows are 128 B and
// XOR-swizzled on the 16-B chunk index (chunk ^= row & 7) so the 16 rows read by one
// ds_read_b128 lane group spread over the banks.
#include "vtd_common.h"

namespace vtd {

namespace {

constexpr int BM = 128, BN = 128, KB = 128;  // KB = bytes of K per tile row
constexpr int NT = 256;
constexpr int TILE_BYTES = BM * KB;          // 16 KiB per operand per buffer

struct EpiArgs {
  const float* bias;
  const float* rowadd; int rowadd_period; int rowadd_ncols;
  int act;
  const float* resid; int ldr;
  void* out; int ldo; int out_dtype;
  void* out2; int ldo2;
  int scatter_tokens;
};

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * KB + ((chunk ^ (row & 7)) << 4);
}

__device__ __forceinline__ void epi_store(const EpiArgs& e, int M, int N, int m, int n,
                                          float v) {
  if (m >= M || n >= N) return;
  if (e.bias) v += e.bias[n];
  if (e.rowadd && n < e.rowadd_ncols) v += e.rowadd[m % e.rowadd_period];
  v = apply_act(e.act, v);
  if (e.resid) v += e.resid[(int64_t)m * e.ldr + n];
  int64_t idx;
  if (e.scatter_tokens > 0) {
    // keras Reshape((17, -1)) of a (B, T, 17) tensor (vtd.py:461-463): flat index
    // f = t*17 + n inside image b lands at row f / T, column f % T of (B, 17, T).
    const int T = e.scatter_tokens;
    int b = m / T, t = m - b * T;
    int f = t * VTD_MAX_DETECT + n;
    idx = ((int64_t)b * VTD_MAX_DETECT + f / T) * e.ldo + (f % T);
  } else {
    idx = (int64_t)m * e.ldo + n;
  }
  if (e.out_dtype == VTD_F32) static_cast<float*>(e.out)[idx] = v;
  else static_cast<bf16_t*>(e.out)[idx] = f32_to_bf16(v);
  if (e.out2) static_cast<bf16_t*>(e.out2)[(int64_t)m * e.ldo2 + n] = f32_to_bf16(v);
}

__device__ __forceinline__ void gload4(i32x4 (&ra)[4], i32x4 (&rb)[4], const char* ga,
                                       const char* gb, const int64_t (&offa)[4],
                                       const int64_t (&offb)[4], int kt) {
  const int64_t o = (int64_t)kt * KB;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ra[i] = *reinterpret_cast<const i32x4*>(ga + offa[i] + o);
    rb[i] = *reinterpret_cast<const i32x4*>(gb + offb[i] + o);
  }
}
__device__ __forceinline__ void swrite4(const i32x4 (&ra)[4], const i32x4 (&rb)[4],
                                        char* lds_a, char* lds_b, int srow, int schunk,
                                        int buf) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int o = buf * TILE_BYTES + swz(srow + 32 * i, schunk);
    *reinterpret_cast<i32x4*>(lds_a + o) = ra[i];
    *reinterpret_cast<i32x4*>(lds_b + o) = rb[i];
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void gemm_tn_kernel(
    int M, int N, int K, const T* __restrict__ A, int lda, const T* __restrict__ Bt,
    int ldb, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* lds_a = smem;                        // [2][TILE_BYTES]
  char* lds_b = smem + 2 * TILE_BYTES;       // [2][TILE_BYTES]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  // global -> register staging: 4 chunks of 16 B per thread per operand
  const int srow = tid >> 3, schunk = tid & 7;
  const char* ga = reinterpret_cast<const char*>(A) + schunk * 16;
  const char* gb = reinterpret_cast<const char*>(Bt) + schunk * 16;
  const int64_t lda_b = (int64_t)lda * sizeof(T), ldb_b = (int64_t)ldb * sizeof(T);
  int64_t offa[4], offb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    offa[i] = (int64_t)min(m0 + srow + 32 * i, M - 1) * lda_b;
    offb[i] = (int64_t)min(n0 + srow + 32 * i, N - 1) * ldb_b;
  }
  i32x4 ra_[4], rb_[4];

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  const int nk = K * (int)sizeof(T) / KB;

  gload4(ra_, rb_, ga, gb, offa, offb, 0);
  swrite4(ra_, rb_, lds_a, lds_b, srow, schunk, 0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload4(ra_, rb_, ga, gb, offa, offb, kt + 1);
    const char* la = lds_a + buf * TILE_BYTES;
    const char* lb = lds_b + buf * TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + fg;
      i32x4 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = *reinterpret_cast<const i32x4*>(la + swz(wm * 64 + i * 16 + fr, c));
        bfr[i] = *reinterpret_cast<const i32x4*>(lb + swz(wn * 64 + i * 16 + fr, c));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (sizeof(T) == 2) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, af[i]), __builtin_bit_cast(bf16x8, bfr[j]),
                acc[i][j], 0, 0, 0);
          } else {
            const f32x4 a4 = __builtin_bit_cast(f32x4, af[i]);
            const f32x4 b4 = __builtin_bit_cast(f32x4, bfr[j]);
#pragma unroll
            for (int t = 0; t < 4; ++t)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t], b4[t], acc[i][j],
                                                                0, 0, 0);
          }
        }
    }
    if (kt + 1 < nk) swrite4(ra_, rb_, lds_a, lds_b, srow, schunk, buf ^ 1);
    __syncthreads();
  }

  // epilogue: C/D map col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int m = m0 + wm * 64 + i * 16 + fg * 4 + r;
        int n = n0 + wn * 64 + j * 16 + fr;
        epi_store(e, M, N, m, n, acc[i][j][r]);
      }
}

}  // namespace

int gemm_launch(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                int dtype, const vtd_epilogue* epi, hipStream_t stream, double flops) {
  VTD_CHECK_ARG(M > 0 && N > 0 && K > 0, "gemm: M, N, K must be positive");
  VTD_CHECK_ARG(K % VTD_KALIGN == 0, "gemm: K must be a multiple of VTD_KALIGN");
  VTD_CHECK_ARG(A && Bt && epi && epi->out, "gemm: null pointer");
  VTD_CHECK_ARG(lda >= K && ldb >= K && lda % 8 == 0 && ldb % 8 == 0,
                "gemm: lda/ldb must be >= K and multiples of 8");
  VTD_CHECK_ARG(dtype == VTD_F32 || dtype == VTD_BF16, "gemm: bad dtype");
  VTD_CHECK_ARG(epi->out_dtype == VTD_F32 || epi->out_dtype == VTD_BF16,
                "gemm: bad out dtype");
  VTD_CHECK_ARG(!epi->rowadd || epi->rowadd_period > 0, "gemm: rowadd_period");
  VTD_CHECK_ARG(epi->scatter_tokens <= 0 || N <= VTD_MAX_DETECT,
                "gemm: scatter epilogue needs N <= 17");
  EpiArgs e{epi->bias, epi->rowadd, epi->rowadd_period,
            epi->rowadd ? epi->rowadd_ncols : 0, epi->act, epi->resid, epi->ldr,
            epi->out, epi->ldo, epi->out_dtype, epi->out2, epi->ldo2,
            epi->scatter_tokens};
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM);
  const size_t lds = 4 * TILE_BYTES;
  ProfScope ps(stream, PROF_GEMM, flops > 0 ? flops : 2.0 * M * N * (double)K);
  if (dtype == VTD_BF16)
    hipLaunchKernelGGL(gemm_tn_kernel<bf16_t>, grid, dim3(NT), lds, stream, M, N, K,
                       static_cast<const bf16_t*>(A), lda,
                       static_cast<const bf16_t*>(Bt), ldb, e);
  else
    hipLaunchKernelGGL(gemm_tn_kernel<float>, grid, dim3(NT), lds, stream, M, N, K,
                       static_cast<const float*>(A), lda, static_cast<const float*>(Bt),
                       ldb, e);
  VTD_LAUNCH_CHECK("gemm");
  return VTD_OK;
}

}  // namespace vtd

extern "C" int vtd_gemm(int M, int N, int K, const void* A_dev, int lda,
                        const void* Bt_dev, int ldb, int dtype, const vtd_epilogue* epi,
                        void* stream) {
  return vtd::gemm_launch(M, N, K, A_dev, lda, Bt_dev, ldb, dtype, epi,
                          static_cast<hipStream_t>(stream), 0.0);
}
