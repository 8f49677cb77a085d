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

// Four consecutive columns n..n+3 of row m (row-vector epilogue of the staged path).
__device__ __forceinline__ void epi_store4(const EpiArgs& e, int M, int N, int m, int n,
                                           f32x4 v) {
  if (m >= M) return;
  const bool full = (n + 3 < N) && e.scatter_tokens <= 0 && (e.ldo & 3) == 0 &&
                    (!e.resid || (e.ldr & 3) == 0) && (!e.out2 || (e.ldo2 & 3) == 0);
  if (!full) {
#pragma unroll
    for (int j = 0; j < 4; ++j) epi_store(e, M, N, m, n + j, v[j]);
    return;
  }
  if (e.bias) {
    const f32x4 b = *reinterpret_cast<const f32x4*>(e.bias + n);
    v += b;
  }
  if (e.rowadd) {
    const float ra = e.rowadd[m % e.rowadd_period];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += (n + j < e.rowadd_ncols) ? ra : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = apply_act(e.act, v[j]);
  if (e.resid) v += *reinterpret_cast<const f32x4*>(e.resid + (int64_t)m * e.ldr + n);
  const int64_t idx = (int64_t)m * e.ldo + n;
  if (e.out_dtype == VTD_F32) {
    *reinterpret_cast<f32x4*>(static_cast<float*>(e.out) + idx) = v;
  } else {
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = static_cast<short>(f32_to_bf16(v[j]));
    *reinterpret_cast<bf16x4*>(static_cast<bf16_t*>(e.out) + idx) = o;
  }
  if (e.out2) {
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = static_cast<short>(f32_to_bf16(v[j]));
    *reinterpret_cast<bf16x4*>(static_cast<bf16_t*>(e.out2) + (int64_t)m * e.ldo2 + n) = o;
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

// ============================================================================
// bf16 "big" kernel: 256 x 256 tile, BK = 64, 512 threads = 8 waves (2 M x 4 N), each
// wave 128 x 64 outputs = 8 x 4 blocks of v_mfma_f32_16x16x32_bf16.
// Operands go HBM/L2 -> LDS directly with global_load_lds_dwordx4 (no VGPR staging):
// one wave-instruction writes 1 KiB = 8 rows of 128 B, lane-linear in LDS; the
// chunk ^= row & 7 swizzle is applied on the per-lane GLOBAL source address and again
// on the ds_read, so the LDS image is the same as the 128-tile kernel's.
// Two LDS stages of 64 KiB (A 32 KiB + B 32 KiB).  Tile t+1's DMA stays in flight while
// tile t is computed: counted `s_waitcnt vmcnt(8)` (8 DMA instructions per wave per
// tile) + raw s_barrier, never __syncthreads() (its fence would drain the DMA).
// Tiles are remapped so consecutive tiles (sharing an A panel) run on one XCD (T1).
// ============================================================================
constexpr int BBM = 256, BBN = 256, BNT = 512;
constexpr int BSTAGE = (BBM + BBN) * KB;     // 64 KiB per stage
static_assert(8 * 32 * 68 * 4 <= 2 * BSTAGE, "epilogue staging must fit the stages");

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

__device__ __forceinline__ void glds16(const char* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ void issue_tile(char* smem, const char* const (&srcA)[4],
                                           const char* const (&srcB)[4], int lds_piece,
                                           int kt, int stage) {
  char* base = smem + stage * BSTAGE;
  const int64_t ko = (int64_t)kt * KB;
#pragma unroll
  for (int j = 0; j < 4; ++j) glds16(srcA[j] + ko, base + lds_piece + j * 8 * KB);
#pragma unroll
  for (int j = 0; j < 4; ++j) glds16(srcB[j] + ko, base + BBM * KB + lds_piece + j * 8 * KB);
}

__global__ __launch_bounds__(BNT) void gemm_tn_bf16_256_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda,
    const bf16_t* __restrict__ Bt, int ldb, int tiles_m, int tiles_n, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // ---- XCD-aware bijective tile remap: blocks b, b+8, ... share an XCD
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = tile / tiles_n, tn = tile - (tile / tiles_n) * tiles_n;
  const int m0 = tm * BBM, n0 = tn * BBN;

  // ---- DMA source addresses: this wave fills rows [wave*32, wave*32+32) of the A tile
  // and of the B tile, as 4 pieces of 8 rows; lane l -> row +(l>>3), logical chunk
  // (l & 7) ^ (l >> 3) (the row's swizzle), so the LDS image is row*128 + (c^(row&7))*16.
  const int prow = lane >> 3;
  const int pchunk = (lane & 7) ^ prow;
  const char* srcA[4];
  const char* srcB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wave * 32 + j * 8 + prow;
    srcA[j] = reinterpret_cast<const char*>(A + (int64_t)min(m0 + row, M - 1) * lda) + pchunk * 16;
    srcB[j] = reinterpret_cast<const char*>(Bt + (int64_t)min(n0 + row, N - 1) * ldb) + pchunk * 16;
  }
  const int lds_piece = wave * 32 * KB;       // byte offset of this wave's first piece

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  const int nk = K / 64;
  issue_tile(smem, srcA, srcB, lds_piece, 0, 0);
  if (nk > 1) issue_tile(smem, srcA, srcB, lds_piece, 1, 1);

  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const char* la = smem + (kt & 1) * BSTAGE;
    const char* lb = la + BBM * KB;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + fg;
      bf16x8 af[8], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(lb + swz(wn * 64 + j * 16 + fr, c));
#pragma unroll
      for (int i = 0; i < 8; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(la + swz(wm * 128 + i * 16 + fr, c));
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + 2 < nk) issue_tile(smem, srcA, srcB, lds_piece, kt + 2, kt & 1);
  }

  // ---- epilogue staged through LDS (the stages are free after the last barrier):
  // each wave owns a private 32 x 68-float region (8 waves x 8.5 KiB); pass p stages
  // accumulator rows i = 2p, 2p+1 (32 rows x 64 cols), then reads them back as row
  // vectors so bias / activation / residual / store use 16-B coalesced accesses.
  constexpr int ES = 68;      // row stride (floats): rows 4 apart hit opposite bank halves
  float* ep = reinterpret_cast<float*>(smem) + wave * 32 * ES;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r2 = 0; r2 < 4; ++r2)
          ep[(i * 16 + fg * 4 + r2) * ES + j * 16 + fr] = acc[p * 2 + i][j][r2];
#pragma unroll 4
    for (int it = 0; it < 8; ++it) {
      const int row = it * 4 + (lane >> 4), col = (lane & 15) * 4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(ep + row * ES + col);
      epi_store4(e, M, N, m0 + wm * 128 + p * 32 + row, n0 + wn * 64 + col, v);
    }
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
  const int tiles_m = (M + BBM - 1) / BBM, tiles_n = (N + BBN - 1) / BBN;
  if (dtype == VTD_BF16 && tiles_m * tiles_n >= 128) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_bf16_256_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BSTAGE);
      attr = true;
    }
    hipLaunchKernelGGL(gemm_tn_bf16_256_kernel, dim3(tiles_m * tiles_n), dim3(BNT),
                       2 * BSTAGE, stream, M, N, K, static_cast<const bf16_t*>(A), lda,
                       static_cast<const bf16_t*>(Bt), ldb, tiles_m, tiles_n, e);
  } else if (dtype == VTD_BF16)
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
