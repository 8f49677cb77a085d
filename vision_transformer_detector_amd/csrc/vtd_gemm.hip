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
#include <stdlib.h>

#include <algorithm>
#include <mutex>

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
  const void* resid; int ldr;      // same dtype as out (f32, or the bf16 residual stream)
  void* out; int ldo; int out_dtype;
  void* out2; int ldo2;
  int scatter_tokens;
  // LayerNorm folded into this GEMM (A = the raw residual stream): per row (mean, rstd),
  // per column colsum[n] = sum_k Bt[n][k]; acc -> (acc - mean * colsum) * rstd first
  const float2* lnstat; const float* colsum;
  // partial LayerNorm statistics of the stored bf16 rows (fold path producer): per row m
  // and 64-column block b, statout[m * stat_ld + b] = (block mean, sum of squared
  // deviations from it) -- centred, so rows with |mean| >> std lose nothing (Chan merge in
  // ln_stats_finalize_kernel)
  float2* statout; int stat_ld;
  // out_dtype VTD_FP8 (MX-fp8 GEMMs, fast epilogue): e4m3 out + E8M0 scales [n/128][s_rows][4]
  uint8_t* sout; int64_t s_rows;
  float* dets;                     // fused transform_predictions (N == 6, fp32 out)
  // fused LayerNorm finalize (pp2 consumers of the fold path): the producer's per-row
  // per-64-column centred partials, `lnslots` per row; the kernel merges them itself (as
  // ln_stats_finalize_kernel) instead of reading lnstat
  const float2* lnpart; int lnslots; int lnD; float lneps;
  // tile order (pp2): 0 = row-major (an XCD walks all n-tiles of consecutive m-rows); g > 0 =
  // n-groups of g tiles, m-rows inside a group (an XCD keeps a group's weight panels in L2)
  int ngw;
};

// bf16 output row vector store of the fast epilogues; build-time A/B knob VTD_OUT_NT: 1 =
// non-temporal (streaming) stores, so the output stream does not evict the weight panels
#ifndef VTD_OUT_NT
#define VTD_OUT_NT 0
#endif
__device__ __forceinline__ void store_out16(void* p, i32x4 v) {
  if constexpr (VTD_OUT_NT) __builtin_nontemporal_store(v, reinterpret_cast<i32x4*>(p));
  else *reinterpret_cast<i32x4*>(p) = v;
}

// tile index -> (tm, tn) for EpiArgs::ngw (bijective; the last n-group may be narrower)
__device__ __forceinline__ void tile_coords(int tile, int tiles_m, int tiles_n, int ngw, int& tm,
                                            int& tn) {
  if (ngw <= 0 || ngw >= tiles_n) {
    tm = tile / tiles_n;
    tn = tile - tm * tiles_n;
    return;
  }
  const int full = tiles_n / ngw, gsz = tiles_m * ngw;
  const int g = tile / gsz;
  if (g < full) {
    const int r = tile - g * gsz;
    tm = r / ngw;
    tn = g * ngw + (r - tm * ngw);
  } else {
    const int lw = tiles_n - full * ngw, r = tile - full * gsz;
    tm = r / lw;
    tn = full * ngw + (r - tm * lw);
  }
}

// v of another lane of the same 16-lane row by a DPP control (0 where the source is out
// of the row)
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// v[l] + v[l ^ 16] and v[l] + v[l ^ 32] by the gfx950 lane-swap instructions (no LDS)
__device__ __forceinline__ float xsum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// sum of the 8 bf16 values packed in o
__device__ __forceinline__ float bf16x8_sum(const i32x4& o) {
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w)
    s += __uint_as_float((uint32_t)o[w] << 16) + __uint_as_float((uint32_t)o[w] & 0xffff0000u);
  return s;
}
// sum of squared deviations from `mean` of the 8 bf16 values packed in o
__device__ __forceinline__ float bf16x8_m2(const i32x4& o, float mean) {
  float q = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const float lo = __uint_as_float((uint32_t)o[w] << 16) - mean;
    const float hi = __uint_as_float((uint32_t)o[w] & 0xffff0000u) - mean;
    q += lo * lo + hi * hi;
  }
  return q;
}
// total over the 8 consecutive lanes of a half-row, in all 8 lanes: DPP quad xor 1,
// quad xor 2, then row_half_mirror (lane i <-> 7 - i: the other quad)
__device__ __forceinline__ float sum8_dpp(float t) {
  t += dpp_f32<0xB1>(t);
  t += dpp_f32<0x4E>(t);
  return t + dpp_f32<0x141>(t);
}

__device__ __forceinline__ float resid_at(const EpiArgs& e, int64_t i) {
  return e.out_dtype == VTD_F32 ? static_cast<const float*>(e.resid)[i]
                                : bf16_to_f32(static_cast<const bf16_t*>(e.resid)[i]);
}
__device__ __forceinline__ f32x4 bf16x4_to_f32(uint32_t lo, uint32_t hi) {
  return f32x4{__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
               __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
}
// 8 contiguous residual values (16-B aligned): BF = bf16 residual (one 16-B load)
template <bool BF>
__device__ __forceinline__ void load_resid8(const EpiArgs& e, int64_t i, f32x4& r0, f32x4& r1) {
  if constexpr (BF) {
    const i32x4 w = *reinterpret_cast<const i32x4*>(static_cast<const bf16_t*>(e.resid) + i);
    r0 = bf16x4_to_f32((uint32_t)w[0], (uint32_t)w[1]);
    r1 = bf16x4_to_f32((uint32_t)w[2], (uint32_t)w[3]);
  } else {
    const float* p = static_cast<const float*>(e.resid) + i;
    r0 = *reinterpret_cast<const f32x4*>(p);
    r1 = *reinterpret_cast<const f32x4*>(p + 4);
  }
}

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * KB + ((chunk ^ (row & 7)) << 4);
}

__device__ __forceinline__ void epi_store(const EpiArgs& e, int M, int N, int m, int n,
                                          float v) {
  if (m >= M || n >= N) return;
  if (e.lnstat) {
    const float2 st = e.lnstat[m];
    v = (v - st.x * e.colsum[n]) * st.y;
  }
  if (e.bias) v += e.bias[n];
  if (e.rowadd && n < e.rowadd_ncols) v += e.rowadd[m % e.rowadd_period];
  v = apply_act(e.act, v);
  if (e.resid) v += resid_at(e, (int64_t)m * e.ldr + n);
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
  if (e.dets) e.dets[(int64_t)m * 6 + n] = decode_transform(n, v);
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
  const bool full = (n + 3 < N) && e.scatter_tokens <= 0 && !e.dets && (e.ldo & 3) == 0 &&
                    (!e.resid || (e.ldr & 3) == 0) && (!e.out2 || (e.ldo2 & 3) == 0);
  if (!full) {
#pragma unroll
    for (int j = 0; j < 4; ++j) epi_store(e, M, N, m, n + j, v[j]);
    return;
  }
  if (e.lnstat) {
    const float2 st = e.lnstat[m];
    v = (v - st.x * *reinterpret_cast<const f32x4*>(e.colsum + n)) * st.y;
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
  if (e.resid) {
    const int64_t ri = (int64_t)m * e.ldr + n;
    if (e.out_dtype == VTD_F32) {
      v += *reinterpret_cast<const f32x4*>(static_cast<const float*>(e.resid) + ri);
    } else {
      const uint2 w = *reinterpret_cast<const uint2*>(static_cast<const bf16_t*>(e.resid) + ri);
      v += bf16x4_to_f32(w.x, w.y);
    }
  }
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


// ============================================================================
// bf16 "ping-pong" kernel: same tile (256 x 256, BK 64), LDS image, DMA staging and
// epilogue as gemm_tn_bf16_256_kernel, but the 8 waves run as two groups offset by one
// barrier: G0 = waves 0-3 (A rows 0-127), G1 = waves 4-7 (A rows 128-255).  Each SIMD
// holds one wave of each group, so while one group issues its MFMAs the other issues
// its LDS reads and DMA (the two pipes overlap instead of alternating).
//
// A K-tile is 4 phases; a phase = [L: ds_reads (+ DMA)] barrier [C: 16 MFMAs] barrier,
// computing one 64 x 32 quadrant of the wave's 128 x 64 tile:
//   P0: a <- A quad 0, b0 <- B quad 0, DMA A of tile t+1 | C: acc[0..3][0..1]
//   P1: b1 <- B quad 1, DMA B of tile t+1                | C: acc[0..3][2..3]
//   P2: a <- A quad 1                                    | C: acc[4..7][2..3]
//   P3: s_waitcnt vmcnt(0) (tile t+1 landed)             | C: acc[4..7][0..1]
// Barrier bookkeeping (event e = e-th workgroup barrier; G1 runs one extra barrier
// first, G0 one extra last): G0's L_p ends at event 2p+1, G1's at 2p+2.  Hazards:
//   RAW (DMA -> ds_read): every wave drains its DMA (vmcnt(0)) in L_{4t+3}, before
//     event 8t+8; the first read of tile t+1 (G0, L_{4t+4}) starts after event 8t+8.
//   WAR (ds_read -> DMA into the same stage): the last reads of tile t-1 (L_{4t-2},
//     retired by the lgkmcnt wait in C_{4t-2}) finish before event 8t-1; the DMA of
//     tile t+1 into that stage issues in L_{4t}, after event 8t.
// ============================================================================
// ---- specialized epilogue (EPI = act | out_bf16 << 2 | resid << 3), full tiles only
constexpr int EPI_GENERIC = -1;
__host__ __device__ constexpr int epi_code(int act, bool out_bf16, bool resid) {
  return act | (out_bf16 ? 4 : 0) | (resid ? 8 : 0);
}

template <int ACT>
__device__ __forceinline__ float act_ct(float x) {
  if constexpr (ACT == VTD_ACT_GELU_TANH) return act_gelu(x);
  else if constexpr (ACT == VTD_ACT_MISH) return act_mish(x);
  else return x;
}
// the activation of 8 values (two f32x4), pairwise through the packed VALU
template <int ACT>
__device__ __forceinline__ void act_ct8(f32x4& v0, f32x4& v1) {
  if constexpr (ACT == VTD_ACT_GELU_TANH || ACT == VTD_ACT_MISH) {
    f32x2 p[4] = {v0.xy, v0.zw, v1.xy, v1.zw};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      p[i] = ACT == VTD_ACT_GELU_TANH ? act_gelu2(p[i]) : act_mish2(p[i]);
    v0 = f32x4{p[0].x, p[0].y, p[1].x, p[1].y};
    v1 = f32x4{p[2].x, p[2].y, p[3].x, p[3].y};
  }
}

// Rare runtime modes kept on the fast epilogues (one launch per forward each): the
// position-embedding row add of the patch embedding (vtd.py:305; before the activation,
// columns < rowadd_ncols only) and the bf16 copy of the last encoder residual (out2, the
// head's input).  8 contiguous columns n .. n + 7 of row m.
__device__ __forceinline__ void epi_rowadd8(const EpiArgs& e, int m, int n, f32x4& v0,
                                            f32x4& v1) {
  const float ra = e.rowadd[m % e.rowadd_period];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v0[j] += (n + j < e.rowadd_ncols) ? ra : 0.f;
    v1[j] += (n + 4 + j < e.rowadd_ncols) ? ra : 0.f;
  }
}
__device__ __forceinline__ void epi_out2_8(const EpiArgs& e, int m, int n, f32x4 v0, f32x4 v1) {
  const i32x4 o = {(int)pack_bf16x2(v0[0], v0[1]), (int)pack_bf16x2(v0[2], v0[3]),
                   (int)pack_bf16x2(v1[0], v1[1]), (int)pack_bf16x2(v1[2], v1[3])};
  *reinterpret_cast<i32x4*>(static_cast<bf16_t*>(e.out2) + (int64_t)m * e.ldo2 + n) = o;
}

// LayerNorm fold of 8 contiguous columns of row m (c0, c1 = colsum of those columns).
// lst (the pp2 kernels): the (mean, rstd) of the wave's 128 rows, loaded before the K
// loop, lane l holding local rows l (lst[0]) and 64 + l (lst[1]); lr = m's local row.
__device__ __forceinline__ void epi_lnfold8(const EpiArgs& e, const float2* lst, int m, int lr,
                                            f32x4 c0, f32x4 c1, f32x4& v0, f32x4& v1) {
  float2 st;
  if (lst) {
    const float2 h = (lr & 64) ? lst[1] : lst[0];
    st.x = __shfl(h.x, lr & 63);
    st.y = __shfl(h.y, lr & 63);
  } else {
    st = e.lnstat[m];
  }
  v0 = (v0 - st.x * c0) * st.y;
  v1 = (v1 - st.x * c1) * st.y;
}

// Writes the wave's 128 x 64 accumulator tile: 4 passes of 32 rows staged through the
// wave's private LDS region; each lane then owns 8 consecutive columns of a row, so
// residual reads and output writes are 16-B per lane (one 128-B line per 8 lanes).
template <int EPI, bool kDiagNoStore = false, int PR = 32>
__device__ __forceinline__ void epilogue_fast(const f32x4 (&acc)[8][4], float* ep, int lane,
                                              int m_base, int n_base, const EpiArgs& e,
                                              const float2* lst = nullptr) {
  constexpr int ACT = EPI & 3;
  constexpr bool OUT_BF16 = (EPI & 4) != 0;
  constexpr bool RESID = (EPI & 8) != 0;
  constexpr int ES = 68;
  constexpr int NB = PR / 16;            // accumulator row blocks per pass
  constexpr int NIT = PR / 8;            // row-vector iterations per pass
  const int fr = lane & 15, fg = lane >> 4;
  const int c8 = (lane & 7) * 8, rsub = lane >> 3;
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(e.bias + n_base + c8);
  const f32x4 b1 = *reinterpret_cast<const f32x4*>(e.bias + n_base + c8 + 4);
  f32x4 cs0 = {}, cs1 = {};
  if (e.lnstat) {
    cs0 = *reinterpret_cast<const f32x4*>(e.colsum + n_base + c8);
    cs1 = *reinterpret_cast<const f32x4*>(e.colsum + n_base + c8 + 4);
  }
  if (e.scatter_tokens == -2) m_base &= 255;   // timing diagnostic (VTD_GEMM_VARIANT=5)
#pragma unroll
  for (int p = 0; p < 128 / PR; ++p) {
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r2 = 0; r2 < 4; ++r2)
          ep[(i * 16 + fg * 4 + r2) * ES + j * 16 + fr] = acc[p * NB + i][j][r2];
    f32x4 rv[NIT][2];
    if constexpr (RESID) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int64_t m = m_base + p * PR + it * 8 + rsub;
        load_resid8<OUT_BF16>(e, m * e.ldr + n_base + c8, rv[it][0], rv[it][1]);
      }
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int row = it * 8 + rsub;
      f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + row * ES + c8);
      f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + row * ES + c8 + 4);
      if (e.lnstat) epi_lnfold8(e, lst, m_base + p * PR + row, p * PR + row, cs0, cs1, v0, v1);
      v0 += b0;
      v1 += b1;
      if (e.rowadd) epi_rowadd8(e, m_base + p * PR + row, n_base + c8, v0, v1);
      act_ct8<ACT>(v0, v1);
      if constexpr (RESID) {
        v0 += rv[it][0];
        v1 += rv[it][1];
      }
      if (e.out2) epi_out2_8(e, m_base + p * PR + row, n_base + c8, v0, v1);
      const int64_t idx = (int64_t)(m_base + p * PR + row) * e.ldo + n_base + c8;
      if constexpr (kDiagNoStore) {
        if (v0[0] != v0[0] && v1[3] != v1[3]) static_cast<float*>(e.out)[idx] = v0[1];
      } else if constexpr (OUT_BF16) {
        if (e.out_dtype == VTD_FP8) {
          // the next MX GEMM's operand: a 32-column block = 4 consecutive lanes (c8 / 8
          // = 0..3 or 4..7), block amax by DPP quad xor 1 / xor 2; bf16-rounded values so
          // the bytes equal vtd_quantize_mx8 of the bf16 output
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v0[j] = bf16_round(v0[j]);
            v1[j] = bf16_round(v1[j]);
          }
          float am = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) am = fmaxf(am, fmaxf(fabsf(v0[j]), fabsf(v1[j])));
          am = fmaxf(am, dpp_f32<0xB1>(am));
          am = fmaxf(am, dpp_f32<0x4E>(am));
          const int E = mx8_exponent(am);
          const float inv = __uint_as_float((uint32_t)(127 - E) << 23);
          const uint2 qv = {mx8_pack4(v0[0], v0[1], v0[2], v0[3], inv),
                            mx8_pack4(v1[0], v1[1], v1[2], v1[3], inv)};
          *reinterpret_cast<uint2*>(static_cast<uint8_t*>(e.out) + idx) = qv;
          if ((lane & 3) == 0) {
            const int n = n_base + c8, b = n >> 5;
            e.sout[((int64_t)(b >> 2) * e.s_rows + m_base + p * PR + row) * 4 + (b & 3)] =
                (uint8_t)(E + 127);
          }
          continue;
        }
        const i32x4 o = {(int)pack_bf16x2(v0[0], v0[1]), (int)pack_bf16x2(v0[2], v0[3]),
                         (int)pack_bf16x2(v1[0], v1[1]), (int)pack_bf16x2(v1[2], v1[3])};
        store_out16(static_cast<bf16_t*>(e.out) + idx, o);
        if (e.statout) {           // the row's 64 columns live in 8 consecutive lanes
          // block mean, then the centred sum of squares (DPP sums, no LDS traffic)
          const float mean = sum8_dpp(bf16x8_sum(o)) * (1.f / 64.f);
          const float m2 = sum8_dpp(bf16x8_m2(o, mean));
          if ((lane & 7) == 7)
            e.statout[(int64_t)(m_base + p * PR + row) * e.stat_ld + (n_base >> 6)] =
                float2{mean, m2};
        }
      } else {
        float* op = static_cast<float*>(e.out) + idx;
        *reinterpret_cast<f32x4*>(op) = v0;
        *reinterpret_cast<f32x4*>(op + 4) = v1;
      }
    }
  }
}
// global stores the fast epilogue issues per wave (used for counted vmcnt waits)
template <int EPI, int PR = 32>
constexpr int epilogue_fast_stores() {
  return (128 / PR) * (PR / 8) * ((EPI & 4) ? 1 : 2);
}

// Runtime-flag epilogue for partial tiles and rare modes (rowadd, scatter, out2): the
// accumulators are staged into LDS inline (static register indices), and only the
// LDS -> global loop is kept rolled (keeps the kernel small).
template <int PR = 32>
__device__ __forceinline__ void epilogue_generic_pass(const float* ep, int lane, int M, int N,
                                                      int m_base, int n_base, const EpiArgs& e) {
  constexpr int ES = 68;
#pragma unroll 1
  for (int it = 0; it < PR / 4; ++it) {
    const int row = it * 4 + (lane >> 4), col = (lane & 15) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(ep + row * ES + col);
    epi_store4(e, M, N, m_base + row, n_base + col, v);
  }
}

template <int PR = 32>
__device__ __forceinline__ void epilogue_generic(const f32x4 (&acc)[8][4], float* ep, int lane,
                                                 int M, int N, int m_base, int n_base,
                                                 const EpiArgs& e) {
  constexpr int ES = 68;
  constexpr int NB = PR / 16;
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int p = 0; p < 128 / PR; ++p) {
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r2 = 0; r2 < 4; ++r2)
          ep[(i * 16 + fg * 4 + r2) * ES + j * 16 + fr] = acc[p * NB + i][j][r2];
    epilogue_generic_pass<PR>(ep, lane, M, N, m_base + p * PR, n_base, e);
  }
}

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int I0, int J0>
__device__ __forceinline__ void pp_mfma(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2],
                                        const bf16x8 (&b)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[I0 + i][J0 + j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s], b[j][s], acc[I0 + i][J0 + j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ void pp_load_a(bf16x8 (&a)[4][2], const char* la, int row0, int fr,
                                          int fg) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      a[i][s] = *reinterpret_cast<const bf16x8*>(la + swz(row0 + i * 16 + fr, 4 * s + fg));
}
__device__ __forceinline__ void pp_load_b(bf16x8 (&b)[2][2], const char* lb, int row0, int fr,
                                          int fg) {
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      b[j][s] = *reinterpret_cast<const bf16x8*>(lb + swz(row0 + j * 16 + fr, 4 * s + fg));
}

// ---- transposed-accumulator operand path (variant 9) -----------------------------------
// MFMA operands swapped (D = B-tile x A-tile^T): a lane's 4 accumulator rows are 4
// consecutive OUTPUT COLUMNS of one output row.  The B-group read is permuted so that
// blocks j = 0 / 1 of a 32-column half hold columns 8*fg + 0..3 / 8*fg + 4..7: each lane
// then owns 8 contiguous columns of a row and the epilogue stores 16 B per lane straight
// from registers (no LDS staging).  The permuted read rows {0-3, 8-11, 16-19, 24-27} + 4j
// would 2-way conflict under chunk ^ (row & 7); the B groups use
// chunk ^ (row & 7) ^ ((row >> 2) & 4) instead (conflict-free for every ds_read_b128 lane
// group of this pattern, checked exhaustively over the four wave offsets).
__device__ __forceinline__ int swz_t(int row, int chunk) {
  return row * KB + ((chunk ^ (row & 7) ^ ((row >> 2) & 4)) << 4);
}
__device__ __forceinline__ int perm_t(int j, int fr) { return 8 * (fr >> 2) + 4 * j + (fr & 3); }

__device__ __forceinline__ void pp_load_b_t(bf16x8 (&b)[2][2], const char* lb, int row0, int fr,
                                            int fg) {
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      b[j][s] = *reinterpret_cast<const bf16x8*>(lb + swz_t(row0 + perm_t(j, fr), 4 * s + fg));
}

template <int I0, int J0>
__device__ __forceinline__ void pp_mfma_t(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2],
                                          const bf16x8 (&b)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[I0 + i][J0 + j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][s], a[i][s], acc[I0 + i][J0 + j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

// The ping-pong K loop.  Precondition: K-tile 0 is in stage 0 and visible to all waves
// (its DMA drained and a workgroup barrier passed).  Postcondition: every wave has
// finished every section (re-aligned), all DMA of this loop has landed.
__device__ __forceinline__ void pp_mainloop(f32x4 (&acc)[8][4], char* smem,
                                            const char* const (&srcA)[4],
                                            const char* const (&srcB)[4], int lds_piece,
                                            int nk, int wm, int arow, int brow, int fr,
                                            int fg) {
  if (wm == 1) pp_barrier();                 // stagger G1 by one barrier
  bf16x8 a[4][2], b0[2][2], b1[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    const char* la = smem + (kt & 1) * BSTAGE;
    const char* lb = la + BBM * KB;
    char* nxt = smem + ((kt + 1) & 1) * BSTAGE;
    const bool pf = kt + 1 < nk;
    const int64_t ko = (int64_t)(kt + 1) * KB;
    // ---- P0
    pp_load_a(a, la, arow, fr, fg);
    pp_load_b(b0, lb, brow, fr, fg);
    if (pf) {
#pragma unroll
      for (int j = 0; j < 4; ++j) glds16(srcA[j] + ko, nxt + lds_piece + j * 8 * KB);
    }
    pp_barrier();
    pp_mfma<0, 0>(acc, a, b0);
    pp_barrier();
    // ---- P1
    pp_load_b(b1, lb, brow + 32, fr, fg);
    if (pf) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        glds16(srcB[j] + ko, nxt + BBM * KB + lds_piece + j * 8 * KB);
    }
    pp_barrier();
    pp_mfma<0, 2>(acc, a, b1);
    pp_barrier();
    // ---- P2
    pp_load_a(a, la, arow + 64, fr, fg);
    pp_barrier();
    pp_mfma<4, 2>(acc, a, b1);
    pp_barrier();
    // ---- P3
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_barrier();
    pp_mfma<4, 0>(acc, a, b0);
    pp_barrier();
  }
  if (wm == 0) pp_barrier();                 // re-align: every wave past its last section
}

// ---------------------------------------------------------------------------------
// Ping-pong K loop v2: each 64 KiB stage holds four 16 KiB DMA groups, one per operand
// quadrant a phase reads:  X0 = A rows {0-63, 128-191} (A quad 0 of both wave groups),
// X1 = A rows {64-127, 192-255}, Y0 = B rows {0-31, 64-95, 128-159, 192-223} (B quad 0
// of every wn), Y1 = the other B rows.  Group row gr -> LDS offset gr*128 + swizzled chunk.
// A group is re-filled as soon as its last reader has retired, two tiles ahead:
//   tile t, P0: DMA X1(t+1)  | reads X0(t), Y0(t) | wait vmcnt(10) -> Y1(t) landed
//           P1:              | reads Y1(t)        | wait vmcnt(8)  -> X1(t) landed
//           P2: DMA X0(t+2)  | reads X1(t)        |
//           P3: DMA Y0,Y1(t+2)|                   | wait vmcnt(10) -> X0,Y0(t+1) landed
// (2 DMA instructions per group per wave; waits count the younger DMA in issue order;
// any phase whose younger DMA may be missing near the end of K waits vmcnt(0).)
// WAR (event numbers as for the v1 loop): X1(t+1) overwrites X1(t-1), last read in
// tile t-1's P2 (retired by event 8t-1) and issued after event 8t; X0(t+2) overwrites
// X0(t) read in P0 (retired by 8t+3), issued after 8t+4; Y0/Y1(t+2) overwrite Y0/Y1(t)
// read in P0/P1 (retired by 8t+5), issued after 8t+6.
__device__ __forceinline__ int grp_tile_row(int g, int gr) {
  return g < 2 ? (gr & 64) * 2 + g * 64 + (gr & 63)          // X0 / X1 (A rows)
               : (gr >> 5) * 64 + (g - 2) * 32 + (gr & 31);  // Y0 / Y1 (B rows)
}

// DMA source addressing of one tile, from wave-uniform scalars only (the per-lane part,
// row-in-piece and swizzled chunk, is rederived from the lane id at each issue): keeps
// 8 x 64-bit per-lane pointers out of the K loop's register budget.
struct PP2Src {
  const bf16_t* A; const bf16_t* Bt;
  int lda, ldb, mlast, nlast, m0, n0;   // mlast = M - 1, nlast = N - 1
};

__device__ __forceinline__ void pp2_sources(PP2Src& src, const bf16_t* A, int lda, int M,
                                            const bf16_t* Bt, int ldb, int N, int m0, int n0,
                                            int, int) {
  src.A = A; src.Bt = Bt; src.lda = lda; src.ldb = ldb;
  src.mlast = M - 1; src.nlast = N - 1; src.m0 = m0; src.n0 = n0;
}

__device__ __forceinline__ int opaque_lane() {
  int l = __lane_id();
  asm volatile("" : "+v"(l));
  return l;
}

template <int G>
__device__ __forceinline__ void pp2_issue(char* smem, const PP2Src& src, int wave, int kt,
                                          int stage) {
  const int lane = opaque_lane();    // rederive per issue: no hoisted 64-bit pointers
  const int prow = lane >> 3, pchunk = (lane & 7) ^ prow;
  char* dst = smem + stage * BSTAGE + G * 16384 + wave * 2 * 1024;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int tr = grp_tile_row(G, (wave * 2 + j) * 8 + prow);
    const char* g;
    if constexpr (G < 2)
      g = reinterpret_cast<const char*>(src.A + (int64_t)min(src.m0 + tr, src.mlast) * src.lda +
                                        kt * 64) + pchunk * 16;
    else
      g = reinterpret_cast<const char*>(src.Bt + (int64_t)min(src.n0 + tr, src.nlast) * src.ldb +
                                        kt * 64) + pchunk * 16;
    glds16(g, dst + j * 1024);
  }
}

// Buffer-resource DMA source (variant 8): one SRD per operand based at the tile's first
// row; the 8 per-lane row offsets (clamped row * ld + swizzled chunk, bytes) are computed
// once, and the K offset goes in the instruction's SGPR soffset, so an issue is
// s_mov m0 + buffer_load_dwordx4 ... lds with no VALU address arithmetic.
struct PP2BufSrc {
  __amdgpu_buffer_rsrc_t ra, rb;
  int off[4][2];
};

template <bool TR>
__device__ __forceinline__ void pp2b_sources(PP2BufSrc& s, const bf16_t* A, int lda, int M,
                                             const bf16_t* Bt, int ldb, int N, int m0, int n0,
                                             int wave, int lane, int k0 = 0) {
  // records = bytes from the tile base to the end of the operand (clamped to 32 bits); all
  // offsets are in range because rows are clamped to the last valid row.  k0: first K
  // element of the loop (stream-K segments), folded into the base.
  const int64_t ra_bytes = (int64_t)(M - m0) * lda * 2 - 2 * k0,
                rb_bytes = (int64_t)(N - n0) * ldb * 2 - 2 * k0;
  s.ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(A + (int64_t)m0 * lda + k0), 0,
                                           (int)std::min<int64_t>(ra_bytes, 0x7fffffff), 0x00020000);
  s.rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(Bt + (int64_t)n0 * ldb + k0), 0,
                                           (int)std::min<int64_t>(rb_bytes, 0x7fffffff), 0x00020000);
  const int prow = lane >> 3, pchunk = (lane & 7) ^ prow;
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int tr = grp_tile_row(g, (wave * 2 + j) * 8 + prow);
      // transposed variant: B groups use swz_t (group row bit 4 = wave & 1 flips chunk bit 2)
      const int bchunk = TR ? pchunk ^ ((wave & 1) << 2) : pchunk;
      s.off[g][j] = g < 2 ? min(tr, M - 1 - m0) * lda * 2 + pchunk * 16
                          : min(tr, N - 1 - n0) * ldb * 2 + bchunk * 16;
    }
}

// cache policy of the operand DMA (buffer aux bits: 1 sc0, 2 nt, 16 sc1); build-time A/B knob
#ifndef VTD_A_LOAD_AUX
#define VTD_A_LOAD_AUX 0
#endif
#ifndef VTD_B_LOAD_AUX
#define VTD_B_LOAD_AUX 0
#endif
template <int G>
__device__ __forceinline__ void pp2_issue(char* smem, const PP2BufSrc& src, int wave, int kt,
                                          int stage) {
  char* dst = smem + stage * BSTAGE + G * 16384 + wave * 2 * 1024;
#pragma unroll
  for (int j = 0; j < 2; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(G < 2 ? src.ra : src.rb,
                                             (lds_void_t*)(dst + j * 1024), 16, src.off[G][j],
                                             kt * 128, 0, G < 2 ? VTD_A_LOAD_AUX : VTD_B_LOAD_AUX);
}

// DG (timing diagnostics only, wrong outputs): bit 0 = P0 skips its B reads (stale b0),
// bit 1 = no DMA after the prologue, bit 2 = no LDS reads after the first K-tile,
// bit 3 = every DMA re-fetches K-tile 0 (L2-resident source, same instruction count),
// bit 4 = (schedule, correct) Y0(t+2) issued in P2 with X0(t+2) instead of in P3,
// bit 7 = the steady-state counted waits leave 8 more DMA instructions in flight (reads may
// see unlanded data: a latency probe)
template <bool TR, class Src, int DG = 0>
__device__ __forceinline__ void pp2_mainloop(f32x4 (&acc)[8][4], char* smem, const Src& src,
                                             int nk, int wave, int wm, int wn, int fr, int fg) {
  // prologue: tile 0 complete, tile 1's X0/Y0/Y1 in flight
  pp2_issue<0>(smem, src, wave, 0, 0);
  pp2_issue<2>(smem, src, wave, 0, 0);
  pp2_issue<3>(smem, src, wave, 0, 0);
  pp2_issue<1>(smem, src, wave, 0, 0);
  if (nk > 1) {
    pp2_issue<0>(smem, src, wave, 1, 1);
    pp2_issue<2>(smem, src, wave, 1, 1);
    pp2_issue<3>(smem, src, wave, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  pp_barrier();
  if (wm == 1) pp_barrier();                 // stagger G1 by one barrier
  const int ra = wm * 64, rb = wn * 32;      // group rows of this wave's quads
  bf16x8 a[4][2], b0[2][2], b1[2][2];
  if constexpr (DG != 0) {
    pp_load_a(a, smem, ra, fr, fg);
    pp_load_b(b0, smem + 2 * 16384, rb, fr, fg);
    pp_load_b(b1, smem + 3 * 16384, rb, fr, fg);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const char* st = smem + (kt & 1) * BSTAGE;
    const bool n1 = kt + 1 < nk && !(DG & 2), n2 = kt + 2 < nk && !(DG & 2);
    constexpr bool RD = !(DG & 4);
    // ---- P0
    if (RD) pp_load_a(a, st + 0 * 16384, ra, fr, fg);
    if constexpr (TR) { if (RD && !(DG & 1)) pp_load_b_t(b0, st + 2 * 16384, rb, fr, fg); }
    else if (RD && !(DG & 1)) pp_load_b(b0, st + 2 * 16384, rb, fr, fg);
    if (n1) pp2_issue<1>(smem, src, wave, (DG & 8) ? 0 : kt + 1, (kt + 1) & 1);
    if (n1) {
      if constexpr ((DG & 128) != 0) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pp_barrier();
    if constexpr (TR) pp_mfma_t<0, 0>(acc, a, b0);
    else pp_mfma<0, 0>(acc, a, b0);
    pp_barrier();
    // ---- P1
    if constexpr (TR) { if (RD) pp_load_b_t(b1, st + 3 * 16384, rb, fr, fg); }
    else if (RD) pp_load_b(b1, st + 3 * 16384, rb, fr, fg);
    if (n1) {
      if constexpr ((DG & 128) != 0) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pp_barrier();
    if constexpr (TR) pp_mfma_t<0, 2>(acc, a, b1);
    else pp_mfma<0, 2>(acc, a, b1);
    pp_barrier();
    // ---- P2
    if (RD) pp_load_a(a, st + 1 * 16384, ra, fr, fg);
    if (n2) pp2_issue<0>(smem, src, wave, (DG & 8) ? 0 : kt + 2, kt & 1);
    if constexpr ((DG & 16) != 0) {
      if (n2) pp2_issue<2>(smem, src, wave, (DG & 8) ? 0 : kt + 2, kt & 1);
    }

    pp_barrier();
    if constexpr (TR) pp_mfma_t<4, 2>(acc, a, b1);
    else pp_mfma<4, 2>(acc, a, b1);
    pp_barrier();
    // ---- P3
    if (n2) {
      if constexpr ((DG & 16) == 0)
        pp2_issue<2>(smem, src, wave, (DG & 8) ? 0 : kt + 2, kt & 1);
      pp2_issue<3>(smem, src, wave, (DG & 8) ? 0 : kt + 2, kt & 1);
      if constexpr ((DG & 128) != 0) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pp_barrier();
    if constexpr (TR) pp_mfma_t<4, 0>(acc, a, b0);
    else pp_mfma<4, 0>(acc, a, b0);
    pp_barrier();
  }
  if (wm == 0) pp_barrier();                 // re-align
}

// Epilogue of the transposed variant, full tiles: lane (fr, fg) of wave (wm, wn) holds,
// for accumulator row block i and column half jp, output row m_base + 16 i + fr and the 8
// contiguous columns n_base + 32 jp + 8 fg + 0..7 (acc[i][2 jp] = first 4, acc[i][2 jp + 1]
// = last 4).  Bias is loaded once; residual rows are fetched 4 row blocks at a time.
template <int EPI>
__device__ __forceinline__ void epilogue_direct(const f32x4 (&acc)[8][4], int lane, int m_base,
                                                int n_base, const EpiArgs& e,
                                                const float2* lst = nullptr) {
  constexpr int ACT = EPI & 3;
  constexpr bool OUT_BF16 = (EPI & 4) != 0;
  constexpr bool RESID = (EPI & 8) != 0;
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 bias[2][2], cs[2][2] = {};
#pragma unroll
  for (int jp = 0; jp < 2; ++jp)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bias[jp][h] = *reinterpret_cast<const f32x4*>(e.bias + n_base + 32 * jp + 8 * fg + 4 * h);
      if (e.lnstat)
        cs[jp][h] = *reinterpret_cast<const f32x4*>(e.colsum + n_base + 32 * jp + 8 * fg + 4 * h);
    }
#pragma unroll
  for (int i0 = 0; i0 < 8; i0 += 4) {
    f32x4 rv[4][2][2];
    if constexpr (RESID) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          load_resid8<OUT_BF16>(e, (int64_t)(m_base + 16 * (i0 + i) + fr) * e.ldr + n_base +
                                       32 * jp + 8 * fg, rv[i][jp][0], rv[i][jp][1]);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float tsum = 0.f;
      i32x4 ob[2];                     // the stored bf16 values (statistics pass below)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        f32x4 v0 = acc[i0 + i][2 * jp];
        f32x4 v1 = acc[i0 + i][2 * jp + 1];
        const int mrow = m_base + 16 * (i0 + i) + fr, ncol = n_base + 32 * jp + 8 * fg;
        if (e.lnstat)
          epi_lnfold8(e, lst, mrow, 16 * (i0 + i) + fr, cs[jp][0], cs[jp][1], v0, v1);
        v0 += bias[jp][0];
        v1 += bias[jp][1];
        if (e.rowadd) epi_rowadd8(e, mrow, ncol, v0, v1);
        act_ct8<ACT>(v0, v1);
        if constexpr (RESID) {
          v0 += rv[i][jp][0];
          v1 += rv[i][jp][1];
        }
        if (e.out2) epi_out2_8(e, mrow, ncol, v0, v1);
        const int64_t idx = (int64_t)mrow * e.ldo + ncol;
        if constexpr (OUT_BF16) {
          const i32x4 o = {(int)pack_bf16x2(v0[0], v0[1]), (int)pack_bf16x2(v0[2], v0[3]),
                           (int)pack_bf16x2(v1[0], v1[1]), (int)pack_bf16x2(v1[2], v1[3])};
          store_out16(static_cast<bf16_t*>(e.out) + idx, o);
          if (e.statout) {
            ob[jp] = o;
            tsum += bf16x8_sum(o);
          }
        } else {
          float* op = static_cast<float*>(e.out) + idx;
          *reinterpret_cast<f32x4*>(op) = v0;
          *reinterpret_cast<f32x4*>(op + 4) = v1;
        }
      }
      if (OUT_BF16 && e.statout) {   // the row's 64 columns: lanes fr, fr + 16, + 32, + 48
        // block mean (lane-swap butterfly: every lane holds it), then the centred sum of
        // squares of the same stored values
        const float mean = xsum32(xsum16(tsum)) * (1.f / 64.f);
        const float m2 = xsum32(xsum16(bf16x8_m2(ob[0], mean) + bf16x8_m2(ob[1], mean)));
        if (fg == 0)
          e.statout[(int64_t)(m_base + 16 * (i0 + i) + fr) * e.stat_ld + (n_base >> 6)] =
              float2{mean, m2};
      }
    }
  }
}

// Transposed variant, partial tiles and the runtime-flag modes: 32-row passes staged
// through the wave's LDS region (a lane's 4 values are 4 contiguous columns: one 16-B
// LDS store each), then the shared LDS -> global pass (bounds, rowadd, scatter, out2).
// Staging keeps the accumulators in registers (32 inlined epi_store4 calls on registers
// would not).
__device__ __forceinline__ void epilogue_direct_generic(const f32x4 (&acc)[8][4], float* ep,
                                                        int lane, int M, int N, int m_base,
                                                        int n_base, const EpiArgs& e) {
  constexpr int ES = 68;
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        *reinterpret_cast<f32x4*>(ep + (i * 16 + fr) * ES + 32 * (jj >> 1) + 8 * fg +
                                  4 * (jj & 1)) = acc[p * 2 + i][jj];
    epilogue_generic_pass<32>(ep, lane, M, N, m_base + p * 32, n_base, e);
  }
}

template <int EPI, bool BUF = false, bool TR = false, int DG = 0>
__global__ __launch_bounds__(BNT) void gemm_tn_bf16_pp2_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda,
    const bf16_t* __restrict__ Bt, int ldb, int tiles_m, int tiles_n, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int tm, tn;
  tile_coords(tile, tiles_m, tiles_n, e.ngw, tm, tn);
  const int m0 = tm * BBM, n0 = tn * BBN;
  using Src = std::conditional_t<BUF, PP2BufSrc, PP2Src>;
  Src src;
  if constexpr (BUF)
    pp2b_sources<TR>(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane);
  else
    pp2_sources(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane);
  // LayerNorm-fold row statistics of the wave's 128 rows: issued before the K loop (the
  // oldest vector-memory op, so the loop's counted waits retire it), used in the epilogue
  float2 lst[2] = {float2{0.f, 0.f}, float2{0.f, 0.f}};
  if (e.lnpart) {
    // fused finalize: the tile's 256 rows of partials (contiguous, 16 B per lane) go to LDS
    // past the two stages by DMA, issued before the prologue's DMAs (its counted wait
    // retires them); merged after the K loop
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(e.lnpart + (int64_t)m0 * e.lnslots), 0,
        (M - m0) * e.lnslots * 8, 0x00020000);
    for (int c = wave; c < 2 * e.lnslots; c += 8)   // 256 rows x slots x 8 B / 1 KiB
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rp, (lds_void_t*)(smem + 2 * BSTAGE + c * 1024), 16,
                                               c * 1024 + lane * 16, 0, 0, 0);
  } else if (e.lnstat) {
    lst[0] = e.lnstat[min(m0 + wm * 128 + lane, M - 1)];
    lst[1] = e.lnstat[min(m0 + wm * 128 + 64 + lane, M - 1)];
  }
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  pp2_mainloop<TR, Src, DG>(acc, smem, src, K / 64, wave, wm, wn, fr, fg);
  const int m_base = m0 + wm * 128, n_base = n0 + wn * 64;
  if (e.lnpart) {
    // the arithmetic of ln_stats_finalize_kernel, row by row (the loop's barriers made every
    // wave's DMA visible)
    const int S = e.lnslots;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const float2* pr =
          reinterpret_cast<const float2*>(smem + 2 * BSTAGE) + (wm * 128 + hh * 64 + lane) * S;
      const float mb = pr[0].x;
      float ds = 0.f, qq = 0.f;
      for (int b = 0; b < S; ++b) {
        const float2 t = pr[b];
        ds += t.x - mb;
        qq += t.y;
      }
      const float dmean = ds / S;
      float between = 0.f;
      for (int b = 0; b < S; ++b) {
        const float dv = (pr[b].x - mb) - dmean;
        between += dv * dv;
      }
      const float var = (qq + 64.f * between) / e.lnD;
      lst[hh] = float2{mb + dmean, 1.f / sqrtf(var + e.lneps)};
    }
  }
  if constexpr (TR) {
    if constexpr (EPI != EPI_GENERIC) {
      if (m0 + BBM <= M && n0 + BBN <= N) {
        epilogue_direct<EPI>(acc, lane, m_base, n_base, e, lst);
        return;
      }
    }
    epilogue_direct_generic(acc, reinterpret_cast<float*>(smem) + wave * 32 * 68, lane, M, N,
                            m_base, n_base, e);
    return;
  }
  float* ep = reinterpret_cast<float*>(smem) + wave * 32 * 68;
  if constexpr (EPI != EPI_GENERIC) {
    if (m0 + BBM <= M && n0 + BBN <= N) {
      epilogue_fast<EPI>(acc, ep, lane, m_base, n_base, e, lst);
      return;
    }
  }
  epilogue_generic(acc, ep, lane, M, N, m_base, n_base, e);
}

// ---------------------------------------------------------------------------------
// Stream-K pp2 ("pp2sk"): the pp2 tile, main loop and epilogues in a persistent grid of G
// workgroups (G = CUs, a multiple of 8) that balances the last tiles over every CU instead
// of leaving a partial final round (an N = 768 layer at C2 B = 256 is 588 tiles = 2.3
// rounds of 256 CUs: a third of its time runs on 76 CUs).
//   data-parallel part: tiles [0, dp_tiles), dp_tiles a multiple of G; workgroup b on XCD
//     x = b % 8 (hardware round-robin, tools/probes/xcc_probe.hip) takes tile
//     i G + x G/8 + b/8 in round i, so an XCD walks contiguous tiles (shared A panels);
//   stream-K part: tiles [dp_tiles, T) are dealt to the XCDs as contiguous whole-tile
//     blocks, and each XCD's block of K-steps is cut evenly over its G/8 workgroups.  A
//     workgroup's range covers one or more (partial) tiles; a tile split between workgroups
//     gets each contributor's fp32 accumulators in a private slot (slot 0 for a range's first
//     tile, 1 for its last), and the contributor that arrives last (per-tile counter, vector
//     atomic, no waiting anywhere: no co-residency assumption) sums the slots in K order --
//     the same order whoever arrives last, so results are deterministic -- and runs the
//     epilogue.  All contributors of a tile share the XCD's L2 and every slot is written at
//     most once per launch, so workgroup-scope release / acquire fences order the slots
//     and the counter.
struct SkArgs {
  int dp_tiles;
  float* partial;     // [G][2][512 threads][32] float4
  int* counters;      // [T], zero between launches (the last arriver resets its tile's)
};

template <int EPI, bool TR>
__device__ __forceinline__ void pp2_tile_epilogue(const f32x4 (&acc)[8][4], char* smem, int lane,
                                                  int wave, int M, int N, int m0, int n0,
                                                  int m_base, int n_base, const EpiArgs& e,
                                                  const float2* lst) {
  if constexpr (TR) {
    if constexpr (EPI != EPI_GENERIC) {
      if (m0 + BBM <= M && n0 + BBN <= N) {
        epilogue_direct<EPI>(acc, lane, m_base, n_base, e, lst);
        return;
      }
    }
    epilogue_direct_generic(acc, reinterpret_cast<float*>(smem) + wave * 32 * 68, lane, M, N,
                            m_base, n_base, e);
  } else {
    float* ep = reinterpret_cast<float*>(smem) + wave * 32 * 68;
    if constexpr (EPI != EPI_GENERIC) {
      if (m0 + BBM <= M && n0 + BBN <= N) {
        epilogue_fast<EPI>(acc, ep, lane, m_base, n_base, e, lst);
        return;
      }
    }
    epilogue_generic(acc, ep, lane, M, N, m_base, n_base, e);
  }
}

template <int EPI, bool TR>
__global__ __launch_bounds__(BNT) void gemm_tn_bf16_pp2sk_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda,
    const bf16_t* __restrict__ Bt, int ldb, int tiles_m, int tiles_n, EpiArgs e, SkArgs sk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_last;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  const int G = gridDim.x, GX = G >> 3;
  const int b = blockIdx.x, x = b & 7, j = b >> 3;
  const int T = tiles_m * tiles_n, nk = K / 64;
  // work items: the data-parallel tiles, then this workgroup's stream-K range
  const int ndp = sk.dp_tiles > x * GX + j ? (sk.dp_tiles - (x * GX + j) + G - 1) / G : 0;
  const int tsk = T - sk.dp_tiles;
  const int t_lo = sk.dp_tiles + (int)((int64_t)x * tsk / 8);
  const int t_hi = sk.dp_tiles + (int)((int64_t)(x + 1) * tsk / 8);
  const int S = (t_hi - t_lo) * nk;
  const int W = max(1, (S + GX - 1) / GX);
  const int s0 = min(j * W, S), s1 = min(s0 + W, S);
  int item = 0, st = s0;
#pragma unroll 1
  while (item < ndp || st < s1) {
    int t, k0, k1, tl = 0;
    if (item < ndp) {
      t = x * GX + j + item * G;
      k0 = 0;
      k1 = nk;
      ++item;
    } else {
      tl = st / nk;
      t = t_lo + tl;
      k0 = st - tl * nk;
      k1 = min(nk, s1 - tl * nk);
      st = tl * nk + k1;
    }
    const int tm = t / tiles_n, tn = t - tm * tiles_n;
    const int m0 = tm * BBM, n0 = tn * BBN;
    PP2BufSrc src;
    pp2b_sources<TR>(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane, k0 * 64);
    float2 lst[2] = {float2{0.f, 0.f}, float2{0.f, 0.f}};
    if (e.lnstat) {
      lst[0] = e.lnstat[min(m0 + wm * 128 + lane, M - 1)];
      lst[1] = e.lnstat[min(m0 + wm * 128 + 64 + lane, M - 1)];
    }
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[i][q] = f32x4{0.f, 0.f, 0.f, 0.f};
    pp2_mainloop<TR, PP2BufSrc, 0>(acc, smem, src, k1 - k0, wave, wm, wn, fr, fg);
    if (k0 != 0 || k1 != nk) {
      // a split tile: contributors are this XCD's workgroup slots jf..jl (K order)
      const int jf = (tl * nk) / W, jl = (tl * nk + nk - 1) / W;
      const int slot = (s0 / nk == tl) ? 0 : 1;
      float4* mine = reinterpret_cast<float4*>(sk.partial) + ((int64_t)(b * 2 + slot) * BNT) * 32;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          mine[(i * 4 + q) * BNT + tid] =
              float4{acc[i][q][0], acc[i][q][1], acc[i][q][2], acc[i][q][3]};
      // stores acknowledged by the XCD's L2 (L1 is write-through) before the count: every
      // contributor of a tile runs on this XCD and shares that L2, so workgroup-scope
      // ordering suffices (an agent-scope release would write back the whole L2)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __syncthreads();
      if (tid == 0) {
        const int old = __hip_atomic_fetch_add(sk.counters + t, 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == jl - jf;
      }
      __syncthreads();
      if (!s_last) continue;
      // each slot is written at most once per launch (a range's first / last split tile),
      // so no L1 line of it can be stale here: a workgroup-scope acquire orders the loads
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (tid == 0) sk.counters[t] = 0;     // ready for the next launch
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
      for (int jj = jf; jj <= jl; ++jj) {     // the same order whoever arrives last
        const int cslot = ((jj * W) / nk == tl) ? 0 : 1;
        const float4* p = reinterpret_cast<const float4*>(sk.partial) +
                          ((int64_t)((jj * 8 + x) * 2 + cslot) * BNT) * 32;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 v = p[(i * 4 + q) * BNT + tid];
            acc[i][q] += f32x4{v.x, v.y, v.z, v.w};
          }
      }
    }
    pp2_tile_epilogue<EPI, TR>(acc, smem, lane, wave, M, N, m0, n0, m0 + wm * 128,
                               n0 + wn * 64, e, lst);
    __syncthreads();                // the epilogue's LDS staging before the next prologue
  }
}

// ---------------------------------------------------------------------------------
// Persistent pp2 ("pp2p"): LDS = stage 0 | stage 1 | 32 KiB epilogue region (160 KiB).
// Per tile: K loop -> DMA of the NEXT tile's prologue (K-tiles 0 and 1) -> this tile's
// epilogue through the private region -> next K loop.  The epilogue's S global stores
// are younger than the next prologue's DMA, so the next loop's first waits add S to
// their counts (vmcnt counts in issue order) and the stores drain under the first
// ~1.5 K-tiles of compute instead of stalling the CU.
// Epilogue region: per wave 16 rows x 64 floats (4 KiB), column XOR-swizzled by
// ((row >> 2) & 3) << 4 so the accumulator writes of lanes 4 rows apart use different
// bank halves; the 16-B row-vector reads keep 4 contiguous floats.
constexpr int EPR_BYTES = 8 * 16 * 64 * 4;   // 32 KiB
static_assert(2 * BSTAGE + EPR_BYTES <= 163840, "LDS budget");

__device__ __forceinline__ int epx(int row, int col) {     // float index in a wave region
  return row * 64 + (col ^ (((row >> 2) & 3) << 4));
}

template <int EPI>
__device__ __forceinline__ void epilogue_fast_x(const f32x4 (&acc)[8][4], float* ep, int lane,
                                                int m_base, int n_base, const EpiArgs& e) {
  constexpr int ACT = EPI & 3;
  constexpr bool OUT_BF16 = (EPI & 4) != 0;
  constexpr bool RESID = (EPI & 8) != 0;
  const int fr = lane & 15, fg = lane >> 4;
  const int c8 = (lane & 7) * 8, rsub = lane >> 3;
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(e.bias + n_base + c8);
  const f32x4 b1 = *reinterpret_cast<const f32x4*>(e.bias + n_base + c8 + 4);
#pragma unroll
  for (int p = 0; p < 8; ++p) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r2 = 0; r2 < 4; ++r2) ep[epx(fg * 4 + r2, j * 16 + fr)] = acc[p][j][r2];
    f32x4 rv[2][2];
    if constexpr (RESID) {
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        load_resid8<OUT_BF16>(e, (int64_t)(m_base + p * 16 + it * 8 + rsub) * e.ldr + n_base + c8,
                              rv[it][0], rv[it][1]);
      }
    }
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int row = it * 8 + rsub;
      f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + epx(row, c8)) + b0;
      f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + epx(row, c8 + 4)) + b1;
      act_ct8<ACT>(v0, v1);
      if constexpr (RESID) {
        v0 += rv[it][0];
        v1 += rv[it][1];
      }
      const int64_t idx = (int64_t)(m_base + p * 16 + row) * e.ldo + n_base + c8;
      if constexpr (OUT_BF16) {
        const i32x4 o = {(int)pack_bf16x2(v0[0], v0[1]), (int)pack_bf16x2(v0[2], v0[3]),
                         (int)pack_bf16x2(v1[0], v1[1]), (int)pack_bf16x2(v1[2], v1[3])};
        store_out16(static_cast<bf16_t*>(e.out) + idx, o);
      } else {
        float* op = static_cast<float*>(e.out) + idx;
        *reinterpret_cast<f32x4*>(op) = v0;
        *reinterpret_cast<f32x4*>(op + 4) = v1;
      }
    }
  }
}

__device__ __forceinline__ void epilogue_generic_x(const f32x4 (&acc)[8][4], float* ep, int lane,
                                                   int M, int N, int m_base, int n_base,
                                                   const EpiArgs& e) {
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r2 = 0; r2 < 4; ++r2) ep[epx(fg * 4 + r2, j * 16 + fr)] = acc[p][j][r2];
#pragma unroll 1
    for (int it = 0; it < 4; ++it) {
      const int row = it * 4 + (lane >> 4), col = (lane & 15) * 4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(ep + epx(row, col));
      epi_store4(e, M, N, m_base + p * 16 + row, n_base + col, v);
    }
  }
}

#define VTD_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

// K loop of pp2 without its prologue (K-tile 0 landed + barrier passed, K-tile 1's
// X0/Y0/Y1 in flight).  kPost: S fast-epilogue stores sit between the prologue DMA and
// this loop's DMA (see the comment above pp2p); waits that cover them add S.
// Fragment loads that rederive their LDS addresses from an opaque copy of the lane id:
// the compiler cannot hoist the 12 swizzled base addresses across the K loop, so they
// do not compete with the accumulators for registers (a spill + reload there would add
// a vmcnt(0) that drains the DMA and epilogue-store pipeline).
__device__ __forceinline__ void pp_load_a_o(bf16x8 (&a)[4][2], const char* la, int row0) {
  const int l = opaque_lane();
  pp_load_a(a, la, row0, l & 15, l >> 4);
}
__device__ __forceinline__ void pp_load_b_o(bf16x8 (&b)[2][2], const char* lb, int row0) {
  const int l = opaque_lane();
  pp_load_b(b, lb, row0, l & 15, l >> 4);
}

template <int S>
__device__ __forceinline__ void pp2_loop(f32x4 (&acc)[8][4], char* smem, const PP2Src& src,
                                         int nk, int wave, int wm, int wn, int fr, int fg,
                                         bool post) {
  if (wm == 1) pp_barrier();
  const int ra = wm * 64, rb = wn * 32;
  bf16x8 a[4][2], b0[2][2], b1[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    const char* st = smem + (kt & 1) * BSTAGE;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    const bool p0 = post && kt == 0, p01 = post && kt <= 1;
    pp_load_a_o(a, st + 0 * 16384, ra);
    pp_load_b_o(b0, st + 2 * 16384, rb);
    if (n1) pp2_issue<1>(smem, src, wave, kt + 1, (kt + 1) & 1);
    if (!n1) VTD_VMCNT(0);
    else if (p01) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(10 + S) : "memory");
    else VTD_VMCNT(10);
    pp_barrier();
    pp_mfma<0, 0>(acc, a, b0);
    pp_barrier();
    pp_load_b_o(b1, st + 3 * 16384, rb);
    if (!n1) VTD_VMCNT(0);
    else if (p0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + S) : "memory");
    else VTD_VMCNT(8);
    pp_barrier();
    pp_mfma<0, 2>(acc, a, b1);
    pp_barrier();
    pp_load_a_o(a, st + 1 * 16384, ra);
    if (n2) pp2_issue<0>(smem, src, wave, kt + 2, kt & 1);
    pp_barrier();
    pp_mfma<4, 2>(acc, a, b1);
    pp_barrier();
    if (n2) {
      pp2_issue<2>(smem, src, wave, kt + 2, kt & 1);
      pp2_issue<3>(smem, src, wave, kt + 2, kt & 1);
      if (p0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(10 + S) : "memory");
      else VTD_VMCNT(10);
    } else {
      VTD_VMCNT(0);
    }
    pp_barrier();
    pp_mfma<4, 0>(acc, a, b0);
    pp_barrier();
  }
  if (wm == 0) pp_barrier();
}

template <int EPI>
__global__ __launch_bounds__(BNT) void gemm_tn_bf16_pp2p_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda,
    const bf16_t* __restrict__ Bt, int ldb, int tiles_m, int tiles_n, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int S = EPI < 0 ? 0 : epilogue_fast_stores<(EPI < 0 ? 0 : EPI), 16>();
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  const int nk = K / 64;
  const int nwg = tiles_m * tiles_n;
  const int q = nwg >> 3, r = nwg & 7;
  float* ep = reinterpret_cast<float*>(smem + 2 * BSTAGE) + wave * 16 * 64;
  int t = blockIdx.x;
  if (t >= nwg) return;
  auto origin = [&](int tt, int& m0, int& n0) {
    const int x = tt & 7;
    const int tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (tt >> 3);
    const int tm = tile / tiles_n;
    m0 = tm * BBM;
    n0 = (tile - tm * tiles_n) * BBN;
  };
  auto prologue = [&](const PP2Src& src) {
    pp2_issue<0>(smem, src, wave, 0, 0);
    pp2_issue<2>(smem, src, wave, 0, 0);
    pp2_issue<3>(smem, src, wave, 0, 0);
    pp2_issue<1>(smem, src, wave, 0, 0);
    if (nk > 1) {
      pp2_issue<0>(smem, src, wave, 1, 1);
      pp2_issue<2>(smem, src, wave, 1, 1);
      pp2_issue<3>(smem, src, wave, 1, 1);
    }
  };
  int m0, n0;
  origin(t, m0, n0);
  PP2Src src;
  pp2_sources(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane);
  prologue(src);
  bool post = false;
  for (;;) {
    if (nk > 1) {
      if (post) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 + S) : "memory");
      else VTD_VMCNT(6);
    } else {
      if (post) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S) : "memory");
      else VTD_VMCNT(0);
    }
    pp_barrier();
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    pp2_loop<S>(acc, smem, src, nk, wave, wm, wn, fr, fg, post);
    const int m_base = m0 + wm * 128, n_base = n0 + wn * 64;
    const bool full = m0 + BBM <= M && n0 + BBN <= N;
    const int tn = t + gridDim.x;
    if (tn < nwg) {                          // next tile's prologue before this epilogue
      origin(tn, m0, n0);
      pp2_sources(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane);
      prologue(src);
    }
    if (EPI != EPI_GENERIC && full) {
      epilogue_fast_x<(EPI < 0 ? 0 : EPI)>(acc, ep, lane, m_base, n_base, e);
      post = true;
    } else {
      epilogue_generic_x(acc, ep, lane, M, N, m_base, n_base, e);
      post = false;
    }
    if (tn >= nwg) break;
    t = tn;
  }
}

template <int EPI, bool kDiagSkipEpilogue>
__global__ __launch_bounds__(BNT) void gemm_tn_bf16_pingpong_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda,
    const bf16_t* __restrict__ Bt, int ldb, int tiles_m, int tiles_n, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = tile / tiles_n, tn = tile - (tile / tiles_n) * tiles_n;
  const int m0 = tm * BBM, n0 = tn * BBN;

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
  const int lds_piece = wave * 32 * KB;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  const int nk = K / 64;
  const int arow = wm * 128, brow = wn * 64;

  // prologue: tile 0 -> stage 0, visible to all waves
  issue_tile(smem, srcA, srcB, lds_piece, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_barrier();
  pp_mainloop(acc, smem, srcA, srcB, lds_piece, nk, wm, arow, brow, fr, fg);

  if constexpr (kDiagSkipEpilogue && EPI >= 0) {   // diag (VTD_GEMM_VARIANT=3): no stores
    epilogue_fast<EPI, true>(acc, reinterpret_cast<float*>(smem) + wave * 32 * 68, lane,
                             m0 + wm * 128, n0 + wn * 64, e);
    return;
  }
  if constexpr (kDiagSkipEpilogue) {         // timing diagnostic only (VTD_GEMM_VARIANT=2)
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (s != s) static_cast<float*>(e.out)[tid] = s;
    return;
  }
  float* ep = reinterpret_cast<float*>(smem) + wave * 32 * 68;
  const int m_base = m0 + wm * 128, n_base = n0 + wn * 64;
  if constexpr (EPI != EPI_GENERIC) {
    if (m0 + BBM <= M && n0 + BBN <= N) {
      epilogue_fast<EPI>(acc, ep, lane, m_base, n_base, e);
      return;
    }
  }
  epilogue_generic(acc, ep, lane, M, N, m_base, n_base, e);
}


// ============================================================================
// Persistent variant of the ping-pong kernel: gridDim.x blocks (one per CU) walk the
// tiles t = blockIdx.x, +gridDim.x, ...  After a tile's K loop the block issues the DMA
// of the NEXT tile's K-tile 0 into stage 0, then runs this tile's epilogue staged in
// stage 1 (16-row passes, 34.8 KiB) and continues without draining its stores: the
// next tile's first wait is vmcnt(#epilogue stores) (those are younger than the DMA), so
// the stores drain while the next tile's first K-tile is computed.
// ============================================================================
template <int EPI>
__global__ __launch_bounds__(BNT) void gemm_tn_bf16_persistent_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda,
    const bf16_t* __restrict__ Bt, int ldb, int tiles_m, int tiles_n, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  const int nk = K / 64;
  const int arow = wm * 128, brow = wn * 64;
  const int nwg = tiles_m * tiles_n;
  const int q = nwg >> 3, r = nwg & 7;
  const int prow = lane >> 3;
  const int pchunk = (lane & 7) ^ prow;
  const int lds_piece = wave * 32 * KB;
  float* ep = reinterpret_cast<float*>(smem + BSTAGE) + wave * 16 * 68;
  constexpr int PR = 16;

  auto tile_origin = [&](int t, int& m0, int& n0) {
    const int x = t & 7;
    const int tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (t >> 3);
    const int tm = tile / tiles_n;
    m0 = tm * BBM;
    n0 = (tile - tm * tiles_n) * BBN;
  };
  auto sources = [&](int m0, int n0, const char* (&sa)[4], const char* (&sb)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wave * 32 + j * 8 + prow;
      sa[j] = reinterpret_cast<const char*>(A + (int64_t)min(m0 + row, M - 1) * lda) + pchunk * 16;
      sb[j] = reinterpret_cast<const char*>(Bt + (int64_t)min(n0 + row, N - 1) * ldb) + pchunk * 16;
    }
  };

  int t = blockIdx.x;
  if (t >= nwg) return;
  int m0, n0;
  tile_origin(t, m0, n0);
  const char* srcA[4];
  const char* srcB[4];
  sources(m0, n0, srcA, srcB);
  issue_tile(smem, srcA, srcB, lds_piece, 0, 0);
  int pending_stores = 0;                    // epilogue stores younger than the DMA
  for (;;) {
    if (pending_stores == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(epilogue_fast_stores<(EPI < 0 ? 0 : EPI), 16>()) : "memory");
    pp_barrier();
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    pp_mainloop(acc, smem, srcA, srcB, lds_piece, nk, wm, arow, brow, fr, fg);

    const int m_base = m0 + wm * 128, n_base = n0 + wn * 64;
    const bool full = m0 + BBM <= M && n0 + BBN <= N;
    const int tn = t + gridDim.x;
    const int cm0 = m0, cn0 = n0;
    if (tn < nwg) {                          // next tile's K-tile 0 -> stage 0 (free)
      tile_origin(tn, m0, n0);
      sources(m0, n0, srcA, srcB);
      issue_tile(smem, srcA, srcB, lds_piece, 0, 0);
    }
    (void)cm0; (void)cn0;
    if constexpr (EPI != EPI_GENERIC) {
      if (full) {
        epilogue_fast<EPI, false, PR>(acc, ep, lane, m_base, n_base, e);
        pending_stores = 1;
      } else {
        epilogue_generic<PR>(acc, ep, lane, M, N, m_base, n_base, e);
        pending_stores = 0;
      }
    } else {
      epilogue_generic<PR>(acc, ep, lane, M, N, m_base, n_base, e);
      pending_stores = 0;
    }
    if (tn >= nwg) break;
    t = tn;
    // every wave's staging reads of stage 1 are done before the next K loop DMAs into it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}



// ============================================================================
// MX-fp8 kernel (VTD_FP8 mode): A, Bt are OCP e4m3 bytes with one E8M0
// scale per 32 K-elements (vtd_mx8.hip layout s[k / 128][rows][4]); D += A Bt^T via
// v_mfma_scale_f32_16x16x128_f8f6f4 (block-scaled, twice the bf16 MFMA rate per clock).
// Tile 256 x 256, K-step 128 elements = 128 B per row, so the operand staging is the
// bf16 256 kernel's byte for byte (DMA 8 rows x 128 B per wave instruction); per stage
// 1 KiB of A scales and 1 KiB of B scales follow (each wave DMAs 128 B of each: lanes 0-7).
// Wave (wm, wn) computes 128 x 64 outputs = 8 x 4 blocks of 16 x 16.  Operand layout of
// the instruction (measured, tools/mx8_probe.py): lane group g = lane / 16 supplies
// K-elements [16 g, 16 g + 16) in its first 16 bytes and [64 + 16 g, 64 + 16 g + 16) in
// its last 16, and its scale byte covers the 32-block [32 g, 32 g + 32) of the
// instruction's K order.  So lane (fr, fg) reads 16-B chunks fg and fg + 4 of the row:
// the instruction's block g is then exactly the quantizer's block g of the K-step and
// the lane's scale is byte fg of the row's scale dword.  LDS chunk c of row r sits at
// position c ^ (r & 7) (the bf16 kernels' image): conflict-free for both reads of every
// ds_read_b128 lane group (exhaustive check in tools/swizzle_check.py).
// Two barriers per K-step (the structure of gemm_tn_bf16_256_kernel).
// ============================================================================
constexpr int MX_SCALES = (BBM + BBN) * KB;   // scale blocks after the A and B tiles
constexpr int MX_STAGE = MX_SCALES + 2048;     // 66 KiB per stage

__device__ __forceinline__ int mx_swz(int row) { return row & 7; }

__device__ __forceinline__ int mx_lds_scale(const char* p) {
  return *reinterpret_cast<const int*>(p);
}

template <int EPI>
__global__ __launch_bounds__(BNT) void gemm_mx8_kernel(
    int M, int N, int K, const uint8_t* __restrict__ A, int lda, const uint8_t* __restrict__ sA,
    int64_t sa_rows, const uint8_t* __restrict__ Bt, int ldb, const uint8_t* __restrict__ sB,
    int64_t sb_rows, int tiles_m, int tiles_n, EpiArgs e) {
  typedef __attribute__((ext_vector_type(8))) int i32x8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int tm, tn;
  tile_coords(tile, tiles_m, tiles_n, e.ngw, tm, tn);
  const int m0 = tm * BBM, n0 = tn * BBN;

  // operand DMA through buffer resources based at the tile's first row: wave fills tile
  // rows wave*32 + 8 j + (lane >> 3), position lane & 7; one per-lane offset, the piece
  // (j * 8 rows) and K-step in the scalar soffset; rows past M / N read as zero (range
  // check).  Scales: lanes 0-7 of wave w copy the dwords of tile rows 32 w + 4 lane .. + 3.
  const int prow = lane >> 3;
  const int pchunk = (lane & 7) ^ mx_swz(prow);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(A + (int64_t)m0 * lda), 0,
      (int)std::min<int64_t>((int64_t)(M - m0) * lda, 0x7fffffff), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(Bt + (int64_t)n0 * ldb), 0,
      (int)std::min<int64_t>((int64_t)(N - n0) * ldb, 0x7fffffff), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(sA), 0, (int)std::min<int64_t>(sa_rows * K / 32, 0x7fffffff), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(sB), 0, (int)std::min<int64_t>(sb_rows * K / 32, 0x7fffffff), 0x00020000);
  const int voa = (wave * 32 + prow) * lda + pchunk * 16;
  const int vob = (wave * 32 + prow) * ldb + pchunk * 16;
  const int vsa = (m0 + wave * 32 + 4 * (lane & 7)) * 4;
  const int vsb = (n0 + wave * 32 + 4 * (lane & 7)) * 4;
  const int lds_piece = wave * 32 * KB;
  auto issue = [&](int kt, int stage) {
    char* base = smem + stage * MX_STAGE;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)(base + lds_piece + j * 8 * KB), 16,
                                               voa, kt * KB + j * 8 * lda, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (lds_void_t*)(base + BBM * KB + lds_piece + j * 8 * KB), 16, vob,
          kt * KB + j * 8 * ldb, 0, 0);
    if (lane < 8) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_void_t*)(base + MX_SCALES + wave * 128),
                                               16, vsa, (int)(kt * sa_rows * 4), 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsb, (lds_void_t*)(base + MX_SCALES + 1024 + wave * 128), 16, vsb,
          (int)(kt * sb_rows * 4), 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  // fragment row offsets: chunk positions 2 fg, 2 fg + 1 under the row's swizzle
  const int sw = mx_swz(fr);
  const int off0 = (fg ^ sw) * 16, off1 = ((fg + 4) ^ sw) * 16;
  const char* pa0 = smem + (wm * 128 + fr) * KB + off0;
  const char* pa1 = smem + (wm * 128 + fr) * KB + off1;
  const char* pb0 = smem + BBM * KB + (wn * 64 + fr) * KB + off0;
  const char* pb1 = smem + BBM * KB + (wn * 64 + fr) * KB + off1;
  const char* psa = smem + MX_SCALES + (wm * 128 + fr) * 4;
  const char* psb = smem + MX_SCALES + 1024 + (wn * 64 + fr) * 4;
  const int nk = K / 128;
  issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // per-lane bases + immediate block offsets (16 rows = 2 KiB apart): no per-block
    // address registers
    const int so = (kt & 1) * MX_STAGE;
    i32x8 bfr[4];
    int sbv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const i32x4 lo = *reinterpret_cast<const i32x4*>(pb0 + so + j * 16 * KB);
      const i32x4 hi = *reinterpret_cast<const i32x4*>(pb1 + so + j * 16 * KB);
      bfr[j] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      sbv[j] = mx_lds_scale(psb + so + j * 64) >> (8 * fg);
    }
#pragma unroll
    for (int hs = 0; hs < 4; ++hs) {
      i32x8 afr[2];
      int sav[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int blk = 2 * hs + i;
        const i32x4 lo = *reinterpret_cast<const i32x4*>(pa0 + so + blk * 16 * KB);
        const i32x4 hi = *reinterpret_cast<const i32x4*>(pa1 + so + blk * 16 * KB);
        afr[i] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        sav[i] = mx_lds_scale(psa + so + blk * 64) >> (8 * fg);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[2 * hs + i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              afr[i], bfr[j], acc[2 * hs + i][j], 0, 0, 0, sav[i], 0, sbv[j]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + 2 < nk) issue(kt + 2, kt & 1);
  }

  float* ep = reinterpret_cast<float*>(smem) + wave * 32 * 68;
  const int m_base = m0 + wm * 128, n_base = n0 + wn * 64;
  if constexpr (EPI != EPI_GENERIC) {
    if (m0 + BBM <= M && n0 + BBN <= N) {
      epilogue_fast<EPI>(acc, ep, lane, m_base, n_base, e);
      return;
    }
  }
  epilogue_generic(acc, ep, lane, M, N, m_base, n_base, e);
}

// ---------------------------------------------------------------------------------
// Ping-pong MX-fp8 GEMM ("mxp"): pp2's K loop (four 16-KiB DMA groups per stage, the
// two wave groups offset by one barrier, counted vmcnt) on MX-fp8 operands.  A K-step of
// 128 fp8 elements is 128 B per row, the same LDS image as a bf16 K-step of 64: the DMA,
// the swizzle and the fragment reads are pp2's byte for byte, and a bf16 pair of
// fragments (chunks fg and fg + 4 of a row) IS the MX operand of
// v_mfma_scale_f32_16x16x128_f8f6f4 (lane group fg supplies K [16 fg, +16) and
// [64 + 16 fg, +16): tools/mx8_probe.py).  One MX MFMA replaces the two bf16 k-substeps at
// the same cycles, so a phase is 8 MFMAs of 32 cycles.
// Scales: per stage, 1 KiB of A scales (256 rows x 4 block bytes) rides with group X0 and
// 1 KiB of B scales with Y0 (lanes 0-7 of every wave, 128 B each: 3 DMA instructions in
// those groups, 2 in X1 / Y1); a wave reads all 8 A and 4 B scale dwords of the tile in
// P0, so X0(t+2) / Y0(t+2) overwrite them under the same WAR argument as their operands.
// Waits (youngest first, per tile: X1 2, X0 3, Y0 3, Y1 2): P0 vmcnt(12) -> Y0, Y1(t);
// P1 vmcnt(10) -> X1(t); P3 vmcnt(12) -> X0, Y0(t+1).
constexpr int MXP_STAGE = BSTAGE + 2048;      // 66 KiB

struct MxpSrc {
  __amdgpu_buffer_rsrc_t ra, rb, rsa, rsb;
  int off[4][2];
  int vsa, vsb, sa4, sb4;                    // scale voffsets, scale K-step strides (bytes)
};

template <int G>
__device__ __forceinline__ void mxp_issue(char* smem, const MxpSrc& src, int wave, int lane,
                                          int kt, int stage) {
  char* st = smem + stage * MXP_STAGE;
  char* dst = st + G * 16384 + wave * 2 * 1024;
#pragma unroll
  for (int j = 0; j < 2; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(G < 2 ? src.ra : src.rb,
                                             (lds_void_t*)(dst + j * 1024), 16, src.off[G][j],
                                             kt * 128, 0, 0);
  if constexpr (G == 0 || G == 2) {
    if (lane < 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          G == 0 ? src.rsa : src.rsb, (lds_void_t*)(st + BSTAGE + (G == 0 ? 0 : 1024) + wave * 128),
          16, G == 0 ? src.vsa : src.vsb, kt * (G == 0 ? src.sa4 : src.sb4), 0, 0);
  }
}

typedef __attribute__((ext_vector_type(8))) int i32x8_t;
__device__ __forceinline__ i32x8_t mx_operand(const bf16x8& lo, const bf16x8& hi) {
  return __builtin_shufflevector(__builtin_bit_cast(i32x4, lo), __builtin_bit_cast(i32x4, hi), 0,
                                 1, 2, 3, 4, 5, 6, 7);
}

template <int I0, int J0>
__device__ __forceinline__ void mxp_mfma(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2],
                                         const bf16x8 (&b)[2][2], const int (&sa)[8],
                                         const int (&sb)[4]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
          mx_operand(a[i][0], a[i][1]), mx_operand(b[j][0], b[j][1]), acc[I0 + i][J0 + j], 0, 0,
          0, sa[I0 + i], 0, sb[J0 + j]);
  // pin the cluster inside its phase: without these the compiler sinks every scaled MFMA
  // of the K-step past the phase barriers to the end of the loop body (no ping-pong left)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[I0 + i][J0 + j]));
  __builtin_amdgcn_s_setprio(0);
}

template <int EPI>
__global__ __launch_bounds__(BNT) void gemm_mx8_pp_kernel(
    int M, int N, int K, const uint8_t* __restrict__ A, int lda, const uint8_t* __restrict__ sA,
    int64_t sa_rows, const uint8_t* __restrict__ Bt, int ldb, const uint8_t* __restrict__ sB,
    int64_t sb_rows, int tiles_m, int tiles_n, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int tm, tn;
  tile_coords(tile, tiles_m, tiles_n, e.ngw, tm, tn);
  const int m0 = tm * BBM, n0 = tn * BBN;
  MxpSrc src;
  {
    const int64_t ra_bytes = (int64_t)(M - m0) * lda, rb_bytes = (int64_t)(N - n0) * ldb;
    src.ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(A + (int64_t)m0 * lda), 0,
                                               (int)std::min<int64_t>(ra_bytes, 0x7fffffff), 0x00020000);
    src.rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(Bt + (int64_t)n0 * ldb), 0,
                                               (int)std::min<int64_t>(rb_bytes, 0x7fffffff), 0x00020000);
    src.rsa = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sA), 0,
                                                (int)std::min<int64_t>(sa_rows * K / 32, 0x7fffffff), 0x00020000);
    src.rsb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sB), 0,
                                                (int)std::min<int64_t>(sb_rows * K / 32, 0x7fffffff), 0x00020000);
    const int prow = lane >> 3, pchunk = (lane & 7) ^ prow;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int tr = grp_tile_row(g, (wave * 2 + j) * 8 + prow);
        src.off[g][j] = g < 2 ? min(tr, M - 1 - m0) * lda + pchunk * 16
                              : min(tr, N - 1 - n0) * ldb + pchunk * 16;
      }
    // scales: lanes 0-7 of wave w copy the dwords of tile rows 32 w + 4 l .. + 3 (rows past
    // the end read beyond sa_rows / sb_rows fall outside the records: zero)
    src.vsa = (m0 + wave * 32 + 4 * (lane & 7)) * 4;
    src.vsb = (n0 + wave * 32 + 4 * (lane & 7)) * 4;
    src.sa4 = (int)(sa_rows * 4);
    src.sb4 = (int)(sb_rows * 4);
  }
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  const int nk = K / 128;
  // prologue: tile 0 complete, tile 1's X0 / Y0 / Y1 in flight
  mxp_issue<0>(smem, src, wave, lane, 0, 0);
  mxp_issue<2>(smem, src, wave, lane, 0, 0);
  mxp_issue<3>(smem, src, wave, lane, 0, 0);
  mxp_issue<1>(smem, src, wave, lane, 0, 0);
  if (nk > 1) {
    mxp_issue<0>(smem, src, wave, lane, 1, 1);
    mxp_issue<2>(smem, src, wave, lane, 1, 1);
    mxp_issue<3>(smem, src, wave, lane, 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  pp_barrier();
  if (wm == 1) pp_barrier();                 // stagger G1 by one barrier
  const int ra = wm * 64, rb = wn * 32;      // group rows of this wave's quads
  const int sa_row = wm * 128 + fr, sb_row = wn * 64 + fr;
  bf16x8 a[4][2], b0[2][2], b1[2][2];
  int sa[8], sb[4];
  for (int kt = 0; kt < nk; ++kt) {
    const char* st = smem + (kt & 1) * MXP_STAGE;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    // ---- P0 (also every scale of the tile: X0 / Y0 refill them two tiles ahead)
    pp_load_a(a, st + 0 * 16384, ra, fr, fg);
    pp_load_b(b0, st + 2 * 16384, rb, fr, fg);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      sa[i] = *reinterpret_cast<const int*>(st + BSTAGE + (sa_row + 16 * i) * 4) >> (8 * fg);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      sb[j] = *reinterpret_cast<const int*>(st + BSTAGE + 1024 + (sb_row + 16 * j) * 4) >> (8 * fg);
    if (n1) mxp_issue<1>(smem, src, wave, lane, kt + 1, (kt + 1) & 1);
    if (n1) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_barrier();
    mxp_mfma<0, 0>(acc, a, b0, sa, sb);
    pp_barrier();
    // ---- P1
    pp_load_b(b1, st + 3 * 16384, rb, fr, fg);
    if (n1) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_barrier();
    mxp_mfma<0, 2>(acc, a, b1, sa, sb);
    pp_barrier();
    // ---- P2
    pp_load_a(a, st + 1 * 16384, ra, fr, fg);
    if (n2) mxp_issue<0>(smem, src, wave, lane, kt + 2, kt & 1);
    pp_barrier();
    mxp_mfma<4, 2>(acc, a, b1, sa, sb);
    pp_barrier();
    // ---- P3
    if (n2) {
      mxp_issue<2>(smem, src, wave, lane, kt + 2, kt & 1);
      mxp_issue<3>(smem, src, wave, lane, kt + 2, kt & 1);
      asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pp_barrier();
    mxp_mfma<4, 0>(acc, a, b0, sa, sb);
    pp_barrier();
  }
  if (wm == 0) pp_barrier();                 // re-align
  float* ep = reinterpret_cast<float*>(smem) + wave * 32 * 68;
  const int m_base = m0 + wm * 128, n_base = n0 + wn * 64;
  if constexpr (EPI != EPI_GENERIC) {
    if (m0 + BBM <= M && n0 + BBN <= N) {
      epilogue_fast<EPI>(acc, ep, lane, m_base, n_base, e);
      return;
    }
  }
  epilogue_generic(acc, ep, lane, M, N, m_base, n_base, e);
}
}  // namespace

bool gemm_pp3_launch(int M, int N, int K, const bf16_t* A, int lda, const bf16_t* Bt,
                     int ldb, const vtd_epilogue* epi, int code, int num_cu,
                     hipStream_t stream);

// 10 = auto (default): 9 when the epilogue has an activation, else 8
// 9 = 8 with transposed accumulators + register-direct epilogue;
// 8 = ping-pong v2 with buffer-resource DMA; 6 = same with global_load_lds;
// 7 = persistent v2; 1 = ping-pong v1; 4 = persistent; 0 = 2-barrier;
// 11 = persistent pp3 (vtd_gemm_pp3.hip); 2, 3, 5 = timing diagnostics (wrong outputs)
int gemm_variant() {
  static const int variant = [] {
    const char* v = getenv("VTD_GEMM_VARIANT");
    return v ? atoi(v) : 10;
  }();
  return variant;
}

// Fewest 256 x 256 tiles for which the bf16 path takes the 256-tile kernels (below: the
// 128 x 128 gemm_tn_kernel).  VTD_PP2_MIN_TILES overrides (A/B of the head's small GEMMs).
int pp2_min_tiles() {
  static const int t = [] {
    const char* v = getenv("VTD_PP2_MIN_TILES");
    return v ? std::max(1, atoi(v)) : 128;
  }();
  return t;
}

// Stream-K (gemm_tn_bf16_pp2sk_kernel) for the default variant when the data-parallel grid's
// last round would leave CUs idle: VTD_GEMM_SK = 0 off (default), 1 when the last round
// is under 85% full, 2 always (tests).  Measured slower on every forward shape (DESIGN.md,
// "What did not pay in round 2"): a split tile's fp32 partials (256 KiB) cost more than
// the K-steps they balance, and ranges starting at different K-steps lose the lockstep
// L2 sharing of the data-parallel rounds.  Returns the data-parallel tile count (a multiple
// of G), or -1 for the plain pp2 launch.  The partial-sum slots and tile counters are
// allocated once per device on first use (never under stream capture: a capture that
// finds them missing runs pp2).
struct SkWorkspace {
  float* partial = nullptr;
  int* counters = nullptr;
  int tiles_cap = 0;
};
constexpr int kSkTilesCap = 1 << 20;

int gemm_sk_mode() {       // read per call: tests switch it inside one process
  const char* v = getenv("VTD_GEMM_SK");
  return v ? atoi(v) : 0;
}

int sk_dp_tiles(int T, int nk, int G, hipStream_t stream, SkArgs& sk) {
  const int mode = gemm_sk_mode();
  if (mode == 0 || G % 8 != 0 || T > kSkTilesCap || nk < 2) return -1;
  const int rounds = (T + G - 1) / G;
  if (mode == 1 && (T >= (int)(0.85 * rounds * G) || nk < 4)) return -1;
  static SkWorkspace ws[64];
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
  {
    std::lock_guard<std::mutex> g(mu);
    SkWorkspace& w = ws[dev];
    if (!w.partial) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
        return -1;
      float* p = nullptr;
      int* c = nullptr;
      if (hipMalloc(reinterpret_cast<void**>(&p), (size_t)G * 2 * BNT * 32 * 16) != hipSuccess)
        return -1;
      if (hipMalloc(reinterpret_cast<void**>(&c), (size_t)kSkTilesCap * sizeof(int)) != hipSuccess ||
          hipMemset(c, 0, (size_t)kSkTilesCap * sizeof(int)) != hipSuccess) {
        (void)hipFree(p);
        return -1;
      }
      w.partial = p;
      w.counters = c;
      w.tiles_cap = G;
    }
    if (w.tiles_cap < G) return -1;
    sk.partial = w.partial;
    sk.counters = w.counters;
  }
  sk.dp_tiles = T / G >= 1 ? (T / G - 1) * G : 0;
  return sk.dp_tiles;
}

template <int C>
void launch_pp2sk(int G, hipStream_t stream, int M, int N, int K, const bf16_t* A, int lda,
                  const bf16_t* Bt, int ldb, int tiles_m, int tiles_n, const EpiArgs& e,
                  const SkArgs& sk) {
  if constexpr (C == 4 || C == 12 || C == 5 || C == 6 || C == 13 || C == 14)
    hipLaunchKernelGGL((gemm_tn_bf16_pp2sk_kernel<C, (C & 3) != 0>), dim3(G), dim3(BNT),
                       2 * BSTAGE, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e, sk);
}

// Whether vtd_gemm can emit the partial LayerNorm statistics (epilogue.statout) for this
// problem: every tile full and on the pp2b / pp2t fast epilogues with a bf16 output.
bool gemm_emits_stats(int M, int N, int dtype, const vtd_epilogue* e) {
  const int tiles = ((M + BBM - 1) / BBM) * ((N + BBN - 1) / BBN);
  const int v = gemm_variant();
  auto a16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  return dtype == VTD_BF16 && e->out_dtype == VTD_BF16 && tiles >= pp2_min_tiles() && N > 64 &&
         M % BBM == 0 && N % BBN == 0 && (v == 8 || v == 9 || v == 10) && e->bias &&
         e->scatter_tokens <= 0 && e->ldo % 8 == 0 && a16(e->out) && a16(e->bias) &&
         (!e->resid || (e->ldr % 8 == 0 && a16(e->resid))) &&
         (!e->out2 || (e->ldo2 % 8 == 0 && a16(e->out2))) && e->stat_ld >= N / 64 &&
         reinterpret_cast<uintptr_t>(e->statout) % 8 == 0;
}

// Whether vtd_gemm_mx8 can write its output as MX-fp8 (out_dtype VTD_FP8): the fast
// epilogue on every tile, no residual or rare modes.
bool gemm_mx8_emits_fp8(int M, int N, const vtd_epilogue* e) {
  auto a16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  return M % BBM == 0 && N % BBN == 0 && e->bias && a16(e->bias) && !e->resid && !e->rowadd &&
         !e->out2 && e->scatter_tokens <= 0 && !e->lnstat && e->ldo % 16 == 0 && a16(e->out) &&
         e->scale_out && e->scale_rows >= M && e->scale_rows % 4 == 0;
}

int gemm_launch_ln(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                   int dtype, const vtd_epilogue* epi, hipStream_t stream, double flops,
                   const float* lnpart, int lnslots, int lnD, float lneps);
int ln_stats_finalize_launch(const float* part, int64_t rows, int slots, int D, float eps,
                             float* stat, hipStream_t st);

int gemm_launch(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                int dtype, const vtd_epilogue* epi, hipStream_t stream, double flops) {
  return gemm_launch_ln(M, N, K, A, lda, Bt, ldb, dtype, epi, stream, flops, nullptr, 0, 0, 0.f);
}

// A GEMM whose LayerNorm-fold row statistics (epi->lnstat) are still the producer's partials
// (lnpart, lnslots per row; the fold path): the pp2 kernels merge them themselves when every
// tile is full and the default fast epilogue runs; otherwise ln_stats_finalize first writes
// epi->lnstat (the unfused sequence).  lnpart == nullptr: a plain gemm_launch.
int gemm_launch_ln(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                   int dtype, const vtd_epilogue* epi, hipStream_t stream, double flops,
                   const float* lnpart, int lnslots, int lnD, float lneps) {
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
  VTD_CHECK_ARG(!epi->lnstat || (epi->colsum && reinterpret_cast<uintptr_t>(epi->lnstat) % 8 == 0 &&
                                 reinterpret_cast<uintptr_t>(epi->colsum) % 16 == 0),
                "gemm: lnstat needs colsum (16-B aligned) and 8-B alignment");
  VTD_CHECK_ARG(!epi->detections || (N == 6 && epi->out_dtype == VTD_F32 &&
                                      epi->scatter_tokens <= 0),
                "gemm: detections (fused transform_predictions) need N == 6 and an fp32 output");
  if (epi->statout && !gemm_emits_stats(M, N, dtype, epi))
    return fail(VTD_ERR_UNSUPPORTED, "gemm: statout needs full 256 x 256 tiles on the bf16 "
                                     "fast epilogues (see gemm_emits_stats)");
  EpiArgs e{epi->bias, epi->rowadd, epi->rowadd_period,
            epi->rowadd ? epi->rowadd_ncols : 0, epi->act, epi->resid, epi->ldr,
            epi->out, epi->ldo, epi->out_dtype, epi->out2, epi->ldo2,
            epi->scatter_tokens, reinterpret_cast<const float2*>(epi->lnstat), epi->colsum,
            reinterpret_cast<float2*>(epi->statout), epi->stat_ld, epi->scale_out,
            epi->scale_rows, epi->detections};
  {
    // pp2 tile order: weight-panel groups of 4 n-tiles (3 at 6) walked down the m-rows keep
    // an XCD's B panels in its L2 (measured per shape, tools/r2_ngw*.sh: qkv / mlp1 / head1
    // -3.3..-4 %, mlp2 -1.7 %); narrower N stays row-major.  VTD_GEMM_NGW overrides (read per
    // call: A/B in one process; 0 = row-major)
    const int tn = (N + BBN - 1) / BBN;
    const char* v = getenv("VTD_GEMM_NGW");
    e.ngw = v ? atoi(v) : tn >= 8 ? 4 : tn == 6 ? 3 : 0;
  }
  // fused LayerNorm finalize only on the default pp2 path (see below); elsewhere the
  // finalize kernel writes lnstat first
  if (lnpart && !(dtype == VTD_BF16 && N > 64 && gemm_variant() == 10 &&
                  ((M + BBM - 1) / BBM) * ((N + BBN - 1) / BBN) >= pp2_min_tiles())) {
    const int rc = ln_stats_finalize_launch(lnpart, M, lnslots, lnD, lneps,
                                            const_cast<float*>(epi->lnstat), stream);
    if (rc) return rc;
    lnpart = nullptr;
  }
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM);
  const size_t lds = 4 * TILE_BYTES;
  ProfScope ps(stream, PROF_GEMM, flops > 0 ? flops : 2.0 * M * N * (double)K);
  const int tiles_m = (M + BBM - 1) / BBM, tiles_n = (N + BBN - 1) / BBN;
  // N <= 64 (the Dense(17) head projection): 128 x 128 tiles waste 8x less MFMA work
  if (dtype == VTD_BF16 && tiles_m * tiles_n >= pp2_min_tiles() && N > 64) {
    static bool attr = false;
    if (!attr) {
      const void* fns[] = {
          reinterpret_cast<const void*>(&gemm_tn_bf16_256_kernel),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pingpong_kernel<EPI_GENERIC, true>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pingpong_kernel<EPI_GENERIC, false>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pingpong_kernel<4, true>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_persistent_kernel<EPI_GENERIC>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<EPI_GENERIC>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pp2p_kernel<EPI_GENERIC>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<EPI_GENERIC, true>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<EPI_GENERIC, true, true>),
#define VTD_PP_FN(C) reinterpret_cast<const void*>(&gemm_tn_bf16_pingpong_kernel<C, false>), \
                     reinterpret_cast<const void*>(&gemm_tn_bf16_pp2p_kernel<C>), \
                     reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C>), \
                     reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, true>), \
                     reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, true, true>), \
                     reinterpret_cast<const void*>(&gemm_tn_bf16_persistent_kernel<C>),
          VTD_PP_FN(0) VTD_PP_FN(1) VTD_PP_FN(2) VTD_PP_FN(4) VTD_PP_FN(5) VTD_PP_FN(6)
          VTD_PP_FN(8) VTD_PP_FN(9) VTD_PP_FN(10) VTD_PP_FN(12) VTD_PP_FN(13) VTD_PP_FN(14)
#undef VTD_PP_FN
      };
      for (const void* f : fns)
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  2 * BSTAGE + EPR_BYTES);
      const void* skfns[] = {
          reinterpret_cast<const void*>(&gemm_tn_bf16_pp2sk_kernel<4, false>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pp2sk_kernel<12, false>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pp2sk_kernel<5, true>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pp2sk_kernel<6, true>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pp2sk_kernel<13, true>),
          reinterpret_cast<const void*>(&gemm_tn_bf16_pp2sk_kernel<14, true>)};
      for (const void* f : skfns)        // + 4 B of static LDS (the last-arriver flag)
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BSTAGE);
      attr = true;
    }
    const int variant = gemm_variant();
    const dim3 g(tiles_m * tiles_n), b(BNT);
    const bf16_t* a16 = static_cast<const bf16_t*>(A);
    const bf16_t* b16 = static_cast<const bf16_t*>(Bt);
    if (variant == 0) {
      hipLaunchKernelGGL(gemm_tn_bf16_256_kernel, g, b, 2 * BSTAGE, stream, M, N, K, a16,
                         lda, b16, ldb, tiles_m, tiles_n, e);
    } else if (variant == 2) {
      hipLaunchKernelGGL((gemm_tn_bf16_pingpong_kernel<EPI_GENERIC, true>), g, b, 2 * BSTAGE,
                         stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e);
    } else if (variant == 3) {
      hipLaunchKernelGGL((gemm_tn_bf16_pingpong_kernel<4, true>), g, b, 2 * BSTAGE,
                         stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e);
    } else {
      // rowadd / out2 ride on the fast epilogues of every variant except the persistent
      // pp2p (7) and pp3 (11), whose epilogues do not implement them
      const bool rare_ok = variant != 7 && variant != 11 &&
                           (!e.out2 || (e.ldo2 % 8 == 0 && reinterpret_cast<uintptr_t>(e.out2) % 16 == 0));
      const bool fast = e.bias && !e.dets && (rare_ok || (!e.rowadd && !e.out2 && !e.lnstat)) &&
                        (e.scatter_tokens <= 0 || variant == 5) &&
                        e.ldo % 8 == 0 && (!e.resid || e.ldr % 8 == 0) &&
                        reinterpret_cast<uintptr_t>(e.out) % 16 == 0 &&
                        reinterpret_cast<uintptr_t>(e.bias) % 16 == 0 &&
                        (!e.resid || reinterpret_cast<uintptr_t>(e.resid) % 16 == 0);
      const int code = fast ? epi_code(e.act, e.out_dtype == VTD_BF16, e.resid != nullptr)
                            : EPI_GENERIC;
      static const int num_cu = [] {
        int dev = 0, n = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n;
      }();
      const bool persistent = variant == 4;
      const bool pp2 = variant == 6;
      const bool pp2p = variant == 7;
      // measured (gemm_bench, same box): 9 wins on activation epilogues (mlp1 -5 %,
      // mlp2 -1.5 %), 8 on plain / f32+residual ones (attn_out -10 %, mlp3 -4 %)
      const bool pp2t = variant == 9 || (variant == 10 && e.act != VTD_ACT_NONE);
      const bool pp2b = variant == 8 || (variant == 10 && !pp2t);
      if (variant == 5) e.scatter_tokens = -2;      // diag: all tiles store to rows 0..255
      // 21..27: main-loop timing diagnostics (pp2_mainloop DG = variant - 20; wrong outputs)
      // on the plain bf16 epilogue; other epilogues run the default kernels
      if (((variant > 20 && variant < 37) || variant == 40) && code == 4) {
        static bool dattr = false;
        const void* dfn[] = {
#define VTD_DG_FN(D) reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<4, true, false, D>),
            VTD_DG_FN(1) VTD_DG_FN(2) VTD_DG_FN(3) VTD_DG_FN(4) VTD_DG_FN(5) VTD_DG_FN(6) VTD_DG_FN(7)
            VTD_DG_FN(8) VTD_DG_FN(9) VTD_DG_FN(10) VTD_DG_FN(11) VTD_DG_FN(12) VTD_DG_FN(13)
            VTD_DG_FN(14) VTD_DG_FN(15) VTD_DG_FN(16) VTD_DG_FN(128)
#undef VTD_DG_FN
        };
        if (!dattr) {
          for (const void* f : dfn)
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BSTAGE);
          dattr = true;
        }
        void* args[] = {&M, &N, &K, (void*)&a16, &lda, (void*)&b16, &ldb,
                        const_cast<int*>(&tiles_m), const_cast<int*>(&tiles_n), &e};
        (void)hipLaunchKernel(dfn[variant == 40 ? 16 : variant - 21], g, b, args, 2 * BSTAGE, stream);
        VTD_LAUNCH_CHECK("gemm");
        return VTD_OK;
      }
      const dim3 gp(std::min(tiles_m * tiles_n, num_cu));
      // pp3 (vtd_gemm_pp3.hip, persistent, one DMA pipeline across tiles): opt-in
      // variant 11.  Isolated it beats pp2 on long-K bf16 layers (mlp2 768 x 3072 -> 1536:
      // 417 vs 463 us, operands L2/MALL-warm) but inside the forward, where A arrives from
      // HBM, its 64-B-row DMA groups cost more than they save (15.3k vs 15.6k img/s).
      if (variant == 11 && code != EPI_GENERIC &&
          gemm_pp3_launch(M, N, K, a16, lda, b16, ldb, epi, code, num_cu, stream)) {
        VTD_LAUNCH_CHECK("gemm");
        return VTD_OK;
      }
      // stream-K on the bf16-output epilogues of the default variant (act: transposed
      // accumulators, as pp2t; none: pp2b)
      SkArgs sk{};
      const bool sk_code = code == 4 || code == 12 || code == 5 || code == 6 || code == 13 ||
                           code == 14;
      const int skdp = variant == 10 && sk_code
                           ? sk_dp_tiles(tiles_m * tiles_n, K / 64, num_cu, stream, sk)
                           : -1;
      if (lnpart) {
        if (variant == 10 && code != EPI_GENERIC && skdp < 0 && M % BBM == 0 && N % BBN == 0 &&
            2 * lnslots * 1024 <= EPR_BYTES) {
          e.lnpart = reinterpret_cast<const float2*>(lnpart);
          e.lnslots = lnslots; e.lnD = lnD; e.lneps = lneps;
        } else {
          const int rc = ln_stats_finalize_launch(lnpart, M, lnslots, lnD, lneps,
                                                  const_cast<float*>(reinterpret_cast<const float*>(e.lnstat)),
                                                  stream);
          if (rc) return rc;
        }
        lnpart = nullptr;
      }
      const int lds_pp2 = 2 * BSTAGE + (e.lnpart ? 2 * e.lnslots * 1024 : 0);
      switch (code) {
#define VTD_PP_CASE(C)                                                                      \
  case C:                                                                                   \
    if (skdp >= 0)                                                                          \
      launch_pp2sk<C>(num_cu, stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e, sk); \
    else if (pp2p)                                                                          \
      hipLaunchKernelGGL((gemm_tn_bf16_pp2p_kernel<C>), gp, b, 2 * BSTAGE + EPR_BYTES,      \
                         stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e);         \
    else if (pp2b)                                                                          \
      hipLaunchKernelGGL((gemm_tn_bf16_pp2_kernel<C, true>), g, b, lds_pp2, stream, M,      \
                         N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e);                    \
    else if (pp2t)                                                                          \
      hipLaunchKernelGGL((gemm_tn_bf16_pp2_kernel<C, true, true>), g, b, lds_pp2, stream,   \
                         M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e);                 \
    else if (pp2)                                                                           \
      hipLaunchKernelGGL((gemm_tn_bf16_pp2_kernel<C>), g, b, 2 * BSTAGE, stream, M, N, K,  \
                         a16, lda, b16, ldb, tiles_m, tiles_n, e);                          \
    else if (persistent)                                                                    \
      hipLaunchKernelGGL((gemm_tn_bf16_persistent_kernel<C>), gp, b, 2 * BSTAGE, stream, M, \
                         N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e);                    \
    else                                                                                    \
      hipLaunchKernelGGL((gemm_tn_bf16_pingpong_kernel<C, false>), g, b, 2 * BSTAGE, stream, \
                         M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e);                 \
    break;
        VTD_PP_CASE(0) VTD_PP_CASE(1) VTD_PP_CASE(2)
        VTD_PP_CASE(4) VTD_PP_CASE(5) VTD_PP_CASE(6)
        VTD_PP_CASE(8) VTD_PP_CASE(9) VTD_PP_CASE(10)
        VTD_PP_CASE(12) VTD_PP_CASE(13) VTD_PP_CASE(14)
#undef VTD_PP_CASE
        default:
          if (pp2p)
            hipLaunchKernelGGL((gemm_tn_bf16_pp2p_kernel<EPI_GENERIC>), gp, b,
                               2 * BSTAGE + EPR_BYTES, stream, M, N, K, a16, lda, b16, ldb,
                               tiles_m, tiles_n, e);
          else if (pp2b)
            hipLaunchKernelGGL((gemm_tn_bf16_pp2_kernel<EPI_GENERIC, true>), g, b, 2 * BSTAGE,
                               stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e);
          else if (pp2t)
            hipLaunchKernelGGL((gemm_tn_bf16_pp2_kernel<EPI_GENERIC, true, true>), g, b,
                               2 * BSTAGE, stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n,
                               e);
          else if (pp2)
            hipLaunchKernelGGL((gemm_tn_bf16_pp2_kernel<EPI_GENERIC>), g, b, 2 * BSTAGE,
                               stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e);
          else if (persistent)
            hipLaunchKernelGGL((gemm_tn_bf16_persistent_kernel<EPI_GENERIC>), gp, b,
                               2 * BSTAGE, stream, M, N, K, a16, lda, b16, ldb, tiles_m,
                               tiles_n, e);
          else
            hipLaunchKernelGGL((gemm_tn_bf16_pingpong_kernel<EPI_GENERIC, false>), g, b,
                               2 * BSTAGE, stream, M, N, K, a16, lda, b16, ldb, tiles_m,
                               tiles_n, e);
      }
    }
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


int gemm_mx8_launch(int M, int N, int K, const uint8_t* A, int lda, const uint8_t* sA,
                    int64_t sa_rows, const uint8_t* Bt, int ldb, const uint8_t* sB,
                    int64_t sb_rows, const vtd_epilogue* epi, hipStream_t stream,
                    double flops) {
  VTD_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 128 == 0, "gemm_mx8: K must be a multiple of 128");
  VTD_CHECK_ARG(A && Bt && sA && sB && epi && epi->out, "gemm_mx8: null pointer");
  VTD_CHECK_ARG(lda >= K && ldb >= K && lda % 16 == 0 && ldb % 16 == 0,
                "gemm_mx8: lda/ldb must be >= K and multiples of 16");
  VTD_CHECK_ARG(sa_rows >= M && sb_rows >= N && sa_rows % 4 == 0 && sb_rows % 4 == 0,
                "gemm_mx8: scale row counts must cover M / N and be multiples of 4");
  VTD_CHECK_ARG(epi->out_dtype == VTD_F32 || epi->out_dtype == VTD_BF16 ||
                    epi->out_dtype == VTD_FP8, "gemm_mx8: bad out dtype");
  VTD_CHECK_ARG(!epi->rowadd || epi->rowadd_period > 0, "gemm_mx8: rowadd_period");
  VTD_CHECK_ARG(epi->scatter_tokens <= 0 || N <= VTD_MAX_DETECT,
                "gemm_mx8: scatter epilogue needs N <= 17");
  VTD_CHECK_ARG(!epi->lnstat || (epi->colsum && reinterpret_cast<uintptr_t>(epi->lnstat) % 8 == 0 &&
                                 reinterpret_cast<uintptr_t>(epi->colsum) % 16 == 0),
                "gemm_mx8: lnstat needs colsum (16-B aligned) and 8-B alignment");
  if (epi->statout) return fail(VTD_ERR_UNSUPPORTED, "gemm_mx8: statout is not supported");
  if (epi->detections)
    return fail(VTD_ERR_UNSUPPORTED, "gemm_mx8: fused detections are not supported");
  if (epi->out_dtype == VTD_FP8 && !gemm_mx8_emits_fp8(M, N, epi))
    return fail(VTD_ERR_UNSUPPORTED, "gemm_mx8: an MX-fp8 output needs full 256 x 256 tiles, a "
                                     "bias, no residual / rowadd / out2 / scatter, ldo % 16 and "
                                     "scale_rows >= M, % 4");
  EpiArgs e{epi->bias, epi->rowadd, epi->rowadd_period,
            epi->rowadd ? epi->rowadd_ncols : 0, epi->act, epi->resid, epi->ldr,
            epi->out, epi->ldo, epi->out_dtype, epi->out2, epi->ldo2,
            epi->scatter_tokens, reinterpret_cast<const float2*>(epi->lnstat), epi->colsum,
            reinterpret_cast<float2*>(epi->statout), epi->stat_ld, epi->scale_out,
            epi->scale_rows, epi->detections};
  ProfScope ps(stream, PROF_GEMM, flops > 0 ? flops : 2.0 * M * N * (double)K);
  const int tiles_m = (M + BBM - 1) / BBM, tiles_n = (N + BBN - 1) / BBN;
  {
    const char* v = getenv("VTD_GEMM_NGW");     // tile order as in gemm_launch
    e.ngw = v ? atoi(v) : tiles_n >= 8 ? 4 : tiles_n == 6 ? 3 : 0;
  }
  static bool attr = false;
  if (!attr) {
#define VTD_MX_FN(C) reinterpret_cast<const void*>(&gemm_mx8_kernel<C>), \
                     reinterpret_cast<const void*>(&gemm_mx8_pp_kernel<C>),
    const void* fns[] = {VTD_MX_FN(EPI_GENERIC) VTD_MX_FN(0) VTD_MX_FN(1) VTD_MX_FN(2)
                         VTD_MX_FN(4) VTD_MX_FN(5) VTD_MX_FN(6) VTD_MX_FN(8) VTD_MX_FN(9)
                         VTD_MX_FN(10) VTD_MX_FN(12) VTD_MX_FN(13) VTD_MX_FN(14)};
#undef VTD_MX_FN
    for (const void* f : fns)
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                std::max(2 * MX_STAGE, 2 * MXP_STAGE));
    attr = true;
  }
  const bool fast = e.bias && !e.rowadd && e.scatter_tokens <= 0 && !e.out2 &&
                    e.ldo % 8 == 0 && (!e.resid || e.ldr % 8 == 0) &&
                    reinterpret_cast<uintptr_t>(e.out) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(e.bias) % 16 == 0 &&
                    (!e.resid || reinterpret_cast<uintptr_t>(e.resid) % 16 == 0);
  const int code = fast ? epi_code(e.act, e.out_dtype != VTD_F32, e.resid != nullptr)
                        : EPI_GENERIC;
  const dim3 g(tiles_m * tiles_n), b(BNT);
  // 1 (default): ping-pong MX kernel; 0: the two-barrier MX kernel
  static const int mxv = [] {
    const char* v = getenv("VTD_MX_VARIANT");
    return v ? atoi(v) : 1;
  }();
  switch (code) {
#define VTD_MX_CASE(C)                                                                     \
  case C:                                                                                  \
    if (mxv == 1)                                                                          \
      hipLaunchKernelGGL((gemm_mx8_pp_kernel<C>), g, b, 2 * MXP_STAGE, stream, M, N, K, A, \
                         lda, sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);     \
    else                                                                                   \
      hipLaunchKernelGGL((gemm_mx8_kernel<C>), g, b, 2 * MX_STAGE, stream, M, N, K, A, lda,\
                         sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);          \
    break;
    VTD_MX_CASE(0) VTD_MX_CASE(1) VTD_MX_CASE(2) VTD_MX_CASE(4) VTD_MX_CASE(5)
    VTD_MX_CASE(6) VTD_MX_CASE(8) VTD_MX_CASE(9) VTD_MX_CASE(10) VTD_MX_CASE(12)
    VTD_MX_CASE(13) VTD_MX_CASE(14)
#undef VTD_MX_CASE
    default:
      if (mxv == 1)
        hipLaunchKernelGGL((gemm_mx8_pp_kernel<EPI_GENERIC>), g, b, 2 * MXP_STAGE, stream, M, N,
                           K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);
      else
        hipLaunchKernelGGL((gemm_mx8_kernel<EPI_GENERIC>), g, b, 2 * MX_STAGE, stream, M, N, K,
                           A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);
  }
  VTD_LAUNCH_CHECK("gemm_mx8");
  return VTD_OK;
}
}  // namespace vtd

extern "C" int vtd_gemm(int M, int N, int K, const void* A_dev, int lda,
                        const void* Bt_dev, int ldb, int dtype, const vtd_epilogue* epi,
                        void* stream) {
  return vtd::gemm_launch(M, N, K, A_dev, lda, Bt_dev, ldb, dtype, epi,
                          static_cast<hipStream_t>(stream), 0.0);
}

extern "C" int vtd_gemm_mx8(int M, int N, int K, const uint8_t* A_dev, int lda,
                            const uint8_t* sA_dev, int64_t sa_rows, const uint8_t* Bt_dev,
                            int ldb, const uint8_t* sB_dev, int64_t sb_rows,
                            const vtd_epilogue* epi, void* stream) {
  return vtd::gemm_mx8_launch(M, N, K, A_dev, lda, sA_dev, sa_rows, Bt_dev, ldb, sB_dev, sb_rows,
                              epi, static_cast<hipStream_t>(stream), 0.0);
}
