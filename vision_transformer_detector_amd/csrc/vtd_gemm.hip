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
#include <type_traits>

#include "vtd_common.h"
#include "vtd_gemm_epi.h"

namespace vtd {

namespace {

constexpr int BM = 128, BN = 128, KB = 128;  // KB = bytes of K per tile row
constexpr int NT = 256;
constexpr int TILE_BYTES = BM * KB;          // 16 KiB per operand per buffer


__device__ __forceinline__ int swz(int row, int chunk) {
  return row * KB + ((chunk ^ (row & 7)) << 4);
}


__device__ __forceinline__ void gload4(i32x4 (&ra)[4], i32x4 (&rb)[4], const char* ga,
                                       const char* gb, const int64_t (&offa)[4],
                                       const int64_t (&offb)[4], int kt, int aw) {
  // A: the split-bf16 wrap (EpiArgs::aw) -- B reads K-step kt, A stored step kt or kt - aw
  const int64_t o = (int64_t)kt * KB, oa = (int64_t)(kt >= aw ? kt - aw : kt) * KB;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ra[i] = *reinterpret_cast<const i32x4*>(ga + offa[i] + oa);
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

  gload4(ra_, rb_, ga, gb, offa, offb, 0, e.aw);
  swrite4(ra_, rb_, lds_a, lds_b, srow, schunk, 0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload4(ra_, rb_, ga, gb, offa, offb, kt + 1, e.aw);
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
// Skinny bf16 GEMM for the detection head's narrow layers at B x 17 rows and its Dense(17)
// projection (vtd.py:454-493): a 256-thread workgroup computes 64 rows x 32 columns, one
// wave 16 rows x 32 columns with v_mfma_f32_16x16x32_bf16.  The workgroup's 32 rows of Bt
// (rows past N zero) are staged once in LDS as the GEMM's 128-B-row image per 64-wide K slab
// (chunk ^ (row & 7): conflict-free ds_read_b128 B reads); A goes straight to registers in
// chunks of SK_CH K-steps, the next chunk's loads in flight while one is multiplied.  These
// layers are latency-bound: the 128 x 128 kernel ran 17-51 workgroups per layer through
// dependent register-staged K-steps, the 256-tile kernel needs >= 128 tiles.
// K % 64 == 0, K <= SK_KMAX.  Split-bf16 operands (EpiArgs::aw > 0, K = 3 P): Bt rows are
// [hi | hi | lo], so only their columns [P, 3P) = [hi | lo] are staged (2 P <= SK_KMAX) and
// K-step s reads staged step s, or s - P / 32 once past it; A wraps after 2 P.
constexpr int SK_ROWS = 64, SK_CH = 8, SK_KMAX = 2048;
__global__ __launch_bounds__(256) void gemm_skinny_kernel(int M, int N, int K,
                                                          const bf16_t* __restrict__ A, int lda,
                                                          const bf16_t* __restrict__ Bt, int ldb,
                                                          EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * SK_ROWS + wave * 16, n0 = blockIdx.y * 32;
  const int nks = K >> 5;                         // 32-wide K-steps
  const bf16_t* ap = A + (int64_t)min(m0 + fr, M - 1) * lda + 8 * g;
  i32x4 a0[SK_CH], a1[SK_CH];
  const int aw2 = 2 * e.aw;                       // the split-bf16 A wrap in 32-wide steps
  auto load = [&](i32x4 (&a)[SK_CH], int s0) {
#pragma unroll
    for (int j = 0; j < SK_CH; ++j) {  // past the end: re-read the last step (no branches)
      const int sa = min(s0 + j, nks - 1);
      a[j] = *reinterpret_cast<const i32x4*>(ap + (sa >= aw2 ? sa - aw2 : sa) * 32);
    }
  };
  load(a0, 0);
  // Bt rows n0 .. n0 + 31: slab t = k / 64, row r, 16-B chunk c at t * 4096 + r * 128 + (c ^ (r & 7)) * 16.
  // Eight chunks per thread in flight at once (a load-store loop waited out one load latency
  // per chunk: 8-12 serial round trips at the head's K = 544-768); a thread's chunks are
  // 256 apart, stepped as (row, chunk) without a division per chunk.
  {
    const int bo = e.aw * 32;                     // first staged column (P, or 0)
    const int kc = (K - bo) >> 3, nch = 32 * kc;
    const int dr = 256 / kc, dc = 256 - dr * kc;
    int r0 = tid / kc, c0 = tid - r0 * kc;
    for (int i0 = tid; i0 < nch; i0 += 8 * 256) {
      i32x4 v[8];
      int rr[8], cc[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        rr[u] = r0;
        cc[u] = c0;
        v[u] = i32x4{0, 0, 0, 0};
        if (i0 + u * 256 < nch && n0 + r0 < N)
          v[u] = *reinterpret_cast<const i32x4*>(Bt + (int64_t)(n0 + r0) * ldb + bo + c0 * 8);
        r0 += dr;
        c0 += dc;
        if (c0 >= kc) {
          c0 -= kc;
          ++r0;
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + u * 256 < nch) {
          const int r = rr[u], t = cc[u] >> 3, c = cc[u] & 7;
          *reinterpret_cast<i32x4*>(smem + t * 4096 + r * 128 + ((c ^ (r & 7)) << 4)) = v[u];
        }
    }
  }
  __syncthreads();
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  auto compute = [&](const i32x4 (&a)[SK_CH], int s0) {
#pragma unroll
    for (int j = 0; j < SK_CH; ++j) {
      const int st = s0 + j;
      if (st < nks) {
        const int sb = st >= e.aw ? st - e.aw : st;   // staged B step (split-bf16 wrap)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const int r = 16 * cb + fr, c = 4 * (sb & 1) + g;
          const bf16x8 b = *reinterpret_cast<const bf16x8*>(smem + (sb >> 1) * 4096 + r * 128 +
                                                            ((c ^ (r & 7)) << 4));
          acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[j]), b,
                                                            acc[cb], 0, 0, 0);
        }
      }
    }
  };
  for (int s0 = 0; s0 < nks; s0 += 2 * SK_CH) {
    if (s0 + SK_CH < nks) load(a1, s0 + SK_CH);
    compute(a0, s0);
    if (s0 + 2 * SK_CH < nks) load(a0, s0 + 2 * SK_CH);
    if (s0 + SK_CH < nks) compute(a1, s0 + SK_CH);
  }
  // D layout: column n0 + 16 cb + fr, rows 4 g + r
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) epi_store(e, M, N, m0 + 4 * g + r, n0 + 16 * cb + fr, acc[cb][r]);
}

constexpr int BBM = 256, BBN = 256, BNT = 512;
#ifndef VTD_TRS
#define VTD_TRS 0
#endif
// K-loop phases per K-step of the bf16 256 x 256 kernel: 2 (pp2_mainloop_2ph, the default:
// C2 forward +1.6-2.2 %, mlp1 -5 %, head2 -6.5 %, profiles/r05_pp2_2phase_ab.log) or 4
// (pp2_mainloop; -DVTD_PP2_PH=4 A/B builds).  The f32 and MX-fp8 kernels keep four phases
// (two measured -1.1 % / -0.3 %).
#ifndef VTD_PP2_PH
#define VTD_PP2_PH 2
#endif
constexpr int BSTAGE = (BBM + BBN) * KB;     // 64 KiB per stage
static_assert(8 * 32 * 68 * 4 + 8 * 128 * 8 <= 2 * BSTAGE,
              "epilogue staging + LayerNorm-fold row tables must fit the stages");

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

// ============================================================================
// bf16 "pp2" kernel (VTD_GEMM_VARIANT=10): 256 x 256 tile, BK 64, 512 threads = 8 waves in
// 2 (M) x 4 (N), each 128 x 64 outputs = 8 x 4 blocks of v_mfma_f32_16x16x32_bf16.  The
// waves run as two groups offset by one barrier (G0 = waves 0-3, G1 = waves 4-7; each SIMD
// holds one wave of each), so one group's MFMAs overlap the other's LDS reads and DMA.
// Operands go HBM/L2 -> LDS by buffer_load_dwordx4 ... lds into four 16 KiB DMA groups
// per 64 KiB stage (pp2_mainloop).  The default (and, in the product library, the only)
// 256-tile bf16 kernel; the MX-fp8 ping-pong kernel below shares its pieces.
// ============================================================================

// Writes the wave's 128 x 64 accumulator tile: 4 passes of 32 rows staged through the
// wave's private LDS region; each lane then owns 8 consecutive columns of a row, so
// residual reads and output writes are 16-B per lane (one 128-B line per 8 lanes).
// DG (diagnostic build only, wrong outputs): 1 = no partial statistics, 2 = no residual
// loads, 4 = no output stores (values kept live), 8 = no epilogue at all
// lst (EPI_LNF): the wave's LayerNorm-fold row statistics in LDS, local rows 0..127
// pf (multi-tile workgroups): issues the next tile's first K-stage DMA.  Called once the
// epilogue's own operand loads are in flight (bias, then the residual rows of the first two
// passes), so that no wait on those loads also waits for the DMA (vmcnt retires in order).
struct NoPF {
  __device__ void operator()() const {}
};

// Four (mean, rstd) rows of the wave's LayerNorm-fold table at byte offsets addr + O0..O3
// (LDS address = the low 32 bits of the generic pointer).  Inline asm with its own wait:
// reads the compiler schedules itself get a vmcnt(0) after the next tile's LDS-bound DMA
// (pf), which would serialise the epilogue behind that prefetch.
template <int O0, int O1, int O2, int O3>
__device__ __forceinline__ void lds_read4_b64(const void* p, float2 (&o)[4]) {
  const uint32_t a = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p));
  asm volatile(
      "ds_read_b64 %0, %4 offset:%5\n\tds_read_b64 %1, %4 offset:%6\n\t"
      "ds_read_b64 %2, %4 offset:%7\n\tds_read_b64 %3, %4 offset:%8\n\ts_waitcnt lgkmcnt(0)"
      : "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3])
      : "v"(a), "i"(O0), "i"(O1), "i"(O2), "i"(O3)
      : "memory");
}
// EPI_S3 (split-bf16 output): o = the hi words of v0, v1 already stored at idx; the lo
// piece at idx + s3 ([hi | lo])
__device__ __forceinline__ void store_s3(const EpiArgs& e, int64_t idx, const i32x4& o, f32x4 v0,
                                         f32x4 v1) {
  const i32x4 lo = {(int)pack_lo_bf16x2(v0[0], v0[1], (uint32_t)o[0]),
                    (int)pack_lo_bf16x2(v0[2], v0[3], (uint32_t)o[1]),
                    (int)pack_lo_bf16x2(v1[0], v1[1], (uint32_t)o[2]),
                    (int)pack_lo_bf16x2(v1[2], v1[3], (uint32_t)o[3])};
  bf16_t* p = static_cast<bf16_t*>(e.out) + idx;
  store_out16(p + e.s3, lo);
}
// TRL: the accumulators are in the transposed layout (lane (fr, fg): row 16 i + fr, columns
// 32 jp + 8 fg .. + 7 in acc[i][2 jp], acc[i][2 jp + 1]): staged with ds_write_b128
template <int EPI, int PR = 32, int DG = 0, typename PF = NoPF, bool TRL = false>
__device__ __forceinline__ void epilogue_fast(const f32x4 (&acc)[8][4], float* ep, int lane,
                                              int m_base, int n_base, const EpiArgs& e,
                                              const float2* lst = nullptr, PF pf = PF{}) {
  constexpr int ACT = EPI & 3;
  constexpr bool OUT_BF16 = (EPI & 4) != 0;
  constexpr bool RESID = (EPI & 8) != 0 && !(DG & 2);
  constexpr bool NOBIAS = (EPI & EPI_PARTIAL) != 0;   // split-K partial: raw fp32 sums
  constexpr bool LNF = (EPI & EPI_LNF) != 0, STAT = (EPI & EPI_STAT) != 0 && !(DG & 1);
  constexpr bool F8O = (EPI & EPI_F8O) != 0;
  // staging image: 64-float rows, 16-B chunk c of row r at chunk c ^ (r & 7) -- conflict-free
  // for both the ds_write_b32 scatter of the accumulators and the ds_read_b128 row reads
  // (a 68-float pitch left the reads 2-way conflicted: SQ_LDS_BANK_CONFLICT ~20 % of the
  // LDS cycles of the query/key/value and attention-output kernels)
  auto sidx = [](int row, int col) { return row * 64 + (((col >> 2) ^ (row & 7)) << 2) + (col & 3); };
  constexpr int NB = PR / 16;            // accumulator row blocks per pass
  constexpr int NIT = PR / 8;            // row-vector iterations per pass
  const int fr = lane & 15, fg = lane >> 4;
  const int c8 = (lane & 7) * 8, rsub = lane >> 3;
  f32x4 b0 = {}, b1 = {};
  if constexpr (!NOBIAS) {
    b0 = *reinterpret_cast<const f32x4*>(e.bias + n_base + c8);
    b1 = *reinterpret_cast<const f32x4*>(e.bias + n_base + c8 + 4);
  }
  f32x4 cs0 = {}, cs1 = {};
  if constexpr (LNF) {
    cs0 = *reinterpret_cast<const f32x4*>(e.colsum + n_base + c8);
    cs1 = *reinterpret_cast<const f32x4*>(e.colsum + n_base + c8 + 4);
  }
  // bf16 residual stream: each pass's rows loaded as raw 16-B words one pass ahead (the rows
  // of pass p + 1 are in flight while pass p is staged and stored; they are rows this wave
  // alone writes, so the in-place update cannot overtake the prefetch)
  constexpr bool RPRE = RESID && OUT_BF16;
  i32x4 rraw[2][NIT];
  auto load_raw = [&](int pp, i32x4 (&dst)[NIT]) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int64_t m = m_base + pp * PR + it * 8 + rsub;
      dst[it] = *reinterpret_cast<const i32x4*>(static_cast<const bf16_t*>(e.resid) + m * e.ldr +
                                                n_base + c8);
    }
  };
  if constexpr (RPRE) load_raw(0, rraw[0]);
  else pf();
#pragma unroll
  for (int p = 0; p < 128 / PR; ++p) {
    if constexpr (TRL) {
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          *reinterpret_cast<f32x4*>(ep + sidx(i * 16 + fr, 32 * (jj >> 1) + 8 * fg + 4 * (jj & 1))) =
              acc[p * NB + i][jj];
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r2 = 0; r2 < 4; ++r2)
            ep[sidx(i * 16 + fg * 4 + r2, j * 16 + fr)] = acc[p * NB + i][j][r2];
    }
    if constexpr (RPRE) {
      if (p + 1 < 128 / PR) load_raw(p + 1, rraw[(p + 1) & 1]);
      if (p == 0) pf();
    }
    // LayerNorm fold, with a prefetch (pf): rows p * PR + it * 8 + rsub read up front by
    // lds_read4_b64 (without one, each row's pair is read where it is used)
    constexpr bool ASM_ST = LNF && !std::is_same<PF, NoPF>::value;
    float2 stv[4];
    if constexpr (ASM_ST) {
      static_assert(PR == 32, "the fold's table reads assume 32-row passes");
      if (p == 0) lds_read4_b64<0, 64, 128, 192>(lst + rsub, stv);
      else if (p == 1) lds_read4_b64<256, 320, 384, 448>(lst + rsub, stv);
      else if (p == 2) lds_read4_b64<512, 576, 640, 704>(lst + rsub, stv);
      else lds_read4_b64<768, 832, 896, 960>(lst + rsub, stv);
    }
    f32x4 rv[NIT][2];
    // STAT: lanes with (lane & 7) == it keep row it * 8 + rsub's (mean, M2): after the pass,
    // lanes (lane & 7) < NIT hold 32 distinct rows, stored by ONE instruction (the slot-major
    // statout plane makes them 256 contiguous bytes)
    [[maybe_unused]] float2 stkeep = float2{0.f, 0.f};
    if constexpr (RESID && !RPRE) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int64_t m = m_base + p * PR + it * 8 + rsub;
        load_resid8<OUT_BF16>(e, m * e.ldr + n_base + c8, rv[it][0], rv[it][1]);
      }
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int row = it * 8 + rsub;
      f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + sidx(row, c8));
      f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + sidx(row, c8 + 4));
      if constexpr (ASM_ST) epi_lnfold8_st(stv[it], cs0, cs1, v0, v1);
      else if constexpr (LNF) epi_lnfold8_st(lst[p * PR + row], cs0, cs1, v0, v1);
      v0 += b0;
      v1 += b1;
      if constexpr ((EPI & EPI_RA) != 0) epi_rowadd8(e, m_base + p * PR + row, n_base + c8, v0, v1);
      act_ct8<ACT>(v0, v1);
      if constexpr (RPRE) {
        const i32x4 w = rraw[p & 1][it];
        v0 += bf16x4_to_f32((uint32_t)w[0], (uint32_t)w[1]);
        v1 += bf16x4_to_f32((uint32_t)w[2], (uint32_t)w[3]);
      } else if constexpr (RESID) {
        v0 += rv[it][0];
        v1 += rv[it][1];
      }
      if constexpr ((EPI & EPI_O2) != 0) epi_out2_8(e, m_base + p * PR + row, n_base + c8, v0, v1);
      const int64_t idx = (int64_t)(m_base + p * PR + row) * e.ldo + n_base + c8;
      if constexpr (OUT_BF16) {
        if constexpr (F8O) {
          // the next MX GEMM's operand: a 32-column block = 4 consecutive lanes (c8 / 8
          // = 0..3 or 4..7), block amax by DPP quad xor 1 / xor 2; bf16-rounded values so
          // the bytes equal vtd_quantize_mx8 of the bf16 output
          bf16_round4(v0);
          bf16_round4(v1);
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
        if constexpr (DG & 4) asm volatile("" ::"v"(o));
        else store_out16(static_cast<bf16_t*>(e.out) + idx, o);
        if constexpr ((EPI & EPI_S3) != 0) store_s3(e, idx, o, v0, v1);
        if constexpr (STAT) {      // the row's 64 columns live in 8 consecutive lanes
          // block mean, then the centred sum of squares (DPP sums, no LDS traffic)
          f32x2 pv[4];
          bf16x8_unpack(o, pv);
          const float mean = sum8_dpp(pairs_sum(pv)) * (1.f / 64.f);
          const float m2 = sum8_dpp(pairs_m2(pv, mean));
          if ((lane & 7) == it) stkeep = float2{mean, m2};
        }
      } else {
        float* op = static_cast<float*>(e.out) + idx;
        *reinterpret_cast<f32x4*>(op) = v0;
        *reinterpret_cast<f32x4*>(op + 4) = v1;
      }
    }
    if constexpr (OUT_BF16 && STAT && !F8O) {
      static_assert(NIT <= 8, "one statistics row per lane of an 8-lane group");
      if ((lane & 7) < NIT)
        e.statout[(int64_t)(n_base >> 6) * e.stat_ld + m_base + p * PR + (lane & 7) * 8 + rsub] =
            stkeep;
    }
  }
}
// global stores the fast epilogue issues per wave (used for counted vmcnt waits)
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

// F32: the fp32 parity mode's operands (a 16-B fragment = 4 f32 K-elements): four
// v_mfma_f32_16x16x4_f32 per fragment pair (exact fp32 fma chain), the K-element t of lane
// group fg being K index 4 (4 s + fg) + t of the 32-wide K-step -- the same LDS image and
// reads as bf16, four times the MFMAs per byte.  Consecutive MFMAs hit different accumulators
// (the f32 MFMA's dependent latency exceeds its issue time).
template <int I0, int J0, bool F32 = false>
__device__ __forceinline__ void pp_mfma(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2],
                                        const bf16x8 (&b)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
  if constexpr (F32) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                __builtin_bit_cast(f32x4, a[i][s])[t], __builtin_bit_cast(f32x4, b[j][s])[t],
                acc[I0 + i][J0 + j], 0, 0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[I0 + i][J0 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s], b[j][s], acc[I0 + i][J0 + j], 0, 0, 0);
  }
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

template <int I0, int J0, bool F32 = false>
__device__ __forceinline__ void pp_mfma_t(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2],
                                          const bf16x8 (&b)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
  if constexpr (F32) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                __builtin_bit_cast(f32x4, b[j][s])[t], __builtin_bit_cast(f32x4, a[i][s])[t],
                acc[I0 + i][J0 + j], 0, 0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[I0 + i][J0 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][s], a[i][s], acc[I0 + i][J0 + j], 0, 0, 0);
  }
  __builtin_amdgcn_s_setprio(0);
}

// ---------------------------------------------------------------------------------
// pp2 K loop: each 64 KiB stage holds four 16 KiB DMA groups, one per operand quadrant a
// phase reads:  X0 = A rows {0-63, 128-191} (A quad 0 of both wave groups), X1 = A rows
// {64-127, 192-255}, Y0 = B rows {0-31, 64-95, 128-159, 192-223} (B quad 0 of every wn),
// Y1 = the other B rows.  Group row gr -> LDS offset gr*128 + swizzled chunk.  A group is
// re-filled as soon as its last reader has retired, two tiles ahead:
//   tile t, P0: DMA X1(t+1)  | reads X0(t), Y0(t) | wait vmcnt(10) -> Y1(t) landed
//           P1:              | reads Y1(t)        | wait vmcnt(8)  -> X1(t) landed
//           P2: DMA X0(t+2)  | reads X1(t)        |
//           P3: DMA Y0,Y1(t+2)|                   | wait vmcnt(10) -> X0,Y0(t+1) landed
// (2 DMA instructions per group per wave; waits count the younger DMA in issue order;
// any phase whose younger DMA may be missing near the end of K waits vmcnt(0).)
// WAR (event e = e-th workgroup barrier; G1 runs one extra barrier first, G0 one extra
// last): X1(t+1) overwrites X1(t-1), last read in tile t-1's P2 (retired by event 8t-1)
// and issued after event 8t; X0(t+2) overwrites X0(t) read in P0 (retired by 8t+3), issued
// after 8t+4; Y0/Y1(t+2) overwrite Y0/Y1(t) read in P0/P1 (retired by 8t+5), issued after
// 8t+6.
__device__ __forceinline__ int grp_tile_row(int g, int gr) {
  return g < 2 ? (gr & 64) * 2 + g * 64 + (gr & 63)          // X0 / X1 (A rows)
               : (gr >> 5) * 64 + (g - 2) * 32 + (gr & 31);  // Y0 / Y1 (B rows)
}

// DMA source addressing of one tile, from wave-uniform scalars only (the per-lane part,
// row-in-piece and swizzled chunk, is rederived from the lane id at each issue): keeps
// 8 x 64-bit per-lane pointers out of the K loop's register budget.
// AW: the kernel may read a split-bf16 A operand (EpiArgs::aw) -- A's K-step of loop step kt
// is kt + ak0, minus aw once past it; !AW: kt (k0 folded into A's base), no scalar arithmetic
// per DMA issue (the bf16 forward's kernels: -0.14 % at C2, profiles/r06_awrap_ab.log)
struct PP2BufSrc {
  __amdgpu_buffer_rsrc_t ra, rb;
  int off[4][2];
  int ak0, aw;
};
template <bool AW>
struct PP2Src : PP2BufSrc {};
// the pp2 epilogue codes whose kernels take the wrap: the split-bf16 output, the f32-output
// codes (the split-bf16 forward's query/key/value and residual layers), split-K partials and
// the generic epilogue; a wrapped A operand never runs the other codes (pp2_code)
constexpr bool pp2_wraps(int code) {
  return code == EPI_GENERIC || (code & EPI_S3) != 0 || (code & 4) == 0;
}

template <bool TR, typename T = bf16_t, bool AW = true>
__device__ __forceinline__ void pp2b_sources(PP2Src<AW>& s, const T* A, int lda, int M,
                                             const T* Bt, int ldb, int N, int m0, int n0,
                                             int wave, int lane, int k0 = 0, bool valid = true,
                                             int aw = 0) {
  // records = bytes from the tile base to the end of the operand (clamped to 32 bits); all
  // offsets are in range because rows are clamped to the last valid row.  k0: first K
  // element of the loop (split-K ranges), folded into B's base; A's K-step offset instead
  // (ak0: the split-bf16 wrap aw counts stored K-steps from the row start)
  constexpr int ES = (int)sizeof(T);
  const int ka0 = AW ? 0 : k0;               // the K offset folded into A's base
  const int64_t ra_bytes = (int64_t)(M - m0) * lda * ES - ES * ka0,
                rb_bytes = (int64_t)(N - n0) * ldb * ES - ES * k0;
  s.ak0 = AW ? k0 * ES / 128 : 0;
  s.aw = AW ? aw : 0;
  // !valid: zero records -- every load out of range (no memory traffic)
  s.ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(A + (int64_t)m0 * lda + ka0), 0,
                                           valid ? (int)std::min<int64_t>(ra_bytes, 0x7fffffff) : 0,
                                           0x00020000);
  s.rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(Bt + (int64_t)n0 * ldb + k0), 0,
                                           valid ? (int)std::min<int64_t>(rb_bytes, 0x7fffffff) : 0,
                                           0x00020000);
  const int prow = lane >> 3, pchunk = (lane & 7) ^ prow;
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int tr = grp_tile_row(g, (wave * 2 + j) * 8 + prow);
      // transposed variant: B groups use swz_t (group row bit 4 = wave & 1 flips chunk bit 2)
      const int bchunk = TR ? pchunk ^ ((wave & 1) << 2) : pchunk;
      s.off[g][j] = g < 2 ? min(tr, M - 1 - m0) * lda * ES + pchunk * 16
                          : min(tr, N - 1 - n0) * ldb * ES + bchunk * 16;
    }
}

template <int G, bool AW>
__device__ __forceinline__ void pp2_issue(char* smem, const PP2BufSrc& src, int wave, int kt,
                                          int stage) {
  char* dst = smem + stage * BSTAGE + G * 16384 + wave * 2 * 1024;
  int ks = kt;
  if constexpr (G < 2 && AW) {
    ks += src.ak0;
    ks = ks >= src.aw ? ks - src.aw : ks;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(G < 2 ? src.ra : src.rb,
                                             (lds_void_t*)(dst + j * 1024), 16, src.off[G][j],
                                             ks * 128, 0, 0);
}

// pre: K-tile 0 was issued by the caller (pp2_prefetch, during the previous output tile's
// epilogue, whose LDS staging lies past stage 0): wait until every wave has left that epilogue
// before K-tile 1 is loaded over it.
// NB (diagnostic build, VTD_PP2_DG & 32, wrong outputs): the K loop's per-phase barriers
// dropped -- the cost of the ping-pong synchronisation itself
template <bool TR, bool F32 = false, bool NB = false, bool AW = true>
__device__ __forceinline__ void pp2_mainloop(f32x4 (&acc)[8][4], char* smem, const PP2Src<AW>& src,
                                             int nk, int wave, int wm, int wn, int fr, int fg,
                                             uint64_t* t_prologue = nullptr, bool pre = false) {
  // prologue: tile 0 complete, tile 1's X0/Y0/Y1 in flight
  if (!pre) {
    pp2_issue<0, AW>(smem, src, wave, 0, 0);
    pp2_issue<2, AW>(smem, src, wave, 0, 0);
    pp2_issue<3, AW>(smem, src, wave, 0, 0);
    pp2_issue<1, AW>(smem, src, wave, 0, 0);
  } else {
    pp_barrier();
  }
  if (nk > 1) {
    pp2_issue<0, AW>(smem, src, wave, 1, 1);
    pp2_issue<2, AW>(smem, src, wave, 1, 1);
    pp2_issue<3, AW>(smem, src, wave, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  pp_barrier();
  if (t_prologue) *t_prologue = __builtin_amdgcn_s_memtime();   // diagnostic stamps only
  if (wm == 1) pp_barrier();                 // stagger G1 by one barrier
  const int ra = wm * 64, rb = wn * 32;      // group rows of this wave's quads
  bf16x8 a[4][2], b0[2][2], b1[2][2];
  // one K-step; n1 / n2 = K-tiles kt + 1 / kt + 2 exist.  The steady-state steps (both) and the
  // last two are separate compile-time bodies: no per-phase branches in the main loop
  auto step = [&](int kt, auto t1, auto t2) {
    const char* st = smem + (kt & 1) * BSTAGE;
    constexpr bool n1 = decltype(t1)::value, n2 = decltype(t2)::value;
    // ---- P0
    pp_load_a(a, st + 0 * 16384, ra, fr, fg);
    if constexpr (TR) pp_load_b_t(b0, st + 2 * 16384, rb, fr, fg);
    else pp_load_b(b0, st + 2 * 16384, rb, fr, fg);
    if constexpr (n1) pp2_issue<1, AW>(smem, src, wave, kt + 1, (kt + 1) & 1);
    if constexpr (n1) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (!NB) pp_barrier();
    if constexpr (TR) pp_mfma_t<0, 0, F32>(acc, a, b0);
    else pp_mfma<0, 0, F32>(acc, a, b0);
    if constexpr (!NB) pp_barrier();
    // ---- P1
    if constexpr (TR) pp_load_b_t(b1, st + 3 * 16384, rb, fr, fg);
    else pp_load_b(b1, st + 3 * 16384, rb, fr, fg);
    if constexpr (n1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (!NB) pp_barrier();
    if constexpr (TR) pp_mfma_t<0, 2, F32>(acc, a, b1);
    else pp_mfma<0, 2, F32>(acc, a, b1);
    if constexpr (!NB) pp_barrier();
    // ---- P2
    pp_load_a(a, st + 1 * 16384, ra, fr, fg);
    if constexpr (n2) pp2_issue<0, AW>(smem, src, wave, kt + 2, kt & 1);
    if constexpr (!NB) pp_barrier();
    if constexpr (TR) pp_mfma_t<4, 2, F32>(acc, a, b1);
    else pp_mfma<4, 2, F32>(acc, a, b1);
    if constexpr (!NB) pp_barrier();
    // ---- P3
    if constexpr (n2) {
      pp2_issue<2, AW>(smem, src, wave, kt + 2, kt & 1);
      pp2_issue<3, AW>(smem, src, wave, kt + 2, kt & 1);
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if constexpr (!NB) pp_barrier();
    if constexpr (TR) pp_mfma_t<4, 0, F32>(acc, a, b0);
    else pp_mfma<4, 0, F32>(acc, a, b0);
    if constexpr (!NB) pp_barrier();
  };
  int kt = 0;
  for (; kt + 2 < nk; ++kt) step(kt, std::true_type{}, std::true_type{});
  if (kt + 1 < nk) step(kt++, std::true_type{}, std::false_type{});
  step(kt, std::false_type{}, std::false_type{});
  if (wm == 0) pp_barrier();                 // re-align
}

// 32-MFMA cluster: row blocks I0..I0+3 against all four column blocks
template <int I0, bool TR, bool F32>
__device__ __forceinline__ void pp_mfma32(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2],
                                          const bf16x8 (&b0)[2][2], const bf16x8 (&b1)[2][2]) {
  if constexpr (TR) {
    pp_mfma_t<I0, 0, F32>(acc, a, b0);
    pp_mfma_t<I0, 2, F32>(acc, a, b1);
  } else {
    pp_mfma<I0, 0, F32>(acc, a, b0);
    pp_mfma<I0, 2, F32>(acc, a, b1);
  }
}

// Two-phase K-step (the same stages, DMA groups and LDS image as pp2_mainloop): phase X
// reads A quad X0 and both B quads and runs row blocks 0-3 x all columns (32 MFMAs), phase Y
// reads A quad X1 and runs row blocks 4-7 -- four barriers per K-step instead of eight.
// Windows (e = workgroup barrier events, G1 one event behind G0): G0 reads X(t) in
// (4t-1, 4t), Y(t) in (4t+1, 4t+2); G1 in (4t, 4t+1), (4t+2, 4t+3).
//   X(t): DMA X1(t+1)         -> stage (t+1)&1 | wait vmcnt(8): X1(t) landed
//   Y(t): DMA X0,Y0,Y1(t+2)   -> stage t&1     | wait vmcnt(8): X0,Y0,Y1(t+1) landed
// WAR: X1(t+1) overwrites X1(t-1), whose last reads (G1, Y(t-1)) retired by 4t-1; the X(t)
// windows open at 4t-1 (G0) / 4t (G1).  X0,Y0,Y1(t+2) overwrite tile t's, last read by G1 in
// X(t), retired by 4t+1; the Y(t) windows open at 4t+1 / 4t+2.  RAW: every wave waits for its
// own DMA before the barrier that opens the readers' window.
template <bool TR, bool F32 = false, bool AW = true>
__device__ __forceinline__ void pp2_mainloop_2ph(f32x4 (&acc)[8][4], char* smem,
                                                 const PP2Src<AW>& src, int nk, int wave, int wm,
                                                 int wn, int fr, int fg,
                                                 uint64_t* t_prologue = nullptr) {
  // prologue: X0,Y0,Y1,X1(0) complete; X0,Y0,Y1(1) in flight
  pp2_issue<0, AW>(smem, src, wave, 0, 0);
  pp2_issue<2, AW>(smem, src, wave, 0, 0);
  pp2_issue<3, AW>(smem, src, wave, 0, 0);
  pp2_issue<1, AW>(smem, src, wave, 0, 0);
  if (nk > 1) {
    pp2_issue<0, AW>(smem, src, wave, 1, 1);
    pp2_issue<2, AW>(smem, src, wave, 1, 1);
    pp2_issue<3, AW>(smem, src, wave, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  pp_barrier();
  if (t_prologue) *t_prologue = __builtin_amdgcn_s_memtime();   // diagnostic stamps only
  if (wm == 1) pp_barrier();                 // stagger G1 by one barrier
  const int ra = wm * 64, rb = wn * 32;
  bf16x8 a[4][2], b0[2][2], b1[2][2];
  auto step = [&](int kt, auto t1, auto t2) {
    const char* st = smem + (kt & 1) * BSTAGE;
    constexpr bool n1 = decltype(t1)::value, n2 = decltype(t2)::value;
    // ---- X
    pp_load_a(a, st + 0 * 16384, ra, fr, fg);
    if constexpr (TR) {
      pp_load_b_t(b0, st + 2 * 16384, rb, fr, fg);
      pp_load_b_t(b1, st + 3 * 16384, rb, fr, fg);
    } else {
      pp_load_b(b0, st + 2 * 16384, rb, fr, fg);
      pp_load_b(b1, st + 3 * 16384, rb, fr, fg);
    }
    if constexpr (n1) {
      pp2_issue<1, AW>(smem, src, wave, kt + 1, (kt + 1) & 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pp_barrier();
    pp_mfma32<0, TR, F32>(acc, a, b0, b1);
    pp_barrier();
    // ---- Y
    pp_load_a(a, st + 1 * 16384, ra, fr, fg);
    if constexpr (n2) {
      pp2_issue<0, AW>(smem, src, wave, kt + 2, kt & 1);
      pp2_issue<2, AW>(smem, src, wave, kt + 2, kt & 1);
      pp2_issue<3, AW>(smem, src, wave, kt + 2, kt & 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      // last K-step: every LDS read retired before the barrier, so that G0, released
      // into its epilogue by the next one, cannot overwrite a stage G1 is still reading
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    pp_barrier();
    pp_mfma32<4, TR, F32>(acc, a, b0, b1);
    // the last Y-phase barrier is G0's alone (G1's Y-phase barrier above): G0's epilogue then
    // runs beside G1's last MFMA cluster instead of waiting for it (no re-align barrier)
    if (n1 || n2 || wm == 0) pp_barrier();
  };
  int kt = 0;
  for (; kt + 2 < nk; ++kt) step(kt, std::true_type{}, std::true_type{});
  if (kt + 1 < nk) step(kt++, std::true_type{}, std::false_type{});
  step(kt, std::false_type{}, std::false_type{});
}

// Epilogue of the transposed variant, full tiles: lane (fr, fg) of wave (wm, wn) holds,
// for accumulator row block i and column half jp, output row m_base + 16 i + fr and the 8
// contiguous columns n_base + 32 jp + 8 fg + 0..7 (acc[i][2 jp] = first 4, acc[i][2 jp + 1]
// = last 4).  Bias is loaded once; residual rows are fetched 4 row blocks at a time.
template <int EPI, int DG = 0, typename PF = NoPF>
__device__ __forceinline__ void epilogue_direct(const f32x4 (&acc)[8][4], int lane, int m_base,
                                                int n_base, const EpiArgs& e,
                                                const float2* lst = nullptr, PF pf = PF{}) {
  constexpr int ACT = EPI & 3;
  constexpr bool OUT_BF16 = (EPI & 4) != 0;
  constexpr bool RESID = (EPI & 8) != 0 && !(DG & 2);
  constexpr bool LNF = (EPI & EPI_LNF) != 0, STAT = (EPI & EPI_STAT) != 0 && !(DG & 1);
  constexpr bool F8O = (EPI & EPI_F8O) != 0;
  static_assert(!(F8O && (STAT || (EPI & EPI_S3) != 0)), "MX-fp8 output: no statistics / split");
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 bias[2][2], cs[2][2] = {};
#pragma unroll
  for (int jp = 0; jp < 2; ++jp)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bias[jp][h] = *reinterpret_cast<const f32x4*>(e.bias + n_base + 32 * jp + 8 * fg + 4 * h);
      if constexpr (LNF)
        cs[jp][h] = *reinterpret_cast<const f32x4*>(e.colsum + n_base + 32 * jp + 8 * fg + 4 * h);
    }
  // bf16 residual: the second half's rows (raw 16-B words) are loaded while the first half
  // is computed
  constexpr bool RPRE = RESID && OUT_BF16;
  i32x4 rraw[2][4][2];
  auto load_raw = [&](int h0, i32x4 (&dst)[4][2]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp)
        dst[i][jp] = *reinterpret_cast<const i32x4*>(
            static_cast<const bf16_t*>(e.resid) + (int64_t)(m_base + 16 * (h0 + i) + fr) * e.ldr +
            n_base + 32 * jp + 8 * fg);
  };
  if constexpr (RPRE) load_raw(0, rraw[0]);
  else pf();
#pragma unroll
  for (int i0 = 0; i0 < 8; i0 += 4) {
    f32x4 rv[4][2][2];
    float2 st[4];                      // LayerNorm fold: the (mean, rstd) of rows 16 (i0 + i) + fr
    if constexpr (LNF && !std::is_same<PF, NoPF>::value) {   // see epilogue_fast
      if (i0 == 0) lds_read4_b64<0, 128, 256, 384>(lst + fr, st);
      else lds_read4_b64<512, 640, 768, 896>(lst + fr, st);
    } else if constexpr (LNF) {
#pragma unroll
      for (int i = 0; i < 4; ++i) st[i] = lst[16 * (i0 + i) + fr];
    }
    // STAT: lanes with fg == i keep row block i's statistics; after the four blocks the 64
    // lanes hold 64 consecutive rows: one store (slot-major statout plane)
    [[maybe_unused]] float2 stkeep = float2{0.f, 0.f};
    if constexpr (RPRE) {
      if (i0 == 0) {
        load_raw(4, rraw[1]);
        pf();
      }
    } else if constexpr (RESID) {
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
        if constexpr (LNF)
          epi_lnfold8_st(st[i], cs[jp][0], cs[jp][1], v0, v1);
        v0 += bias[jp][0];
        v1 += bias[jp][1];
        if constexpr ((EPI & EPI_RA) != 0) epi_rowadd8(e, mrow, ncol, v0, v1);
        act_ct8<ACT>(v0, v1);
        if constexpr (RPRE) {
          const i32x4 w = rraw[i0 >> 2][i][jp];
          v0 += bf16x4_to_f32((uint32_t)w[0], (uint32_t)w[1]);
          v1 += bf16x4_to_f32((uint32_t)w[2], (uint32_t)w[3]);
        } else if constexpr (RESID) {
          v0 += rv[i][jp][0];
          v1 += rv[i][jp][1];
        }
        if constexpr ((EPI & EPI_O2) != 0) epi_out2_8(e, mrow, ncol, v0, v1);
        const int64_t idx = (int64_t)mrow * e.ldo + ncol;
        if constexpr (F8O) {
          // the next MX GEMM's operand: the 32-column block 32 jp .. + 31 of row mrow is the
          // lanes fr, fr + 16, fr + 32, fr + 48 (fg = 0..3): block amax by the two lane swaps;
          // bf16-rounded values, so the bytes equal vtd_quantize_mx8 of the bf16 output
          bf16_round4(v0);
          bf16_round4(v1);
          float am = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) am = fmaxf(am, fmaxf(fabsf(v0[j]), fabsf(v1[j])));
          am = xmax32(xmax16(am));
          const int E = mx8_exponent(am);
          const float inv = __uint_as_float((uint32_t)(127 - E) << 23);
          const uint2 qv = {mx8_pack4(v0[0], v0[1], v0[2], v0[3], inv),
                            mx8_pack4(v1[0], v1[1], v1[2], v1[3], inv)};
          *reinterpret_cast<uint2*>(static_cast<uint8_t*>(e.out) + idx) = qv;
          if (fg == 0) {
            const int b = (n_base + 32 * jp) >> 5;
            e.sout[((int64_t)(b >> 2) * e.s_rows + mrow) * 4 + (b & 3)] = (uint8_t)(E + 127);
          }
          continue;
        }
        if constexpr (OUT_BF16) {
          const i32x4 o = {(int)pack_bf16x2(v0[0], v0[1]), (int)pack_bf16x2(v0[2], v0[3]),
                           (int)pack_bf16x2(v1[0], v1[1]), (int)pack_bf16x2(v1[2], v1[3])};
          if constexpr (DG & 4) asm volatile("" ::"v"(o));
          else store_out16(static_cast<bf16_t*>(e.out) + idx, o);
          if constexpr ((EPI & EPI_S3) != 0) store_s3(e, idx, o, v0, v1);
          if constexpr (STAT) {
            ob[jp] = o;
            tsum += bf16x8_sum(o);
          }
        } else {
          float* op = static_cast<float*>(e.out) + idx;
          *reinterpret_cast<f32x4*>(op) = v0;
          *reinterpret_cast<f32x4*>(op + 4) = v1;
        }
      }
      if constexpr (OUT_BF16 && STAT) {   // the row's 64 columns: lanes fr, fr + 16, + 32, + 48
        // block mean (lane-swap butterfly: every lane holds it), then the centred sum of
        // squares of the same stored values
        const float mean = xsum32(xsum16(tsum)) * (1.f / 64.f);
        const float m2 = xsum32(xsum16(bf16x8_m2(ob[0], mean) + bf16x8_m2(ob[1], mean)));
        if (fg == i) stkeep = float2{mean, m2};
      }
    }
    if constexpr (OUT_BF16 && STAT)
      e.statout[(int64_t)(n_base >> 6) * e.stat_ld + m_base + 16 * (i0 + fg) + fr] = stkeep;
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

#if VTD_DIAG
constexpr int kStampSlots = 16384;
__device__ uint64_t g_pp2_stamps[kStampSlots * 6];
#endif

// ksplit > 1 (split-K, EPI_PARTIAL or EPI_GENERIC without bias / activation): the grid holds
// ksplit x tiles workgroups; workgroup v (after the XCD remap) takes split v / tiles of tile
// v % tiles (neighbours on an XCD share a K range, so their panels are the same lines) and
// writes its fp32 partial tile at e.out + split * e.split_stride; gemm_splitk_epilogue_kernel
// sums the splits and applies the layer's epilogue.
template <int EPI, bool TR = false, int DG = 0>
__global__ __launch_bounds__(BNT) void gemm_tn_bf16_pp2_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda,
    const bf16_t* __restrict__ Bt, int ldb, int tiles_m, int tiles_n, EpiArgs e, int ksplit) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nt = tiles_m * tiles_n, nwg = nt * ksplit;
  const int bid = blockIdx.x;
#if VTD_DIAG
  if (e.dsl > 0 && bid < 256 && ((bid >> 3) & 1))
    for (int i = 0; i < e.dsl; ++i) __builtin_amdgcn_s_sleep(8);
#endif
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int v = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  // one K range (the forward's launches): no division by the tile count or split count
  const int split = ksplit > 1 ? v / nt : 0, tile = v - split * nt;
  int tm, tn;
  tile_coords(tile, e.to, tm, tn);
  const int m0 = tm * BBM, n0 = tn * BBN;
  const int nk_all = K / 64, nks = ksplit > 1 ? (nk_all + ksplit - 1) / ksplit : nk_all;
  const int k0 = split * nks, nk = min(nks, nk_all - k0);   // host: every split non-empty
  if (ksplit > 1) e.out = static_cast<float*>(e.out) + split * e.split_stride;
  PP2Src<pp2_wraps(EPI)> src;
  pp2b_sources<TR>(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane, k0 * 64, true, e.aw);
  // LayerNorm-fold row statistics of the wave's 128 rows: issued before the K loop (the
  // oldest vector-memory op, so the loop's counted waits retire it), used in the epilogue
  float2 lst[2] = {float2{0.f, 0.f}, float2{0.f, 0.f}};
  if constexpr (EPI != EPI_GENERIC && (EPI & EPI_LNF) != 0) {
    lst[0] = e.lnstat[min(m0 + wm * 128 + lane, M - 1)];
    lst[1] = e.lnstat[min(m0 + wm * 128 + 64 + lane, M - 1)];
  }
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  uint64_t ts[4] = {0, 0, 0, 0};
  [[maybe_unused]] uint64_t rt0 = 0;
  if constexpr ((DG & 16) != 0) {
    ts[0] = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (VTD_PP2_PH == 2 && (DG & 32) == 0)
    pp2_mainloop_2ph<TR>(acc, smem, src, nk, wave, wm, wn, fr, fg, (DG & 16) ? &ts[1] : nullptr);
  else
    pp2_mainloop<TR, false, (DG & 32) != 0>(acc, smem, src, nk, wave, wm, wn, fr, fg,
                                             (DG & 16) ? &ts[1] : nullptr);
  if constexpr ((DG & 16) != 0) ts[2] = __builtin_amdgcn_s_memtime();
  const int m_base = m0 + wm * 128, n_base = n0 + wn * 64;
#if VTD_DIAG
  // DG & 16 (diagnostic build): per-workgroup s_memtime stamps of wave 0 -- start, prologue
  // landed, main loop done, epilogue stores issued -- and s_memrealtime (100 MHz) at the start
  // and the end, at g_pp2_stamps[bid]
  auto stamp = [&]() {
    if constexpr ((DG & 16) != 0) {
      ts[3] = __builtin_amdgcn_s_memtime();
      if (wave == 0 && lane == 0 && bid < kStampSlots) {
        g_pp2_stamps[bid * 6 + 0] = ts[0];
        g_pp2_stamps[bid * 6 + 1] = ts[1];
        g_pp2_stamps[bid * 6 + 2] = ts[2];
        g_pp2_stamps[bid * 6 + 3] = ts[3];
        g_pp2_stamps[bid * 6 + 4] = rt0;
        g_pp2_stamps[bid * 6 + 5] = __builtin_amdgcn_s_memrealtime();
      }
    }
  };
#else
  auto stamp = [&]() {};
#endif
  // LayerNorm fold: the wave's 128 row statistics into a wave-private LDS table past the
  // epilogue staging regions (stages are free after the main loop's last barrier); the
  // epilogues read a row's pair from it (a broadcast ds_read_b64, no lane shuffles)
  float2* const lds_st = reinterpret_cast<float2*>(smem + 8 * 32 * 68 * 4) + wave * 128;
  if constexpr (EPI != EPI_GENERIC && (EPI & EPI_LNF) != 0) {
    lds_st[lane] = lst[0];
    lds_st[64 + lane] = lst[1];
  }
  if constexpr ((DG & 8) != 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  if constexpr (TR) {
    if constexpr (EPI != EPI_GENERIC) {
      if (m0 + BBM <= M && n0 + BBN <= N) {
        // VTD_TRS (A/B builds): the transposed accumulators staged through LDS by 16-B writes
        // and stored as whole-line row vectors (epilogue_fast) instead of register-direct
        if constexpr (VTD_TRS && (EPI & 4) != 0 && (EPI & EPI_F8O) == 0)
          epilogue_fast<EPI, 32, DG, NoPF, true>(acc, reinterpret_cast<float*>(smem) + wave * 32 * 68,
                                                 lane, m_base, n_base, e, lds_st);
        else
          epilogue_direct<EPI, DG>(acc, lane, m_base, n_base, e, lds_st);
        stamp();
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
      epilogue_fast<EPI, 32, DG>(acc, ep, lane, m_base, n_base, e, lds_st);
      stamp();
      return;
    }
  }
  epilogue_generic(acc, ep, lane, M, N, m_base, n_base, e);
}

#if VTD_DIAG
// Diagnostic build only (round 4, measured: the forward 18.9k vs 20.0k img/s with two tiles
// per workgroup -- the next tile's K loop cannot start before the epilogue's stores are
// acknowledged, vmcnt counting them with the prefetch; profiles/r04_tpw_trs_ab.log).
// Several tiles per workgroup (knob VTD_KNOB_GEMM_TPW > 1, the forward's epilogue codes):
// pp2's K loop and epilogues in a tile loop; a tile's epilogue issues the next tile's first
// K-stage into stage 0 (the epilogue's LDS lies past it), so that the next K loop starts on
// landed operands, and the workgroup is not relaunched per tile.
template <int EPI, bool TR>
__global__ __launch_bounds__(BNT) void gemm_tn_bf16_pp2_mt_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda,
    const bf16_t* __restrict__ Bt, int ldb, int tiles_m, int tiles_n, EpiArgs e) {
  constexpr int DG = 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane0 = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nt = tiles_m * tiles_n;
  // the grid's nwg workgroups take tiles v, v + nwg, v + 2 nwg, ... (XCD-remapped v): the
  // tiles in flight at any time are one contiguous range of the tile order, as in the
  // one-tile launch (L2 reuse of the A / B panels)
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int v = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int tile = v;
  const int nk = K / 64, k0 = 0;
  int tm, tn;
  tile_coords(tile, e.to, tm, tn);
  // epilogue LDS (32-row staging per wave, then the LayerNorm-fold statistics table) past
  // stage 0: the next tile's first K-stage lands there during the epilogue
  char* const epb = smem + BSTAGE;
  uint64_t ts[4] = {0, 0, 0, 0};
  [[maybe_unused]] uint64_t rt0 = 0;
  if constexpr ((DG & 16) != 0) {
    ts[0] = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  bool pre = false;
  for (;;) {
    const int m0 = tm * BBM, n0 = tn * BBN;
    // per-lane addressing is rederived inside each tile (the opaque copy of the lane id keeps
    // the compiler from hoisting it out of the tile loop, where it would stay live through
    // the epilogue), so a one-tile workgroup has the register budget of a loop-free kernel
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int fr = lane & 15, fg = lane >> 4;
    float* const ep = reinterpret_cast<float*>(epb) + wave * 32 * 68;
    float2* const lds_st = reinterpret_cast<float2*>(epb + 8 * 32 * 68 * 4) + wave * 128;
    PP2Src<pp2_wraps(EPI)> src;
    pp2b_sources<TR>(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane, k0 * 64, true, e.aw);
    // LayerNorm-fold row statistics of the wave's 128 rows: issued before the K loop (older
    // than the K loop's DMAs, so its counted waits retire them), used in the epilogue
    float2 lst[2] = {float2{0.f, 0.f}, float2{0.f, 0.f}};
    if constexpr (EPI != EPI_GENERIC && (EPI & EPI_LNF) != 0) {
      lst[0] = e.lnstat[min(m0 + wm * 128 + lane, M - 1)];
      lst[1] = e.lnstat[min(m0 + wm * 128 + 64 + lane, M - 1)];
    }
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    pp2_mainloop<TR>(acc, smem, src, nk, wave, wm, wn, fr, fg,
                     ((DG & 16) && !pre) ? &ts[1] : nullptr, pre);
    if constexpr ((DG & 16) != 0) {
      if (!pre) ts[2] = __builtin_amdgcn_s_memtime();
    }
    const int m_base = m0 + wm * 128, n_base = n0 + wn * 64;
    // the statistics table (wave-private; the epilogues read a row's pair with a broadcast
    // ds_read_b64, no lane shuffles)
    if constexpr (EPI != EPI_GENERIC && (EPI & EPI_LNF) != 0) {
      lds_st[lane] = lst[0];
      lds_st[64 + lane] = lst[1];
    }
    // next tile of this workgroup: its K-tile 0 is loaded into stage 0 now (every wave has
    // left the K loop: stages are free), under this tile's epilogue
    const bool more = tile + nwg < nt;
    int tm2 = tm, tn2 = tn;
    if (more) tile_coords(tile + nwg, e.to, tm2, tn2);
    // issued unconditionally (out-of-range, traffic-free loads after the last tile): the
    // same instruction sequence on both paths keeps the compiler's counted waits for the
    // epilogue's own loads exact, instead of the minimum over a branch merge
    auto prefetch = [&]() {
      PP2Src<pp2_wraps(EPI)> nsrc;
      pp2b_sources<TR>(nsrc, A, lda, M, Bt, ldb, N, tm2 * BBM, tn2 * BBN, wave, lane, k0 * 64,
                       more, e.aw);
      pp2_issue<0, pp2_wraps(EPI)>(smem, nsrc, wave, 0, 0);
      pp2_issue<2, pp2_wraps(EPI)>(smem, nsrc, wave, 0, 0);
      pp2_issue<3, pp2_wraps(EPI)>(smem, nsrc, wave, 0, 0);
      pp2_issue<1, pp2_wraps(EPI)>(smem, nsrc, wave, 0, 0);
    };
    if constexpr ((DG & 8) != 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
      prefetch();
    } else {
      bool done = false;
      if constexpr (EPI != EPI_GENERIC) {
        if (m0 + BBM <= M && n0 + BBN <= N) {
          if constexpr (TR) epilogue_direct<EPI, DG>(acc, lane, m_base, n_base, e, lds_st, prefetch);
          else epilogue_fast<EPI, 32, DG>(acc, ep, lane, m_base, n_base, e, lds_st, prefetch);
          done = true;
        }
      }
      if (!done) {
        prefetch();
        if constexpr (TR) epilogue_direct_generic(acc, ep, lane, M, N, m_base, n_base, e);
        else epilogue_generic(acc, ep, lane, M, N, m_base, n_base, e);
      }
    }
    if (!more) {
      // the last epilogue issued traffic-free out-of-range DMAs into stage 0: drain them
      // before the workgroup (and its LDS allocation) ends
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      break;
    }
    tile += nwg;
    tm = tm2;
    tn = tn2;
    pre = true;
  }
}
#endif  // VTD_DIAG

// The fp32 parity mode's 256 x 256-tile kernel: pp2's staging, ping-pong schedule and
// epilogues with f32 operands (a 128-B K-step row = 32 f32) on v_mfma_f32_16x16x4_f32
// (pp_mfma<.., true>).  MFMA-bound: a K-step's 64 KiB of operands feed 16x the MFMA cycles
// of the bf16 kernel's.
template <int EPI, bool TR>
__global__ __launch_bounds__(BNT) void gemm_tn_f32_pp2_kernel(
    int M, int N, int K, const float* __restrict__ A, int lda, const float* __restrict__ Bt,
    int ldb, int tiles_m, int tiles_n, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nt = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nt >> 3, r = nt & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int tm, tn;
  tile_coords(tile, e.to, tm, tn);
  const int m0 = tm * BBM, n0 = tn * BBN;
  PP2Src<false> src;
  pp2b_sources<TR, float>(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane, 0);
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  // four phases: with four f32 MFMAs per fragment pair the clusters are long enough (the
  // two-phase step measured -1.1 %, profiles/r05_pp2_2phase_ab.log)
  pp2_mainloop<TR, true>(acc, smem, src, K / 32, wave, wm, wn, fr, fg);
  const int m_base = m0 + wm * 128, n_base = n0 + wn * 64;
  if constexpr (TR) {
    if constexpr (EPI != EPI_GENERIC) {
      if (m0 + BBM <= M && n0 + BBN <= N) {
        epilogue_direct<EPI>(acc, lane, m_base, n_base, e);
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
      epilogue_fast<EPI>(acc, ep, lane, m_base, n_base, e);
      return;
    }
  }
  epilogue_generic(acc, ep, lane, M, N, m_base, n_base, e);
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

// TR: the transposed-accumulator variant (operands swapped, B rows permuted, as pp_mfma_t):
// a lane's accumulators are 8 contiguous output columns of one row, for the register-direct
// epilogue; sb then holds the scales of the permuted B rows the lane supplies
template <int I0, int J0, bool TR = false>
__device__ __forceinline__ void mxp_mfma(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2],
                                         const bf16x8 (&b)[2][2], const int (&sa)[8],
                                         const int (&sb)[4]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if constexpr (TR)
        acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            mx_operand(b[j][0], b[j][1]), mx_operand(a[i][0], a[i][1]), acc[I0 + i][J0 + j], 0,
            0, 0, sb[J0 + j], 0, sa[I0 + i]);
      else
        acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            mx_operand(a[i][0], a[i][1]), mx_operand(b[j][0], b[j][1]), acc[I0 + i][J0 + j], 0,
            0, 0, sa[I0 + i], 0, sb[J0 + j]);
  // pin the cluster inside its phase: without these the compiler sinks every scaled MFMA
  // of the K-step past the phase barriers to the end of the loop body (no ping-pong left)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[I0 + i][J0 + j]));
  __builtin_amdgcn_s_setprio(0);
}

template <int EPI, bool TR = false>
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
  tile_coords(tile, e.to, tm, tn);
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
    // transposed variant: B groups in the swz_t image (as pp2b_sources)
    const int bchunk = TR ? pchunk ^ ((wave & 1) << 2) : pchunk;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int tr = grp_tile_row(g, (wave * 2 + j) * 8 + prow);
        src.off[g][j] = g < 2 ? min(tr, M - 1 - m0) * lda + pchunk * 16
                              : min(tr, N - 1 - n0) * ldb + bchunk * 16;
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
  // scale bytes: a lane's K-block is fg, i.e. byte fg of each row's scale dword, read as a
  // byte (the instruction takes byte 0 of the scale register: no shift); the lane-constant
  // offsets are hoisted, the row-block steps are immediates (TR: perm_t(1, fr) =
  // perm_t(0, fr) + 4)
  const int sa_lane = BSTAGE + (wm * 128 + fr) * 4 + fg;
  const int sb_lane = BSTAGE + 1024 + (TR ? wn * 64 + perm_t(0, fr) : wn * 64 + fr) * 4 + fg;
  bf16x8 a[4][2], b0[2][2], b1[2][2];
  int sa[8], sb[4];
  // one K-step, the last two peeled at compile time (as pp2_mainloop)
  auto step = [&](int kt, auto t1, auto t2) {
    const char* st = smem + (kt & 1) * MXP_STAGE;
    constexpr bool n1 = decltype(t1)::value, n2 = decltype(t2)::value;
    // ---- P0 (also every scale of the tile: X0 / Y0 refill them two tiles ahead)
    pp_load_a(a, st + 0 * 16384, ra, fr, fg);
    if constexpr (TR) pp_load_b_t(b0, st + 2 * 16384, rb, fr, fg);
    else pp_load_b(b0, st + 2 * 16384, rb, fr, fg);
    const uint8_t* ssa = reinterpret_cast<const uint8_t*>(st) + sa_lane;
    const uint8_t* ssb = reinterpret_cast<const uint8_t*>(st) + sb_lane;
#pragma unroll
    for (int i = 0; i < 8; ++i) sa[i] = ssa[64 * i];
#pragma unroll
    for (int j = 0; j < 4; ++j)     // TR: block j of a 32-row half holds rows perm_t(j & 1, fr)
      sb[j] = ssb[TR ? 4 * (32 * (j >> 1) + 4 * (j & 1)) : 64 * j];
    if constexpr (n1) mxp_issue<1>(smem, src, wave, lane, kt + 1, (kt + 1) & 1);
    if constexpr (n1) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_barrier();
    mxp_mfma<0, 0, TR>(acc, a, b0, sa, sb);
    pp_barrier();
    // ---- P1
    if constexpr (TR) pp_load_b_t(b1, st + 3 * 16384, rb, fr, fg);
    else pp_load_b(b1, st + 3 * 16384, rb, fr, fg);
    if constexpr (n1) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_barrier();
    mxp_mfma<0, 2, TR>(acc, a, b1, sa, sb);
    pp_barrier();
    // ---- P2
    pp_load_a(a, st + 1 * 16384, ra, fr, fg);
    if constexpr (n2) mxp_issue<0>(smem, src, wave, lane, kt + 2, kt & 1);
    pp_barrier();
    mxp_mfma<4, 2, TR>(acc, a, b1, sa, sb);
    pp_barrier();
    // ---- P3
    if constexpr (n2) {
      mxp_issue<2>(smem, src, wave, lane, kt + 2, kt & 1);
      mxp_issue<3>(smem, src, wave, lane, kt + 2, kt & 1);
      asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    } else if constexpr (n1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      // last K-step: every LDS read retired before the barrier, so that G0, released into its
      // epilogue (LDS staging over the stages) by the next one, cannot overwrite fragments G1
      // is still reading
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    pp_barrier();
    mxp_mfma<4, 0, TR>(acc, a, b0, sa, sb);
    // the last P3 barrier is G0's alone: G0's epilogue runs beside G1's last MFMA cluster
    // instead of waiting for it (as pp2_mainloop_2ph; G1 ran one extra barrier first)
    if (n1 || wm == 0) pp_barrier();
  };
  int kt = 0;
  for (; kt + 2 < nk; ++kt) step(kt, std::true_type{}, std::true_type{});
  if (kt + 1 < nk) step(kt++, std::true_type{}, std::false_type{});
  step(kt, std::false_type{}, std::false_type{});
  float* ep = reinterpret_cast<float*>(smem) + wave * 32 * 68;
  const int m_base = m0 + wm * 128, n_base = n0 + wn * 64;
  if constexpr (TR) {
    if constexpr (EPI != EPI_GENERIC) {
      if (m0 + BBM <= M && n0 + BBN <= N) {
        epilogue_direct<EPI>(acc, lane, m_base, n_base, e);
        return;
      }
    }
    epilogue_direct_generic(acc, ep, lane, M, N, m_base, n_base, e);
    return;
  }
  if constexpr (EPI != EPI_GENERIC) {
    if (m0 + BBM <= M && n0 + BBN <= N) {
      epilogue_fast<EPI>(acc, ep, lane, m_base, n_base, e);
      return;
    }
  }
  epilogue_generic(acc, ep, lane, M, N, m_base, n_base, e);
}
}  // namespace

#ifndef VTD_DIAG
#define VTD_DIAG 0
#endif
#if VTD_DIAG
// Diagnostic build only (`make diag`, vtd_gemm_w4.hip): the one-wave-per-SIMD w4 (bf16) and
// x4 (MX-fp8) kernels, measured slower than / equal to the ping-pong kernels in the forward
// (profiles/r03_fwd_ab.log, r03_bench_c5_b128_fp8_mx3_s2.log) and therefore not in the product
// library.  VTD_GEMM_VARIANT = 12 selects w4; VTD_MX_VARIANT = 2 selects x4, 3 x4 for K >= 2048.
bool gemm_w4_launch(int M, int N, int K, const bf16_t* A, int lda, const bf16_t* Bt, int ldb,
                    const vtd_epilogue* epi, int ngw, hipStream_t stream);
void gemm_mx8_x4_launch(int M, int N, int K, const uint8_t* A, int lda, const uint8_t* sA,
                        int64_t sa_rows, const uint8_t* Bt, int ldb, const uint8_t* sB,
                        int64_t sb_rows, const vtd_epilogue* epi, int ngw, hipStream_t stream);
int mx_variant() {
  const char* v = getenv("VTD_MX_VARIANT");
  return v ? atoi(v) : 1;
}
int gemm_variant() {
  const char* v = getenv("VTD_GEMM_VARIANT");
  return v ? atoi(v) : 10;
}
#endif

// Fewest 256 x 256 tiles for which the bf16 path takes the 256-tile kernels (below: the
// 128 x 128 gemm_tn_kernel; measured within noise from 1 to 128 tiles on the head's GEMMs).
// 64 since round 5: the N = 768 layers of C2 at B = 64 in two parts (75 tiles each) ran the
// 128 x 128 kernel at 161 us per launch against 27-43 us for the whole batch on pp2
// (profiles/r05_b64_split_trace_*.txt); with 64 the split B = 64 forward is +15 %
// (profiles/r05_b64_split_ab.log).  VTD_MIN_BIG_TILES overrides (A/B).
int min_big_tiles() {
  static const int t = [] {
    const char* v = getenv("VTD_MIN_BIG_TILES");
    return v ? std::max(1, atoi(v)) : 64;
  }();
  return t;
}
#define kMinBigTiles min_big_tiles()

// pp2 / w4 tile order: weight-panel groups of 4 n-tiles (3 at 6) walked down the m-rows keep
// an XCD's B panels in its L2 (measured per shape, round 2: qkv / mlp1 / head1 -3.3..-4 %,
// mlp2 -1.7 %); narrower N stays row-major.  VTD_GEMM_NGW overrides (0 = row-major).
int tile_group_width(int tiles_n) {
  const int k = knob(VTD_KNOB_GEMM_NGW);
  return k >= 0 ? k : tiles_n >= 8 ? 4 : tiles_n == 6 ? 3 : 0;
}

// The epilogue codes pp2 has a specialised (compile-time) kernel for: the activation /
// bf16 output / residual bits and the fold, statistics and row-add combinations the forward
// uses.  Every other combination runs the generic epilogue, which applies the fold, the row
// add and out2 at run time but does NOT write partial statistics (gemm_emits_stats).
#define VTD_PP2_CODES(X)                                                                     \
  X(0) X(1) X(2) X(4) X(5) X(6) X(8) X(9) X(10) X(12) X(13) X(14) X(EPI_PARTIAL)               \
  X(4 | EPI_LNF) X(5 | EPI_LNF) X(6 | EPI_LNF) X(4 | EPI_STAT) X(5 | EPI_STAT)                \
  X(6 | EPI_STAT) X(12 | EPI_STAT) X(13 | EPI_STAT) X(14 | EPI_STAT)                          \
  X(4 | EPI_STAT | EPI_RA) X(4 | EPI_RA) X(4 | EPI_S3) X(5 | EPI_S3) X(6 | EPI_S3)

constexpr bool pp2_specialised(int code) {
#define VTD_PP_IS(C) code == (C) ||
  return VTD_PP2_CODES(VTD_PP_IS) false;
#undef VTD_PP_IS
}

// whether the pp2 kernel can take its fast (specialised) epilogues for this epilogue
bool pp2_fast_epilogue(const vtd_epilogue* e) {
  auto al16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  return e->bias && !e->detections && e->scatter_tokens <= 0 && e->ldo % 8 == 0 &&
         (e->out_dtype != VTD_BF16X3 || (e->ldo / 2) % 8 == 0) &&
         (!e->resid || e->ldr % 8 == 0) && al16(e->out) && al16(e->bias) &&
         (!e->resid || al16(e->resid)) && (!e->out2 || (e->ldo2 % 8 == 0 && al16(e->out2)));
}

// the pp2 epilogue code for this epilogue: its specialised kernel when one exists, else
// EPI_GENERIC
int pp2_code(const vtd_epilogue* e) {
  if (!pp2_fast_epilogue(e)) return EPI_GENERIC;
  const bool s3 = e->out_dtype == VTD_BF16X3;
  const int code = epi_code(e->act, e->out_dtype == VTD_BF16 || s3, e->resid != nullptr) |
                   (e->lnstat ? EPI_LNF : 0) | (e->statout ? EPI_STAT : 0) |
                   (e->rowadd ? EPI_RA : 0) | (e->out2 ? EPI_O2 : 0) | (s3 ? EPI_S3 : 0);
  return pp2_specialised(code) ? code : EPI_GENERIC;
}

// Whether vtd_gemm can emit the partial LayerNorm statistics (epilogue.statout) for this
// problem: every tile full and on a specialised 256-tile epilogue with the statistics bit
// (the generic epilogue does not write them; e.g. the fold + residual + statistics of a
// single-layer MLP has no specialised kernel: its caller takes the row-statistics pass).
bool gemm_emits_stats(int M, int N, int dtype, const vtd_epilogue* e) {
  const int tiles = ((M + BBM - 1) / BBM) * ((N + BBN - 1) / BBN);
  auto a16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  if (!(dtype == VTD_BF16 && e->out_dtype == VTD_BF16 && tiles >= kMinBigTiles && N > 64 &&
        M % BBM == 0 && N % BBN == 0 && e->bias && e->statout &&
        e->scatter_tokens <= 0 && e->ldo % 8 == 0 && a16(e->out) && a16(e->bias) &&
        (!e->resid || (e->ldr % 8 == 0 && a16(e->resid))) &&
        (!e->out2 || (e->ldo2 % 8 == 0 && a16(e->out2))) && e->stat_ld >= M &&
        reinterpret_cast<uintptr_t>(e->statout) % 8 == 0))
    return false;
  return (pp2_code(e) & EPI_STAT) != 0 && pp2_code(e) != EPI_GENERIC;
}

// The skinny kernel for problems the 256-tile kernels do not take (< kMinBigTiles tiles or
// N <= 64): the head's Dense(17) projection (any M) and its narrow layers, when every
// 32-column block re-reads A at most 10 times (N <= 320) -- wider layers keep the 128 x 128
// kernel's A reuse.  VTD_KNOB_SKINNY = 0 disables it; a value >= 64 sets the N threshold.
constexpr int kSkinnyMaxN = 320;
bool skinny_choice(int M, int N, int K) {
  const int kn = knob(VTD_KNOB_SKINNY);
  const int max_n = kn >= 64 ? kn : kSkinnyMaxN;
  return kn != 0 && N <= max_n && K % 64 == 0 && M > 0;
}

// Whether vtd_gemm_mx8 can write its output as MX-fp8 (out_dtype VTD_FP8): the fast
// epilogue on every tile, no residual or rare modes.
bool gemm_mx8_emits_fp8(int M, int N, const vtd_epilogue* e) {
  auto a16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  return M % BBM == 0 && N % BBN == 0 && e->bias && a16(e->bias) && !e->resid && !e->rowadd &&
         !e->out2 && e->scatter_tokens <= 0 && !e->lnstat && e->ldo % 16 == 0 && a16(e->out) &&
         e->scale_out && e->scale_rows >= M && e->scale_rows % 4 == 0;
}

int ln_stats_finalize_launch(const float* part, int64_t rows, int slots, int D, float eps,
                             float* stat, hipStream_t st);

// multi-tile pp2 dynamic LDS: stage 0, then stage 1 overlapped by the epilogue staging and
// the statistics table (stage 0 takes the next tile's first K-stage during an epilogue)
constexpr size_t kPP2LdsMax = BSTAGE + 8 * 32 * 68 * 4 + 8 * 128 * 8;
static_assert(kPP2LdsMax <= 160 * 1024 && kPP2LdsMax >= 2 * BSTAGE, "pp2 LDS");
// the epilogue codes with a multi-tile kernel: the forward's query/key/value and mlp1
// (LayerNorm fold), attention_output / mlp3 (residual + statistics), mlp2
constexpr bool pp2_mt_code(int c) {
  return c == (4 | EPI_LNF) || c == (5 | EPI_LNF) || c == (12 | EPI_STAT) || c == 5 || c == 12;
}
// tiles per pp2 workgroup (knob VTD_KNOB_GEMM_TPW)
inline int pp2_tpw() { return std::max(1, knob(VTD_KNOB_GEMM_TPW)); }

template <int C>
void pp2_launch(bool tr, dim3 g, hipStream_t stream, int M, int N, int K, const bf16_t* A, int lda,
                const bf16_t* Bt, int ldb, int tiles_m, int tiles_n, const EpiArgs& e,
                int ksplit = 1) {
#if VTD_DIAG
  if constexpr (pp2_mt_code(C)) {
    if (ksplit == 1 && e.tpw > 1) {
      const dim3 gm((tiles_m * tiles_n + e.tpw - 1) / e.tpw);
      if (tr)
        hipLaunchKernelGGL((gemm_tn_bf16_pp2_mt_kernel<C, true>), gm, dim3(BNT), kPP2LdsMax,
                           stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
      else
        hipLaunchKernelGGL((gemm_tn_bf16_pp2_mt_kernel<C, false>), gm, dim3(BNT), kPP2LdsMax,
                           stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
      return;
    }
  }
#endif
  if (tr)
    hipLaunchKernelGGL((gemm_tn_bf16_pp2_kernel<C, true>), g, dim3(BNT), 2 * BSTAGE, stream, M,
                       N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e, ksplit);
  else
    hipLaunchKernelGGL((gemm_tn_bf16_pp2_kernel<C, false>), g, dim3(BNT), 2 * BSTAGE, stream, M,
                       N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e, ksplit);
}

void pp2_set_attributes() {
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
#define VTD_PP_FN(C) reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, false>), \
                     reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, true>),
    const void* fns[] = {VTD_PP_FN(EPI_GENERIC) VTD_PP2_CODES(VTD_PP_FN)};
#undef VTD_PP_FN
    for (const void* f : fns)
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BSTAGE);
#if VTD_DIAG
#define VTD_MT_FN(C) reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_mt_kernel<C, false>), \
                     reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_mt_kernel<C, true>),
    const void* mts[] = {VTD_MT_FN(4 | EPI_LNF) VTD_MT_FN(5 | EPI_LNF) VTD_MT_FN(12 | EPI_STAT)
                         VTD_MT_FN(5) VTD_MT_FN(12)};
#undef VTD_MT_FN
    for (const void* f : mts)
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPP2LdsMax);
#endif
  });
}

// Split-K reduction + the layer's epilogue: out[m][n..n+3] = epilogue(sum over the splits of
// part[s][m][n..n+3]) through the shared row-vector epilogue (bias, activation, residual,
// scatter, out2, fused decode; bounds), one thread per 4 columns.  The splits are summed in
// split order (deterministic).
__global__ __launch_bounds__(256) void gemm_splitk_epilogue_kernel(
    const float* __restrict__ part, int ksplit, int64_t stride, int M, int N, int ldp,
    EpiArgs e) {
  const int nq = (N + 3) >> 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)M * nq) return;
  const int m = (int)(i / nq), n = (int)(i - (int64_t)m * nq) * 4;
  const float* p = part + (int64_t)m * ldp + n;
  f32x4 v = *reinterpret_cast<const f32x4*>(p);
  for (int s = 1; s < ksplit; ++s) v += *reinterpret_cast<const f32x4*>(p + s * stride);
  epi_store4(e, M, N, m, n, v);
}

int gemm_launch_ln(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                   int dtype, const vtd_epilogue* epi, hipStream_t stream, double flops,
                   const float* lnpart, int lnslots, int lnD, float lneps);

// the f32 256-tile kernel: the f32-output codes the fp32 mode's forward uses (bias,
// activation, f32 residual, the position-embedding row add); anything else generic
#define VTD_F32_CODES(X) X(0) X(1) X(2) X(8) X(9) X(10) X(EPI_RA)
void f32_pp2_launch(int M, int N, int K, const float* A, int lda, const float* Bt, int ldb,
                    const vtd_epilogue* epi, int tiles_m, int tiles_n, hipStream_t stream) {
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
#define VTD_F32_FN(C) reinterpret_cast<const void*>(&gemm_tn_f32_pp2_kernel<C, false>), \
                      reinterpret_cast<const void*>(&gemm_tn_f32_pp2_kernel<C, true>),
    const void* fns[] = {VTD_F32_FN(EPI_GENERIC) VTD_F32_CODES(VTD_F32_FN)};
#undef VTD_F32_FN
    for (const void* f : fns)
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BSTAGE);
  });
  EpiArgs e = make_epi_args(epi);
  e.ngw = tile_group_width(tiles_n);
  e.to = make_tile_order(tiles_m, tiles_n, e.ngw);
  int code = EPI_GENERIC;
  if (pp2_fast_epilogue(epi) && epi->out_dtype == VTD_F32 && !epi->lnstat && !epi->statout &&
      !epi->out2) {
    const int c = epi_code(e.act, false, e.resid != nullptr) | (e.rowadd ? EPI_RA : 0);
#define VTD_F32_IS(C) c == (C) ||
    if (VTD_F32_CODES(VTD_F32_IS) false) code = c;
#undef VTD_F32_IS
  }
  const bool tr = e.act != VTD_ACT_NONE;
  const dim3 g(tiles_m * tiles_n);
  switch (code) {
#define VTD_F32_CASE(C)                                                                         \
  case C:                                                                                       \
    if (tr) hipLaunchKernelGGL((gemm_tn_f32_pp2_kernel<C, true>), g, dim3(BNT), 2 * BSTAGE,     \
                               stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);          \
    else hipLaunchKernelGGL((gemm_tn_f32_pp2_kernel<C, false>), g, dim3(BNT), 2 * BSTAGE,       \
                            stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);             \
    break;
    VTD_F32_CODES(VTD_F32_CASE)
#undef VTD_F32_CASE
    default:
      if (tr) hipLaunchKernelGGL((gemm_tn_f32_pp2_kernel<EPI_GENERIC, true>), g, dim3(BNT),
                                 2 * BSTAGE, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
      else hipLaunchKernelGGL((gemm_tn_f32_pp2_kernel<EPI_GENERIC, false>), g, dim3(BNT),
                              2 * BSTAGE, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
  }
}

int gemm_launch(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                int dtype, const vtd_epilogue* epi, hipStream_t stream, double flops) {
  return gemm_launch_ln(M, N, K, A, lda, Bt, ldb, dtype, epi, stream, flops, nullptr, 0, 0, 0.f);
}

// dtype VTD_BF16X3 (include/vtd.h "Split-bf16 operands"): a bf16 GEMM over K = 3 P whose A
// rows are stored [hi | lo] (lda >= 2 P) and read as [hi | lo | hi] -- EpiArgs::aw = 2 P / 64
// K-steps, after which the loop's A column returns to 0.  Returns aw (0: not split) and the
// kernels' dtype (VTD_BF16) in dtype, or -1 when the shape cannot be split.
int split_a_wrap(int& dtype, int K, int lda) {
  if (dtype != VTD_BF16X3) return 0;
  if (K % (3 * VTD_KALIGN) != 0 || lda < 2 * (K / 3)) return -1;
  dtype = VTD_BF16;
  return 2 * (K / 3) / 64;
}

// A GEMM whose LayerNorm-fold row statistics (epi->lnstat) are still the producer's partials
// (lnpart, lnslots per row; the fold path): ln_stats_finalize first writes epi->lnstat.
// lnpart == nullptr: a plain gemm_launch.
int gemm_launch_ln(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                   int dtype, const vtd_epilogue* epi, hipStream_t stream, double flops,
                   const float* lnpart, int lnslots, int lnD, float lneps) {
  VTD_CHECK_ARG(M > 0 && N > 0 && K > 0, "gemm: M, N, K must be positive");
  VTD_CHECK_ARG(K % VTD_KALIGN == 0, "gemm: K must be a multiple of VTD_KALIGN");
  VTD_CHECK_ARG(A && Bt && epi && epi->out, "gemm: null pointer");
  VTD_CHECK_ARG(dtype == VTD_F32 || dtype == VTD_BF16 || dtype == VTD_BF16X3, "gemm: bad dtype");
  const bool split_a = dtype == VTD_BF16X3;
  const int aw = split_a_wrap(dtype, K, lda);
  VTD_CHECK_ARG(aw >= 0, "gemm: a split-bf16 A operand needs K = 3 P with P % 64 == 0 and "
                         "lda >= 2 P");
  VTD_CHECK_ARG((split_a || lda >= K) && ldb >= K && lda % 8 == 0 && ldb % 8 == 0,
                "gemm: lda/ldb must be >= K and multiples of 8");
  VTD_CHECK_ARG(epi->out_dtype == VTD_F32 || epi->out_dtype == VTD_BF16 ||
                    (epi->out_dtype == VTD_BF16X3 && dtype == VTD_BF16),
                "gemm: bad out dtype (VTD_BF16X3 output: bf16 operands only)");
  VTD_CHECK_ARG(epi->out_dtype != VTD_BF16X3 ||
                    (epi->ldo % 2 == 0 && epi->ldo / 2 >= N && !epi->out2 && !epi->detections &&
                     !epi->resid && !epi->statout),
                "gemm: a split-bf16 output needs ldo % 2 == 0, ldo / 2 >= N, no out2 / "
                "detections / residual / statistics");
  VTD_CHECK_ARG(!epi->rowadd || epi->rowadd_period > 0, "gemm: rowadd_period");
  VTD_CHECK_ARG(epi->scatter_tokens <= 0 || N <= VTD_MAX_DETECT,
                "gemm: scatter epilogue needs N <= 17");
  VTD_CHECK_ARG(!epi->lnstat || (epi->colsum && reinterpret_cast<uintptr_t>(epi->lnstat) % 8 == 0 &&
                                 reinterpret_cast<uintptr_t>(epi->colsum) % 16 == 0),
                "gemm: lnstat needs colsum (16-B aligned) and 8-B alignment");
  VTD_CHECK_ARG(!epi->detections || (N == 6 && epi->out_dtype == VTD_F32 &&
                                      epi->scatter_tokens <= 0),
                "gemm: detections (fused transform_predictions) need N == 6 and an fp32 output");
  // (a split-bf16 A operand runs the wrap-capable codes only, none of which writes statistics)
  if (epi->statout && (split_a || !gemm_emits_stats(M, N, dtype, epi)))
    return fail(VTD_ERR_UNSUPPORTED, "gemm: statout needs full 256 x 256 tiles on the bf16 "
                                     "fast epilogues and bf16 operands (see gemm_emits_stats)");
  if (lnpart) {
    const int rc = ln_stats_finalize_launch(lnpart, M, lnslots, lnD, lneps,
                                            const_cast<float*>(epi->lnstat), stream);
    if (rc) return rc;
  }
  ProfScope ps(stream, PROF_GEMM, flops > 0 ? flops : 2.0 * M * N * (double)K);
  const int tiles_m = (M + BBM - 1) / BBM, tiles_n = (N + BBN - 1) / BBN;
  // Kernel choice.  >= kMinBigTiles 256 x 256 tiles: pp2.  Fewer: the skinny kernel for
  // narrow layers (N <= 320, its Bt image in LDS), else pp2 as well -- a few-tile problem
  // (small batches: qkv at B = 8 has 63 tiles) runs one round of pp2 tiles at its K loop's
  // rate, where the 128 x 128 register-staged kernel took 4-8x longer (C2 B = 8: 50 launches
  // of 87-193 us per forward, profiles/r06_small_batch_pp2_ab.log); VTD_SMALL_PP2=0 restores it.
  // N <= 64 (the Dense(17) head projection): 128 x 128 tiles waste 8x less MFMA work.
  static const bool small_pp2 = [] {
    const char* v = getenv("VTD_SMALL_PP2");
    return !v || atoi(v) != 0;
  }();
  const bool big = tiles_m * tiles_n >= kMinBigTiles && N > 64;
  const bool skinny = dtype == VTD_BF16 && K - 32 * aw <= SK_KMAX && skinny_choice(M, N, K);
  const bool few = small_pp2 && N > 64 && !skinny;
  if (dtype == VTD_BF16 && (big || few)) {
    const bf16_t* a16 = static_cast<const bf16_t*>(A);
    const bf16_t* b16 = static_cast<const bf16_t*>(Bt);
    const int ngw = tile_group_width(tiles_n);
#if VTD_DIAG
    if (gemm_variant() == 12 && epi->out_dtype != VTD_BF16X3 && aw == 0) {   // (w4: no split)
      if (!gemm_w4_launch(M, N, K, a16, lda, b16, ldb, epi, ngw, stream))
        return fail(VTD_ERR_HIP, "gemm: w4 kernel attributes could not be set");
      VTD_LAUNCH_CHECK("gemm");
      return VTD_OK;
    }
#endif
    pp2_set_attributes();
    EpiArgs e = make_epi_args(epi);
    e.aw = aw;
    e.ngw = ngw;
    e.to = make_tile_order(tiles_m, tiles_n, e.ngw);
    e.tpw = VTD_DIAG ? pp2_tpw() : 1;   // several tiles per workgroup: diagnostic build only
#if VTD_DIAG
    static const int pp2_sleep = getenv("VTD_PP2_SLEEP") ? atoi(getenv("VTD_PP2_SLEEP")) : 0;
    e.dsl = pp2_sleep;
#endif
    // a wrapped (split-bf16) A operand: the codes whose kernels take the wrap (pp2_wraps)
    const int code = aw > 0 && !pp2_wraps(pp2_code(epi)) ? EPI_GENERIC : pp2_code(epi);
    // transposed accumulators + register-direct epilogue for activation layers (mlp1 -5 %,
    // mlp2 -1.5 %), LDS-staged row vectors for the others (attn_out -10 %, mlp3 -4 %);
    // knob VTD_KNOB_GEMM_TR: 0 = never, 1 = always
    const int ktr = knob(VTD_KNOB_GEMM_TR);
    const bool tr = ktr >= 0 ? ktr != 0 : e.act != VTD_ACT_NONE;
    const dim3 g(tiles_m * tiles_n);
#if VTD_DIAG
    const size_t lds = 2 * BSTAGE;
    // epilogue ablation (wrong outputs): VTD_PP2_DG = the DG bits of epilogue_fast /
    // epilogue_direct, for the plain / residual / statistics codes gemm_bench uses
    static const int pp2_dg = getenv("VTD_PP2_DG") ? atoi(getenv("VTD_PP2_DG")) : 0;
    if (pp2_dg > 0 && aw == 0) {
      bool done = true;
      auto dg = [&](auto c) {
        constexpr int C = decltype(c)::value;
        static std::once_flag once[kMaxDevices];
        once_per_device(once, [] {
          for (const void* f : {reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, false, 1>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, true, 1>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, false, 2>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, true, 2>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, false, 4>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, true, 4>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, false, 8>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, true, 8>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, false, 16>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, true, 16>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, false, 32>),
                                reinterpret_cast<const void*>(&gemm_tn_bf16_pp2_kernel<C, true, 32>)})
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BSTAGE);
        });
#define VTD_DG_L(D)                                                                                \
  if (pp2_dg == D) {                                                                               \
    if (tr) hipLaunchKernelGGL((gemm_tn_bf16_pp2_kernel<C, true, D>), g, dim3(BNT), lds,           \
                               stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e, 1);       \
    else hipLaunchKernelGGL((gemm_tn_bf16_pp2_kernel<C, false, D>), g, dim3(BNT), lds,             \
                            stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e, 1);          \
  }
        VTD_DG_L(1) VTD_DG_L(2) VTD_DG_L(4) VTD_DG_L(8) VTD_DG_L(16) VTD_DG_L(32)
#undef VTD_DG_L
      };
      switch (code) {
        case 4: dg(std::integral_constant<int, 4>{}); break;
        case 5: dg(std::integral_constant<int, 5>{}); break;
        case 12: dg(std::integral_constant<int, 12>{}); break;
        case 13: dg(std::integral_constant<int, 13>{}); break;
        case 12 | EPI_STAT: dg(std::integral_constant<int, 12 | EPI_STAT>{}); break;
        case 13 | EPI_STAT: dg(std::integral_constant<int, 13 | EPI_STAT>{}); break;
        case 4 | EPI_LNF: dg(std::integral_constant<int, 4 | EPI_LNF>{}); break;
        case 5 | EPI_LNF: dg(std::integral_constant<int, 5 | EPI_LNF>{}); break;
        default: done = false;
      }
      if (done) {
        VTD_LAUNCH_CHECK("gemm");
        return VTD_OK;
      }
    }
#endif
    switch (code) {
#define VTD_PP_CASE(C) \
  case C: pp2_launch<C>(tr, g, stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e); break;
      VTD_PP2_CODES(VTD_PP_CASE)
#undef VTD_PP_CASE
      default:
        pp2_launch<EPI_GENERIC>(tr, g, stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, e);
    }
  } else if (dtype == VTD_F32 && big && knob(VTD_KNOB_F32_PP2) != 0) {
    // (f32: few-tile problems stay on the 128 x 128 kernel -- the f32 256-tile kernel measured
    // 1.7x slower there, C2 B = 8 f32 557 -> 328 img/s)
    f32_pp2_launch(M, N, K, static_cast<const float*>(A), lda, static_cast<const float*>(Bt), ldb,
                   epi, tiles_m, tiles_n, stream);
  } else if (skinny) {
    EpiArgs e = make_epi_args(epi);
    e.aw = aw;
    const dim3 grid((M + SK_ROWS - 1) / SK_ROWS, (N + 31) / 32);
    const size_t lds = (size_t)32 * (K - 32 * aw) * 2;   // the staged Bt columns
    static std::once_flag once[kMaxDevices];
    once_per_device(once, [] {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_skinny_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 32 * SK_KMAX * 2);
    });
    hipLaunchKernelGGL(gemm_skinny_kernel, grid, dim3(256), lds, stream, M, N, K,
                       static_cast<const bf16_t*>(A), lda, static_cast<const bf16_t*>(Bt), ldb, e);
  } else {
    EpiArgs e = make_epi_args(epi);
    e.aw = aw;
    dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM);
    const size_t lds = 4 * TILE_BYTES;
    if (dtype == VTD_BF16)
      hipLaunchKernelGGL(gemm_tn_kernel<bf16_t>, grid, dim3(NT), lds, stream, M, N, K,
                         static_cast<const bf16_t*>(A), lda, static_cast<const bf16_t*>(Bt), ldb,
                         e);
    else
      hipLaunchKernelGGL(gemm_tn_kernel<float>, grid, dim3(NT), lds, stream, M, N, K,
                         static_cast<const float*>(A), lda, static_cast<const float*>(Bt), ldb, e);
  }
  VTD_LAUNCH_CHECK("gemm");
  return VTD_OK;
}

// Split-K for few-tile, long-K bf16 problems (the detection head's Dense layers at
// B x 17 rows): the number of K splits that brings the 256 x 256-tile grid near one full
// round of the chip (kSplitTarget workgroups), every split keeping >= kSplitMinSteps K-steps
// so its operand traffic stays well above its 256 KiB fp32 partial tile; 1 = no split.
// Fixed targets (not the device's CU count) so that workspace sizing needs no device.
// VTD_SPLITK=0 / knob VTD_KNOB_SPLITK = 0 disables it.
constexpr int kSplitTargetDefault = 256, kSplitMinSteps = 8;
int gemm_splitk_choice(int M, int N, int K, int dtype, int target) {
  const int ks = knob(VTD_KNOB_SPLITK);
  if (ks == 0) return 1;
  // knob value >= 64: the workgroup target itself (A/B of the concurrent micro-batch halves);
  // target > 0: the caller's (vtd_forward: 256 / the concurrent parts)
  const int kSplitTarget = ks >= 64 ? ks : target > 0 ? target : kSplitTargetDefault;
  if ((dtype != VTD_BF16 && dtype != VTD_BF16X3) || N <= 64 || K % 64 != 0 || M <= 0) return 1;
  const int tiles = ((M + BBM - 1) / BBM) * ((N + BBN - 1) / BBN);
  const int nk = K / 64;
  if (tiles >= (3 * kSplitTarget) / 4) return 1;
  // a layer the skinny kernel takes (gemm_launch) stays unsplit
  const int k_staged = dtype == VTD_BF16X3 ? 2 * (K / 3) : K;   // the skinny kernel's Bt in LDS
  if (tiles < kMinBigTiles && k_staged <= SK_KMAX && skinny_choice(M, N, K)) return 1;
  const int s = std::min((kSplitTarget + tiles - 1) / tiles, nk / kSplitMinSteps);
  if (s < 2) return 1;
  const int nks = (nk + s - 1) / s;
  return (nk + nks - 1) / nks;               // every split non-empty
}

// C = epilogue(A Bt^T) as ksplit pp2 K-ranges writing fp32 partial tiles into part
// ([ksplit][M][N] floats), then gemm_splitk_epilogue_kernel.  Same products as the unsplit
// kernels, summed in a different order (fp32).
int gemm_splitk_launch(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                       int dtype, const vtd_epilogue* epi, float* part, int ksplit,
                       hipStream_t stream, double flops) {
  VTD_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 64 == 0 && N % 4 == 0,
                "gemm_splitk: M, N, K positive, K % 64, N % 4");
  VTD_CHECK_ARG(A && Bt && epi && epi->out && part, "gemm_splitk: null pointer");
  VTD_CHECK_ARG(dtype == VTD_BF16 || dtype == VTD_BF16X3, "gemm_splitk: bf16 operands only");
  const bool split_a = dtype == VTD_BF16X3;
  const int aw = split_a_wrap(dtype, K, lda);
  VTD_CHECK_ARG(aw >= 0, "gemm_splitk: a split-bf16 A operand needs K = 3 P with P % 64 == 0 "
                         "and lda >= 2 P");
  // the reduce kernel reads the partials as 16-B vectors (N % 4 keeps every row aligned)
  VTD_CHECK_ARG(reinterpret_cast<uintptr_t>(part) % 16 == 0,
                "gemm_splitk: part_dev must be 16-byte aligned");
  VTD_CHECK_ARG((split_a || lda >= K) && ldb >= K && lda % 8 == 0 && ldb % 8 == 0,
                "gemm_splitk: lda/ldb must be >= K and multiples of 8");
  VTD_CHECK_ARG(ksplit >= 2 && ksplit <= K / 64, "gemm_splitk: ksplit");
  // (the LayerNorm fold applies in the reduction's epilogue; partial statistics are not written)
  VTD_CHECK_ARG(!epi->statout, "gemm_splitk: LayerNorm partial statistics are not supported");
  VTD_CHECK_ARG(!epi->lnstat || (epi->colsum && reinterpret_cast<uintptr_t>(epi->lnstat) % 8 == 0 &&
                                 reinterpret_cast<uintptr_t>(epi->colsum) % 16 == 0),
                "gemm_splitk: lnstat needs colsum (16-B aligned) and 8-B alignment");
  const int nk = K / 64, nks = (nk + ksplit - 1) / ksplit;
  VTD_CHECK_ARG((ksplit - 1) * nks < nk, "gemm_splitk: an empty split");
  ProfScope ps(stream, PROF_GEMM, flops > 0 ? flops : 2.0 * M * N * (double)K);
  pp2_set_attributes();
  const int tiles_m = (M + BBM - 1) / BBM, tiles_n = (N + BBN - 1) / BBN;
  EpiArgs pe{};
  pe.out = part; pe.ldo = N; pe.out_dtype = VTD_F32;
  pe.ngw = tile_group_width(tiles_n);
  pe.to = make_tile_order(tiles_m, tiles_n, pe.ngw);
  pe.split_stride = (int64_t)M * N;
  pe.aw = aw;
  const bf16_t* a16 = static_cast<const bf16_t*>(A);
  const bf16_t* b16 = static_cast<const bf16_t*>(Bt);
  const dim3 g(tiles_m * tiles_n * ksplit);
  if (N % 8 == 0)
    pp2_launch<EPI_PARTIAL>(false, g, stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, pe,
                            ksplit);
  else
    pp2_launch<EPI_GENERIC>(false, g, stream, M, N, K, a16, lda, b16, ldb, tiles_m, tiles_n, pe,
                            ksplit);
  VTD_LAUNCH_CHECK("gemm_splitk");
  const EpiArgs e = make_epi_args(epi);
  const int64_t work = (int64_t)M * ((N + 3) / 4);
  hipLaunchKernelGGL(gemm_splitk_epilogue_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256),
                     0, stream, part, ksplit, (int64_t)M * N, M, N, N, e);
  VTD_LAUNCH_CHECK("gemm_splitk_epilogue");
  return VTD_OK;
}

// the MX-fp8 epilogue codes with a transposed-accumulator kernel: the activation layers
// without a residual (bias + act, f32 / bf16 / MX-fp8 out) and the generic path of partial
// tiles.  C5 per launch (profiles/r05_mx_transposed_ab.log): mlp1 (MX-fp8 out) -5 %, mlp2
// -3 %; the residual layer mlp3 +3 % (not transposed)
#define VTD_MX_TR_CODES(X) X(EPI_GENERIC) X(0) X(1) X(2) X(4) X(5) X(6) X(5 | EPI_F8O) \
  X(6 | EPI_F8O)
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
  EpiArgs e = make_epi_args(epi);
  ProfScope ps(stream, PROF_GEMM, flops > 0 ? flops : 2.0 * M * N * (double)K);
  const int tiles_m = (M + BBM - 1) / BBM, tiles_n = (N + BBN - 1) / BBN;
  e.ngw = tile_group_width(tiles_n);
  e.to = make_tile_order(tiles_m, tiles_n, e.ngw);
#if VTD_DIAG
  // 3: x4 for the long-K layers (K >= 2048: the MLP's inner and last), ping-pong otherwise
  const int mxv = mx_variant();
  if (mxv == 2 || (mxv == 3 && K >= 2048)) {
    gemm_mx8_x4_launch(M, N, K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows, epi, e.ngw, stream);
    VTD_LAUNCH_CHECK("gemm_mx8");
    return VTD_OK;
  }
#endif
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
#define VTD_MX_FN(C) reinterpret_cast<const void*>(&gemm_mx8_pp_kernel<C>),
#define VTD_MXT_FN(C) reinterpret_cast<const void*>(&gemm_mx8_pp_kernel<C, true>),
    const void* fns[] = {VTD_MX_FN(EPI_GENERIC) VTD_MX_FN(0) VTD_MX_FN(1) VTD_MX_FN(2)
                         VTD_MX_FN(4) VTD_MX_FN(5) VTD_MX_FN(6) VTD_MX_FN(8) VTD_MX_FN(9)
                         VTD_MX_FN(10) VTD_MX_FN(12) VTD_MX_FN(13) VTD_MX_FN(14)
                         VTD_MX_FN(4 | EPI_F8O) VTD_MX_FN(5 | EPI_F8O) VTD_MX_FN(6 | EPI_F8O)
                         VTD_MX_TR_CODES(VTD_MXT_FN)};
#undef VTD_MX_FN
#undef VTD_MXT_FN
    for (const void* f : fns)
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * MXP_STAGE);
  });
  const bool fast = e.bias && !e.rowadd && e.scatter_tokens <= 0 && !e.out2 &&
                    e.ldo % 8 == 0 && (!e.resid || e.ldr % 8 == 0) &&
                    reinterpret_cast<uintptr_t>(e.out) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(e.bias) % 16 == 0 &&
                    (!e.resid || reinterpret_cast<uintptr_t>(e.resid) % 16 == 0);
  const int code = fast ? epi_code(e.act, e.out_dtype != VTD_F32, e.resid != nullptr) |
                              (e.out_dtype == VTD_FP8 ? EPI_F8O : 0)
                        : EPI_GENERIC;
  const dim3 g(tiles_m * tiles_n), b(BNT);
  // transposed accumulators + register-direct epilogue for the activation layers (as the bf16
  // kernels; knob VTD_KNOB_GEMM_TR = 0 keeps the staged epilogue everywhere)
  // (1: every layer without a residual, also query/key/value and the plain ones)
  const int ktr = knob(VTD_KNOB_GEMM_TR);
  const bool tr = !e.resid && (ktr == 1 || (ktr != 0 && e.act != VTD_ACT_NONE));
  if (tr) {
    switch (code) {
#define VTD_MXT_CASE(C)                                                                         \
  case C:                                                                                       \
    hipLaunchKernelGGL((gemm_mx8_pp_kernel<C, true>), g, b, 2 * MXP_STAGE, stream, M, N, K, A,  \
                       lda, sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);            \
    VTD_LAUNCH_CHECK("gemm_mx8");                                                               \
    return VTD_OK;
      VTD_MX_TR_CODES(VTD_MXT_CASE)
#undef VTD_MXT_CASE
      default: break;
    }
  }
  switch (code) {
#define VTD_MX_CASE(C)                                                                       \
  case C:                                                                                    \
    hipLaunchKernelGGL((gemm_mx8_pp_kernel<C>), g, b, 2 * MXP_STAGE, stream, M, N, K, A, lda, \
                       sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);              \
    break;
    VTD_MX_CASE(0) VTD_MX_CASE(1) VTD_MX_CASE(2) VTD_MX_CASE(4) VTD_MX_CASE(5)
    VTD_MX_CASE(6) VTD_MX_CASE(8) VTD_MX_CASE(9) VTD_MX_CASE(10) VTD_MX_CASE(12)
    VTD_MX_CASE(13) VTD_MX_CASE(14) VTD_MX_CASE(4 | EPI_F8O) VTD_MX_CASE(5 | EPI_F8O)
    VTD_MX_CASE(6 | EPI_F8O)
#undef VTD_MX_CASE
    default:
      hipLaunchKernelGGL((gemm_mx8_pp_kernel<EPI_GENERIC>), g, b, 2 * MXP_STAGE, stream, M, N, K,
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

extern "C" int vtd_gemm_splitk(int M, int N, int K, const void* A_dev, int lda,
                               const void* Bt_dev, int ldb, int dtype, const vtd_epilogue* epi,
                               float* part_dev, size_t part_bytes, int ksplit, void* stream) {
  if (ksplit < 2 || part_bytes < (size_t)ksplit * (size_t)std::max(M, 0) * std::max(N, 0) * 4)
    return vtd::fail(VTD_ERR_INVALID_ARG, "gemm_splitk: ksplit < 2 or part_bytes too small");
  return vtd::gemm_splitk_launch(M, N, K, A_dev, lda, Bt_dev, ldb, dtype, epi, part_dev, ksplit,
                                 static_cast<hipStream_t>(stream), 0.0);
}

extern "C" int vtd_gemm_splitk_choice(int M, int N, int K, int dtype) {
  return vtd::gemm_splitk_choice(M, N, K, dtype, 0);
}

#if VTD_DIAG
// present in the diagnostic build only (tests select the w4 / x4 comparisons by it)
extern "C" int vtd_diag_build(void) { return 1; }
// the pp2 kernel's per-workgroup stamps (VTD_PP2_DG=16): n slots of 6 uint64 each
extern "C" int vtd_diag_read_stamps(uint64_t* host, int n) {
  n = std::min(n, vtd::kStampSlots);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(vtd::g_pp2_stamps), (size_t)n * 6 * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
#endif
