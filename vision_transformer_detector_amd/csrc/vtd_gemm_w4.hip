// "w4" (VTD_GEMM_VARIANT=12, opt-in): the bf16 Dense-layer GEMM with ONE wave per SIMD (vtd.py:297, 364-412, 454-493 as
// C = act(A Bt^T + bias + rowadd) + resid; A [M][lda] and Bt [N][ldb] both K-contiguous).
//
// Tile 256 x 256, BK = 64, 256 threads = 4 waves in 2 (M) x 2 (N); each wave owns a
// 128 x 128 output block = 8 x 8 blocks of v_mfma_f32_16x16x32_bf16, 256 fp32 accumulators
// per lane (the register file is 512 per lane at one wave per SIMD: accumulators in AGPRs,
// two fragment sets and the DMA offsets in VGPRs).  Against the 8-wave ping-pong pp2 tile
// (128 x 64 per wave) every operand byte read from LDS feeds twice the MFMA work (128 KiB
// of LDS reads per K-step instead of 192) and a K-step is 1 barrier instead of 8.
//
// Staging: both operands HBM/L2 -> LDS by buffer_load_dwordx4 ... lds (1 KiB = 8 rows of
// 128 B per wave-instruction, 16 per wave per K-step), two 64 KiB stages.  LDS rows are
// 128 B with the 16-B chunk XOR-swizzled (A: chunk ^ (row & 7); B: the permuted-read
// swizzle below), applied on the per-lane SOURCE address so the LDS image stays
// lane-linear.  Fragments are double-buffered in registers (F0 = k 0..31 of a K-step,
// F1 = k 32..63).  One K-step (kt, stage s = kt & 1), one barrier:
//
//   MFMA F0: 64, read F1(kt)             2 ds_read_b128 per 8 MFMAs (stage s)
//   lgkmcnt(0); vmcnt(0); barrier        every wave has read all of stage s (WAR) and tile
//                                        kt+1 (stage s^1, the only DMA in flight) landed (RAW)
//   MFMA F1: 64, DMA tile kt+2 -> s,     2 DMA instructions + 2 ds_read_b128 per 8 MFMAs
//     read F0(kt+1) (stage s^1)
//
// Tile kt + 2's DMA thus has one K-step to land.  Counted waits are inline asm and the
// barrier raw s_barrier (a __syncthreads() fence would drain the in-flight DMA).
//
// Epilogue: the MFMA operands are swapped (D = B-block x A-block^T) and the B fragment rows
// permuted so that a lane holds 8 contiguous output columns of one output row: bias,
// LayerNorm fold, activation, residual and the 16-B stores go straight from registers.
// Partial tiles and the rare modes (scatter, fused decode, unaligned) stage through LDS
// into the shared row-vector epilogue (epi_store4).
#include <algorithm>
#include <mutex>

#include "vtd_common.h"
#include "vtd_gemm_epi.h"

namespace vtd {

namespace {

typedef __attribute__((address_space(3))) void w4_lds_t;

constexpr int W4_T = 256;                      // 4 waves, one per SIMD
constexpr int W4_TILE = 256;                   // output tile W4_TILE x W4_TILE
constexpr int W4_OPND = W4_TILE * 128;         // 32 KiB: one operand's K-step (128-B rows)
constexpr int W4_STAGE = 2 * W4_OPND;          // 64 KiB
constexpr int W4_LDS = 2 * W4_STAGE;           // 128 KiB
constexpr int W4_ES = 132;                     // generic epilogue: floats per staged row
static_assert(4 * 32 * W4_ES * 4 <= W4_LDS, "generic epilogue staging must fit the stages");

// A image: chunk ^ (row & 7) -- rows 16 i + fr of one ds_read_b128 lane group hit 8 distinct
// 16-B slots twice, conflict-free for the 4 x 16-lane groups (pp2's derivation).
__device__ __forceinline__ int w4_swz_a(int row, int chunk) {
  return row * 128 + ((chunk ^ (row & 7)) << 4);
}
// B image: the fragment rows are permuted (w4_perm) so that a lane's accumulators are 8
// contiguous output columns; the permuted rows {0-3, 8-11, 16-19, 24-27} + 4 jj would
// 2-way conflict under chunk ^ (row & 7); chunk ^ (row & 7) ^ ((row >> 2) & 4) is
// conflict-free for them.
__device__ __forceinline__ int w4_swz_b(int row, int chunk) {
  return row * 128 + ((chunk ^ (row & 7) ^ ((row >> 2) & 4)) << 4);
}
// B row read by lane fr for block jj (0 / 1) of a 32-column group: blocks 0 / 1 then hold
// output columns 8 (fr >> 2) + 0..3 / 4..7 in the lanes' 4 accumulator rows.
__device__ __forceinline__ int w4_perm(int jj, int fr) { return 8 * (fr >> 2) + 4 * jj + (fr & 3); }

struct W4Src {
  __amdgpu_buffer_rsrc_t ra, rb;
  int offa[8], offb[8];     // per lane: byte offset of its 16 B in DMA piece j (row, chunk)
};

// Wave w fills rows 64 w .. 64 w + 63 of the A and B stage images, piece j = rows
// 64 w + 8 j + (lane >> 3).  Rows past the matrix are clamped to its last row (their
// outputs are never stored), so every offset is in range.
__device__ __forceinline__ void w4_sources(W4Src& s, const bf16_t* A, int lda, int M,
                                           const bf16_t* Bt, int ldb, int N, int m0, int n0,
                                           int wave, int lane) {
  const int64_t ra_bytes = (int64_t)(M - m0) * lda * 2, rb_bytes = (int64_t)(N - n0) * ldb * 2;
  s.ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(A + (int64_t)m0 * lda), 0,
                                           (int)std::min<int64_t>(ra_bytes, 0x7fffffff), 0x00020000);
  s.rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(Bt + (int64_t)n0 * ldb), 0,
                                           (int)std::min<int64_t>(rb_bytes, 0x7fffffff), 0x00020000);
  const int prow = lane >> 3, c = lane & 7;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = wave * 64 + 8 * j + prow;
    // LDS slot (r, c) holds logical chunk c ^ swizzle(r)
    s.offa[j] = min(r, M - 1 - m0) * lda * 2 + ((c ^ prow) << 4);
    s.offb[j] = min(r, N - 1 - n0) * ldb * 2 + ((c ^ prow ^ (((j >> 1) & 1) << 2)) << 4);
  }
}

#ifndef VTD_DIAG
#define VTD_DIAG 0
#endif
// DG (VTD_DIAG builds only; timing diagnostics, WRONG outputs): bit 0 = no DMA after the
// prologue (every K-step reads stale stages), bit 1 = every DMA re-fetches K-tile 0 (the
// same instruction stream from L2-resident lines)
__device__ __forceinline__ void w4_dma(char* stage, const W4Src& s, int wave, int kt, int j) {
  char* da = stage + wave * 64 * 128 + j * 1024;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(s.ra, (w4_lds_t*)da, 16, s.offa[j], kt * 128, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(s.rb, (w4_lds_t*)(da + W4_OPND), 16, s.offb[j],
                                           kt * 128, 0, 0);
}

__device__ __forceinline__ void w4_dma_a(char* stage, const W4Src& s, int wave, int kt, int j) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(s.ra, (w4_lds_t*)(stage + wave * 64 * 128 + j * 1024),
                                           16, s.offa[j], kt * 128, 0, 0);
}
__device__ __forceinline__ void w4_dma_b(char* stage, const W4Src& s, int wave, int kt, int j) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      s.rb, (w4_lds_t*)(stage + W4_OPND + wave * 64 * 128 + j * 1024), 16, s.offb[j], kt * 128, 0,
      0);
}

__device__ __forceinline__ void w4_fence() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void w4_barrier() {
  w4_fence();
  __builtin_amdgcn_s_barrier();
  w4_fence();
}

// fragments of one 32-deep half of a K-step: a[i] = A rows 16 i + fr, b[j] = B rows of
// block j (permuted), chunk 4 h + fg
struct W4Frag {
  bf16x8 a[8], b[8];
};
// reads number r and r + 1 of the 16 (B blocks 0-7, then A blocks 0-7), r = 2 g
__device__ __forceinline__ void w4_read2(W4Frag& f, const char* stage, int g, int aoff,
                                         int boff0, int boff1) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int r = 2 * g + t;
    if (r < 8)
      f.b[r] = *reinterpret_cast<const bf16x8*>(stage + W4_OPND + ((r & 1) ? boff1 : boff0) +
                                                (r >> 1) * 32 * 128);
    else
      f.a[r - 8] = *reinterpret_cast<const bf16x8*>(stage + aoff + (r - 8) * 16 * 128);
  }
}
// 8 MFMAs: output row block i, all 8 column blocks
__device__ __forceinline__ void w4_mfma_row(f32x4 (&acc)[8][8], const W4Frag& f, int i) {
#pragma unroll
  for (int j = 0; j < 8; ++j)
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.b[j], f.a[i], acc[i][j], 0, 0, 0);
}

// One K-step kt (stage st = kt & 1 holds tile kt, F0(kt) in f0; see the file comment).
// F1(kt) is read during F0(kt)'s MFMAs; the barrier
// then retires both every wave's reads of stage st (WAR for tile kt + 2's DMA, issued during
// F1's MFMAs) and tile kt + 1's DMA (RAW for F0(kt + 1)'s reads, also during F1's MFMAs).
template <bool PF, bool NN, int DG>
__device__ __forceinline__ void w4_kstep(f32x4 (&acc)[8][8], W4Frag& f0, W4Frag& f1, char* smem,
                                          const W4Src& src, int kt, int wave, int aoff0,
                                          int aoff1, int b00, int b01, int b10, int b11) {
  char* st = smem + (kt & 1) * W4_STAGE;
  char* nx = smem + ((kt + 1) & 1) * W4_STAGE;
  w4_fence();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w4_read2(f1, st, i, aoff1, b10, b11);
    w4_mfma_row(acc, f0, i);
    w4_fence();
  }
  w4_fence();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile kt + 1 (the only DMA in flight)
  w4_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (PF && !(DG & 1)) w4_dma(st, src, wave, (DG & 2) ? 0 : kt + 2, i);
    if (NN) w4_read2(f0, nx, i, aoff0, b00, b01);
    w4_mfma_row(acc, f1, i);
    w4_fence();
  }
}

// Two-barrier K-step (VTD_W4_SCHED=2): F1(kt) is read during the first quarter of F0's
// MFMAs, so stage st is free a quarter of the way into the K-step and tile kt + 2's B
// operand is DMA'd during F0's remaining MFMAs (its A operand during F1's):
//   rows 0-3 of F0's MFMAs, read F1(kt) (4 per 8 MFMAs);  lgkmcnt(0); barrier A (stage st read
//     by every wave)
//   rows 4-7, DMA B(kt+2) (2 per 8 MFMAs);  vmcnt(8 | 0); barrier B (tile kt+1 landed: the 8
//     youngest are kt+2's)
//   F1's MFMAs, DMA A(kt+2) (1 per 8 MFMAs), read F0(kt+1) (stage st^1)
// (Issuing DMA while F1's reads are in flight made the compiler spill: not done.)
template <bool PF, bool NN, int DG>
__device__ __forceinline__ void w4_kstep2(f32x4 (&acc)[8][8], W4Frag& f0, W4Frag& f1, char* smem,
                                          const W4Src& src, int kt, int wave, int aoff0,
                                          int aoff1, int b00, int b01, int b10, int b11) {
  char* st = smem + (kt & 1) * W4_STAGE;
  char* nx = smem + ((kt + 1) & 1) * W4_STAGE;
  constexpr bool DMA = PF && !(DG & 1);
  const int kd = (DG & 2) ? 0 : kt + 2;
  w4_fence();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w4_read2(f1, st, 2 * i, aoff1, b10, b11);
    w4_read2(f1, st, 2 * i + 1, aoff1, b10, b11);
    w4_mfma_row(acc, f0, i);
    w4_fence();
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  w4_barrier();                                         // A
#pragma unroll
  for (int i = 4; i < 8; ++i) {
    if (DMA) {
      w4_dma_b(st, src, wave, kd, 2 * (i - 4));
      w4_dma_b(st, src, wave, kd, 2 * (i - 4) + 1);
    }
    w4_mfma_row(acc, f0, i);
    w4_fence();
  }
  if (DMA) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  w4_barrier();                                         // B
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (DMA) w4_dma_a(st, src, wave, kd, i);
    if (NN) w4_read2(f0, nx, i, aoff0, b00, b01);
    w4_mfma_row(acc, f1, i);
    w4_fence();
  }
}

// DMA of a tile's K-tiles 0 and 1 into stages 0 and 1 (the stages must be free: no wave
// reads them any more)
__device__ __forceinline__ void w4_issue_k01(char* smem, const W4Src& src, int wave, int nk) {
#pragma unroll
  for (int j = 0; j < 8; ++j) w4_dma(smem, src, wave, 0, j);
  if (nk > 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) w4_dma(smem + W4_STAGE, src, wave, 1, j);
  }
}

template <int SCHED, int DG>
__device__ __forceinline__ void w4_mainloop(f32x4 (&acc)[8][8], char* smem, const W4Src& src,
                                            int nk, int wave, int wm, int wn, int lane) {
  const int fr = lane & 15, fg = lane >> 4;
  // per-lane LDS offsets of the two K-halves' fragments (block offsets are immediates)
  const int aoff0 = w4_swz_a(wm * 128 + fr, fg), aoff1 = w4_swz_a(wm * 128 + fr, 4 + fg);
  const int brow0 = wn * 128 + w4_perm(0, fr), brow1 = wn * 128 + w4_perm(1, fr);
  const int b00 = w4_swz_b(brow0, fg), b01 = w4_swz_b(brow1, fg);          // K-half 0
  const int b10 = w4_swz_b(brow0, 4 + fg), b11 = w4_swz_b(brow1, 4 + fg);  // K-half 1

  // K-tiles 0 and 1 were issued by w4_issue_k01 (for this tile, possibly during the previous
  // tile's epilogue): at least 16 vector-memory operations are younger than K-tile 0's last
  // DMA (K-tile 1's, or the previous epilogue's stores and this tile's column loads), so
  // vmcnt(16) retires K-tile 0; with one K-tile only, everything is waited for
  if (nk > 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  w4_barrier();
  W4Frag f0, f1;
#pragma unroll
  for (int g = 0; g < 8; ++g) w4_read2(f0, smem, g, aoff0, b00, b01);
  int kt = 0;
#define VTD_W4_STEP(PF, NN)                                                                   \
  if constexpr (SCHED == 2)                                                                   \
    w4_kstep2<PF, NN, DG>(acc, f0, f1, smem, src, kt, wave, aoff0, aoff1, b00, b01, b10, b11); \
  else                                                                                        \
    w4_kstep<PF, NN, DG>(acc, f0, f1, smem, src, kt, wave, aoff0, aoff1, b00, b01, b10, b11);
  for (; kt + 2 < nk; ++kt) {
    VTD_W4_STEP(true, true)
  }
  if (kt + 1 < nk) {
    VTD_W4_STEP(false, true)
    ++kt;
  }
  VTD_W4_STEP(false, false)
#undef VTD_W4_STEP
}

// ---- epilogues ---------------------------------------------------------------------
// An accumulator block read out of its AGPRs at the point of use: the "a" constraints keep
// the accumulators' whole live range in the AGPR class (otherwise the register allocator
// splits it at the loop exit and copies all 256 into VGPRs at once, spilling).
__device__ __forceinline__ f32x4 w4_acc(const f32x4& a) {
  f32x4 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v[r]) : "a"(a[r]));
  return v;
}

// Lane (fr, fg) of wave (wm, wn) holds output row m_base + 16 i + fr, columns
// n_base + 32 jp + 8 fg + 0..7 = acc[i][2 jp] (first 4), acc[i][2 jp + 1] (last 4).
// bias / colsum of a lane's 32 columns (4 x 8), loaded before the K loop (oldest memory
// ops: the prologue's counted wait retires them, no load latency left in the epilogue)
// EPI bit 16 (w4 only): the LayerNorm fold (epilogue.lnstat / colsum) is on
constexpr int W4_LNFOLD = 16;
// EPI bit 32 (the MX-fp8 x4 kernel only): MX-fp8 output (out_dtype VTD_FP8, e.sout scales)
constexpr int W4_FP8OUT = 32;
// xmax16 / xmax32: vtd_gemm_epi.h
template <int EPI>
struct W4Cols {
  static constexpr int NC = (EPI & W4_LNFOLD) ? 4 : 1;
  f32x4 bias[4][2], cs[NC][2];
};
template <int EPI>
__device__ __forceinline__ void w4_load_cols(W4Cols<EPI>& c, const EpiArgs& e, int n_base,
                                             int lane) {
  const int fg = lane >> 4;
#pragma unroll
  for (int jp = 0; jp < 4; ++jp)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int n = n_base + 32 * jp + 8 * fg + 4 * h;
      c.bias[jp][h] = *reinterpret_cast<const f32x4*>(e.bias + n);
      if constexpr ((EPI & W4_LNFOLD) != 0)
        c.cs[jp][h] = *reinterpret_cast<const f32x4*>(e.colsum + n);
    }
}

// residual rows of a lane: row block i, column pair jp, 16-B word w
// (f32 residual: loaded two row blocks ahead of their use inside the epilogue)
template <int EPI>
struct W4Resid {
  static constexpr int RW = (EPI & 4) ? 1 : 2;     // 16-B residual loads per 8 columns
  i32x4 r[8][4][RW];
};
template <int EPI>
__device__ __forceinline__ void w4_load_resid(W4Resid<EPI>& rr, const EpiArgs& e, int lane,
                                              int m_base, int n_base, int i) {
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t base = (int64_t)(m_base + 16 * i + fr) * e.ldr + n_base + 8 * fg;
#pragma unroll
  for (int jp = 0; jp < 4; ++jp)
#pragma unroll
    for (int w = 0; w < W4Resid<EPI>::RW; ++w) {
      if constexpr ((EPI & 4) != 0)
        rr.r[i][jp][w] =
            *reinterpret_cast<const i32x4*>(static_cast<const bf16_t*>(e.resid) + base + 32 * jp);
      else
        rr.r[i][jp][w] = *reinterpret_cast<const i32x4*>(static_cast<const float*>(e.resid) +
                                                         base + 32 * jp + 4 * w);
    }
}
template <int EPI>
constexpr bool w4_resid_preloaded() {
  return (EPI & 8) != 0 && (EPI & 4) != 0;         // residual, bf16 stream
}
// bf16 residual: row blocks 0 .. W4_RPRE - 1 are loaded before the next tile's K-tile DMA is
// issued (their waits never include that DMA); the epilogue loads the others two row blocks
// ahead of their use (by then the DMA has had that long to land)
constexpr int W4_RPRE = 3;

// issue_next(): the next tile's K-tile DMA, issued as early as the epilogue allows: before
// row block 0 without a residual, else right after the last residual load (a residual
// load's wait must not include that DMA: vmcnt counts in issue order)
template <int EPI, class F>
__device__ __forceinline__ void w4_epilogue_direct(const f32x4 (&acc)[8][8], int lane, int m_base,
                                                   int n_base, const EpiArgs& e,
                                                   const float2* lst, const W4Cols<EPI>& cols,
                                                   W4Resid<EPI>& rres, F&& issue_next) {
  constexpr int ACT = EPI & 3;
  constexpr bool LNF = (EPI & W4_LNFOLD) != 0;
  constexpr bool OUT_BF16 = (EPI & 4) != 0;
  constexpr bool RESID = (EPI & 8) != 0;
  constexpr int RW = W4Resid<EPI>::RW;
  constexpr bool FP8OUT = (EPI & W4_FP8OUT) != 0;
  const int fr = lane & 15, fg = lane >> 4;
  // residual rows two row blocks ahead of their use (one wave per SIMD: nothing else hides
  // a load's latency); bf16: the first W4_RPRE preloaded by the caller
  auto& rr = rres.r;
  auto load_rows = [&](int i) { w4_load_resid<EPI>(rres, e, lane, m_base, n_base, i); };
  constexpr int PRE = w4_resid_preloaded<EPI>() ? W4_RPRE : 0;   // row blocks already loaded
  if constexpr (RESID) {
#pragma unroll
    for (int i = PRE; i < 2; ++i) load_rows(i);
  } else {
    issue_next();
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if constexpr (RESID) {
      if (i + 2 < 8 && i + 2 >= PRE) load_rows(i + 2);
      if (i + 2 == 7 || (i == 0 && PRE >= 8)) issue_next();
    }
    w4_fence();                    // one row block at a time: no hoisted accumulator copies
    const int lr = 16 * i + fr, mrow = m_base + lr;
    float tsum[2] = {0.f, 0.f};
    i32x4 ob[4];
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      f32x4 v0 = w4_acc(acc[i][2 * jp]), v1 = w4_acc(acc[i][2 * jp + 1]);
      const int ncol = n_base + 32 * jp + 8 * fg;
      if constexpr (LNF)
        epi_lnfold8(e, lst, mrow, lr, cols.cs[jp][0], cols.cs[jp][1], v0, v1);
      v0 += cols.bias[jp][0];
      v1 += cols.bias[jp][1];
      if (e.rowadd) epi_rowadd8(e, mrow, ncol, v0, v1);
      act_ct8<ACT>(v0, v1);
      if constexpr (RESID) {
        if constexpr (OUT_BF16) {
          const i32x4 w = rr[i][jp][0];
          v0 += bf16x4_to_f32((uint32_t)w[0], (uint32_t)w[1]);
          v1 += bf16x4_to_f32((uint32_t)w[2], (uint32_t)w[3]);
        } else {
          v0 += __builtin_bit_cast(f32x4, rr[i][jp][0]);
          v1 += __builtin_bit_cast(f32x4, rr[i][jp][RW - 1]);
        }
      }
      if (e.out2) epi_out2_8(e, mrow, ncol, v0, v1);
      const int64_t idx = (int64_t)mrow * e.ldo + ncol;
      if constexpr (FP8OUT) {
        // the next MX GEMM's operand: the 32-column block 32 jp .. + 31 of this row is held
        // by lanes fr + 16 g (g = 0..3, 8 columns each): block amax by the two lane swaps,
        // of bf16-rounded values (bytes = vtd_quantize_mx8 of the bf16 output)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v0[j] = bf16_round(v0[j]);
          v1[j] = bf16_round(v1[j]);
        }
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
      } else if constexpr (OUT_BF16) {
        const i32x4 o = {(int)pack_bf16x2(v0[0], v0[1]), (int)pack_bf16x2(v0[2], v0[3]),
                         (int)pack_bf16x2(v1[0], v1[1]), (int)pack_bf16x2(v1[2], v1[3])};
        store_out16(static_cast<bf16_t*>(e.out) + idx, o);
        ob[jp] = o;
        tsum[jp >> 1] += bf16x8_sum(o);
      } else {
        float* op = static_cast<float*>(e.out) + idx;
        *reinterpret_cast<f32x4*>(op) = v0;
        *reinterpret_cast<f32x4*>(op + 4) = v1;
      }
    }
    if (OUT_BF16 && !FP8OUT && e.statout) {
      // LayerNorm partials of the two 64-column blocks: a block's 64 values of this row are
      // in lanes fr, fr + 16, + 32, + 48 (jp = 2 b, 2 b + 1)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const float mean = xsum32(xsum16(tsum[b])) * (1.f / 64.f);
        const float m2 =
            xsum32(xsum16(bf16x8_m2(ob[2 * b], mean) + bf16x8_m2(ob[2 * b + 1], mean)));
        if (fg == 0)
          e.statout[(int64_t)((n_base >> 6) + b) * e.stat_ld + mrow] = float2{mean, m2};
      }
    }
  }
}

// Partial tiles and the runtime-flag modes: 32-row passes through the wave's LDS region
// (the stages are free: every wave passed the last K-step's barrier A), then epi_store4
// (bounds, rowadd, scatter, out2, fused decode).
__device__ __forceinline__ void w4_epilogue_generic(const f32x4 (&acc)[8][8], float* ep, int lane,
                                                    int M, int N, int m_base, int n_base,
                                                    const EpiArgs& e) {
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<f32x4*>(ep + (ii * 16 + fr) * W4_ES + 32 * (j >> 1) + 8 * fg +
                                  4 * (j & 1)) = w4_acc(acc[2 * p + ii][j]);
#pragma unroll 1
    for (int it = 0; it < 16; ++it) {
      const int row = it * 2 + (lane >> 5), col = (lane & 31) * 4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(ep + row * W4_ES + col);
      epi_store4(e, M, N, m_base + 32 * p + row, n_base + col, v);
    }
  }
}

// tile vb's (m0, n0): XCD-aware bijective remap (blocks b, b + 8, ... share an XCD: each
// XCD walks one contiguous chunk of the tile order) + n-group tile order
__device__ __forceinline__ void w4_tile(int vb, int tiles_m, int tiles_n, int ngw, int& m0,
                                        int& n0) {
  const int nwg = tiles_m * tiles_n;
  const int xcd = vb & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (vb >> 3);
  int tm, tn;
  tile_coords(tile, tiles_m, tiles_n, ngw, tm, tn);
  m0 = tm * W4_TILE;
  n0 = tn * W4_TILE;
}

// Persistent: a grid of min(tiles, CUs) workgroups; workgroup b takes tiles vb = b, b + G,
// ... (G a multiple of 8 keeps each XCD on its chunk).  The next tile's K-tiles 0 and 1 are
// DMA'd into the stages while the current tile's epilogue runs (it reads no LDS), so a
// tile's prologue load latency is hidden behind the previous tile's epilogue.
template <int EPI, int SCHED = 1, int DG = 0>
__global__ __launch_bounds__(W4_T, 1) void gemm_tn_bf16_w4_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ Bt,
    int ldb, int tiles_m, int tiles_n, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int T = tiles_m * tiles_n, G = gridDim.x, nk = K / 64;
  int vb = blockIdx.x;
  if (vb >= T) return;                         // uniform per workgroup
  int m0, n0;
  w4_tile(vb, tiles_m, tiles_n, e.ngw, m0, n0);
  W4Src src;
  w4_sources(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane);
  w4_issue_k01(smem, src, wave, nk);
  for (;;) {
    // LayerNorm-fold row statistics of the wave's 128 rows (lane l holds rows l, 64 + l) and
    // the lane's bias / colsum columns: used in the epilogue only
    float2 lst[2] = {float2{0.f, 0.f}, float2{0.f, 0.f}};
    if ((EPI & W4_LNFOLD) != 0 || EPI == EPI_GENERIC) {
      lst[0] = e.lnstat[min(m0 + wm * 128 + lane, M - 1)];
      lst[1] = e.lnstat[min(m0 + wm * 128 + 64 + lane, M - 1)];
    }
    const int m_base = m0 + wm * 128, n_base = n0 + wn * 128;
    const bool full = m0 + W4_TILE <= M && n0 + W4_TILE <= N;
    W4Cols<EPI> cols;
    if constexpr (EPI != EPI_GENERIC) {
      if (full) w4_load_cols(cols, e, n_base, lane);
    }
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    w4_mainloop<SCHED, DG>(acc, smem, src, nk, wave, wm, wn, lane);
    // every wave passed the last K-step's barrier: no LDS read of this tile is pending
    const int vn = vb + G;
    const bool more = vn < T;
    int m1 = 0, n1 = 0;
    if (more) w4_tile(vn, tiles_m, tiles_n, e.ngw, m1, n1);
    if constexpr (EPI != EPI_GENERIC) {
      if (full) {
        W4Resid<EPI> rr;
        if constexpr (w4_resid_preloaded<EPI>()) {
#pragma unroll
          for (int i = 0; i < W4_RPRE; ++i) w4_load_resid<EPI>(rr, e, lane, m_base, n_base, i);
        }
        w4_epilogue_direct<EPI>(acc, lane, m_base, n_base, e, lst, cols, rr, [&] {
          if (more) {
            w4_sources(src, A, lda, M, Bt, ldb, N, m1, n1, wave, lane);
            w4_issue_k01(smem, src, wave, nk);
          }
        });
        if (!more) return;
        vb = vn;
        m0 = m1;
        n0 = n1;
        continue;
      }
    }
    // staged epilogue: it uses the stages, so the next tile's DMA waits for every wave
    w4_epilogue_generic(acc, reinterpret_cast<float*>(smem) + wave * 32 * W4_ES, lane, M, N,
                        m_base, n_base, e);
    if (!more) return;
    w4_fence();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    w4_barrier();
    vb = vn;
    m0 = m1;
    n0 = n1;
    w4_sources(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane);
    w4_issue_k01(smem, src, wave, nk);
  }
}

template <int C, int SCHED = 1, int DG = 0>
void w4_launch(dim3 g, hipStream_t stream, int M, int N, int K, const bf16_t* A, int lda,
               const bf16_t* Bt, int ldb, int tiles_m, int tiles_n, const EpiArgs& e) {
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
    (void)hipFuncSetAttribute(
        reinterpret_cast<const void*>(&gemm_tn_bf16_w4_kernel<C, SCHED, DG>),
        hipFuncAttributeMaxDynamicSharedMemorySize, W4_LDS);
  });
  hipLaunchKernelGGL((gemm_tn_bf16_w4_kernel<C, SCHED, DG>), g, dim3(W4_T), W4_LDS, stream, M, N,
                     K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
}

// K-step schedule (VTD_W4_SCHED, read per call: A/B in one process; both exact):
// 1 = one barrier per K-step, 2 = two (earlier DMA of tile kt + 2)
int w4_sched() {
  const char* v = getenv("VTD_W4_SCHED");
  return v && atoi(v) == 2 ? 2 : 1;
}


// ============================================================================
// "x4": the MX-fp8 GEMM (VTD_FP8 mode) on the w4 structure: A, Bt are
// OCP e4m3 bytes with one E8M0 scale per 32 K-elements (vtd_mx8.hip layout: scales
// s[k / 128][rows][4]); D += A Bt^T by v_mfma_scale_f32_16x16x128_f8f6f4.  One wave per
// SIMD, tile 256 x 256, K-step 128 elements = 128 B per row (the bf16 w4 staging byte for
// byte) + 1 KiB of A scales and 1 KiB of B scales per stage (lanes 0-15 of each wave DMA
// 256 B of each).  Accumulators, B-row permutation and the epilogues are w4's.
//
// A scaled MFMA consumes a whole K-step of both operands (32 B per lane: chunks fg and
// 4 + fg of the row, scale byte fg -- the convention the ping-pong MX kernel measured), so
// w4's double-buffered half-K-step fragments do not exist here.  Instead the wave's 128 x 128
// block is four quadrants of 16 MFMAs over operand halves A0 / A1 (row blocks 0-3 / 4-7)
// and B0 / B1 (column blocks 0-3 / 4-7), 4 x 36 VGPRs in all, walked in a zig-zag so that
// every half is re-read one or two quadrants before its next use:
//   K-step t, bf = the B half step t starts with (t even: B0, odd: B1), bs = the other:
//     q0 (A0, bf): read bs(t), A1(t)
//     q1 (A0, bs)
//     lgkmcnt(0); vmcnt(0); barrier     stage t & 1 read by every wave (WAR for tile t + 2),
//                                       tile t + 1 landed (RAW)
//     q2 (A1, bs): read A0(t + 1); DMA tile t + 2 -> stage t & 1
//     q3 (A1, bf): read bs(t + 1)      (= the half step t + 1 starts with)
// ============================================================================
constexpr int X4_SCL = 1024;                       // one operand's scales of a K-step
constexpr int X4_STAGE = 2 * W4_OPND + 2 * X4_SCL; // 66 KiB
constexpr int X4_LDS = 2 * X4_STAGE;               // 132 KiB

struct X4Src {
  __amdgpu_buffer_rsrc_t ra, rb, rsa, rsb, nul;   // nul: no records (every access out of range)
  int va, vb0, vb1;   // per lane: row lane >> 3 of a DMA piece + its swizzled chunk (B: pieces
                      // j with bit 1 of j clear / set)
  int vsa, vsb;       // per lane: the scale dword of row 64 w + l in a K-step
  int pa, pb;         // wave-uniform: bytes from the tile base to the wave's first row
  int lda, ldb, sa4, sb4;
};

// Rows past the matrix read as zero (out of the records: no clamping, no per-piece offsets)
__device__ __forceinline__ void x4_sources(X4Src& s, const uint8_t* A, int lda, int M,
                                           const uint8_t* sA, int64_t sa_rows, const uint8_t* Bt,
                                           int ldb, int N, const uint8_t* sB, int64_t sb_rows,
                                           int K, int m0, int n0, int wave, int lane) {
  const int64_t ra_bytes = (int64_t)(M - m0) * lda, rb_bytes = (int64_t)(N - n0) * ldb;
  s.ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(A + (int64_t)m0 * lda), 0,
                                           (int)std::min<int64_t>(ra_bytes, 0x7fffffff), 0x00020000);
  s.rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(Bt + (int64_t)n0 * ldb), 0,
                                           (int)std::min<int64_t>(rb_bytes, 0x7fffffff), 0x00020000);
  // scale rows past sa_rows / sb_rows fall outside the records (read as zero; never stored)
  s.rsa = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sA), 0,
                                            (int)std::min<int64_t>(sa_rows * K / 32, 0x7fffffff), 0x00020000);
  s.rsb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sB), 0,
                                            (int)std::min<int64_t>(sb_rows * K / 32, 0x7fffffff), 0x00020000);
  s.nul = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sA), 0, 0, 0x00020000);
  const int prow = lane >> 3, c = lane & 7;
  s.va = prow * lda + ((c ^ prow) << 4);
  s.vb0 = prow * ldb + ((c ^ prow) << 4);
  s.vb1 = prow * ldb + ((c ^ prow ^ 4) << 4);
  s.vsa = (m0 + wave * 64 + lane) * 4;
  s.vsb = (n0 + wave * 64 + lane) * 4;
  s.pa = wave * 64 * lda;
  s.pb = wave * 64 * ldb;
  s.lda = lda;
  s.ldb = ldb;
  s.sa4 = (int)(sa_rows * 4);
  s.sb4 = (int)(sb_rows * 4);
}

// DMA piece j (rows 64 w + 8 j .. + 7) of K-step kt of both operands; live = false: the
// same instructions against the empty descriptor (the loop's tail K-steps: nothing is read)
__device__ __forceinline__ void x4_dma(char* stage, const X4Src& s, int wave, int kt, int j,
                                       bool live = true) {
  char* da = stage + wave * 64 * 128 + j * 1024;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(live ? s.ra : s.nul, (w4_lds_t*)da, 16, s.va,
                                           s.pa + 8 * j * s.lda + kt * 128, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(live ? s.rb : s.nul, (w4_lds_t*)(da + W4_OPND), 16,
                                           ((j >> 1) & 1) ? s.vb1 : s.vb0,
                                           s.pb + 8 * j * s.ldb + kt * 128, 0, 0);
}
// the wave's 64 rows of A and B scales of K-step kt (one dword = one row per lane)
__device__ __forceinline__ void x4_dma_scales(char* stage, const X4Src& s, int wave, int kt,
                                              bool live = true) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(live ? s.rsa : s.nul,
                                           (w4_lds_t*)(stage + 2 * W4_OPND + wave * 256), 4, s.vsa,
                                           kt * s.sa4, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(live ? s.rsb : s.nul,
                                           (w4_lds_t*)(stage + 2 * W4_OPND + X4_SCL + wave * 256),
                                           4, s.vsb, kt * s.sb4, 0, 0);
}

typedef __attribute__((ext_vector_type(8))) int x4_i32x8;
// one operand half: 4 blocks x 32 B (chunks fg and 4 + fg of the row: one MFMA operand) +
// the lane's scale byte of each block's row
struct X4Half {
  x4_i32x8 v[4];
  int s[4];
};
// per-lane LDS offsets (block offsets are immediates)
struct X4Offs {
  int a0, a1;               // A row wm * 128 + fr: chunk fg / 4 + fg
  int b00, b01, b10, b11;   // B rows perm(0 / 1, fr): chunk fg (b0*) / 4 + fg (b1*)
  int sa, sb0, sb1;         // scale byte fg of A row wm * 128 + fr / B rows perm(0 / 1, fr)
};
template <int H>
__device__ __forceinline__ void x4_read_a(X4Half& h, const char* st, const X4Offs& o) {
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int i = 4 * H + b;
    h.v[b].lo = *reinterpret_cast<const i32x4*>(st + o.a0 + i * 16 * 128);
    h.v[b].hi = *reinterpret_cast<const i32x4*>(st + o.a1 + i * 16 * 128);
    h.s[b] = *reinterpret_cast<const uint8_t*>(st + 2 * W4_OPND + o.sa + i * 16 * 4);
  }
}
template <int H>
__device__ __forceinline__ void x4_read_b(X4Half& h, const char* st, const X4Offs& o) {
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int j = 4 * H + b;
    const int blk = (j >> 1) * 32;
    h.v[b].lo = *reinterpret_cast<const i32x4*>(st + W4_OPND + ((j & 1) ? o.b01 : o.b00) + blk * 128);
    h.v[b].hi = *reinterpret_cast<const i32x4*>(st + W4_OPND + ((j & 1) ? o.b11 : o.b10) + blk * 128);
    h.s[b] = *reinterpret_cast<const uint8_t*>(st + 2 * W4_OPND + X4_SCL +
                                               ((j & 1) ? o.sb1 : o.sb0) + blk * 4);
  }
}
// one MFMA row of a quadrant: output row block 4 HA + i, column blocks 4 HB .. 4 HB + 3
// (operands swapped as in w4: D = B-block x A-block^T; scale A = the B rows', scale B = the
// A rows').  Inline asm with the accumulator tied in place ("+a"): the builtin's AGPR form
// has no tied-accumulator variant, so the compiler rotates every result through a
// temporary quad with 4 copies and a 7-cycle hazard NOP per MFMA.  Hazards the compiler
// then no longer sees: a block's next accumulation is >= 16 MFMAs later, nothing but these
// instructions writes the accumulators in the K loop, and x4_mainloop ends with the
// wait states an MFMA result needs before the epilogue's AGPR reads.
template <int HA, int HB>
__device__ __forceinline__ void x4_mfma_row(f32x4 (&acc)[8][8], const X4Half& a, const X4Half& b,
                                            int i) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0]"
                 : "+a"(acc[4 * HA + i][4 * HB + j])
                 : "v"(b.v[j]), "v"(a.v[i]), "v"(b.s[j]), "v"(a.s[i]));
}

// K-step t (stage t & 1 holds tile t; a0 and bf, the B half (index HF) step t starts with,
// hold tile t).  Tile t + 2 is DMA'd when it exists (else the empty descriptor); tile t + 1's
// first halves are read into a0 and bs (B half HS: the half step t + 1 starts with; stale
// stage bytes after the last K-step, never used).  The caller swaps bf / bs every step.
// SCHED 1: one barrier (before q2), tile t + 2's DMA during q2 / q3 (one K-step to land).
// SCHED 2: a first barrier after q0 (stage t read by every wave: its DMA starts in q1) and
// the second before q2 (tile t + 1 landed: vmcnt counts the 6 DMAs issued in q1): 1.25
// K-steps to land.
template <int HF, int DG, int SCHED>
__device__ __forceinline__ void x4_kstep(f32x4 (&acc)[8][8], X4Half& a0, X4Half& a1, X4Half& bf,
                                         X4Half& bs, char* smem, const X4Src& src, int t, int nk,
                                         int wave, int lane, const X4Offs& o) {
  constexpr int HS = 1 - HF;
  char* st = smem + (t & 1) * X4_STAGE;
  const char* nx = smem + ((t + 1) & 1) * X4_STAGE;
  const bool pf = t + 2 < nk && !(DG & 1);
  w4_fence();
  // q0 (A0, bf): read bs(t), A1(t)
  x4_read_b<HS>(bs, st, o);
  x4_read_a<1>(a1, st, o);
#pragma unroll
  for (int i = 0; i < 4; ++i) x4_mfma_row<0, HF>(acc, a0, bf, i);
  w4_fence();
  if constexpr (SCHED == 2) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    w4_barrier();                                     // stage t free
    x4_dma_scales(st, src, wave, t + 2, pf);
  }
  // q1 (A0, bs)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (SCHED == 2 && i < 2) x4_dma(st, src, wave, t + 2, i, pf);
    x4_mfma_row<0, HS>(acc, a0, bs, i);
    w4_fence();
  }
  if constexpr (SCHED == 2) {
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // tile t + 1 (older than q1's 6)
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile t + 1 (the only DMA in flight)
  }
  w4_barrier();
  // q2 (A1, bs): read A0(t + 1), DMA tile t + 2
  x4_read_a<0>(a0, nx, o);
  if (SCHED == 1) x4_dma_scales(st, src, wave, t + 2, pf);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (SCHED == 1) x4_dma(st, src, wave, t + 2, i, pf);
    else if (i < 3) x4_dma(st, src, wave, t + 2, 2 + i, pf);
    x4_mfma_row<1, HS>(acc, a1, bs, i);
    w4_fence();
  }
  // q3 (A1, bf): read bs(t + 1) (bs's last use was q2)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (SCHED == 1) x4_dma(st, src, wave, t + 2, 4 + i, pf);
    else if (i < 3) x4_dma(st, src, wave, t + 2, 5 + i, pf);
    if (i == 0) x4_read_b<HS>(bs, nx, o);
    x4_mfma_row<1, HF>(acc, a1, bf, i);
    w4_fence();
  }
}

// K-tiles 0 and 1 of a tile into stages 0 and 1 (the stages must be free)
__device__ __forceinline__ void x4_issue_k01(char* smem, const X4Src& src, int wave, int lane,
                                             int nk) {
  x4_dma_scales(smem, src, wave, 0);
#pragma unroll
  for (int j = 0; j < 8; ++j) x4_dma(smem, src, wave, 0, j);
  if (nk > 1) {
    x4_dma_scales(smem + X4_STAGE, src, wave, 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) x4_dma(smem + X4_STAGE, src, wave, 1, j);
  }
}

template <int DG, int SCHED>
__device__ __forceinline__ void x4_mainloop(f32x4 (&acc)[8][8], char* smem, const X4Src& src,
                                            int nk, int wave, int wm, int wn, int lane) {
  const int fr = lane & 15, fg = lane >> 4;
  X4Offs o;
  o.a0 = w4_swz_a(wm * 128 + fr, fg);
  o.a1 = w4_swz_a(wm * 128 + fr, 4 + fg);
  const int brow0 = wn * 128 + w4_perm(0, fr), brow1 = wn * 128 + w4_perm(1, fr);
  o.b00 = w4_swz_b(brow0, fg);
  o.b01 = w4_swz_b(brow1, fg);
  o.b10 = w4_swz_b(brow0, 4 + fg);
  o.b11 = w4_swz_b(brow1, 4 + fg);
  o.sa = 4 * (wm * 128 + fr) + fg;
  o.sb0 = 4 * brow0 + fg;
  o.sb1 = 4 * brow1 + fg;
  // K-tile 0 retired (K-tile 1's DMA, or more, is younger), every wave's part visible
  if (nk > 1) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  w4_barrier();
  asm volatile("s_nop 4" ::: "memory");            // accumulator init -> first MFMA srcC
  X4Half a0, a1, b0, b1;
  x4_read_a<0>(a0, smem, o);
  x4_read_b<0>(b0, smem, o);
  // even steps start with B half 0 (bf = b0), odd steps with B half 1 (bf = b1)
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    x4_kstep<0, DG, SCHED>(acc, a0, a1, b0, b1, smem, src, t, nk, wave, lane, o);
    x4_kstep<1, DG, SCHED>(acc, a0, a1, b1, b0, smem, src, t + 1, nk, wave, lane, o);
  }
  if (t < nk) x4_kstep<0, DG, SCHED>(acc, a0, a1, b0, b1, smem, src, t, nk, wave, lane, o);
  // the last MFMAs' results: wait states before any AGPR read (XDL write -> VALU read)
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
}

// Persistent like the w4 kernel (the next tile's K-tiles 0 and 1 are DMA'd during the
// current tile's register-direct epilogue).
// DG (VTD_DIAG builds only; timing diagnostics, WRONG outputs): bit 0 = no DMA after a tile's
// first two K-tiles (the K loop reads stale stages), bit 1 = no epilogue (nothing stored)
template <int EPI, int SCHED, int DG = 0>
__global__ __launch_bounds__(W4_T, 1) void gemm_mx8_x4_kernel(
    int M, int N, int K, const uint8_t* __restrict__ A, int lda, const uint8_t* __restrict__ sA,
    int64_t sa_rows, const uint8_t* __restrict__ Bt, int ldb, const uint8_t* __restrict__ sB,
    int64_t sb_rows, int tiles_m, int tiles_n, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int T = tiles_m * tiles_n, G = gridDim.x, nk = K / 128;
  int vb = blockIdx.x;
  if (vb >= T) return;
  int m0, n0;
  w4_tile(vb, tiles_m, tiles_n, e.ngw, m0, n0);
  X4Src src;
  x4_sources(src, A, lda, M, sA, sa_rows, Bt, ldb, N, sB, sb_rows, K, m0, n0, wave, lane);
  x4_issue_k01(smem, src, wave, lane, nk);
  for (;;) {
    const int m_base = m0 + wm * 128, n_base = n0 + wn * 128;
    const bool full = m0 + W4_TILE <= M && n0 + W4_TILE <= N;
    W4Cols<EPI> cols;
    if constexpr (EPI != EPI_GENERIC) {
      if (full) w4_load_cols(cols, e, n_base, lane);
    }
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    x4_mainloop<DG, SCHED>(acc, smem, src, nk, wave, wm, wn, lane);
    const int vn = vb + G;
    const bool more = vn < T;
    int m1 = 0, n1 = 0;
    if (more) w4_tile(vn, tiles_m, tiles_n, e.ngw, m1, n1);
    if constexpr (DG & 2) {
      if (!more) return;
      vb = vn;
      m0 = m1;
      n0 = n1;
      x4_sources(src, A, lda, M, sA, sa_rows, Bt, ldb, N, sB, sb_rows, K, m0, n0, wave, lane);
      x4_issue_k01(smem, src, wave, lane, nk);
      continue;
    }
    if constexpr (EPI != EPI_GENERIC) {
      if (full) {
        W4Resid<EPI> rr;
        if constexpr (w4_resid_preloaded<EPI>()) {
#pragma unroll
          for (int i = 0; i < W4_RPRE; ++i) w4_load_resid<EPI>(rr, e, lane, m_base, n_base, i);
        }
        w4_epilogue_direct<EPI>(acc, lane, m_base, n_base, e, nullptr, cols, rr, [&] {
          if (more) {
            x4_sources(src, A, lda, M, sA, sa_rows, Bt, ldb, N, sB, sb_rows, K, m1, n1, wave,
                       lane);
            x4_issue_k01(smem, src, wave, lane, nk);
          }
        });
        if (!more) return;
        vb = vn;
        m0 = m1;
        n0 = n1;
        continue;
      }
    }
    w4_epilogue_generic(acc, reinterpret_cast<float*>(smem) + wave * 32 * W4_ES, lane, M, N,
                        m_base, n_base, e);
    if (!more) return;
    w4_fence();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    w4_barrier();
    vb = vn;
    m0 = m1;
    n0 = n1;
    x4_sources(src, A, lda, M, sA, sa_rows, Bt, ldb, N, sB, sb_rows, K, m0, n0, wave, lane);
    x4_issue_k01(smem, src, wave, lane, nk);
  }
}

template <int C, int SCHED, int DG = 0>
void x4_launch(dim3 g, hipStream_t stream, int M, int N, int K, const uint8_t* A, int lda,
               const uint8_t* sA, int64_t sa_rows, const uint8_t* Bt, int ldb, const uint8_t* sB,
               int64_t sb_rows, int tiles_m, int tiles_n, const EpiArgs& e) {
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_mx8_x4_kernel<C, SCHED, DG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, X4_LDS);
  });
  hipLaunchKernelGGL((gemm_mx8_x4_kernel<C, SCHED, DG>), g, dim3(W4_T), X4_LDS, stream, M, N, K, A, lda, sA,
                     sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);
}
// x4 K-step schedule (VTD_X4_SCHED, read per call; both exact): 1 = one barrier per K-step,
// 2 = two (the next-but-one K-tile's DMA starts a quadrant earlier)
int x4_sched() {
  const char* v = getenv("VTD_X4_SCHED");
  return v && atoi(v) == 1 ? 1 : 2;
}

}  // namespace

// The w4 GEMM for a bf16 problem (the caller checked shapes / dtypes and finalized any
// LayerNorm partials into epi->lnstat).  Returns false when it does not apply.
bool gemm_w4_launch(int M, int N, int K, const bf16_t* A, int lda, const bf16_t* Bt, int ldb,
                    const vtd_epilogue* epi, int ngw, hipStream_t stream) {
  // no split-bf16 (VTD_BF16X3) output epilogue here: the caller's pp2 path writes it
  if (epi->out_dtype == VTD_BF16X3) return false;
  EpiArgs e = make_epi_args(epi);
  e.ngw = ngw;
  auto a16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  const bool fast = e.bias && !e.dets && e.scatter_tokens <= 0 && e.ldo % 8 == 0 &&
                    (!e.resid || e.ldr % 8 == 0) && a16(e.out) && a16(e.bias) &&
                    (!e.resid || a16(e.resid)) && (!e.out2 || (e.ldo2 % 8 == 0 && a16(e.out2)));
  // the LayerNorm fold is a compile-time epilogue property (bit 16): its column sums and a
  // residual never share a kernel (no forward layer has both: those go the generic way)
  const int code = fast && !(e.lnstat && e.resid)
                       ? epi_code(e.act, e.out_dtype == VTD_BF16, e.resid != nullptr) |
                             (e.lnstat ? W4_LNFOLD : 0)
                       : EPI_GENERIC;
  const int tiles_m = (M + W4_TILE - 1) / W4_TILE, tiles_n = (N + W4_TILE - 1) / W4_TILE;
  const dim3 g(std::min(tiles_m * tiles_n, device_cu_count()));
#if VTD_DIAG
  // timing diagnostics (wrong outputs), plain bf16 epilogue only: VTD_W4_DG = 1 / 2
  if (const char* dg = getenv("VTD_W4_DG"); dg && atoi(dg) > 0 && code == 4) {
    const int d = atoi(dg);
    if (d == 1) w4_launch<4, 1, 1>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
    else if (d == 2) w4_launch<4, 1, 2>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
    else if (d == 3) w4_launch<4, 2, 1>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
    else w4_launch<4, 2, 2>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
    return true;
  }
#endif
#ifndef VTD_X4_ONLY   // (build-speed aid for the x4 kernel's register tuning)
  const int sched = w4_sched();
  switch (code) {
#define VTD_W4_CASE(C)                                                                       \
  case C:                                                                                    \
    if (sched == 2) w4_launch<C, 2>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e); \
    else w4_launch<C, 1>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);          \
    break;
    VTD_W4_CASE(0) VTD_W4_CASE(1) VTD_W4_CASE(2) VTD_W4_CASE(4) VTD_W4_CASE(5) VTD_W4_CASE(6)
    VTD_W4_CASE(8) VTD_W4_CASE(9) VTD_W4_CASE(10) VTD_W4_CASE(12) VTD_W4_CASE(13)
    VTD_W4_CASE(14) VTD_W4_CASE(16) VTD_W4_CASE(17) VTD_W4_CASE(18) VTD_W4_CASE(20)
    VTD_W4_CASE(21) VTD_W4_CASE(22)
#undef VTD_W4_CASE
    default:
      if (sched == 2) w4_launch<EPI_GENERIC, 2>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
      else w4_launch<EPI_GENERIC, 1>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
  }
#endif
  return true;
}

// The x4 MX-fp8 GEMM (the caller checked shapes and the fp8-output conditions).
void gemm_mx8_x4_launch(int M, int N, int K, const uint8_t* A, int lda, const uint8_t* sA,
                        int64_t sa_rows, const uint8_t* Bt, int ldb, const uint8_t* sB,
                        int64_t sb_rows, const vtd_epilogue* epi, int ngw, hipStream_t stream) {
  EpiArgs e = make_epi_args(epi);
  e.ngw = ngw;
  auto a16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  const bool fast = e.bias && !e.dets && !e.lnstat && e.scatter_tokens <= 0 && e.ldo % 8 == 0 &&
                    (!e.resid || e.ldr % 8 == 0) && a16(e.out) && a16(e.bias) &&
                    (!e.resid || a16(e.resid)) && (!e.out2 || (e.ldo2 % 8 == 0 && a16(e.out2)));
  const bool fp8out = e.out_dtype == VTD_FP8;
  const int code = fast ? epi_code(e.act, e.out_dtype != VTD_F32, e.resid != nullptr) |
                              (fp8out ? W4_FP8OUT : 0)
                        : EPI_GENERIC;
  const int tiles_m = (M + W4_TILE - 1) / W4_TILE, tiles_n = (N + W4_TILE - 1) / W4_TILE;
  const dim3 g(std::min(tiles_m * tiles_n, device_cu_count()));
  const int sched = x4_sched();
#if VTD_DIAG
  // timing diagnostics (wrong outputs), plain bf16 epilogue only: VTD_X4_DG = 1 / 2 / 3
  if (const char* dg = getenv("VTD_X4_DG"); dg && atoi(dg) > 0 && code == 4) {
    const int d = atoi(dg);
    if (d == 1) x4_launch<4, 1, 1>(g, stream, M, N, K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);
    else if (d == 2) x4_launch<4, 1, 2>(g, stream, M, N, K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);
    else x4_launch<4, 1, 3>(g, stream, M, N, K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);
    return;
  }
#endif
#ifdef VTD_X4_ONLY
  if (code == 4) {
    if (x4_sched() == 2) x4_launch<4, 2>(g, stream, M, N, K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);
    else x4_launch<4, 1>(g, stream, M, N, K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows, tiles_m, tiles_n, e);
    return;
  }
#endif
  switch (code) {
#define VTD_X4_CASE(C)                                                                     \
  case C:                                                                                  \
    if (sched == 2)                                                                        \
      x4_launch<C, 2>(g, stream, M, N, K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows,       \
                      tiles_m, tiles_n, e);                                                \
    else                                                                                   \
      x4_launch<C, 1>(g, stream, M, N, K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows,       \
                      tiles_m, tiles_n, e);                                                \
    break;
#ifndef VTD_X4_ONLY
    VTD_X4_CASE(0) VTD_X4_CASE(1) VTD_X4_CASE(2) VTD_X4_CASE(4) VTD_X4_CASE(5) VTD_X4_CASE(6)
    VTD_X4_CASE(8) VTD_X4_CASE(9) VTD_X4_CASE(10) VTD_X4_CASE(12) VTD_X4_CASE(13)
    VTD_X4_CASE(14) VTD_X4_CASE(36) VTD_X4_CASE(37) VTD_X4_CASE(38)
#endif
#undef VTD_X4_CASE
    default:
      if (sched == 2)
        x4_launch<EPI_GENERIC, 2>(g, stream, M, N, K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows,
                                  tiles_m, tiles_n, e);
      else
        x4_launch<EPI_GENERIC, 1>(g, stream, M, N, K, A, lda, sA, sa_rows, Bt, ldb, sB, sb_rows,
                                  tiles_m, tiles_n, e);
  }
}

}  // namespace vtd
