// "w4": the bf16 Dense-layer GEMM with ONE wave per SIMD (vtd.py:297, 364-412, 454-493 as
// C = act(A Bt^T + bias + rowadd) + resid; A [M][lda] and Bt [N][ldb] both K-contiguous).
//
// Tile 256 x 256, BK = 64, 256 threads = 4 waves in 2 (M) x 2 (N); each wave owns a
// 128 x 128 output block = 8 x 8 blocks of v_mfma_f32_16x16x32_bf16, 256 fp32 accumulators
// per lane (the register file is 512 per lane at one wave per SIMD: accumulators in AGPRs,
// two fragment sets and the DMA offsets in VGPRs).  Against the 8-wave ping-pong pp2 tile
// (128 x 64 per wave) every operand byte read from LDS feeds twice the MFMA work (128 KiB
// of LDS reads per K-step instead of 192) and a K-step is 2 barriers instead of 8.
//
// Staging: both operands HBM/L2 -> LDS by buffer_load_dwordx4 ... lds (1 KiB = 8 rows of
// 128 B per wave-instruction, 16 per wave per K-step), two 64 KiB stages.  LDS rows are
// 128 B with the 16-B chunk XOR-swizzled (A: chunk ^ (row & 7); B: the permuted-read
// swizzle below), applied on the per-lane SOURCE address so the LDS image stays
// lane-linear.  Fragments are double-buffered in registers (F0 = k 0..31 of a K-step,
// F1 = k 32..63).  One K-step (kt, stage s = kt & 1):
//
//   MFMA F0: 8, read F1(kt)          16 ds_read_b128
//   MFMA F0: 8                       (F1's reads land meanwhile)
//   lgkmcnt(0); barrier A            every wave has read all of stage s  (WAR)
//   MFMA F0: 48, DMA tile kt+2 -> s  16 DMA instructions, 4 per 8 MFMAs
//   vmcnt(16 | 0); barrier B         tile kt+1 (stage s^1) landed for every wave (RAW)
//   MFMA F1: 64, read F0(kt+1)       2 reads per 8 MFMAs
//
// Tile kt + 2's DMA is issued right after barrier A of K-step kt and retired at barrier B
// of K-step kt + 1: about 1.3 K-steps in flight.  Counted waits are inline asm and barriers raw s_barrier
// (a __syncthreads() fence would drain the in-flight DMA).
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

// One K-step (see the file comment).  PF: tile kt + 2 exists (DMA it); NN: tile kt + 1
// exists (read its first fragments).  Compile-time flags: no branch inside the step.
template <bool PF, bool NN, int DG>
__device__ __forceinline__ void w4_kstep0(f32x4 (&acc)[8][8], W4Frag& f0, W4Frag& f1, char* smem,
                                         const W4Src& src, int kt, int wave, int aoff0,
                                         int aoff1, int b00, int b01, int b10, int b11) {
  char* st = smem + (kt & 1) * W4_STAGE;
  char* nx = smem + ((kt + 1) & 1) * W4_STAGE;
  w4_fence();
  // ---- first quarter of F0's MFMAs, F1 reads (after the first row: the compiler's wait for
  // F0's last reads of the previous step then does not also wait for these)
  w4_mfma_row(acc, f0, 0);
  w4_fence();
#pragma unroll
  for (int g = 0; g < 8; ++g) w4_read2(f1, st, g, aoff1, b10, b11);
  w4_fence();
  w4_mfma_row(acc, f0, 1);
  w4_fence();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  w4_barrier();                                // A: stage st fully read by every wave
  // ---- the rest of F0, DMA of tile kt + 2 into stage st (4 instructions per 8 MFMAs)
#pragma unroll
  for (int i = 2; i < 8; ++i) {
    if (PF && !(DG & 1) && i < 6) {
      w4_dma(st, src, wave, (DG & 2) ? 0 : kt + 2, 2 * (i - 2));
      w4_dma(st, src, wave, (DG & 2) ? 0 : kt + 2, 2 * (i - 2) + 1);
    }
    w4_mfma_row(acc, f0, i);
    w4_fence();
  }
  w4_fence();
  if (PF) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  w4_barrier();                                // B: tile kt + 1 landed for every wave
  // ---- F1's MFMAs, F0 reads of tile kt + 1 (B fragments first: the next K-step's first
  // MFMA row needs all 8 of them)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (NN) w4_read2(f0, nx, i, aoff0, b00, b01);
    w4_mfma_row(acc, f1, i);
    w4_fence();
  }
}

// Schedule 1: one barrier per K-step.  F1(kt) is read during F0(kt)'s MFMAs; the barrier
// then retires both every wave's reads of stage st (WAR for tile kt + 2's DMA, issued during
// F1's MFMAs) and tile kt + 1's DMA (RAW for F0(kt + 1)'s reads, also during F1's MFMAs).
template <bool PF, bool NN, int DG>
__device__ __forceinline__ void w4_kstep1(f32x4 (&acc)[8][8], W4Frag& f0, W4Frag& f1, char* smem,
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

template <int SCHED, int DG>
__device__ __forceinline__ void w4_mainloop(f32x4 (&acc)[8][8], char* smem, const W4Src& src,
                                            int nk, int wave, int wm, int wn, int lane) {
  const int fr = lane & 15, fg = lane >> 4;
  // per-lane LDS offsets of the two K-halves' fragments (block offsets are immediates)
  const int aoff0 = w4_swz_a(wm * 128 + fr, fg), aoff1 = w4_swz_a(wm * 128 + fr, 4 + fg);
  const int brow0 = wn * 128 + w4_perm(0, fr), brow1 = wn * 128 + w4_perm(1, fr);
  const int b00 = w4_swz_b(brow0, fg), b01 = w4_swz_b(brow1, fg);          // K-half 0
  const int b10 = w4_swz_b(brow0, 4 + fg), b11 = w4_swz_b(brow1, 4 + fg);  // K-half 1

  // prologue: tiles 0 and 1 in flight, tile 0 landed
#pragma unroll
  for (int j = 0; j < 8; ++j) w4_dma(smem, src, wave, 0, j);
  if (nk > 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) w4_dma(smem + W4_STAGE, src, wave, 1, j);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  w4_barrier();
  W4Frag f0, f1;
#pragma unroll
  for (int g = 0; g < 8; ++g) w4_read2(f0, smem, g, aoff0, b00, b01);
  int kt = 0;
#define VTD_W4_STEP(PF, NN)                                                                    \
  if constexpr (SCHED == 0)                                                                    \
    w4_kstep0<PF, NN, DG>(acc, f0, f1, smem, src, kt, wave, aoff0, aoff1, b00, b01, b10, b11); \
  else                                                                                         \
    w4_kstep1<PF, NN, DG>(acc, f0, f1, smem, src, kt, wave, aoff0, aoff1, b00, b01, b10, b11);
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
template <int EPI>
__device__ __forceinline__ void w4_epilogue_direct(const f32x4 (&acc)[8][8], int lane, int m_base,
                                                   int n_base, const EpiArgs& e,
                                                   const float2* lst) {
  constexpr int ACT = EPI & 3;
  constexpr bool OUT_BF16 = (EPI & 4) != 0;
  constexpr bool RESID = (EPI & 8) != 0;
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w4_fence();                    // one row block at a time: no hoisted accumulator copies
    const int lr = 16 * i + fr, mrow = m_base + lr;
    f32x4 rv[4][2];
    if constexpr (RESID) {
#pragma unroll
      for (int jp = 0; jp < 4; ++jp)
        load_resid8<OUT_BF16>(e, (int64_t)mrow * e.ldr + n_base + 32 * jp + 8 * fg, rv[jp][0],
                              rv[jp][1]);
    }
    float tsum[2] = {0.f, 0.f};
    i32x4 ob[4];
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      f32x4 v0 = w4_acc(acc[i][2 * jp]), v1 = w4_acc(acc[i][2 * jp + 1]);
      const int ncol = n_base + 32 * jp + 8 * fg;
      // bias / colsum re-read per row block (L1 hits): keeps 64 registers free
      if (e.lnstat)
        epi_lnfold8(e, lst, mrow, lr, *reinterpret_cast<const f32x4*>(e.colsum + ncol),
                    *reinterpret_cast<const f32x4*>(e.colsum + ncol + 4), v0, v1);
      v0 += *reinterpret_cast<const f32x4*>(e.bias + ncol);
      v1 += *reinterpret_cast<const f32x4*>(e.bias + ncol + 4);
      if (e.rowadd) epi_rowadd8(e, mrow, ncol, v0, v1);
      act_ct8<ACT>(v0, v1);
      if constexpr (RESID) {
        v0 += rv[jp][0];
        v1 += rv[jp][1];
      }
      if (e.out2) epi_out2_8(e, mrow, ncol, v0, v1);
      const int64_t idx = (int64_t)mrow * e.ldo + ncol;
      if constexpr (OUT_BF16) {
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
    if (OUT_BF16 && e.statout) {
      // LayerNorm partials of the two 64-column blocks: a block's 64 values of this row are
      // in lanes fr, fr + 16, + 32, + 48 (jp = 2 b, 2 b + 1)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const float mean = xsum32(xsum16(tsum[b])) * (1.f / 64.f);
        const float m2 =
            xsum32(xsum16(bf16x8_m2(ob[2 * b], mean) + bf16x8_m2(ob[2 * b + 1], mean)));
        if (fg == 0)
          e.statout[(int64_t)mrow * e.stat_ld + (n_base >> 6) + b] = float2{mean, m2};
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

template <int EPI, int SCHED = 1, int DG = 0>
__global__ __launch_bounds__(W4_T, 1) void gemm_tn_bf16_w4_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ Bt,
    int ldb, int tiles_m, int tiles_n, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware bijective remap (blocks b, b + 8, ... share an XCD) + n-group tile order
  const int nwg = tiles_m * tiles_n, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int tm, tn;
  tile_coords(tile, tiles_m, tiles_n, e.ngw, tm, tn);
  const int m0 = tm * W4_TILE, n0 = tn * W4_TILE;
  W4Src src;
  w4_sources(src, A, lda, M, Bt, ldb, N, m0, n0, wave, lane);
  // LayerNorm-fold row statistics of the wave's 128 rows (oldest vector-memory ops: the
  // prologue's counted wait retires them); lane l holds rows l and 64 + l
  float2 lst[2] = {float2{0.f, 0.f}, float2{0.f, 0.f}};
  if (e.lnstat) {
    lst[0] = e.lnstat[min(m0 + wm * 128 + lane, M - 1)];
    lst[1] = e.lnstat[min(m0 + wm * 128 + 64 + lane, M - 1)];
  }
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  w4_mainloop<SCHED, DG>(acc, smem, src, K / 64, wave, wm, wn, lane);
  const int m_base = m0 + wm * 128, n_base = n0 + wn * 128;
  if constexpr (EPI != EPI_GENERIC) {
    if (m0 + W4_TILE <= M && n0 + W4_TILE <= N) {
      w4_epilogue_direct<EPI>(acc, lane, m_base, n_base, e, lst);
      return;
    }
  }
  w4_epilogue_generic(acc, reinterpret_cast<float*>(smem) + wave * 32 * W4_ES, lane, M, N,
                      m_base, n_base, e);
}

template <int C, int SCHED, int DG = 0>
void w4_launch(dim3 g, hipStream_t stream, int M, int N, int K, const bf16_t* A, int lda,
               const bf16_t* Bt, int ldb, int tiles_m, int tiles_n, const EpiArgs& e) {
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_bf16_w4_kernel<C, SCHED, DG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, W4_LDS);
  });
  hipLaunchKernelGGL((gemm_tn_bf16_w4_kernel<C, SCHED, DG>), g, dim3(W4_T), W4_LDS, stream, M, N,
                     K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
}

// K-loop schedule (VTD_W4_SCHED, read per call: A/B in one process; both exact):
// 1 = one barrier per K-step (default), 0 = two barriers per K-step
int w4_sched() {
  const char* v = getenv("VTD_W4_SCHED");
  return v && atoi(v) == 0 ? 0 : 1;
}

}  // namespace

// The w4 GEMM for a bf16 problem (the caller checked shapes / dtypes and finalized any
// LayerNorm partials into epi->lnstat).  Returns false when it does not apply.
bool gemm_w4_launch(int M, int N, int K, const bf16_t* A, int lda, const bf16_t* Bt, int ldb,
                    const vtd_epilogue* epi, int ngw, hipStream_t stream) {
  EpiArgs e = make_epi_args(epi);
  e.ngw = ngw;
  auto a16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  const bool fast = e.bias && !e.dets && e.scatter_tokens <= 0 && e.ldo % 8 == 0 &&
                    (!e.resid || e.ldr % 8 == 0) && a16(e.out) && a16(e.bias) &&
                    (!e.resid || a16(e.resid)) && (!e.out2 || (e.ldo2 % 8 == 0 && a16(e.out2)));
  const int code = fast ? epi_code(e.act, e.out_dtype == VTD_BF16, e.resid != nullptr)
                        : EPI_GENERIC;
  const int tiles_m = (M + W4_TILE - 1) / W4_TILE, tiles_n = (N + W4_TILE - 1) / W4_TILE;
  const dim3 g(tiles_m * tiles_n);
#if VTD_DIAG
  // timing diagnostics (wrong outputs), plain bf16 epilogue only: VTD_W4_DG = 1 / 2 / 3
  if (const char* dg = getenv("VTD_W4_DG"); dg && atoi(dg) > 0 && code == 4) {
    const int d = atoi(dg);
    if (d == 1) w4_launch<4, 1, 1>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
    else if (d == 2) w4_launch<4, 1, 2>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
    else w4_launch<4, 0, 1>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
    return true;
  }
#endif
  const int sched = w4_sched();
  switch (code) {
#define VTD_W4_CASE(C)                                                                        \
  case C:                                                                                     \
    if (sched == 1) w4_launch<C, 1>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e); \
    else w4_launch<C, 0>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);          \
    break;
    VTD_W4_CASE(0) VTD_W4_CASE(1) VTD_W4_CASE(2) VTD_W4_CASE(4) VTD_W4_CASE(5) VTD_W4_CASE(6)
    VTD_W4_CASE(8) VTD_W4_CASE(9) VTD_W4_CASE(10) VTD_W4_CASE(12) VTD_W4_CASE(13)
    VTD_W4_CASE(14)
#undef VTD_W4_CASE
    default:
      if (sched == 1)
        w4_launch<EPI_GENERIC, 1>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
      else
        w4_launch<EPI_GENERIC, 0>(g, stream, M, N, K, A, lda, Bt, ldb, tiles_m, tiles_n, e);
  }
  return true;
}

}  // namespace vtd
