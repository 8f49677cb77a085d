// Persistent bf16 GEMM ("pp3") for the Dense layers of the detector (vtd.py:297,
// 364-369 EinsumDense, 389-403, 472-483): C = act(A Bt^T + bias) (+ resid), fast
// epilogues only (bias, GELU/Mish, bf16 or f32 out, f32 residual).  Same tile geometry
// and ping-pong wave groups as the non-persistent kernels in vtd_gemm.hip.
#include <stdlib.h>

#include <algorithm>

#include "vtd_common.h"

namespace vtd {

namespace {

constexpr int BBM = 256, BBN = 256, BNT = 512;
constexpr int BSTAGE = 65536;                 // 64 KiB per stage

typedef __attribute__((address_space(3))) void lds_void_t;

struct P3Epi {
  const float* bias;
  const float* resid; int ldr;
  void* out; int ldo;
};

template <int ACT>
__device__ __forceinline__ float act_ct(float x) {
  if constexpr (ACT == VTD_ACT_GELU_TANH) return act_gelu(x);
  else if constexpr (ACT == VTD_ACT_MISH) return act_mish(x);
  else return x;
}
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

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// ============================================================================
// pp3: persistent 256 x 256 ping-pong kernel with ONE DMA pipeline across tiles.
// gridDim.x blocks (one per CU) walk tiles t = blockIdx.x, +gridDim.x, ... (XCD-remapped
// as above); the K-tiles of all of a block's tiles form one global step sequence g, and
// the DMA of steps g+1 / g+2 is issued during step g whether or not it belongs to the
// next tile, so a tile boundary costs no prologue burst.  The epilogue (registers ->
// global, transposed accumulators, no LDS) is inserted between two steps, with both
// wave groups re-aligned for it; its stores are left in flight and drain under the
// next tile's first ~1.25 K-tiles.  The bias comes from an LDS table filled once per
// launch.
//
// LDS stage (64 KiB) = four 16 KiB DMA groups split by K HALF: GA0 = A rows 0-255,
// k 0-31; GA1 = A, k 32-63; GB0, GB1 likewise for B.  A group row is 64 B; position
// p of logical 16-B chunk c in row r is c ^ (((r >> 3) & 1) << 1), conflict-free for the
// plain A-fragment reads and the permuted B-fragment reads under ds_read_b128's lane
// groups (exhaustive check: tools/swizzle_check.py).
// A K-tile is 4 phases of 16 MFMAs per wave (k-half s, A row blocks lo = 0-3 / hi = 4-7):
//   L0: read A lo s0 + B s0 (8 ds_read_b128) | DMA GB1(g+1) | C0: acc[0..3][*]
//   L1: read A hi s0 (4)        | DMA GA1(g+1) | wait -> GA1(g), GB1(g) | C1: acc[4..7][*]
//   L2: read A lo s1 + B s1 (8) | DMA GB0(g+2) | C2: acc[0..3][*]
//   L3: read A hi s1 (4)        | DMA GA0(g+2) | wait -> GA0(g+1), GB0(g+1) | C3
// Operand registers: one A part (16) + one B part (16).  Every refill is issued 2
// phases after the last read of the group it overwrites (WAR across the staggered
// groups), and every read is at least one phase after the wait that retires it (RAW);
// event numbering as in the pp2 comment.  Each wait has exactly 8 younger DMA
// instructions in steady state; the first step after an epilogue adds its S stores.
// ============================================================================
constexpr int P3_GA0 = 0, P3_GA1 = 16384, P3_GB0 = 32768, P3_GB1 = 49152;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pp3_rsrc(const bf16_t* base, int row0,
                                                           int rows, int ld) {
  // rows past the operand's end read as zero (buffer range check on the row offset)
  const int64_t bytes = (int64_t)(rows - row0) * ld * 2;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(base + (int64_t)row0 * ld), 0,
                                           (int)std::min<int64_t>(bytes, 0x7fffffff),
                                           0x00020000);
}

template <int GRP>
__device__ __forceinline__ void pp3_issue(char* smem, __amdgpu_buffer_rsrc_t rs, int off0,
                                          int off1, int stage, int kt, int wave) {
  char* dst = smem + stage * BSTAGE + GRP * 16384 + wave * 2048;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)dst, 16, off0,
                                           kt * 128 + (GRP & 1) * 64, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + 1024), 16, off1,
                                           kt * 128 + (GRP & 1) * 64, 0, 0);
}

template <int I0>
__device__ __forceinline__ void pp3_mfma(f32x4 (&acc)[8][4], const bf16x8 (&a)[4],
                                         const bf16x8 (&b)[4]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      acc[I0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[I0 + i][j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}
// Residual loads are inline asm: a VGPR-destination load the compiler can see inside the
// persistent loop makes its waitcnt pass put an s_waitcnt vmcnt(0) at the loop head
// (draining the DMA pipeline every K-step).  The block issues its loads and waits for
// them (vmcnt(0): also retires the DMA in flight, issued >= 1 phase earlier) before
// returning the values, so no value is read before it landed.  (The bias comes from an
// LDS table filled at kernel start.)
// residual rows of one 4-block chunk: 16 loads in flight, then one wait
__device__ __forceinline__ void p3_load_resid(f32x4 (&rv)[4][2][2], const float* const (&p)[4][2]) {
  asm volatile(
      "global_load_dwordx4 %0, %16, off\n\t"
      "global_load_dwordx4 %1, %16, off offset:16\n\t"
      "global_load_dwordx4 %2, %17, off\n\t"
      "global_load_dwordx4 %3, %17, off offset:16\n\t"
      "global_load_dwordx4 %4, %18, off\n\t"
      "global_load_dwordx4 %5, %18, off offset:16\n\t"
      "global_load_dwordx4 %6, %19, off\n\t"
      "global_load_dwordx4 %7, %19, off offset:16\n\t"
      "global_load_dwordx4 %8, %20, off\n\t"
      "global_load_dwordx4 %9, %20, off offset:16\n\t"
      "global_load_dwordx4 %10, %21, off\n\t"
      "global_load_dwordx4 %11, %21, off offset:16\n\t"
      "global_load_dwordx4 %12, %22, off\n\t"
      "global_load_dwordx4 %13, %22, off offset:16\n\t"
      "global_load_dwordx4 %14, %23, off\n\t"
      "global_load_dwordx4 %15, %23, off offset:16\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(rv[0][0][0]), "=&v"(rv[0][0][1]), "=&v"(rv[0][1][0]), "=&v"(rv[0][1][1]),
        "=&v"(rv[1][0][0]), "=&v"(rv[1][0][1]), "=&v"(rv[1][1][0]), "=&v"(rv[1][1][1]),
        "=&v"(rv[2][0][0]), "=&v"(rv[2][0][1]), "=&v"(rv[2][1][0]), "=&v"(rv[2][1][1]),
        "=&v"(rv[3][0][0]), "=&v"(rv[3][0][1]), "=&v"(rv[3][1][0]), "=&v"(rv[3][1][1])
      : "v"(p[0][0]), "v"(p[0][1]), "v"(p[1][0]), "v"(p[1][1]), "v"(p[2][0]), "v"(p[2][1]),
        "v"(p[3][0]), "v"(p[3][1])
      : "memory");
}

// Epilogue.  Lane (fr, fg) of wave (wm, wn) holds output row m_base + 16 i + fr, columns
// n_base + 32 jp + 8 fg + 0..7 (acc[i][2 jp] first 4, acc[i][2 jp + 1] last 4).
// FULL: no bounds checks; else rows >= M and 8-column groups >= N (N % 8 == 0) are not
// stored (their loads are clamped to valid addresses).
template <int EPI, bool FULL>
__device__ __forceinline__ void pp3_epilogue(const f32x4 (&acc)[8][4], int lane, int M, int N,
                                             int m_base, int n_base, const P3Epi& e) {
  constexpr int ACT = EPI & 3;
  constexpr bool OUT_BF16 = (EPI & 4) != 0;
  constexpr bool RESID = (EPI & 8) != 0;
  const int fr = lane & 15, fg = lane >> 4;
  bool cok[2] = {true, true};
  int col[2];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    col[jp] = n_base + 32 * jp + 8 * fg;
    if (!FULL) cok[jp] = col[jp] < N;
  }
#pragma unroll
  for (int i0 = 0; i0 < 8; i0 += 4) {
    f32x4 rv[4][2][2];
    if constexpr (RESID) {
      const float* rp[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const int m = FULL ? m_base + 16 * (i0 + i) + fr : min(m_base + 16 * (i0 + i) + fr, M - 1);
          rp[i][jp] = e.resid + (int64_t)m * e.ldr + (FULL ? col[jp] : min(col[jp], N - 8));
        }
      p3_load_resid(rv, rp);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int m = m_base + 16 * (i0 + i) + fr;
        f32x4 v0 = acc[i0 + i][2 * jp];             // bias already in the accumulators
        f32x4 v1 = acc[i0 + i][2 * jp + 1];
        act_ct8<ACT>(v0, v1);
        if constexpr (RESID) {
          v0 += rv[i][jp][0];
          v1 += rv[i][jp][1];
        }
        if (FULL || (m < M && cok[jp])) {
          const int64_t idx = (int64_t)m * e.ldo + col[jp];
          if constexpr (OUT_BF16) {
            const i32x4 o = {(int)pack_bf16x2(v0[0], v0[1]), (int)pack_bf16x2(v0[2], v0[3]),
                             (int)pack_bf16x2(v1[0], v1[1]), (int)pack_bf16x2(v1[2], v1[3])};
            *reinterpret_cast<i32x4*>(static_cast<bf16_t*>(e.out) + idx) = o;
          } else {
            float* op = static_cast<float*>(e.out) + idx;
            *reinterpret_cast<f32x4*>(op) = v0;
            *reinterpret_cast<f32x4*>(op + 4) = v1;
          }
        }
      }
  }
}
// global stores a full-tile epilogue issues after its last wait, per wave: the only
// vector-memory ops younger than the DMA in flight at its end (all 8 row blocks without a
// residual; the second 4-block chunk with one, whose loads retire the first chunk's)
template <int EPI>
constexpr int pp3_post_stores() { return ((EPI & 8) ? 4 : 8) * 2 * ((EPI & 4) ? 1 : 2); }

#define VTD_WAIT_VM(n) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory")

// Bias table: N fp32 at LDS offset 2 * BSTAGE (N <= P3_MAX_BIAS), filled once per launch.
constexpr int P3_MAX_BIAS = 8192;
constexpr int P3_LDS = 2 * BSTAGE + P3_MAX_BIAS * 4;      // 160 KiB
static_assert(P3_LDS <= 163840, "LDS budget");

template <int EPI, int DIAG = 0>
__global__ __launch_bounds__(BNT) void gemm_tn_bf16_pp3_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int lda,
    const bf16_t* __restrict__ Bt, int ldb, int tiles_m, int tiles_n, P3Epi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // stores left in flight by a full-tile epilogue (partial tiles drain theirs)
  constexpr int S = pp3_post_stores<EPI>();
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int fg = lane >> 4, fr = lane & 15;
  const int nk = K >> 6;
  const int nwg = tiles_m * tiles_n;
  const int q = nwg >> 3, r = nwg & 7;
  const int G = gridDim.x;
  const int ntile = (nwg - (int)blockIdx.x + G - 1) / G;   // tiles of this block
  if (ntile <= 0) return;
  const int total = ntile * nk;                             // global steps
  float* sbias = reinterpret_cast<float*>(smem + 2 * BSTAGE);
  for (int c = tid * 4; c < N; c += BNT * 4)
    *reinterpret_cast<f32x4*>(sbias + c) = *reinterpret_cast<const f32x4*>(e.bias + c);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // visible after the first barrier

  // per-lane DMA offsets (tile-invariant): instruction j of wave w fills group rows
  // (2w + j) * 16 + (lane >> 2), position lane & 3
  int offA[2], offB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wave * 2 + j) * 16 + (lane >> 2);
    const int c = (lane & 3) ^ (((row >> 3) & 1) << 1);
    offA[j] = row * lda * 2 + c * 16;
    offB[j] = row * ldb * 2 + c * 16;
  }
  // per-lane fragment read offsets: A block i = rows wm*128 + 16 i + fr; B block jj =
  // permuted rows wn*64 + 32 (jj >> 1) + 8 (fr >> 2) + 4 (jj & 1) + (fr & 3)
  const int a_lane = fr * 64 + ((fg ^ ((fr >> 3) << 1)) << 4) + wm * 128 * 64;
  const int pt = 8 * (fr >> 2) + (fr & 3);
  const int b_lane = pt * 64 + ((fg ^ (((fr >> 2) & 1) << 1)) << 4) + wn * 64 * 64;

  auto origin = [&](int i, int& m0, int& n0) {
    const int t = (int)blockIdx.x + i * G;
    const int x = t & 7;
    const int tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (t >> 3);
    const int tm = tile / tiles_n;
    m0 = __builtin_amdgcn_readfirstlane(tm * BBM);
    n0 = __builtin_amdgcn_readfirstlane((tile - tm * tiles_n) * BBN);
  };
  int cm0, cn0, nm0 = 0, nn0 = 0;
  origin(0, cm0, cn0);
  __amdgpu_buffer_rsrc_t ra_c = pp3_rsrc(A, cm0, M, lda), rb_c = pp3_rsrc(Bt, cn0, N, ldb);
  __amdgpu_buffer_rsrc_t ra_n = ra_c, rb_n = rb_c;
  if (ntile > 1) {
    origin(1, nm0, nn0);
    ra_n = pp3_rsrc(A, nm0, M, lda);
    rb_n = pp3_rsrc(Bt, nn0, N, ldb);
  }
  // DMA of global step h (h in {g+1, g+2}, never more than one tile ahead: nk >= 2)
#define P3_ISSUE(GRP, h)                                                                   \
  do {                                                                                     \
    const int h_ = (h);                                                                    \
    if (h_ < total) {                                                                      \
      const bool nx_ = h_ >= tile_end;                                                     \
      const int kt_ = nx_ ? h_ - tile_end : h_ - tile_end + nk;                            \
      pp3_issue<GRP>(smem, (GRP < 2) ? (nx_ ? ra_n : ra_c) : (nx_ ? rb_n : rb_c),          \
                     (GRP < 2) ? offA[0] : offB[0], (GRP < 2) ? offA[1] : offB[1], h_ & 1, \
                     kt_, wave);                                                           \
    }                                                                                      \
  } while (0)
#define P3_WAIT(last)                                                                      \
  do {                                                                                     \
    if (last) VTD_WAIT_VM(0);                                                              \
    else if (post) VTD_WAIT_VM(8 + S);                                                     \
    else VTD_WAIT_VM(8);                                                                   \
  } while (0)

  int tile_end = nk;                          // global step at which the current tile ends
  // prologue: step 0 complete (all four groups), step 1's GB0/GA0 in flight, then the
  // steady-state invariant at L0(0): GB1(1) and GA1(1) are issued by L0/L1 of step 0
  P3_ISSUE(0, 0); P3_ISSUE(2, 0); P3_ISSUE(1, 0); P3_ISSUE(3, 0);
  P3_ISSUE(2, 1); P3_ISSUE(0, 1);
  if (total > 1) VTD_WAIT_VM(4); else VTD_WAIT_VM(0);
  pp_barrier();
  if (wm == 1) pp_barrier();                  // stagger the second wave group

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool post = false;                          // first step after a full-tile epilogue
  for (int g = 0; g < total; ++g) {
    const char* st = smem + (g & 1) * BSTAGE;
    bf16x8 a[4], b[4];
    // ---- L0
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(st + P3_GA0 + a_lane + i * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      b[j] = *reinterpret_cast<const bf16x8*>(st + P3_GB0 + b_lane + (j >> 1) * 2048 + (j & 1) * 256);
    P3_ISSUE(3, g + 1);
    pp_barrier();
    pp3_mfma<0>(acc, a, b);
    pp_barrier();
    // ---- L1
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(st + P3_GA0 + a_lane + (4 + i) * 1024);
    P3_ISSUE(1, g + 1);
    P3_WAIT(g + 1 >= total);
    pp_barrier();
    pp3_mfma<4>(acc, a, b);
    pp_barrier();
    // ---- L2
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(st + P3_GA1 + a_lane + i * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      b[j] = *reinterpret_cast<const bf16x8*>(st + P3_GB1 + b_lane + (j >> 1) * 2048 + (j & 1) * 256);
    P3_ISSUE(2, g + 2);
    pp_barrier();
    pp3_mfma<0>(acc, a, b);
    pp_barrier();
    // ---- L3
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(st + P3_GA1 + a_lane + (4 + i) * 1024);
    P3_ISSUE(0, g + 2);
    P3_WAIT(g + 2 >= total);
    pp_barrier();
    pp3_mfma<4>(acc, a, b);
    pp_barrier();
    post = false;
    if (g + 1 != tile_end) continue;
    // ---- tile boundary: epilogue
    if (wm == 0) pp_barrier();                // both groups run their epilogues together
    const int m_base = cm0 + wm * 128, n_base = cn0 + wn * 64;
    {                                         // + bias (acc[i][jj] element t: column
      f32x4 bv[4];                            // n_base + 32 (jj >> 1) + 8 fg + 4 (jj & 1) + t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bv[j] = *reinterpret_cast<const f32x4*>(
            sbias + min(n_base + 32 * (j >> 1) + 8 * fg + 4 * (j & 1), N - 4));
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += bv[j];
    }
    if (DIAG == 2) {                          // timing diagnostic: no epilogue (wrong output)
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
      if (t != t) static_cast<float*>(e.out)[lane] = t;
    } else if (cm0 + BBM <= M && cn0 + BBN <= N) {
      pp3_epilogue<EPI, true>(acc, lane, M, N, m_base, n_base, e);
      post = true;
    } else {
      pp3_epilogue<EPI, false>(acc, lane, M, N, m_base, n_base, e);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // uncounted stores: drain
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int tile = (tile_end / nk) - 1;     // index of the tile just finished
    if (wm == 1 && tile + 1 < ntile) pp_barrier();     // re-stagger for the next tile
    tile_end += nk;
    cm0 = nm0; cn0 = nn0; ra_c = ra_n; rb_c = rb_n;
    if (tile + 2 < ntile) {
      origin(tile + 2, nm0, nn0);
      ra_n = pp3_rsrc(A, nm0, M, lda);
      rb_n = pp3_rsrc(Bt, nn0, N, ldb);
    }
  }
#undef P3_WAIT
#undef P3_ISSUE
}


}  // namespace

// EPI = act | out_bf16 << 2 | resid << 3 (vtd_gemm.hip epi_code).  Returns false when the
// problem is not eligible (the caller then uses the non-persistent kernels).
bool gemm_pp3_launch(int M, int N, int K, const bf16_t* A, int lda, const bf16_t* Bt,
                     int ldb, const vtd_epilogue* epi, int code, int num_cu,
                     hipStream_t stream) {
  if (N % 8 != 0 || N > P3_MAX_BIAS || K < 128 || K % 64 != 0 || !epi->bias) return false;
  if (epi->rowadd || epi->out2 || epi->scatter_tokens > 0) return false;
  if ((int64_t)256 * std::max(lda, ldb) * 2 >= 0x7fffffff) return false;
  if (epi->ldo % 8 != 0 || (epi->resid && epi->ldr % 8 != 0)) return false;
  if (epi->resid && epi->out_dtype != VTD_F32) return false;   // f32 residual only
  const int tiles_m = (M + BBM - 1) / BBM, tiles_n = (N + BBN - 1) / BBN;
  const P3Epi e{epi->bias, static_cast<const float*>(epi->resid), epi->ldr, epi->out, epi->ldo};
  // VTD_PP3_GRID: persistent blocks per launch (default one per CU); a smaller grid leaves
  // CUs to a kernel running concurrently on another stream
  static const int grid_cap = [] {
    const char* v = getenv("VTD_PP3_GRID");
    return v ? std::max(1, atoi(v)) : 1 << 30;
  }();
  const dim3 grid(std::min({tiles_m * tiles_n, num_cu, grid_cap})), block(BNT);
  static bool attr = false;
  if (!attr) {
#define VTD_P3_FN(C) reinterpret_cast<const void*>(&gemm_tn_bf16_pp3_kernel<C>),
    const void* fns[] = {VTD_P3_FN(0) VTD_P3_FN(1) VTD_P3_FN(2) VTD_P3_FN(4) VTD_P3_FN(5)
                         VTD_P3_FN(6) VTD_P3_FN(8) VTD_P3_FN(9) VTD_P3_FN(10) VTD_P3_FN(12)
                         VTD_P3_FN(13) VTD_P3_FN(14)};
#undef VTD_P3_FN
    for (const void* f : fns)
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, P3_LDS);
    attr = true;
  }
  static const int diag = [] {
    const char* v = getenv("VTD_PP3_DIAG");
    return v ? atoi(v) : 0;
  }();
  if (diag == 2) {                             // timing diagnostic (wrong outputs)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tn_bf16_pp3_kernel<4, 2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, P3_LDS);
    hipLaunchKernelGGL((gemm_tn_bf16_pp3_kernel<4, 2>), grid, block, P3_LDS, stream, M, N, K,
                       A, lda, Bt, ldb, tiles_m, tiles_n, e);
    return true;
  }
  switch (code) {
#define VTD_P3_CASE(C)                                                                      \
  case C:                                                                                   \
    hipLaunchKernelGGL((gemm_tn_bf16_pp3_kernel<C>), grid, block, P3_LDS, stream, M, N, \
                       K, A, lda, Bt, ldb, tiles_m, tiles_n, e);                            \
    return true;
    VTD_P3_CASE(0) VTD_P3_CASE(1) VTD_P3_CASE(2) VTD_P3_CASE(4) VTD_P3_CASE(5)
    VTD_P3_CASE(6) VTD_P3_CASE(8) VTD_P3_CASE(9) VTD_P3_CASE(10) VTD_P3_CASE(12)
    VTD_P3_CASE(13) VTD_P3_CASE(14)
#undef VTD_P3_CASE
    default:
      return false;
  }
}

}  // namespace vtd
