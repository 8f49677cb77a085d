// Epilogue arguments and the shared epilogue helpers of the bf16 / MX-fp8 GEMM kernels
// (vtd_gemm.hip, vtd_gemm_w4.hip): C = act(A Bt^T + bias + rowadd) + resid, the LayerNorm
// fold / partial statistics, the head's Reshape scatter and the fused decode.
#pragma once

#include <algorithm>

#include "vtd_common.h"

namespace vtd {
namespace {

// n / d for 0 <= n < 2^31 by a multiply-high and a shift (Granlund-Montgomery round-up
// method: s = ceil(log2 d), m = floor(2^32 (2^s - d) / d) + 1, q = (mulhi(n, m) + n) >> s):
// the pp2 tile-order divisions otherwise cost ~300 scalar instructions between a workgroup's
// start and its first DMA
struct FastDiv {
  uint32_t m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  const uint64_t m = ((uint64_t(1) << 32) * ((uint64_t(1) << s) - d)) / d + 1;
  return FastDiv{(uint32_t)m, s};
}
__device__ __forceinline__ int fdiv(int n, FastDiv f) {
  return (int)((__umulhi((uint32_t)n, f.m) + (uint32_t)n) >> f.s);
}
// The grouped tile order of EpiArgs::ngw with its divisors precomputed (make_tile_order)
struct TileOrder {
  int tiles_n, ngw, full, lw, gsz, grouped;
  FastDiv f_tn, f_ngw, f_lw, f_gsz;
};
inline TileOrder make_tile_order(int tiles_m, int tiles_n, int ngw) {
  TileOrder t{};
  t.tiles_n = tiles_n;
  t.grouped = ngw > 0 && ngw < tiles_n;
  t.f_tn = make_fastdiv((uint32_t)std::max(tiles_n, 1));
  if (t.grouped) {
    t.ngw = ngw;
    t.full = tiles_n / ngw;
    t.lw = tiles_n - t.full * ngw;
    t.gsz = tiles_m * ngw;
    t.f_ngw = make_fastdiv((uint32_t)ngw);
    t.f_lw = make_fastdiv((uint32_t)std::max(t.lw, 1));
    t.f_gsz = make_fastdiv((uint32_t)std::max(t.gsz, 1));
  }
  return t;
}

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
  // and 64-column block b, statout[b * stat_ld + m] = (block mean, sum of squared
  // deviations from it) -- slot-major planes (a wave's rows of one block are contiguous);
  // centred, so rows with |mean| >> std lose nothing (Chan merge in ln_stats_finalize_kernel)
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
  // split-K partial launches (pp2, ksplit > 1): split s writes its fp32 partial tile at
  // out + s * split_stride (elements)
  int64_t split_stride;
  // pp2 (ksplit == 1): consecutive tiles per workgroup (<= 1: one); with more than one, the
  // next tile's first K-stage is loaded while the current tile's epilogue runs
  int tpw;
  // the tile order of ngw with precomputed divisors (set with ngw by the 256-tile launchers)
  TileOrder to;
  // out_dtype VTD_BF16X3: width of one piece of the split-bf16 output row [hi | lo] (ldo / 2)
  int s3;
  // split-bf16 A operand (dtype VTD_BF16X3): the stored row [hi | lo] is read as the K' = 3 P
  // row [hi | lo | hi] -- K-step (64 wide) ka of the loop reads stored step ka, or ka - aw
  // once ka >= aw (aw = 2 P / 64); 0 (no wrap: ka - 0) for every other operand
  int aw;
  // diagnostic build only (VTD_PP2_SLEEP): first-round pp2 workgroups in odd XCD slots start
  // dsl x 512 cycles late (epilogue phases of neighbouring CUs out of step); 0 in the product
  int dsl;
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

// tile index -> (tm, tn) for a TileOrder (the same map as the form below, divisions by
// multiply-high)
__device__ __forceinline__ void tile_coords(int tile, const TileOrder& t, int& tm, int& tn) {
  if (!t.grouped) {
    tm = fdiv(tile, t.f_tn);
    tn = tile - tm * t.tiles_n;
    return;
  }
  const int g = fdiv(tile, t.f_gsz);
  if (g < t.full) {
    const int r = tile - g * t.gsz;
    tm = fdiv(r, t.f_ngw);
    tn = g * t.ngw + (r - tm * t.ngw);
  } else {
    const int r = tile - t.full * t.gsz;
    tm = fdiv(r, t.f_lw);
    tn = t.full * t.ngw + (r - tm * t.lw);
  }
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
// max(v[l], v[l ^ 16]) and max(v[l], v[l ^ 32]): the same lane swaps
__device__ __forceinline__ float xmax16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// the 8 bf16 values packed in o as four f32 pairs (element order lo, hi of each word)
__device__ __forceinline__ void bf16x8_unpack(const i32x4& o, f32x2 (&p)[4]) {
#pragma unroll
  for (int w = 0; w < 4; ++w)
    p[w] = f32x2{__uint_as_float((uint32_t)o[w] << 16),
                 __uint_as_float((uint32_t)o[w] & 0xffff0000u)};
}
// sum of 8 unpacked values (pairwise tree through the packed VALU)
__device__ __forceinline__ float pairs_sum(const f32x2 (&p)[4]) {
  const f32x2 t = (p[0] + p[1]) + (p[2] + p[3]);
  return t.x + t.y;
}
// sum of squared deviations from `mean` of 8 unpacked values
__device__ __forceinline__ float pairs_m2(const f32x2 (&p)[4], float mean) {
  const f32x2 m = {mean, mean};
  const f32x2 d0 = p[0] - m, d1 = p[1] - m, d2 = p[2] - m, d3 = p[3] - m;
  const f32x2 q = (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
  return q.x + q.y;
}
// sum of the 8 bf16 values packed in o
__device__ __forceinline__ float bf16x8_sum(const i32x4& o) {
  f32x2 p[4];
  bf16x8_unpack(o, p);
  return pairs_sum(p);
}
// sum of squared deviations from `mean` of the 8 bf16 values packed in o
__device__ __forceinline__ float bf16x8_m2(const i32x4& o, float mean) {
  f32x2 p[4];
  bf16x8_unpack(o, p);
  return pairs_m2(p, mean);
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
  if (e.out_dtype == VTD_F32) {
    static_cast<float*>(e.out)[idx] = v;
  } else if (e.out_dtype == VTD_BF16X3) {         // [hi | lo]
    bf16_t* o = static_cast<bf16_t*>(e.out) + idx;
    const bf16_t h = f32_to_bf16(v);
    o[0] = h;
    o[e.s3] = lo_bf16(v, h);
  } else {
    static_cast<bf16_t*>(e.out)[idx] = f32_to_bf16(v);
  }
  if (e.out2) static_cast<bf16_t*>(e.out2)[(int64_t)m * e.ldo2 + n] = f32_to_bf16(v);
  if (e.dets) e.dets[(int64_t)m * 6 + n] = decode_transform(n, v);
}

// Four consecutive columns n..n+3 of row m (row-vector epilogue of the staged path).
__device__ __forceinline__ void epi_store4(const EpiArgs& e, int M, int N, int m, int n,
                                           f32x4 v) {
  if (m >= M) return;
  const bool full = (n + 3 < N) && e.scatter_tokens <= 0 && !e.dets && (e.ldo & 3) == 0 &&
                    (e.out_dtype != VTD_BF16X3 || (e.s3 & 3) == 0) &&
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
  } else if (e.out_dtype == VTD_BF16X3) {
    const uint32_t h0 = pack_bf16x2(v[0], v[1]), h1 = pack_bf16x2(v[2], v[3]);
    bf16_t* o = static_cast<bf16_t*>(e.out) + idx;
    *reinterpret_cast<uint2*>(o) = uint2{h0, h1};
    *reinterpret_cast<uint2*>(o + e.s3) =
        uint2{pack_lo_bf16x2(v[0], v[1], h0), pack_lo_bf16x2(v[2], v[3], h1)};
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

// ---- specialized epilogue (EPI = act | out_bf16 << 2 | resid << 3), full tiles only
constexpr int EPI_GENERIC = -1;
// pp2 split-K partial launches: fp32 raw sums, no bias / activation / residual (vtd_gemm.hip)
constexpr int EPI_PARTIAL = 16;
// compile-time epilogue modes of the fast (pp2 / MX ping-pong) epilogues: the LayerNorm fold
// (epilogue.lnstat / colsum), the partial row statistics (epilogue.statout) and the MX-fp8
// output (out_dtype VTD_FP8) -- per-row uniform branches gone from the unrolled store loops
constexpr int EPI_LNF = 32, EPI_STAT = 64, EPI_F8O = 128;
// and the rare runtime modes: the position-embedding row add (patch embedding) and the bf16
// copy of an f32 residual stream (out2)
constexpr int EPI_RA = 256, EPI_O2 = 512;
// the split-bf16 output (out_dtype VTD_BF16X3, with the bf16-output bit 4): [hi | lo] over
// two e.s3 wide pieces -- the next split-bf16 GEMM's A operand
constexpr int EPI_S3 = 1024;
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

// LayerNorm fold of 8 contiguous columns with the row's (mean, rstd) st (c0, c1 = colsum of
// those columns).
__device__ __forceinline__ void epi_lnfold8_st(float2 st, f32x4 c0, f32x4 c1, f32x4& v0,
                                               f32x4& v1) {
  v0 = (v0 - st.x * c0) * st.y;
  v1 = (v1 - st.x * c1) * st.y;
}
// The same with the row's statistics fetched by lane shuffles (the w4 kernel): lst = the
// (mean, rstd) of the wave's 128 rows, lane l holding local rows l (lst[0]) and 64 + l
// (lst[1]); lr = m's local row.
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

// EpiArgs from the C-ABI epilogue (ngw: pp2 / w4 tile order; lnpart: not fused)
__host__ inline EpiArgs make_epi_args(const vtd_epilogue* epi) {
  EpiArgs e{epi->bias, epi->rowadd, epi->rowadd_period,
            epi->rowadd ? epi->rowadd_ncols : 0, epi->act, epi->resid, epi->ldr,
            epi->out, epi->ldo, epi->out_dtype, epi->out2, epi->ldo2,
            epi->scatter_tokens, reinterpret_cast<const float2*>(epi->lnstat), epi->colsum,
            reinterpret_cast<float2*>(epi->statout), epi->stat_ld, epi->scale_out,
            epi->scale_rows, epi->detections};
  e.s3 = epi->out_dtype == VTD_BF16X3 ? epi->ldo / 2 : 0;
  e.aw = 0;
  return e;
}

}  // namespace
}  // namespace vtd
