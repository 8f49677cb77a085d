// keras MultiHeadAttention core (vtd.py:364-369; [upstream] key = value = x, scores
// scaled by 1/sqrt(key_dim), softmax over keys) as a flash-style kernel: scores never
// leave registers.
//
// One workgroup = NW waves = 32*NW queries of one (image b, head h); K and V are
// streamed through LDS in tiles of 64 keys, shared by all waves of the workgroup.
// Per wave, per 32-key block, the scores are computed SWAPPED: S^T = K . Q^T with the
// 32x32 MFMA, so lane l owns query (l & 31) and 16 of the block's keys in registers:
// the row max is 15 in-register fmax + one exchange with lane l ^ 32, and the row sum
// needs no exchange until the end.  The exponentiated tile P^T is then directly the B
// operand of O^T += V^T . P^T (the accumulator's rows are the keys being summed), so
// P never touches LDS; V is staged transposed (Vt[d][key]) so the A operand is two
// 8-byte LDS reads per MFMA.
//   bf16: v_mfma_f32_32x32x16_bf16 (8 elements per lane per operand)
//   f32 : v_mfma_f32_32x32x2_f32  (1 element per lane per operand)
// Generic lane map used by both (E = elements per lane): lane half h = l >> 5 supplies
// k = 2E*step + h*E + j; accumulator register rho holds row (rho&3) + 8(rho>>2) + 4h.
#include <stdlib.h>

#include <type_traits>
#include <utility>

#include "vtd_common.h"

namespace vtd {

namespace {

constexpr int KVT = 64;   // keys per LDS tile

template <typename T, int DKP>
struct AttnCfg {
  static constexpr int E = sizeof(T) == 2 ? 8 : 1;          // elements per lane
  static constexpr int KSTEPS = DKP / (2 * E);              // MFMA k-steps over d
  static constexpr int KROW = DKP * (int)sizeof(T) + (sizeof(T) == 2 ? 16 : 4);
  static constexpr int VROW = KVT * (int)sizeof(T) + (sizeof(T) == 2 ? 8 : 4);
  static constexpr int LDS = KVT * KROW + DKP * VROW;
  static constexpr int DB = DKP / 32;                       // 32-wide d blocks
};

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <typename T, int DKP>
__global__ __launch_bounds__(512) void attention_kernel(
    const T* __restrict__ qkv, int N, int heads, int ldqkv, float scale_log2,
    T* __restrict__ out, int ldo) {
  using C = AttnCfg<T, DKP>;
  using OpT = typename std::conditional<sizeof(T) == 2, bf16x8, float>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* k_lds = smem;
  char* v_lds = smem + KVT * C::KROW;

  const int tid = threadIdx.x, nthreads = blockDim.x;
  const int lane = tid & 63, wave = tid >> 6, half = lane >> 5, col = lane & 31;
  const int h = blockIdx.y, b = blockIdx.z;
  const int inner = heads * DKP;
  const int64_t row0 = (int64_t)b * N;
  const int q0 = (blockIdx.x * (nthreads >> 6) + wave) * 32;
  const bool active = q0 < N;

  // ---- Q fragment of this lane's query, kept in registers for the whole kernel
  OpT qf[C::KSTEPS];
  {
    const int q = min(q0 + col, N - 1);
    const T* qp = qkv + (row0 + q) * ldqkv + h * DKP;
#pragma unroll
    for (int s = 0; s < C::KSTEPS; ++s) {
      if constexpr (sizeof(T) == 2)
        qf[s] = *reinterpret_cast<const bf16x8*>(qp + s * 16 + half * 8);
      else
        qf[s] = qp[s * 2 + half];
    }
  }

  f32x16 o[C::DB];
#pragma unroll
  for (int i = 0; i < C::DB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  const int chunks_per_row = DKP * (int)sizeof(T) / 16;   // 16-B chunks per K/V row
  for (int kv0 = 0; kv0 < N; kv0 += KVT) {
    __syncthreads();   // previous tile fully consumed
    // ---- stage K tile [key][d] and V^T tile [d][key]
    for (int c = tid; c < KVT * chunks_per_row; c += nthreads) {
      const int kr = c / chunks_per_row, ch = c - kr * chunks_per_row;
      const int key = min(kv0 + kr, N - 1);
      const T* base = qkv + (row0 + key) * ldqkv + h * DKP + ch * (16 / (int)sizeof(T));
      const i32x4 kv = *reinterpret_cast<const i32x4*>(base + inner);
      const i32x4 vv = *reinterpret_cast<const i32x4*>(base + 2 * inner);
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<i32x4*>(k_lds + kr * C::KROW + ch * 16) = kv;
        const bf16_t* ve = reinterpret_cast<const bf16_t*>(&vv);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          *reinterpret_cast<bf16_t*>(v_lds + (ch * 8 + i) * C::VROW + kr * 2) = ve[i];
      } else {
        const float* ke = reinterpret_cast<const float*>(&kv);
        const float* ve = reinterpret_cast<const float*>(&vv);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          *reinterpret_cast<float*>(k_lds + kr * C::KROW + (ch * 4 + i) * 4) = ke[i];
          *reinterpret_cast<float*>(v_lds + (ch * 4 + i) * C::VROW + kr * 4) = ve[i];
        }
      }
    }
    __syncthreads();
    if (!active) continue;

    // ---- S^T = K . Q^T for the two 32-key blocks of the tile
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
      const char* krow = k_lds + (kb * 32 + col) * C::KROW;
#pragma unroll
      for (int st = 0; st < C::KSTEPS; ++st) {
        OpT a;
        if constexpr (sizeof(T) == 2)
          a = *reinterpret_cast<const bf16x8*>(krow + (st * 16 + half * 8) * 2);
        else
          a = *reinterpret_cast<const float*>(krow + (st * 2 + half) * 4);
        s[kb] = mfma32(a, qf[st], s[kb]);
      }
    }
    // ---- online softmax (base 2; scale folded into scale_log2)
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kv0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        float v = s[kb][r] * scale_log2;
        v = key < N ? v : -INFINITY;
        s[kb][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    m_run = m_new;
    float psum = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = exp2f(s[kb][r] - m_new);
        s[kb][r] = p;
        psum += p;
      }
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int i = 0; i < C::DB; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[i][r] *= alpha;

    // ---- O^T += V^T . P^T
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pb = __builtin_bit_cast(
              bf16x8, i32x4{(int)pack_bf16x2(s[kb][8 * st + 0], s[kb][8 * st + 1]),
                            (int)pack_bf16x2(s[kb][8 * st + 2], s[kb][8 * st + 3]),
                            (int)pack_bf16x2(s[kb][8 * st + 4], s[kb][8 * st + 5]),
                            (int)pack_bf16x2(s[kb][8 * st + 6], s[kb][8 * st + 7])});
          const int key_lo = kb * 32 + 16 * st + 4 * half;   // j = 0..3
#pragma unroll
          for (int db = 0; db < C::DB; ++db) {
            const char* vr = v_lds + (db * 32 + col) * C::VROW;
            const bf16x4 lo = *reinterpret_cast<const bf16x4*>(vr + key_lo * 2);
            const bf16x4 hi = *reinterpret_cast<const bf16x4*>(vr + (key_lo + 8) * 2);
            bf16x8 a;
            a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
            a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
            o[db] = mfma32(a, pb, o[db]);
          }
        }
      } else {
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          const int key = kb * 32 + (t & 3) + 8 * (t >> 2) + 4 * half;
#pragma unroll
          for (int db = 0; db < C::DB; ++db) {
            const float a =
                *reinterpret_cast<const float*>(v_lds + (db * 32 + col) * C::VROW + key * 4);
            o[db] = mfma32(a, s[kb][t], o[db]);
          }
        }
      }
    }
  }
  if (!active) return;

  // ---- normalise and store: lane owns query q0 + col, register rho -> d
  const float l_tot = l_run + __shfl_xor(l_run, 32);
  const float inv = 1.f / l_tot;
  const int q = q0 + col;
  if (q >= N) return;
  T* op = out + (row0 + q) * ldo + h * DKP;
#pragma unroll
  for (int db = 0; db < C::DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = db * 32 + 8 * g + 4 * half;
      if constexpr (sizeof(T) == 2) {
        const uint2 v = {pack_bf16x2(o[db][4 * g + 0] * inv, o[db][4 * g + 1] * inv),
                         pack_bf16x2(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv)};
        *reinterpret_cast<uint2*>(op + d) = v;
      } else {
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = o[db][4 * g + r] * inv;
        *reinterpret_cast<f32x4*>(op + d) = v;
      }
    }
}

// ---------------------------------------------------------------------------------
// bf16 kernel, v2: K and V are staged row-major with 16-B stores (global -> registers
// during the previous chunk's compute -> LDS after it; two LDS buffers, one barrier per
// 64-key chunk).  The A operand of O^T += V^T P^T needs, per lane (d = l & 31 of the
// 32-wide d block, half h = l >> 5), the 8 keys 16s + 8(j>>2) + 4h + (j&3) of column d:
// two ds_read_b64_tr_b16, each delivering one column of a 4-key x 16-d block
// (lane 4q+p of a 16-lane group addresses key q, d 4p..4p+3 of the block).
// V row stride DKP*2 + 64 B shifts consecutive keys by 16 mod 64 banks, so the 4 rows
// x 64 B of a 32-lane tr-read half cover all 64 banks once (conflict-free for DKP 64/128).
// lanes l and l ^ 32 combined by one v_permlane32_swap (no LDS round trip): after the swap
// the two results hold x[l] and x[l ^ 32] in some order, so max / sum of them is the pair's
__device__ __forceinline__ float pair_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
template <int DKP>
struct AttnBf16Cfg {
  static constexpr int KC = 64;                       // keys per chunk
  static constexpr int KS = DKP * 2 + 16;             // K row stride (bytes)
  static constexpr int VS = DKP * 2 + 64;             // V row stride (bytes)
  static constexpr int BUF = KC * KS + KC * VS;
  static constexpr int CPR = DKP * 2 / 16;            // 16-B chunks per row
  static constexpr int NCH = KC * CPR * 2;            // chunks per K+V tile
  static constexpr int KSTEPS = DKP / 16;
  static constexpr int DB = DKP / 32;
};

// MX8: the output is written as the MX-fp8 A operand of the attention-output GEMM (VTD_FP8
// mode) instead of bf16: per 32-column block (lanes l and l ^ 32 of one query hold 16 values
// each) the amax of the bf16-rounded values -> E8M0 scale -> e4m3 bytes, exactly what
// vtd_quantize_mx8 makes of the bf16 output (layout in vtd_mx8.hip: q[row][ldo] bytes,
// s[k / 128][s_rows][4]).
// Grid: one workgroup per (query block of NWG x 32 queries, head, image), 1-D.  The query
// blocks of one (image, head) stream the same K / V chunks, so workgroup ids are remapped
// XCD-aware (xcd_remap != 0): blocks b, b + 8, ... share an XCD and walk one contiguous range
// of (pair, query block) ids, so a pair's query blocks run on one XCD and read its K / V
// through that XCD's L2 once instead of once per XCD from beyond it.
template <int DKP, int NWG, bool MX8 = false>
__global__ __launch_bounds__(64 * NWG, NWG == 4 ? (DKP == 128 ? 2 : 3) : 2) void attention_bf16_kernel(
    const bf16_t* __restrict__ qkv, int N, int heads, int ldqkv, float scale_log2,
    bf16_t* __restrict__ out, int ldo, uint8_t* __restrict__ s8, int64_t s_rows, int nqb,
    int xcd_remap) {
  using C = AttnBf16Cfg<DKP>;
  typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  constexpr int nthreads = 64 * NWG;
  const int lane = tid & 63, wave = tid >> 6, half = lane >> 5, col = lane & 31;
  int v = blockIdx.x;
  if (xcd_remap) {
    const int G = gridDim.x, xcd = v & 7, q8 = G >> 3, r8 = G & 7;
    v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
  }
  const int pair = v / nqb, qb = v - pair * nqb;
  const int b = pair / heads, h = pair - b * heads;
  const int inner = heads * DKP;
  const int64_t row0 = (int64_t)b * N;
  const int q0 = (qb * NWG + wave) * 32;
  const bool active = q0 < N;

  // Q pre-scaled by scale * log2(e) (keras scales the query by 1 / sqrt(key_dim) before
  // Q K^T [upstream]; the log2(e) factor makes the scores log2 units) and rounded to bf16
  // again: a score is then exp2'ed as it leaves the MFMA, with no per-score multiply
  bf16x8 qf[C::KSTEPS];
  {
    const int q = min(q0 + col, N - 1);
    const bf16_t* qp = qkv + (row0 + q) * ldqkv + h * DKP;
#pragma unroll
    for (int st = 0; st < C::KSTEPS; ++st) {
      const i32x4 raw = *reinterpret_cast<const i32x4*>(qp + st * 16 + half * 8);
      i32x4 sc;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        sc[j] = (int)pack_bf16x2(__uint_as_float((uint32_t)raw[j] << 16) * scale_log2,
                                 __uint_as_float((uint32_t)raw[j] & 0xffff0000u) * scale_log2);
      qf[st] = __builtin_bit_cast(bf16x8, sc);
    }
  }
  f32x16 o[C::DB];
#pragma unroll
  for (int i = 0; i < C::DB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  // Running max m_run (log2 units, kept exactly representable in bf16) subtracted INSIDE the
  // score MFMA chain: one extra K-step multiplies the constant A column e_0 (1 at k = 0) by the
  // B column -m_run (k = 0), so each score leaves the matrix core as s - m_run and P is one
  // v_exp_f32 of it.  m_run starts at 0 and is set from the first chunk's max (`first`).
  // SUMMFMA: the row sum l rides in the PV MFMAs as a 32-row block of ones in V^T (every row
  // of osum = sum_k P[k][q] of the bf16 P actually used), instead of one VALU add per score;
  // otherwise l_run sums the fp32 P.  Both only where the registers allow it: the 4-wave
  // workgroups (3 per CU; dkp <= 64 for SUMMFMA).  The 8-wave ones (C5's MX-fp8 epilogue,
  // 2 workgroups per CU at <= 128 VGPRs) keep the running max outside the MFMA chain
  // (OFFM false: P = exp2(s - m_run), m_run from -inf) -- with both tricks they took 141
  // VGPRs, one workgroup per CU: C5 fp8 attention 261 -> 345 us (profiles/r06_s1_*).
  constexpr bool OFFM = NWG == 4;
  constexpr bool SUMMFMA = OFFM && DKP <= 64;
  float m_run = OFFM ? 0.f : -INFINITY, l_run = 0.f;
  const bf16_t one_bf16 = 0x3F80;
  const bf16x8 a_e0 = {(short)(half == 0 ? one_bf16 : 0), 0, 0, 0, 0, 0, 0, 0};
  const bf16x8 a_ones = {(short)one_bf16, (short)one_bf16, (short)one_bf16, (short)one_bf16,
                         (short)one_bf16, (short)one_bf16, (short)one_bf16, (short)one_bf16};
  bf16x8 b_m = {0, 0, 0, 0, 0, 0, 0, 0};        // -m_run at k = 0 (half 0 lanes)
  f32x16 osum;
#pragma unroll
  for (int r = 0; r < 16; ++r) osum[r] = 0.f;

  constexpr int NPASS = (C::NCH + nthreads - 1) / nthreads;
  i32x4 stg[NPASS];
  auto gload = [&](int kv0) {
#pragma unroll
    for (int i = 0; i < NPASS; ++i) {
      const int c = tid + i * nthreads;
      if (c < C::NCH) {
        const int isv = c >= C::KC * C::CPR;
        const int cc = c - isv * C::KC * C::CPR;
        const int kr = cc / C::CPR, ch = cc - kr * C::CPR;
        const int key = min(kv0 + kr, N - 1);
        stg[i] = *reinterpret_cast<const i32x4*>(qkv + (row0 + key) * ldqkv +
                                                 (1 + isv) * inner + h * DKP + ch * 8);
      }
    }
  };
  auto swrite = [&](int buf) {
    char* base = smem + buf * C::BUF;
#pragma unroll
    for (int i = 0; i < NPASS; ++i) {
      const int c = tid + i * nthreads;
      if (c < C::NCH) {
        const int isv = c >= C::KC * C::CPR;
        const int cc = c - isv * C::KC * C::CPR;
        const int kr = cc / C::CPR, ch = cc - kr * C::CPR;
        char* dst = isv ? base + C::KC * C::KS + kr * C::VS + ch * 16 : base + kr * C::KS + ch * 16;
        *reinterpret_cast<i32x4*>(dst) = stg[i];
      }
    }
  };

  const int nchunks = (N + C::KC - 1) / C::KC;
  gload(0);
  swrite(0);
  __syncthreads();
  // per-lane tr-read address pieces: key offset within a 4-key block, d offset
  const int tr_key = 4 * half + ((lane & 15) >> 2);
  const int tr_d = ((lane >> 4) & 1) * 16 + (lane & 3) * 4;
  // one key chunk; LAST = the final chunk (possibly ragged: runtime key-block count and
  // mask, no next-chunk load): every other chunk is full, so its block loop and mask are
  // compile-time (no per-chunk branches)
  auto chunk = [&](int c, auto last_tag) {
    constexpr bool LAST = decltype(last_tag)::value;
    const int kv0 = c * C::KC;
    if (!LAST) gload(kv0 + C::KC);
    if (active) {
      const char* kl = smem + (c & 1) * C::BUF;
      const char* vl = kl + C::KC * C::KS;
      // 32-key blocks of this chunk holding at least one key (the last chunk may be
      // ragged: N = 196 leaves 4 keys in it, one block)
      const int nkb = LAST ? min(2, (N - kv0 + 31) >> 5) : 2;
      const bool ragged = LAST && kv0 + C::KC > N;
      f32x16 s[2];
      const f32x16 zero = {};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        if (kb < nkb) {
          const char* krow = kl + (kb * 32 + col) * C::KS;
          if constexpr (OFFM) s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_e0, b_m, zero, 0, 0, 0);   // -m_run
          else s[kb] = zero;
#pragma unroll
          for (int st = 0; st < C::KSTEPS; ++st)
            s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                *reinterpret_cast<const bf16x8*>(krow + (st * 16 + half * 8) * 2), qf[st],
                s[kb], 0, 0, 0);
        }
      }
      // scores beyond N (ragged last chunk only) are -inf
      if (ragged) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kv0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
            if (key >= N) s[kb][r] = -INFINITY;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        if (kb < nkb) {
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
        }
      mx = pair_max(mx);              // (relative to m_run) lane l ^ 32 holds the other keys
      // deferred rescale: the accumulators are rescaled only when some lane's max grows by
      // more than 8 (log2 units), so exp2 arguments stay <= 8 + 1/8 (P <= 2^8.125, exact in the
      // bf16 P operand's range, l and O in fp32); the final 1/l normalises whatever max was
      // used consistently for O and l.  The first chunk always sets the max.
      if constexpr (OFFM) {
        if (__builtin_amdgcn_ballot_w64(c == 0 || mx > 8.f)) {
          const float m_new = bf16_round(m_run + (c == 0 ? mx : fmaxf(mx, 0.f)));
          const float dlt = m_new - m_run;
          // (first chunk: O and l are still 0; dlt may be any size there)
          const float alpha = c == 0 ? 0.f : __builtin_amdgcn_exp2f(-dlt);
          m_run = m_new;
          b_m[0] = (short)(half == 0 ? f32_to_bf16(-m_new) : 0);
          l_run *= alpha;
          osum[0] *= alpha;
#pragma unroll
          for (int i = 0; i < C::DB; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) s[kb][r] -= dlt;
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          if (kb < nkb) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[kb][r] = __builtin_amdgcn_exp2f(s[kb][r]);
          }
      } else {
        // (absolute scores) rescale only when some lane's max grows by more than 8
        if (__builtin_amdgcn_ballot_w64(mx > m_run + 8.f)) {
          const float m_new = fmaxf(m_run, mx);
          const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
          m_run = m_new;
          l_run *= alpha;
#pragma unroll
          for (int i = 0; i < C::DB; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
        }
        const float nm = -m_run;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          if (kb < nkb) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[kb][r] = __builtin_amdgcn_exp2f(s[kb][r] + nm);
          }
      }
      if constexpr (!SUMMFMA) {
        // scalar fp32 adds (the file is built without SLP packing: packed f32 ops cost more
        // issue cycles beside MFMAs than two scalar ones); even / odd scores summed apart
        float ps0 = 0.f, ps1 = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          if (kb < nkb) {
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              ps0 += s[kb][r];
              ps1 += s[kb][r + 1];
            }
          }
        l_run += ps0 + ps1;
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        if (kb < nkb) {
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const bf16x8 pb = __builtin_bit_cast(
                bf16x8, i32x4{(int)pack_bf16x2(s[kb][8 * st + 0], s[kb][8 * st + 1]),
                              (int)pack_bf16x2(s[kb][8 * st + 2], s[kb][8 * st + 3]),
                              (int)pack_bf16x2(s[kb][8 * st + 4], s[kb][8 * st + 5]),
                              (int)pack_bf16x2(s[kb][8 * st + 6], s[kb][8 * st + 7])});
            const int key0 = kb * 32 + 16 * st + tr_key;
#pragma unroll
            for (int db = 0; db < C::DB; ++db) {
              const char* va = vl + key0 * C::VS + (db * 32 + tr_d) * 2;
              const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)va);
              const bf16x4 hi =
                  __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(va + 8 * C::VS));
              const bf16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
              o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pb, o[db], 0, 0, 0);
            }
            if constexpr (SUMMFMA) osum = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_ones, pb, osum, 0, 0, 0);
          }
        }
    }
    if (!LAST) swrite((c + 1) & 1);
    __syncthreads();
  };
  for (int c = 0; c + 1 < nchunks; ++c) chunk(c, std::false_type{});
  chunk(nchunks - 1, std::true_type{});
  if (!active) return;
  // osum rows hold the whole key sum (both lane halves' keys); l_run holds this half's
  const float inv = 1.f / (SUMMFMA ? osum[0] : pair_sum(l_run));
  const int q = q0 + col;
  if constexpr (!MX8 && DKP == 64) {
    // bf16 output through LDS (free after the loop's last barrier): a lane holds 16-B
    // pieces of one query row spread over 8 columns groups, so direct stores write 16 B
    // per row per instruction; restaged (row stride 144 B: the 16-lane groups of the
    // 8-B writes hit distinct banks) every store instruction writes 8 whole 128-B rows.
    char* wst = smem + wave * (32 * 144);
#pragma unroll
    for (int db = 0; db < C::DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<uint2*>(wst + col * 144 + (db * 32 + 8 * g + 4 * half) * 2) =
            uint2{pack_bf16x2(o[db][4 * g + 0] * inv, o[db][4 * g + 1] * inv),
                  pack_bf16x2(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv)};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // wave-local: own writes landed
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int r = pass * 8 + (lane >> 3), ch = lane & 7;
      if (q0 + r < N)
        *reinterpret_cast<i32x4*>(out + (row0 + q0 + r) * ldo + h * DKP + ch * 8) =
            *reinterpret_cast<const i32x4*>(wst + r * 144 + ch * 16);
    }
    return;
  }
  if (q >= N) return;          // lanes l and l ^ 32 hold the same query: both leave or stay
  if constexpr (MX8) {
    uint8_t* qp = reinterpret_cast<uint8_t*>(out) + (row0 + q) * (int64_t)ldo + h * DKP;
#pragma unroll
    for (int db = 0; db < C::DB; ++db) {
      float v[16];
      float amax = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        v[i] = bf16_round(o[db][i] * inv);
        amax = fmaxf(amax, fabsf(v[i]));
      }
      amax = pair_max(amax);
      const int E = mx8_exponent(amax);
      const float sinv = __uint_as_float((uint32_t)(127 - E) << 23);     // 2^-E, exact
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<uint32_t*>(qp + db * 32 + 8 * g + 4 * half) =
            mx8_pack4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3], sinv);
      if (half == 0) {
        const int k0 = h * DKP + db * 32;
        s8[((int64_t)(k0 >> 7) * s_rows + row0 + q) * 4 + ((k0 >> 5) & 3)] = (uint8_t)(E + 127);
      }
    }
    return;
  }
  bf16_t* op = out + (row0 + q) * ldo + h * DKP;
#pragma unroll
  for (int db = 0; db < C::DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = db * 32 + 8 * g + 4 * half;
      const uint2 v = {pack_bf16x2(o[db][4 * g + 0] * inv, o[db][4 * g + 1] * inv),
                       pack_bf16x2(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv)};
      *reinterpret_cast<uint2*>(op + d) = v;
    }
}

// ---------------------------------------------------------------------------------
// Persistent short-sequence kernel (bf16, DKP = 64, 128 < N <= 256: the C2 shape N = 196).
// At N = 196 the per-(image, head) kernel above spends most of a workgroup's life waiting:
// an exposed Q + first-chunk load, then one barrier + one register-staged chunk per 64 keys.
// Here one workgroup per CU walks the (image, head) pairs p = blockIdx.x + i * gridDim.x and
// the loads never stop:
//   - a pair's whole K and V (NR = N rounded up to 32 rows of 128 B each) arrive by LDS-DMA
//     (buffer_load ... lds, 8 rows = 1 KiB per wave-instruction, no VGPR staging) into one of
//     two slots, issued while the previous pair is computed; its Q arrives the same way in a
//     third area, one pair ahead, and goes to registers at the top of the pair;
//   - the compute of a pair reads only LDS: no barrier between its key chunks;
//   - O is restaged through the pair's own slot (after the compute's barrier) and stored as
//     whole 128-B rows by buffer stores whose range check drops the rows >= N, so every wave
//     issues exactly 4 stores per pair: the next pair's wait is `vmcnt(4)` (the DMAs landed,
//     the stores may still fly).
// LDS images are lane-linear (the DMA writes base + 16 * lane) and swizzled on the source
// address: K and Q rows chunk ^ ((row >> 1) & 7) (the 16 rows of a ds_read_b128 lane group hit
// 16 distinct 16-B bank slots), V rows chunk ^ (((row >> 1) & 1) << 2) (the 4 rows x 64 B of
// a ds_read_b64_tr_b16 half-wave cover the 64 banks once).  Same arithmetic and operation
// order as attention_bf16_kernel: per-image results are identical (tested).
// Waits: counted vmcnt + raw s_barrier only (a __syncthreads fence would drain the DMAs).
__device__ __forceinline__ int swz_kq(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swz_v(int row) { return ((row >> 1) & 1) << 2; }

// TG: the last key block's 8-key row groups (r >> 2 of a lane's 16 scores) that can hold a key
// < N, i.e. ceil((N - 32 (NB - 1)) / 8) (4: no trim).  The groups past it hold only masked keys:
// their exponentials are 0 without being computed, and with TG <= 2 the block's second
// 16-key PV step (and its V reads) is skipped -- at N = 196 the last block holds 4 keys.
template <int NB, int TG = 4>   // key blocks of 32: N in (32 (NB - 1), 32 NB]
__global__ __launch_bounds__(512, 1) void attention_bf16_ps_kernel(
    const bf16_t* __restrict__ qkv, int npairs, int N, int heads, int ldqkv, float scale_log2,
    bf16_t* __restrict__ out, int ldo, int dmode_arg) {
  constexpr int DKP = 64;
  typedef __attribute__((address_space(3))) void lds_void_t;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // diagnostic build only (timing experiments, wrong results; knob VTD_ATTN_DMODE): bit 0
  // reads each image's Q / K / V as head-major [part][head][N][64] blocks, bit 1 skips the
  // compute (DMAs + stores only), bit 2 skips the DMAs (compute on stale LDS), bit 3 replaces
  // the exponential by a multiply, bit 4 skips the V DMAs, bit 5 the K reads of the scores
  // (Q fragments as both operands), bit 6 the V reads of the PV steps (P as both operands),
  // bit 7 an XCD-major pair order (below)
#if VTD_DIAG
  const int dmode = dmode_arg;
#else
  constexpr int dmode = 0;
  (void)dmode_arg;
#endif
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, half = lane >> 5, col = lane & 31;
  const int NR = (N + 31) & ~31;
  const int SLOT = 2 * NR * 128;                 // K image, then V image
  char* const qarea = smem + 2 * SLOT;
  const int inner = heads * DKP;
  const int q0 = wave * 32;
  const bool active = q0 < N && !(dmode & 2);
  const int G = gridDim.x;
  const int ngroups = NR >> 3;                   // 8-row groups per matrix
  const int lrow = lane >> 3, lchunk = lane & 7;
  const uint32_t lds_base =
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(smem);

  // DMA of one matrix (part 0 = Q, 1 = K, 2 = V) of pair p into dst
  auto issue = [&](int p, int part, char* dst) {
    const int b = p / heads, h = p - b * heads;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(qkv + (int64_t)b * N * ldqkv), 0, N * ldqkv * 2, 0x00020000);
    const int colb = (part * inner + h * DKP) * 2;
    const bool skip = (dmode & 4) || ((dmode & 16) && part == 2);
    for (int g = skip ? ngroups : wave; g < ngroups; g += 8) {
      const int r = g * 8 + lrow;
      const int sw = part == 2 ? swz_v(r) : swz_kq(r);
      const int voff = (dmode & 1)
                           ? ((part * heads + h) * N + min(r, N - 1)) * 128 + ((lchunk ^ sw) << 4)
                           : min(r, N - 1) * ldqkv * 2 + colb + ((lchunk ^ sw) << 4);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + g * 1024), 16, voff, 0, 0,
                                               0);
    }
  };

  // bit 7: the workgroups of one XCD (blockIdx % 8) take consecutive pairs (all heads of an
  // image on one XCD's L2) -- needs a grid that is a multiple of 8
  int p = (dmode & 128) ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  if (p >= npairs) return;                       // uniform per workgroup
  issue(p, 1, smem);
  issue(p, 2, smem + NR * 128);
  issue(p, 0, qarea);
  const int tr_key = 4 * half + ((lane & 15) >> 2);
  const int tr_byte = ((lane >> 4) & 1) * 32 + (lane & 3) * 8;   // within a 64-B d block
  for (int it = 0; p < npairs; p += G, ++it) {
    char* const kl = smem + (it & 1) * SLOT;
    const uint32_t kl_addr = lds_base + (it & 1) * SLOT, vl_addr = kl_addr + NR * 128;
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // previous pair's O stores may fly
    __builtin_amdgcn_s_barrier();
    bf16x8 qf[4];
    if (active) {
      const int row = q0 + col;
#pragma unroll
      for (int st = 0; st < 4; ++st)
        qf[st] = *reinterpret_cast<const bf16x8*>(qarea + row * 128 +
                                                   (((st * 2 + half) ^ swz_kq(row)) << 4));
    }
    const int pn = p + G;
    const bool fetch = pn < npairs;
    if (fetch) {
      char* const kn = smem + ((it + 1) & 1) * SLOT;
      issue(pn, 1, kn);
      issue(pn, 2, kn + NR * 128);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Q fragments in registers
    __builtin_amdgcn_s_barrier();
    if (fetch) issue(pn, 0, qarea);

    f32x16 o[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
    float l_run = 0.f;
    if (active) {
      // ---- all NB key blocks of S^T = K . Q^T at once (NB independent MFMA chains): every
      // key is in LDS, so the softmax takes the row's true max in one pass (no running max)
      f32x16 s[NB];
      const int swk = swz_kq(col);             // (row >> 1) & 7 with row = 32 kb + col
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
        const char* krow = kl + (kb * 32 + col) * 128;
#pragma unroll
        for (int st = 0; st < 4; ++st)
          s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              (dmode & 32) ? qf[st]
                           : *reinterpret_cast<const bf16x8*>(krow + (((st * 2 + half) ^ swk) << 4)),
              qf[st], s[kb], 0, 0, 0);
      }
      if (N < NB * 32) {                        // keys >= N of the last block
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = (NB - 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
          if (key >= N) s[NB - 1][r] = -INFINITY;
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < NB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
      mx = pair_max(mx) * scale_log2;
      // ---- P = exp2(S c - max) block by block, each block's four O^T += V^T . P^T MFMAs
      // issued right after its exponentials: the matrix core runs them while the VALU
      // exponentiates the next block (scalar fma / add: packed f32 ops cost more beside MFMAs)
      // V^T fragments by inline-asm tr-reads one block ahead (the compiler's own tr-read
      // would be treated as aliasing the in-flight LDS-DMA and wait vmcnt(0) for the next
      // pair); lane-constant part of the swizzled address hoisted
      const int swv = swz_v(tr_key);            // rows 32 kb + 16 st + tr_key (+ 8): same
      uint32_t va[2];
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const int byte = db * 64 + tr_byte;
        va[db] = vl_addr + tr_key * 128 + (((byte >> 4) ^ swv) << 4) + (byte & 15);
      }
      bf16x4 vf[2][2][2][2];                    // [kb parity][st][db][lo / hi]
      // 16-key PV steps of block kb: 1 for a trimmed last block (TG <= 2)
      auto nsteps = [](int kb) { return (kb == NB - 1 && TG <= 2) ? 1 : 2; };
      auto vread = [&](int kb, bf16x4 (&f)[2][2][2]) {
        if (dmode & 64) return;
#pragma unroll
        for (int st = 0; st < nsteps(kb); ++st)
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            const uint32_t a = va[db] + (kb * 32 + 16 * st) * 128;
            asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f[st][db][0]) : "v"(a));
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:1024" : "=v"(f[st][db][1]) : "v"(a));
          }
      };
      vread(0, vf[0]);
      float ps0 = 0.f, ps1 = 0.f;
      const float nmx = -mx;
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) {
        bf16x8 pb[2];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          float e[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (kb == NB - 1 && ((8 * st + j) >> 2) >= TG) {   // only masked keys: exp = 0
              e[j] = 0.f;
              continue;
            }
            e[j] = (dmode & 8) ? __builtin_fmaf(s[kb][8 * st + j], scale_log2, nmx)
                               : __builtin_amdgcn_exp2f(__builtin_fmaf(s[kb][8 * st + j], scale_log2, nmx));
            if (j & 1) ps1 += e[j];
            else ps0 += e[j];
          }
          pb[st] = __builtin_bit_cast(bf16x8, i32x4{(int)pack_bf16x2(e[0], e[1]),
                                                    (int)pack_bf16x2(e[2], e[3]),
                                                    (int)pack_bf16x2(e[4], e[5]),
                                                    (int)pack_bf16x2(e[6], e[7])});
        }
        if (kb + 1 < NB) {
          vread(kb + 1, vf[(kb + 1) & 1]);
          // the next block's reads (8, or 4 for a trimmed last block) may stay in flight
          if (nsteps(kb + 1) == 2) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
          else asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int st = 0; st < nsteps(kb); ++st)
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            const bf16x4 lo = vf[kb & 1][st][db][0], hi = vf[kb & 1][st][db][1];
            const bf16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16((dmode & 64) ? pb[st] : a, pb[st],
                                                            o[db], 0, 0, 0);
          }
      }
      l_run = ps0 + ps1;
    }
    // every wave done reading this slot's K / V: restage O in it, store whole rows
    __builtin_amdgcn_s_barrier();
    const float inv = 1.f / pair_sum(l_run);
    char* const wst = kl + wave * (32 * 144);
    if (active) {
      // inline asm for the same reason as the tr-reads (a compiler ds_write would wait
      // vmcnt(0) for the next pair's DMA); "memory" keeps the row reads below after them
      const uint32_t wa = kl_addr + wave * (32 * 144) + col * 144 + 8 * half;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint2 v = {pack_bf16x2(o[db][4 * g + 0] * inv, o[db][4 * g + 1] * inv),
                           pack_bf16x2(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv)};
          asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(wa), "v"(v), "n"((db * 32 + 8 * g) * 2)
                       : "memory");
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // wave-local: own writes landed
    {
      const int b = p / heads, h = p - b * heads;
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
          out + (int64_t)b * N * ldo, 0, N * ldo * 2, 0x00020000);
#pragma unroll
      for (int pass = 0; pass < 4; ++pass) {
        const int r = pass * 8 + lrow;
        const i32x4 v = *reinterpret_cast<const i32x4*>(wst + r * 144 + lchunk * 16);
        // rows >= N (and every row of an inactive wave) fall outside the range: dropped
        __builtin_amdgcn_raw_buffer_store_b128(v, ro, ((q0 + r) * ldo + h * DKP + lchunk * 8) * 2,
                                               0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------
// Long-sequence kernel (bf16, DKP = 64, N > 256: C3 N = 1600, C5 N = 576; opt-in, knob
// VTD_KNOB_ATTN_VARIANT 6: measured 12 % / 5 % SLOWER than the streaming kernel at C3 / C5,
// profiles/r05_attn_fl_ab.log -- kept for the record and for its tests).  One workgroup = NW waves x 32 queries of one
// (image, head).  The 64-key chunks of K and V every wave of it reads arrive by LDS-DMA
// (buffer_load ... lds: no VGPR staging, no staging VALU) into a ring of KS slots of 16 KiB,
// KS - 1 chunks ahead: per chunk one counted vmcnt (the wave's own pieces of chunk c), one
// barrier (every piece landed, every wave past chunk c - 1), then the DMA of chunk c + KS - 1
// into the slot chunk c - 1 used.  The per-chunk arithmetic is attention_bf16_kernel's (scores
// swapped, S^T = K Q^T; online softmax with the deferred rescale; P^T as the B operand of
// O^T += V^T P^T) on the persistent kernel's LDS images (128-B rows swizzled on the DMA
// source, V read by ds_read_b64_tr_b16).  <= 128 VGPRs: 4 waves per SIMD.  NW is picked per N
// so that the last workgroup of a pair has no idle waves (N = 1600: 5, N = 576: 6).
template <int CNT>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT) : "memory");
}
template <int NW, int KS>
__global__ __launch_bounds__(64 * NW, 4) void attention_bf16_fl_kernel(
    const bf16_t* __restrict__ qkv, int N, int heads, int ldqkv, float scale_log2,
    bf16_t* __restrict__ out, int ldo, int nqb) {
  constexpr int DKP = 64, KC = 64, SLOT = 2 * KC * 128;
  static_assert(NW >= 4 && NW <= 6 && KS >= 2 && KS <= 4, "fl kernel geometry");
  typedef __attribute__((address_space(3))) void lds_void_t;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  // wave-uniform in an SGPR: the DMA loop, the counted waits and `active` branch on scalars
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, half = lane >> 5, col = lane & 31;
  int v = blockIdx.x;                         // XCD-aware: a pair's query blocks share an XCD
  {
    const int G = gridDim.x, xcd = v & 7, q8 = G >> 3, r8 = G & 7;
    v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
  }
  const int pair = v / nqb, qb = v - pair * nqb;
  const int b = pair / heads, h = pair - b * heads;
  const int inner = heads * DKP;
  const int q0 = (qb * NW + wave) * 32;
  const bool active = q0 < N;
  const uint32_t lds_base =
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(smem);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(qkv + (int64_t)b * N * ldqkv), 0, N * ldqkv * 2, 0x00020000);
  const int lrow = lane >> 3, lchunk = lane & 7;
  const int colk = (inner + h * DKP) * 2, colv = (2 * inner + h * DKP) * 2;
  // this wave's Q fragments (plain loads: the compiler's wait before their first use also
  // retires the first chunks' DMA, once)
  bf16x8 qf[4];
  {
    const int q = min(q0 + col, N - 1);
    const bf16_t* qp = qkv + ((int64_t)b * N + q) * ldqkv + h * DKP;
#pragma unroll
    for (int st = 0; st < 4; ++st) qf[st] = *reinterpret_cast<const bf16x8*>(qp + st * 16 + half * 8);
  }
  const int nch = (N + KC - 1) / KC;
  // a chunk = 8 groups of 8 K rows + 8 groups of 8 V rows; wave w issues groups w, w + NW, ..
  const int my_groups = (8 - wave + NW - 1) / NW;      // 1 or 2
  auto issue = [&](int c) {
    char* dst = smem + (c % KS) * SLOT;
    for (int g = wave; g < 8; g += NW) {
      const int r = g * 8 + lrow;                       // row within the chunk
      const int key = min(c * KC + r, N - 1);
      const int base = key * ldqkv * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + g * 1024), 16,
                                               base + colk + ((lchunk ^ swz_kq(r)) << 4), 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + KC * 128 + g * 1024), 16,
                                               base + colv + ((lchunk ^ swz_v(r)) << 4), 0, 0, 0);
    }
  };
  for (int c = 0; c < KS - 1 && c < nch; ++c) issue(c);

  f32x16 o[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const int tr_key = 4 * half + ((lane & 15) >> 2);
  const int tr_byte = ((lane >> 4) & 1) * 32 + (lane & 3) * 8;
  const int swk = swz_kq(col), swv = swz_v(tr_key);
  uint32_t va0[2];                                      // V tr-read address in a slot, per db
#pragma unroll
  for (int db = 0; db < 2; ++db) {
    const int byte = db * 64 + tr_byte;
    va0[db] = KC * 128 + tr_key * 128 + (((byte >> 4) ^ swv) << 4) + (byte & 15);
  }

  auto chunk = [&](int c, auto last_tag) {
    constexpr bool LAST = decltype(last_tag)::value;
    // the wave's pieces of chunk c landed: pieces of the KS - 2 later chunks may fly
    const int pend = my_groups * 2 * min(KS - 2, nch - 1 - c);
    switch (pend) {
      case 0: vm_wait<0>(); break;
      case 2: vm_wait<2>(); break;
      case 4: vm_wait<4>(); break;
      case 6: vm_wait<6>(); break;
      default: vm_wait<8>(); break;
    }
    __builtin_amdgcn_s_barrier();
    if (!LAST && c + KS - 1 < nch) issue(c + KS - 1);    // into the slot chunk c - 1 used
    if (!active) return;
    const char* kl = smem + (c % KS) * SLOT;
    const uint32_t vs = lds_base + (c % KS) * SLOT;
    const int kv0 = c * KC;
    const int nkb = LAST ? min(2, (N - kv0 + 31) >> 5) : 2;
    const bool ragged = LAST && kv0 + KC > N;
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if (kb < nkb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
        const char* krow = kl + (kb * 32 + col) * 128;
#pragma unroll
        for (int st = 0; st < 4; ++st)
          s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              *reinterpret_cast<const bf16x8*>(krow + (((st * 2 + half) ^ swk) << 4)), qf[st],
              s[kb], 0, 0, 0);
      }
    }
    if (ragged) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kv0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
          if (key >= N) s[kb][r] = -INFINITY;
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
      if (kb < nkb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
      }
    mx = pair_max(mx) * scale_log2;
    // deferred rescale (attention_bf16_kernel): only when some lane's max grows by > 8
    if (__builtin_amdgcn_ballot_w64(mx > m_run + 8.f)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      m_run = m_new;
      l_run *= alpha;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
    }
    const float nm = -m_run;
    float ps0 = 0.f, ps1 = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if (kb < nkb) {
        // V^T fragments of this key block (inline asm: see attention_bf16_ps_kernel)
        bf16x4 vf[2][2][2];
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            const uint32_t a = vs + va0[db] + (kb * 32 + 16 * st) * 128;
            asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(vf[st][db][0]) : "v"(a));
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:1024" : "=v"(vf[st][db][1]) : "v"(a));
          }
        bf16x8 pb[2];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          float e[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            e[j] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kb][8 * st + j], scale_log2, nm));
            if (j & 1) ps1 += e[j];
            else ps0 += e[j];
          }
          pb[st] = __builtin_bit_cast(bf16x8, i32x4{(int)pack_bf16x2(e[0], e[1]),
                                                    (int)pack_bf16x2(e[2], e[3]),
                                                    (int)pack_bf16x2(e[4], e[5]),
                                                    (int)pack_bf16x2(e[6], e[7])});
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            const bf16x4 lo = vf[st][db][0], hi = vf[st][db][1];
            const bf16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pb[st], o[db], 0, 0, 0);
          }
      }
    }
    l_run += ps0 + ps1;
  };
  for (int c = 0; c + 1 < nch; ++c) chunk(c, std::false_type{});
  chunk(nch - 1, std::true_type{});

  // every wave done with the ring: O restaged per wave (32 rows x 144 B) and stored as whole
  // 128-B rows (the buffer range check drops rows >= N)
  __builtin_amdgcn_s_barrier();
  const float inv = 1.f / pair_sum(l_run);
  const uint32_t wst = lds_base + wave * (32 * 144);
  if (active) {
    const uint32_t wa = wst + col * 144 + 8 * half;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint2 vv = {pack_bf16x2(o[db][4 * g + 0] * inv, o[db][4 * g + 1] * inv),
                          pack_bf16x2(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv)};
        asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(wa), "v"(vv), "n"((db * 32 + 8 * g) * 2)
                     : "memory");
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
      out + (int64_t)b * N * ldo, 0, N * ldo * 2, 0x00020000);
  const char* wsp = smem + wave * (32 * 144);
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int r = pass * 8 + lrow;
    i32x4 vv;
    asm volatile("ds_read_b128 %0, %1" : "=v"(vv) : "v"(wst + r * 144 + lchunk * 16) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (active)
      __builtin_amdgcn_raw_buffer_store_b128(vv, ro, ((q0 + r) * ldo + h * DKP + lchunk * 8) * 2,
                                             0, 0);
  }
  (void)wsp;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------
// Persistent short-sequence kernel, 16 queries per wave (bf16, DKP = 64, N in
// (16 (NKB - 1), 16 NKB]; the C2 shape N = 196 is NKB = 13).  The 32-query kernel above runs
// 2 waves per SIMD (7 active of 8 at N = 196) with ~190 registers each: its softmax chains
// (a 56-deep max, exponentials feeding the PV MFMAs) have little else to hide behind.  Here a
// workgroup has NKB waves (one 16-query block each, every wave active at N = 196) with
// <= 128 registers: 3-4 waves per SIMD.  v_mfma_f32_16x16x32_bf16 throughout:
//   S^T block kb (16 keys x 16 queries) = K[16 kb .. +15] . Q^T: lane l holds query
//   q0 + (l & 15) and keys 16 kb + 4 g + r (g = l >> 4, r = 0..3);
//   O^T (64 d x 16 queries) += V^T . P^T per 32-key step ks: P^T's 8 K-elements of lane l are
//   its own scores of blocks 2 ks and 2 ks + 1 (keys 16 (2ks) + 4g + 0..3 and
//   16 (2ks + 1) + 4g + 0..3, all lane-local), and V^T's are the same keys at d = 16 db +
//   (l & 15), two ds_read_b64_tr_b16 (one 4-key x 16-d block per 16-lane group);
//   row max / sum: in-lane trees, then the four lanes l, l ^ 16, l ^ 32, l ^ 48 of a query
//   (gfx950 lane swaps).
// Loads as in the 32-query kernel: K / V of a pair (N rounded up to 32 rows of 128 B: an odd
// last 16-key block pairs with zero P against clamped, finite V rows) by LDS-DMA into one of
// two slots one pair ahead, Q one pair ahead; O restaged through the pair's slot and stored
// as whole 128-B rows (buffer range check drops rows >= N): 2 stores per wave, `vmcnt(2)`.
// LDS images (swizzle on the DMA source): K, Q rows chunk ^ ((row >> 1) & 7) (the 16 rows x
// 16 B of every ds_read_b128 lane group hit 16 distinct bank slots for this read pattern);
// V rows chunk ^ (((row >> 1) & 3) << 1) (the 8 rows x 32 B of a tr-read half-wave cover the
// 64 banks once).  Same operations per score / output as attention_bf16_ps_kernel, summed in
// another order: equal to within fp32 / bf16-P rounding (tested against it and fp64).
#if VTD_DIAG   // diagnostic build only: measured neutral against attention_bf16_ps_kernel at C2
__device__ __forceinline__ int swz_v16(int row) { return ((row >> 1) & 3) << 1; }
__device__ __forceinline__ float xmax16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xadd16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// f(integral_constant<int, I>) for I in the sequence, in order (compile-time indices)
template <int... I, class F>
__device__ __forceinline__ void static_for(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}

template <int OFF>
__device__ __forceinline__ bf16x4 tr_read(uint32_t a) {
  bf16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return v;
}

template <int NKB>
__global__ __launch_bounds__(1024, 1) void attention_bf16_ps16_kernel(
    const bf16_t* __restrict__ qkv, int npairs, int N, int heads, int ldqkv, float scale_log2,
    bf16_t* __restrict__ out, int ldo) {
  constexpr int DKP = 64;
  constexpr int NKS = (NKB + 1) / 2;             // 32-key PV steps
  constexpr int NR = 32 * NKS;                   // LDS rows per matrix
  constexpr int SLOT = 2 * NR * 128;             // K image, then V image
  constexpr int NG = NR / 8;                     // 8-row DMA groups per matrix
  typedef __attribute__((address_space(3))) void lds_void_t;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, fr = lane & 15, g = lane >> 4;
  char* const qarea = smem + 2 * SLOT;
  const int inner = heads * DKP;
  const int q0 = wave * 16;
  const int G = gridDim.x;
  const int lrow = lane >> 3, lchunk = lane & 7;
  const uint32_t lds_base =
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(smem);

  // DMA of one matrix (part 0 = Q, 1 = K, 2 = V) of pair p into dst
  auto issue = [&](int p, int part, char* dst) {
    const int b = p / heads, h = p - b * heads;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(qkv + (int64_t)b * N * ldqkv), 0, N * ldqkv * 2, 0x00020000);
    const int colb = (part * inner + h * DKP) * 2;
    for (int gi = wave; gi < NG; gi += NKB) {
      const int r = gi * 8 + lrow;
      const int sw = part == 2 ? swz_v16(r) : swz_kq(r);
      const int voff = min(r, N - 1) * ldqkv * 2 + colb + ((lchunk ^ sw) << 4);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + gi * 1024), 16, voff, 0,
                                               0, 0);
    }
  };

  int p = blockIdx.x;
  if (p >= npairs) return;                       // uniform per workgroup
  issue(p, 1, smem);
  issue(p, 2, smem + NR * 128);
  issue(p, 0, qarea);
  // lane-constant pieces of the LDS addresses
  const int skq = (fr >> 1) & 7;                 // swz_kq of rows 16 kb + fr and q0 + fr
  const int tr_row = 4 * g + (fr >> 2);          // tr-read: key row within a 16-key block
  const int tr_p = fr & 3;                       // tr-read: 4-d piece within the 16-d block
  const int swv = swz_v16(tr_row);               // (row >> 1) & 3: independent of the block
  for (int it = 0; p < npairs; p += G, ++it) {
    char* const kl = smem + (it & 1) * SLOT;
    const uint32_t kl_addr = lds_base + (it & 1) * SLOT, vl_addr = kl_addr + NR * 128;
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // previous pair's O stores may fly
    __builtin_amdgcn_s_barrier();
    bf16x8 qf[2];
    {
      const int row = q0 + fr;
#pragma unroll
      for (int st = 0; st < 2; ++st)
        qf[st] = *reinterpret_cast<const bf16x8*>(qarea + row * 128 + (((4 * st + g) ^ skq) << 4));
    }
    const int pn = p + G;
    const bool fetch = pn < npairs;
    if (fetch) {
      char* const kn = smem + ((it + 1) & 1) * SLOT;
      issue(pn, 1, kn);
      issue(pn, 2, kn + NR * 128);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Q fragments in registers
    __builtin_amdgcn_s_barrier();
    if (fetch) issue(pn, 0, qarea);

    // ---- S^T blocks: all NKB at once (independent 2-MFMA chains); the row max as a tree
    f32x4 s[2 * NKS];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      s[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const char* krow = kl + (kb * 16 + fr) * 128;
#pragma unroll
      for (int st = 0; st < 2; ++st)
        s[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            *reinterpret_cast<const bf16x8*>(krow + (((4 * st + g) ^ skq) << 4)), qf[st], s[kb],
            0, 0, 0);
    }
    if (N < NKB * 16) {                          // keys >= N of the last block
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((NKB - 1) * 16 + 4 * g + r >= N) s[NKB - 1][r] = -INFINITY;
    }
    float bm[NKB];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
      bm[kb] = fmaxf(fmaxf(s[kb][0], s[kb][1]), fmaxf(s[kb][2], s[kb][3]));
#pragma unroll
    for (int w = 1; w < NKB; w *= 2)
#pragma unroll
      for (int kb = 0; kb + w < NKB; kb += 2 * w) bm[kb] = fmaxf(bm[kb], bm[kb + w]);
    const float mx = xmax16(pair_max(bm[0])) * scale_log2;
    const float nmx = -mx;
    // ---- P = exp2(S c - max), O^T += V^T . P^T per 32-key step; V^T by tr-reads (inline
    // asm: the compiler's tr-read would wait for the in-flight DMA), offsets immediate
    f32x4 o[4];
#pragma unroll
    for (int db = 0; db < 4; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint32_t va[4];
#pragma unroll
    for (int db = 0; db < 4; ++db)
      va[db] = vl_addr + tr_row * 128 + (((2 * db + (tr_p >> 1)) ^ swv) << 4) + (tr_p & 1) * 8;
    float ps[4] = {0.f, 0.f, 0.f, 0.f};
    auto step = [&](auto ks_tag) {
      constexpr int ks = decltype(ks_tag)::value;
      bf16x4 lo[4], hi[4];
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        lo[db] = tr_read<ks * 4096>(va[db]);
        hi[db] = tr_read<ks * 4096 + 2048>(va[db]);
      }
      float e[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        e[j] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[2 * ks][j], scale_log2, nmx));
        ps[j] += e[j];
      }
      if constexpr (2 * ks + 1 < NKB) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          e[4 + j] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[2 * ks + 1][j], scale_log2, nmx));
          ps[j] += e[4 + j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) e[4 + j] = 0.f;   // the odd block past the last: P = 0
      }
      const bf16x8 pb = __builtin_bit_cast(bf16x8, i32x4{(int)pack_bf16x2(e[0], e[1]),
                                                         (int)pack_bf16x2(e[2], e[3]),
                                                         (int)pack_bf16x2(e[4], e[5]),
                                                         (int)pack_bf16x2(e[6], e[7])});
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16x8 a = {lo[db][0], lo[db][1], lo[db][2], lo[db][3],
                          hi[db][0], hi[db][1], hi[db][2], hi[db][3]};
        o[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb, o[db], 0, 0, 0);
      }
    };
    static_for(std::make_integer_sequence<int, NKS>{}, step);
    const float l_run = (ps[0] + ps[1]) + (ps[2] + ps[3]);
    // every wave done reading this slot's K / V: restage O in it, store whole rows
    __builtin_amdgcn_s_barrier();
    const float inv = 1.f / xadd16(pair_sum(l_run));
    char* const wst = kl + wave * (16 * 144);
    {
      // lane: query row fr, d = 16 db + 4 g + 0..3 -> 8 B at byte 32 db + 8 g
      const uint32_t wa = kl_addr + wave * (16 * 144) + fr * 144 + 8 * g;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const uint2 v = {pack_bf16x2(o[db][0] * inv, o[db][1] * inv),
                         pack_bf16x2(o[db][2] * inv, o[db][3] * inv)};
        if (db == 0) asm volatile("ds_write_b64 %0, %1 offset:0" ::"v"(wa), "v"(v) : "memory");
        if (db == 1) asm volatile("ds_write_b64 %0, %1 offset:32" ::"v"(wa), "v"(v) : "memory");
        if (db == 2) asm volatile("ds_write_b64 %0, %1 offset:64" ::"v"(wa), "v"(v) : "memory");
        if (db == 3) asm volatile("ds_write_b64 %0, %1 offset:96" ::"v"(wa), "v"(v) : "memory");
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // wave-local: own writes landed
    {
      const int b = p / heads, h = p - b * heads;
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
          out + (int64_t)b * N * ldo, 0, N * ldo * 2, 0x00020000);
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        const int r = pass * 8 + lrow;
        const i32x4 v = *reinterpret_cast<const i32x4*>(wst + r * 144 + lchunk * 16);
        // rows >= N fall outside the range: dropped
        __builtin_amdgcn_raw_buffer_store_b128(v, ro, ((q0 + r) * ldo + h * DKP + lchunk * 8) * 2,
                                               0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int launch_bf16_ps16(const void* qkv, int B, int N, int heads, int ldqkv, float scale,
                     void* out, int ldo, hipStream_t stream) {
  constexpr int NKB = 13;                        // N in (192, 208]: C2 (N = 196)
  constexpr int NR = 32 * ((NKB + 1) / 2);
  constexpr int lds = 5 * NR * 128;
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_bf16_ps16_kernel<NKB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  });
  const int npairs = B * heads;
  const int kg = knob(VTD_KNOB_ATTN_GRID);
  const int grid = std::min(npairs, kg > 0 ? kg : device_cu_count());
  hipLaunchKernelGGL(attention_bf16_ps16_kernel<NKB>, dim3(grid), dim3(64 * NKB), lds, stream,
                     static_cast<const bf16_t*>(qkv), npairs, N, heads, ldqkv,
                     scale * 1.4426950408889634f, static_cast<bf16_t*>(out), ldo);
  VTD_LAUNCH_CHECK("attention_bf16_ps16");
  return VTD_OK;
}
#endif  // VTD_DIAG

int launch_bf16_ps(const void* qkv, int B, int N, int heads, int ldqkv, float scale, void* out,
                   int ldo, hipStream_t stream, int parts) {
  const int NR = (N + 31) & ~31;
  const int lds = 5 * NR * 128;
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
#define VTD_PS_FN(NB) reinterpret_cast<const void*>(&attention_bf16_ps_kernel<NB, 1>), \
                      reinterpret_cast<const void*>(&attention_bf16_ps_kernel<NB, 2>), \
                      reinterpret_cast<const void*>(&attention_bf16_ps_kernel<NB, 4>),
    for (const void* f : {VTD_PS_FN(5) VTD_PS_FN(6) VTD_PS_FN(7) VTD_PS_FN(8)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 5 * 256 * 128);
#undef VTD_PS_FN
  });
  const int ncu = device_cu_count();
  const int npairs = B * heads;
  // workgroups: one per CU, divided by the concurrent micro-batch parts of a split forward
  // (their attention launches co-run: half the chip each, +0.2 % at C2 B = 256, +0.4 % at
  // B = 64, profiles/r05_attn_grid_ab.log); knob VTD_KNOB_ATTN_GRID overrides
  const int kg = knob(VTD_KNOB_ATTN_GRID);
  const int grid = std::min(npairs, kg > 0 ? kg : ncu / std::max(parts, 1));
  // the last block's 8-key groups holding keys < N (1, 2 or 4 = untrimmed)
  const int tail = N - (NR - 32), tg = tail <= 8 ? 1 : tail <= 16 ? 2 : 4;
#define VTD_PS_PICK(NB) (tg == 1 ? attention_bf16_ps_kernel<NB, 1>                          \
                         : tg == 2 ? attention_bf16_ps_kernel<NB, 2> : attention_bf16_ps_kernel<NB, 4>)
  auto* kern = NR == 160 ? VTD_PS_PICK(5)
               : NR == 192 ? VTD_PS_PICK(6)
               : NR == 224 ? VTD_PS_PICK(7)
                           : VTD_PS_PICK(8);
#undef VTD_PS_PICK
#if VTD_DIAG
  static const int dmode = getenv("VTD_ATTN_DMODE") ? atoi(getenv("VTD_ATTN_DMODE")) : 0;
#else
  constexpr int dmode = 0;
#endif
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, stream, static_cast<const bf16_t*>(qkv),
                     npairs, N, heads, ldqkv, scale * 1.4426950408889634f,
                     static_cast<bf16_t*>(out), ldo, dmode);
  VTD_LAUNCH_CHECK("attention_bf16_ps");
  return VTD_OK;
}

// the long-sequence kernel: waves per workgroup chosen so that the last query block of a pair
// leaves the fewest waves idle (ties: more waves; 4 to 6 -- 8 spills at 128 VGPRs); KS = 3
// ring slots (48 KiB: 3 workgroups of <= 5 waves per CU, 2 of 6)
int launch_bf16_fl(const void* qkv, int B, int N, int heads, int ldqkv, float scale, void* out,
                   int ldo, hipStream_t stream) {
  constexpr int KS = 3, LDS = KS * 2 * 64 * 128;
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
    for (const void* f : {reinterpret_cast<const void*>(&attention_bf16_fl_kernel<4, KS>),
                          reinterpret_cast<const void*>(&attention_bf16_fl_kernel<5, KS>),
                          reinterpret_cast<const void*>(&attention_bf16_fl_kernel<6, KS>)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
  });
  const int nq = (N + 31) / 32;
  int nw = 6, best = 1 << 30;
  for (int w : {6, 5, 4}) {
    const int idle = (nq + w - 1) / w * w - nq;
    if (idle < best) best = idle, nw = w;
  }
  const int nqb = (nq + nw - 1) / nw;
  VTD_CHECK_ARG((int64_t)nqb * heads * B < INT32_MAX && (int64_t)N * ldqkv * 2 < INT32_MAX &&
                    (int64_t)N * ldo * 2 < INT32_MAX,
                "attention: grid / image too large for the long-sequence kernel");
  const dim3 grid(nqb * heads * B);
  const float sl2 = scale * 1.4426950408889634f;
  const bf16_t* q = static_cast<const bf16_t*>(qkv);
  bf16_t* o = static_cast<bf16_t*>(out);
  switch (nw) {
    case 4: hipLaunchKernelGGL((attention_bf16_fl_kernel<4, KS>), grid, dim3(256), LDS, stream, q, N, heads, ldqkv, sl2, o, ldo, nqb); break;
    case 5: hipLaunchKernelGGL((attention_bf16_fl_kernel<5, KS>), grid, dim3(320), LDS, stream, q, N, heads, ldqkv, sl2, o, ldo, nqb); break;
    default: hipLaunchKernelGGL((attention_bf16_fl_kernel<6, KS>), grid, dim3(384), LDS, stream, q, N, heads, ldqkv, sl2, o, ldo, nqb);
  }
  VTD_LAUNCH_CHECK("attention_bf16_fl");
  return VTD_OK;
}

// ---------------------------------------------------------------------------------
// Split-bf16 kernel (the VTD_BF16X3 parity mode; include/vtd.h "Split-bf16 operands").
// Q, K, V arrive as f32 (the query/key/value GEMM's f32 output) and every product runs on
// the bf16 MFMA as three: hi.hi + lo.hi + hi.lo with hi = bf16(v), lo = bf16(v - hi), fp32
// accumulators -- S^T = K Q^T over (K_hi, K_lo) x (Q_hi, Q_lo) and O^T += V^T P^T over
// (V_hi, V_lo) x (P_hi, P_lo), P in fp32 split the same way; the dropped lo.lo term is
// <= 2^-18 of each product.  Softmax statistics stay fp32.  Structure as
// attention_bf16_kernel (32 queries per wave, 64-key chunks register-staged from global
// memory into one of two LDS buffers, one barrier per chunk, the deferred-rescale online
// softmax); the split of K / V happens once per workgroup, in the staging write (hi and lo
// planes with the bf16 kernel's row strides, so the K reads and the V^T tr-reads are the
// bf16 kernel's).  The output is written directly as the attention_output GEMM's split-bf16
// A operand [hi | lo] (two P = ldo / 2 wide pieces), so no split pass follows it.
template <int DKP, int KC_ = 64>
struct AttnX3Cfg {
  static constexpr int KC = KC_;                      // keys per chunk
  static constexpr int NKB = KC / 32;                 // 32-key blocks per chunk
  static constexpr int KS = DKP * 2 + 16;             // K row stride (bytes, per plane)
  static constexpr int VS = DKP * 2 + 64;             // V row stride (bytes, per plane)
  static constexpr int PLANE = KC * KS + KC * VS;     // K then V image of one plane
  static constexpr int BUF = 2 * PLANE;               // hi plane, lo plane
  static constexpr int CPR = DKP / 4;                 // 16-B f32 chunks per row
  static constexpr int NCH = KC * CPR * 2;            // chunks per K + V tile
  static constexpr int KSTEPS = DKP / 16;
  static constexpr int DB = DKP / 32;
};

// 8 f32 values -> split-bf16 (hi, lo) fragments
__device__ __forceinline__ void split8(const f32x4& a, const f32x4& b, bf16x8& hi, bf16x8& lo) {
  const uint32_t h0 = pack_bf16x2(a[0], a[1]), h1 = pack_bf16x2(a[2], a[3]);
  const uint32_t h2 = pack_bf16x2(b[0], b[1]), h3 = pack_bf16x2(b[2], b[3]);
  hi = __builtin_bit_cast(bf16x8, i32x4{(int)h0, (int)h1, (int)h2, (int)h3});
  lo = __builtin_bit_cast(bf16x8, i32x4{(int)pack_lo_bf16x2(a[0], a[1], h0),
                                        (int)pack_lo_bf16x2(a[2], a[3], h1),
                                        (int)pack_lo_bf16x2(b[0], b[1], h2),
                                        (int)pack_lo_bf16x2(b[2], b[3], h3)});
}

template <int DKP, int NWG, int KC = 64, int MINB = 1>
__global__ __launch_bounds__(64 * NWG, MINB) void attention_x3_kernel(
    const float* __restrict__ qkv, int N, int heads, int ldqkv, float scale_log2,
    bf16_t* __restrict__ out, int ldo, int nqb) {
  using C = AttnX3Cfg<DKP, KC>;
  typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  constexpr int nthreads = 64 * NWG;
  const int lane = tid & 63, wave = tid >> 6, half = lane >> 5, col = lane & 31;
  int v = blockIdx.x;                  // XCD-aware: a pair's query blocks share an XCD
  {
    const int G = gridDim.x, xcd = v & 7, q8 = G >> 3, r8 = G & 7;
    v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (v >> 3);
  }
  const int pair = v / nqb, qb = v - pair * nqb;
  const int b = pair / heads, h = pair - b * heads;
  const int inner = heads * DKP;
  const int64_t row0 = (int64_t)b * N;
  const int q0 = (qb * NWG + wave) * 32;
  const bool active = q0 < N;
  const int P = ldo / 2;               // piece width of the split output

  bf16x8 qh[C::KSTEPS], ql[C::KSTEPS];
  {
    const int q = min(q0 + col, N - 1);
    const float* qp = qkv + (row0 + q) * ldqkv + h * DKP;
#pragma unroll
    for (int st = 0; st < C::KSTEPS; ++st)
      split8(*reinterpret_cast<const f32x4*>(qp + st * 16 + half * 8),
             *reinterpret_cast<const f32x4*>(qp + st * 16 + half * 8 + 4), qh[st], ql[st]);
  }
  f32x16 o[C::DB];
#pragma unroll
  for (int i = 0; i < C::DB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  constexpr int NPASS = (C::NCH + nthreads - 1) / nthreads;
  f32x4 stg[NPASS];
  auto gload = [&](int kv0) {
#pragma unroll
    for (int i = 0; i < NPASS; ++i) {
      const int c = tid + i * nthreads;
      if (c < C::NCH) {
        const int isv = c >= C::KC * C::CPR;
        const int cc = c - isv * C::KC * C::CPR;
        const int kr = cc / C::CPR, ch = cc - kr * C::CPR;
        const int key = min(kv0 + kr, N - 1);
        stg[i] = *reinterpret_cast<const f32x4*>(qkv + (row0 + key) * ldqkv +
                                                 (1 + isv) * inner + h * DKP + ch * 4);
      }
    }
  };
  // split once per workgroup: 4 f32 -> 8 B of the hi plane + 8 B of the lo plane
  auto swrite = [&](int buf) {
    char* base = smem + buf * C::BUF;
#pragma unroll
    for (int i = 0; i < NPASS; ++i) {
      const int c = tid + i * nthreads;
      if (c < C::NCH) {
        const int isv = c >= C::KC * C::CPR;
        const int cc = c - isv * C::KC * C::CPR;
        const int kr = cc / C::CPR, ch = cc - kr * C::CPR;
        char* dst = isv ? base + C::KC * C::KS + kr * C::VS + ch * 8 : base + kr * C::KS + ch * 8;
        const uint32_t h0 = pack_bf16x2(stg[i][0], stg[i][1]), h1 = pack_bf16x2(stg[i][2], stg[i][3]);
        *reinterpret_cast<uint2*>(dst) = uint2{h0, h1};
        *reinterpret_cast<uint2*>(dst + C::PLANE) =
            uint2{pack_lo_bf16x2(stg[i][0], stg[i][1], h0), pack_lo_bf16x2(stg[i][2], stg[i][3], h1)};
      }
    }
  };

  const int nchunks = (N + C::KC - 1) / C::KC;
  gload(0);
  swrite(0);
  __syncthreads();
  const int tr_key = 4 * half + ((lane & 15) >> 2);
  const int tr_d = ((lane >> 4) & 1) * 16 + (lane & 3) * 4;
  auto chunk = [&](int c, auto last_tag) {
    constexpr bool LAST = decltype(last_tag)::value;
    const int kv0 = c * C::KC;
    if (!LAST) gload(kv0 + C::KC);
    if (active) {
      const char* kl = smem + (c & 1) * C::BUF;      // hi plane; lo plane at + PLANE
      const char* vl = kl + C::KC * C::KS;
      const int nkb = LAST ? min(C::NKB, (N - kv0 + 31) >> 5) : C::NKB;
      const bool ragged = LAST && kv0 + C::KC > N;
      f32x16 s[C::NKB];
#pragma unroll
      for (int kb = 0; kb < C::NKB; ++kb) {
        if (kb < nkb) {
#pragma unroll
          for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
          const char* krow = kl + (kb * 32 + col) * C::KS;
#pragma unroll
          for (int st = 0; st < C::KSTEPS; ++st) {
            const bf16x8 kh = *reinterpret_cast<const bf16x8*>(krow + (st * 16 + half * 8) * 2);
            const bf16x8 klo =
                *reinterpret_cast<const bf16x8*>(krow + C::PLANE + (st * 16 + half * 8) * 2);
            s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, qh[st], s[kb], 0, 0, 0);
            s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(klo, qh[st], s[kb], 0, 0, 0);
            s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, ql[st], s[kb], 0, 0, 0);
          }
        }
      }
      if (ragged) {
#pragma unroll
        for (int kb = 0; kb < C::NKB; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kv0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
            if (key >= N) s[kb][r] = -INFINITY;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < C::NKB; ++kb)
        if (kb < nkb) {
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
        }
      mx = pair_max(mx) * scale_log2;
      // deferred rescale (attention_bf16_kernel): P <= 256, split exactly as any f32 value
      if (__builtin_amdgcn_ballot_w64(mx > m_run + 8.f)) {
        const float m_new = fmaxf(m_run, mx);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        l_run *= alpha;
#pragma unroll
        for (int i = 0; i < C::DB; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
      }
      float ps0 = 0.f, ps1 = 0.f;
      const float nm = -m_run;
#pragma unroll
      for (int kb = 0; kb < C::NKB; ++kb)
        if (kb < nkb) {
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const float p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kb][r], scale_log2, nm));
            const float p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kb][r + 1], scale_log2, nm));
            s[kb][r] = p0;
            s[kb][r + 1] = p1;
            ps0 += p0;
            ps1 += p1;
          }
        }
      l_run += ps0 + ps1;
#pragma unroll
      for (int kb = 0; kb < C::NKB; ++kb)
        if (kb < nkb) {
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            bf16x8 ph, pl;
            split8(f32x4{s[kb][8 * st + 0], s[kb][8 * st + 1], s[kb][8 * st + 2], s[kb][8 * st + 3]},
                   f32x4{s[kb][8 * st + 4], s[kb][8 * st + 5], s[kb][8 * st + 6], s[kb][8 * st + 7]},
                   ph, pl);
            const int key0 = kb * 32 + 16 * st + tr_key;
#pragma unroll
            for (int db = 0; db < C::DB; ++db) {
              const char* va = vl + key0 * C::VS + (db * 32 + tr_d) * 2;
              const bf16x4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)va);
              const bf16x4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(va + 8 * C::VS));
              const bf16x4 l0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(va + C::PLANE));
              const bf16x4 l1 =
                  __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(va + C::PLANE + 8 * C::VS));
              const bf16x8 vh = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
              const bf16x8 vlo = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
              o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, ph, o[db], 0, 0, 0);
              o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vlo, ph, o[db], 0, 0, 0);
              o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, pl, o[db], 0, 0, 0);
            }
          }
        }
    }
    if (!LAST) swrite((c + 1) & 1);
    __syncthreads();
  };
  for (int c = 0; c + 1 < nchunks; ++c) chunk(c, std::false_type{});
  chunk(nchunks - 1, std::true_type{});
  if (!active) return;
  const float inv = 1.f / pair_sum(l_run);
  if constexpr (DKP == 64) {
    // restaged through the LDS free after the loop's last barrier: per wave a hi and a lo
    // image of its 32 query rows (row stride 144 B), then whole 128-B rows per store
    char* wst = smem + wave * (2 * 32 * 144);
#pragma unroll
    for (int db = 0; db < C::DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float a = o[db][4 * g + 0] * inv, bb = o[db][4 * g + 1] * inv;
        const float cc = o[db][4 * g + 2] * inv, d = o[db][4 * g + 3] * inv;
        const uint32_t h0 = pack_bf16x2(a, bb), h1 = pack_bf16x2(cc, d);
        char* dst = wst + col * 144 + (db * 32 + 8 * g + 4 * half) * 2;
        *reinterpret_cast<uint2*>(dst) = uint2{h0, h1};
        *reinterpret_cast<uint2*>(dst + 32 * 144) =
            uint2{pack_lo_bf16x2(a, bb, h0), pack_lo_bf16x2(cc, d, h1)};
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // wave-local: own writes landed
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int r = pass * 8 + (lane >> 3), ch = lane & 7;
      if (q0 + r < N) {
        bf16_t* op = out + (row0 + q0 + r) * ldo + h * DKP + ch * 8;
        const i32x4 hv = *reinterpret_cast<const i32x4*>(wst + r * 144 + ch * 16);
        const i32x4 lv = *reinterpret_cast<const i32x4*>(wst + 32 * 144 + r * 144 + ch * 16);
        *reinterpret_cast<i32x4*>(op) = hv;
        *reinterpret_cast<i32x4*>(op + P) = lv;
      }
    }
    return;
  }
  const int q = q0 + col;
  if (q >= N) return;
  bf16_t* op = out + (row0 + q) * ldo + h * DKP;
#pragma unroll
  for (int db = 0; db < C::DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = db * 32 + 8 * g + 4 * half;
      const float a = o[db][4 * g + 0] * inv, bb = o[db][4 * g + 1] * inv;
      const float cc = o[db][4 * g + 2] * inv, dd = o[db][4 * g + 3] * inv;
      const uint32_t h0 = pack_bf16x2(a, bb), h1 = pack_bf16x2(cc, dd);
      const uint2 hv = {h0, h1}, lv = {pack_lo_bf16x2(a, bb, h0), pack_lo_bf16x2(cc, dd, h1)};
      *reinterpret_cast<uint2*>(op + d) = hv;
      *reinterpret_cast<uint2*>(op + P + d) = lv;
    }
}

template <int DKP, int KC = 64, int MINB = 1>
int launch_x3(const void* qkv, int B, int N, int heads, int ldqkv, float scale, void* out,
              int ldo, hipStream_t stream) {
  using C = AttnX3Cfg<DKP, KC>;
  constexpr int NWG = 8;
  // the K / V double buffer, or (dkp 64) the output restage: a hi and a lo image of 32 rows
  // x 144 B per wave
  constexpr int LDS = std::max(2 * C::BUF, DKP == 64 ? NWG * 2 * 32 * 144 : 0);
  const int nq = (N + 31) / 32, nqb = (nq + NWG - 1) / NWG;
  VTD_CHECK_ARG((int64_t)nqb * heads * B < INT32_MAX, "attention: grid too large");
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_x3_kernel<DKP, NWG, KC, MINB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
  });
  hipLaunchKernelGGL((attention_x3_kernel<DKP, NWG, KC, MINB>), dim3(nqb * heads * B),
                     dim3(64 * NWG), LDS, stream, static_cast<const float*>(qkv), N, heads, ldqkv,
                     scale * 1.4426950408889634f, static_cast<bf16_t*>(out), ldo, nqb);
  VTD_LAUNCH_CHECK("attention_x3");
  return VTD_OK;
}

template <int DKP, int NWG, bool MX8 = false>
int launch_bf16_v2(const void* qkv, int B, int N, int heads, int ldqkv, float scale,
                   void* out, int ldo, hipStream_t stream, uint8_t* s8 = nullptr,
                   int64_t s_rows = 0) {
  using C = AttnBf16Cfg<DKP>;
  const int nq = (N + 31) / 32, nqb = (nq + NWG - 1) / NWG;
  VTD_CHECK_ARG((int64_t)nqb * heads * B < INT32_MAX, "attention: grid too large");
  const dim3 grid(nqb * heads * B);
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
    (void)hipFuncSetAttribute(
        reinterpret_cast<const void*>(&attention_bf16_kernel<DKP, NWG, MX8>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 2 * C::BUF);
  });
  // XCD-aware order: C3 attention 382.5-383.2 vs 384.0-384.2 us per launch, forward
  // 1,812-1,813 vs 1,783-1,790 img/s (profiles/r03_attn_xcd_order_ab.log); the kernel is
  // VALU-bound, its K / V re-reads were mostly served beyond L2 at no visible cost
  const int xcd_remap = 1;
  hipLaunchKernelGGL((attention_bf16_kernel<DKP, NWG, MX8>), grid, dim3(64 * NWG), 2 * C::BUF,
                     stream, static_cast<const bf16_t*>(qkv), N, heads, ldqkv,
                     scale * 1.4426950408889634f, static_cast<bf16_t*>(out), ldo, s8, s_rows,
                     nqb, xcd_remap);
  VTD_LAUNCH_CHECK("attention_bf16");
  return VTD_OK;
}

template <typename T, int DKP>
int launch(const void* qkv, int B, int N, int heads, int ldqkv, float scale, void* out,
           int ldo, hipStream_t stream) {
  using C = AttnCfg<T, DKP>;
  const int nq = (N + 31) / 32;
  const int nw = nq <= 8 ? nq : 8;
  dim3 grid((nq + nw - 1) / nw, heads, B);
  static std::once_flag once[kMaxDevices];
  once_per_device(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_kernel<T, DKP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
  });
  const float scale_log2 = scale * 1.4426950408889634f;
  hipLaunchKernelGGL((attention_kernel<T, DKP>), grid, dim3(64 * nw), C::LDS, stream,
                     static_cast<const T*>(qkv), N, heads, ldqkv, scale_log2,
                     static_cast<T*>(out), ldo);
  VTD_LAUNCH_CHECK("attention");
  return VTD_OK;
}

}  // namespace

int attention_launch(const void* qkv, int B, int N, int heads, int dkp, int ldqkv,
                     float scale, void* out, int ldo, int dtype, hipStream_t stream,
                     double flops, int parts) {
  VTD_CHECK_ARG(qkv && out, "attention: null pointer");
  VTD_CHECK_ARG(B > 0 && N > 0 && heads > 0, "attention: bad B/N/heads");
  VTD_CHECK_ARG(dkp == 32 || dkp == 64 || dkp == 128, "attention: dkp must be 32/64/128");
  VTD_CHECK_ARG(dtype == VTD_F32 || dtype == VTD_BF16 || dtype == VTD_BF16X3,
                "attention: bad dtype");
  // VTD_BF16X3: f32 qkv in, the split-bf16 operand [hi | lo] out (ldo = 2 P, P >= inner)
  const int owidth = dtype == VTD_BF16X3 ? ldo / 2 : ldo;
  VTD_CHECK_ARG(dtype != VTD_BF16X3 || ldo % 2 == 0,
                "attention: a split-bf16 output needs ldo % 2 == 0");
  VTD_CHECK_ARG(ldqkv >= 3 * heads * dkp && owidth >= heads * dkp,
                "attention: leading dimensions too small");
  VTD_CHECK_ARG(ldqkv % 8 == 0 && owidth % 8 == 0, "attention: ld must be multiple of 8");
  ProfScope ps(stream, PROF_ATTN,
               flops > 0 ? flops : 4.0 * B * heads * (double)N * N * dkp);
  if (dtype == VTD_BF16X3) {
    if (dkp == 32) return launch_x3<32>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
    // dkp 64: 32-key chunks at <= 128 VGPRs, two workgroups per CU (the output restage's
    // 72 KiB of LDS each): C2 attention 208 -> 158 us per layer, bf16x3 forward +1.4 %, C3
    // 769 -> 713 us (profiles/r06_x3_attn_kc32_ab.log); knob VTD_KNOB_ATTN_VARIANT 10: the
    // 64-key chunks at one workgroup per CU (169 VGPRs, 84 KiB)
    if (dkp == 64 && knob(VTD_KNOB_ATTN_VARIANT) != 10)
      return launch_x3<64, 32, 2>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
    if (dkp == 64) return launch_x3<64>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
    return launch_x3<128>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
  }
  if (dtype == VTD_BF16) {
    // knob VTD_KNOB_ATTN_VARIANT (environment read once per process; tests set it per call)
    const int kv = knob(VTD_KNOB_ATTN_VARIANT);
    const int v1 = kv >= 0 ? kv : 4;
    // 4 (default): the persistent kernel where it applies (dkp 64, 128 < N <= 256, whole
    // 128-B rows and 16-B aligned row pitches), else as 2
    const bool ps_ok = dkp == 64 && N > 128 && N <= 256 && ldqkv % 8 == 0 && ldo % 8 == 0 &&
                       (int64_t)N * ldqkv * 2 < INT32_MAX && (int64_t)N * ldo * 2 < INT32_MAX;
    // 5 (diagnostic build): the 16-query-per-wave persistent kernel at N in (192, 208] (C2),
    // else (and in the product library) as 4
#if VTD_DIAG
    if (v1 == 5 && ps_ok && N > 192 && N <= 208)
      return launch_bf16_ps16(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
#endif
    if ((v1 == 4 || v1 == 5) && ps_ok)
      return launch_bf16_ps(qkv, B, N, heads, ldqkv, scale, out, ldo, stream, parts);
    // 6: the long-sequence LDS-DMA kernel (dkp 64, any N; opt-in: measured slower than the
    // streaming kernel at C3 / C5, profiles/r05_attn_fl_ab.log)
    if (dkp == 64 && ldqkv % 8 == 0 && ldo % 8 == 0 && v1 == 6)
      return launch_bf16_fl(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
    if (v1 == 1) {
      if (dkp == 32) return launch<bf16_t, 32>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
      if (dkp == 64) return launch<bf16_t, 64>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
      return launch<bf16_t, 128>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
    }
    // 8-wave workgroups (one (b,h) per WG to N=256): knob 3 always, knob 2 from N = 129, and the
    // default (4) for dkp 64 from N = 257 (C3 / C5: 311-330 vs 339-397 us at C3, 255-257 vs
    // 270-284 us at C5; 2 workgroups per CU at <= 128 VGPRs, profiles/r06_attn_8wave_default_ab.log)
    if (v1 == 3 || (v1 == 2 && N > 128) || (v1 == 4 && dkp == 64 && N > 256)) {
      if (dkp == 32) return launch_bf16_v2<32, 8>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
      if (dkp == 64) return launch_bf16_v2<64, 8>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
      return launch_bf16_v2<128, 8>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
    }
    if (dkp == 32) return launch_bf16_v2<32, 4>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
    if (dkp == 64) return launch_bf16_v2<64, 4>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
    return launch_bf16_v2<128, 4>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
  }
  if (dkp == 32) return launch<float, 32>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
  if (dkp == 64) return launch<float, 64>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
  return launch<float, 128>(qkv, B, N, heads, ldqkv, scale, out, ldo, stream);
}

int attention_mx8_launch(const void* qkv, int B, int N, int heads, int dkp, int ldqkv,
                         float scale, uint8_t* q, int ldq, uint8_t* s, int64_t s_rows,
                         hipStream_t stream, double flops) {
  VTD_CHECK_ARG(qkv && q && s, "attention_mx8: null pointer");
  VTD_CHECK_ARG(B > 0 && N > 0 && heads > 0, "attention_mx8: bad B/N/heads");
  VTD_CHECK_ARG(dkp == 32 || dkp == 64 || dkp == 128, "attention_mx8: dkp must be 32/64/128");
  VTD_CHECK_ARG((heads * dkp) % 128 == 0,
                "attention_mx8: heads * dkp must be a multiple of 128 (whole MX K-steps)");
  VTD_CHECK_ARG(ldqkv >= 3 * heads * dkp && ldqkv % 8 == 0 && ldq >= heads * dkp && ldq % 16 == 0,
                "attention_mx8: leading dimensions (ldqkv % 8, ldq % 16)");
  VTD_CHECK_ARG(s_rows >= (int64_t)B * N, "attention_mx8: s_rows < B * N");
  ProfScope ps(stream, PROF_ATTN,
               flops > 0 ? flops : 4.0 * B * heads * (double)N * N * dkp);
  // the streaming kernel's workgroup size as attention_launch picks it under knob 2 (4 waves
  // up to N = 128, else 8: C5's 576 keys), so that the two give the same bits
  if (N <= 128) {
    if (dkp == 32)
      return launch_bf16_v2<32, 4, true>(qkv, B, N, heads, ldqkv, scale, q, ldq, stream, s, s_rows);
    if (dkp == 64)
      return launch_bf16_v2<64, 4, true>(qkv, B, N, heads, ldqkv, scale, q, ldq, stream, s, s_rows);
    return launch_bf16_v2<128, 4, true>(qkv, B, N, heads, ldqkv, scale, q, ldq, stream, s, s_rows);
  }
  if (dkp == 32)
    return launch_bf16_v2<32, 8, true>(qkv, B, N, heads, ldqkv, scale, q, ldq, stream, s, s_rows);
  if (dkp == 64)
    return launch_bf16_v2<64, 8, true>(qkv, B, N, heads, ldqkv, scale, q, ldq, stream, s, s_rows);
  return launch_bf16_v2<128, 8, true>(qkv, B, N, heads, ldqkv, scale, q, ldq, stream, s, s_rows);
}

}  // namespace vtd

extern "C" int vtd_attention_mx8(const void* qkv_dev, int B, int N, int heads, int dkp,
                                 int ldqkv, float scale, uint8_t* q_dev, int ldq, uint8_t* s_dev,
                                 int64_t s_rows, void* stream) {
  return vtd::attention_mx8_launch(qkv_dev, B, N, heads, dkp, ldqkv, scale, q_dev, ldq, s_dev,
                                   s_rows, static_cast<hipStream_t>(stream), 0.0);
}

extern "C" int vtd_attention(const void* qkv_dev, int B, int N, int heads, int dkp,
                             int ldqkv, float scale, void* out_dev, int ldo, int dtype,
                             void* stream) {
  return vtd::attention_launch(qkv_dev, B, N, heads, dkp, ldqkv, scale, out_dev, ldo,
                               dtype, static_cast<hipStream_t>(stream), 0.0, 1);
}
