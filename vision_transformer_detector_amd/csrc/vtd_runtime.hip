// Host runtime of libvtd.so: error state, graph shapes, workspace plan, the whole
// forward (`model(images, training=False)`, vtd.py:498-583) as one sequence of
// launches on the caller's stream, and optional hipEvent per-launch profiling.
#include <atomic>
#include <algorithm>
#include <cmath>
#include <mutex>
#include <vector>

#include "vtd_common.h"

namespace vtd {

int gemm_launch(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                int dtype, const vtd_epilogue* epi, hipStream_t stream, double flops);
int gemm_launch_ln(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                   int dtype, const vtd_epilogue* epi, hipStream_t stream, double flops,
                   const float* lnpart, int lnslots, int lnD, float lneps);
int attention_launch(const void* qkv, int B, int N, int heads, int dkp, int ldqkv,
                     float scale, void* out, int ldo, int dtype, hipStream_t stream,
                     double flops, int parts = 1);
int layernorm_launch(const void* x, int x_dtype, int64_t rows, int D, int ldx, const float* g,
                     const float* b, float eps, void* y, int ldy, int dtype, hipStream_t st);
int ln_stats_launch(const void* x, int x_dtype, int64_t rows, int D, int ldx, float eps,
                    float* stat, hipStream_t st);
int ln_stats_finalize_launch(const float* part, int64_t rows, int slots, int D, float eps,
                             float* stat, hipStream_t st);
bool gemm_emits_stats(int M, int N, int dtype, const vtd_epilogue* e);
int gemm_splitk_choice(int M, int N, int K, int dtype, int target = 0);
int gemm_splitk_launch(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                       int dtype, const vtd_epilogue* epi, float* part, int ksplit,
                       hipStream_t stream, double flops);
int patches_launch(const float* img, int B, int H, int W, int C, int p, void* out, int ldo,
                   int dtype, hipStream_t st);
int attention_mx8_launch(const void* qkv, int B, int N, int heads, int dkp, int ldqkv,
                         float scale, uint8_t* q, int ldq, uint8_t* s, int64_t s_rows,
                         hipStream_t stream, double flops);
int quantize_mx8_launch(const void* x, int x_dtype, int64_t rows, int K, int ldx, int Kq,
                        uint8_t* q, int ldq, uint8_t* s, int64_t s_rows, hipStream_t st);
int layernorm_mx8_launch(const void* x, int x_dtype, int64_t rows, int D, int ldx,
                         const float* g, const float* b, float eps, uint8_t* q, int ldq, int Kq,
                         uint8_t* s, int64_t s_rows, hipStream_t st);
bool gemm_mx8_emits_fp8(int M, int N, const vtd_epilogue* e);
int split_bf16x3_launch(const float* x, int64_t rows, int K, int ldx, void* y, int ldy, int role,
                        hipStream_t st);
int gemm_mx8_launch(int M, int N, int K, const uint8_t* A, int lda, const uint8_t* sA,
                    int64_t sa_rows, const uint8_t* Bt, int ldb, const uint8_t* sB,
                    int64_t sb_rows, const vtd_epilogue* epi, hipStream_t stream,
                    double flops);

// ------------------------------------------------------------------ errors
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

// ------------------------------------------------------------------ knobs
namespace {
constexpr const char* kKnobEnv[VTD_KNOB_COUNT] = {"VTD_ATTN_VARIANT", "VTD_ATTN_GRID",
                                                  "VTD_GEMM_NGW", "VTD_SPLITK",
                                                  "VTD_JPEG_CHUNK_BITS", "VTD_SKINNY",
                                                  "VTD_F32_PP2", "VTD_STAGGER", "VTD_GEMM_TR",
                                                  "VTD_FIN_WGS", "VTD_GEMM_TPW"};
std::atomic<int> g_knob[VTD_KNOB_COUNT];
std::once_flag g_knob_once;
void knob_init() {
  std::call_once(g_knob_once, [] {
    for (int k = 0; k < VTD_KNOB_COUNT; ++k) {
      const char* v = getenv(kKnobEnv[k]);
      g_knob[k].store(v && *v ? atoi(v) : -1, std::memory_order_relaxed);
    }
  });
}
}  // namespace
int knob(int k) {
  knob_init();
  return g_knob[k].load(std::memory_order_relaxed);
}

// ------------------------------------------------------------------ devices
int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = 0;
  return dev;
}
int device_cu_count() {
  static std::once_flag once[kMaxDevices];
  static int ncu[kMaxDevices];
  const int dev = current_device();
  std::call_once(once[dev], [dev] {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    ncu[dev] = n;
  });
  return ncu[dev];
}

// ------------------------------------------------------------------ profiling
namespace {
struct ProfRecord { int cls; int ev0, ev1; double flops; };
struct ProfState {
  std::mutex mu;
  bool enabled = false;
  std::vector<hipEvent_t> events;
  int next_event = 0;
  std::vector<ProfRecord> pending;
  double ms[VTD_PROF_CLASSES] = {0};
  int64_t launches[VTD_PROF_CLASSES] = {0};
  double flops[VTD_PROF_CLASSES] = {0};
};
ProfState& prof() {
  static ProfState s;
  return s;
}
int prof_event() {  // caller holds the mutex
  ProfState& p = prof();
  if (p.next_event == (int)p.events.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return -1;
    p.events.push_back(e);
  }
  return p.next_event++;
}
}  // namespace

ProfScope::ProfScope(hipStream_t s, int c, double fl) : stream(s), cls(c), slot(-1) {
  ProfState& p = prof();
  if (!p.enabled) return;
  std::lock_guard<std::mutex> g(p.mu);
  int e0 = prof_event(), e1 = prof_event();
  if (e0 < 0 || e1 < 0) return;
  (void)hipEventRecord(p.events[e0], stream);
  p.pending.push_back({c, e0, e1, fl});
  slot = (int)p.pending.size() - 1;
}
ProfScope::~ProfScope() {
  if (slot < 0) return;
  ProfState& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  (void)hipEventRecord(p.events[p.pending[slot].ev1], stream);
}

// ------------------------------------------------------------------ shapes
static int derive(const vtd_config* c, vtd_dims* d) {
  VTD_CHECK_ARG(c && d, "null config/dims");
  VTD_CHECK_ARG(c->batch > 0 && c->image_h > 0 && c->image_w > 0 && c->channels > 0,
                "batch and input_shape must be positive");
  VTD_CHECK_ARG(c->patch_size > 0 && c->embedding_dim > 0 && c->num_heads > 0 &&
                    c->key_dim > 0 && c->mlp_quantities > 0 && c->repeat_times > 0,
                "patch_size, embedding_dim, heads, key_dim, mlp/repeat counts must be > 0");
  VTD_CHECK_ARG(c->mlp_quantities <= VTD_MAX_MLP, "encoder_mlp_quantities too large");
  VTD_CHECK_ARG(c->head_last_units > 0 && c->head_layers > 0 && c->head_repeats > 0 &&
                    c->head_layers * c->head_repeats <= VTD_MAX_HEAD,
                "bad mlp_head configuration");
  VTD_CHECK_ARG(c->dtype == VTD_F32 || c->dtype == VTD_BF16 || c->dtype == VTD_FP8 ||
                    c->dtype == VTD_BF16X3,
                "dtype must be F32, BF16, FP8 or BF16X3");
  VTD_CHECK_ARG(c->key_dim <= 128, "encoder_key_dim > 128 not supported");
  const int p = c->patch_size;
  d->grid_h = (c->image_h + p - 1) / p;
  d->grid_w = (c->image_w + p - 1) / p;
  d->tokens = d->grid_h * d->grid_w;
  d->pad_top = ((d->grid_h - 1) * p + p - c->image_h) / 2;
  d->pad_left = ((d->grid_w - 1) * p + p - c->image_w) / 2;
  d->patch_dim = p * p * c->channels;
  d->patch_dim_p = (int)round_up(d->patch_dim, VTD_KALIGN);
  d->d = c->embedding_dim;
  d->d_p = (int)round_up(d->d, VTD_KALIGN);
  int dkp = c->key_dim <= 32 ? 32 : (c->key_dim <= 64 ? 64 : 128);
  if ((c->num_heads * dkp) % VTD_KALIGN) dkp *= 2;
  VTD_CHECK_ARG(dkp <= 128, "key_dim padding exceeds 128");
  d->key_dim_p = dkp;
  d->inner_p = c->num_heads * dkp;
  d->qkv_p = (int)round_up(3 * d->inner_p, VTD_KALIGN);
  for (int j = 0; j < VTD_MAX_MLP; ++j) d->mlp_units[j] = d->mlp_units_p[j] = 0;
  for (int j = 0; j < c->mlp_quantities; ++j) {      // vtd.py:385-386
    const int64_t u = (int64_t)d->d << (c->mlp_quantities - 1 - j);
    VTD_CHECK_ARG(u < (1 << 24), "encoder MLP width overflow");
    d->mlp_units[j] = (int)u;
    d->mlp_units_p[j] = (int)round_up(u, VTD_KALIGN);
  }
  d->n_head = c->head_layers * c->head_repeats;
  for (int j = 0; j < VTD_MAX_HEAD; ++j) d->head_units[j] = d->head_units_p[j] = 0;
  int idx = 0;
  for (int e = c->head_layers - 1; e >= 0; --e) {     // vtd.py:465-470
    const int64_t u = (int64_t)c->head_last_units << e;
    VTD_CHECK_ARG(u < (1 << 24), "head width overflow");
    for (int r = 0; r < c->head_repeats; ++r, ++idx) {
      d->head_units[idx] = (int)u;
      d->head_units_p[idx] = (int)round_up(u, VTD_KALIGN);
    }
  }
  d->tokens_p = (int)round_up(d->tokens, VTD_KALIGN);
  d->rows = (int64_t)c->batch * d->tokens;
  d->head_rows = (int64_t)c->batch * VTD_MAX_DETECT;
  return VTD_OK;
}

namespace {
struct Plan {
  size_t patches, x, xb, h, stat, pstat, qkv, attn, attn3, mlp0, mlp1, u, head0, head1, q8, s8, q8b,
      s8b, splitk, splitk_bytes, total;
  int k8_max;                       // widest MX-fp8 GEMM K (VTD_FP8)
  int64_t s8_rows;                  // activation scale rows (rows rounded up to 4)
};
// activation / non-MX matrix dtype of a mode (VTD_FP8 keeps everything else in bf16; the
// split-bf16 mode VTD_BF16X3 keeps its activations -- query/key/value, attention -- in f32)
int act_dtype(int dtype) {
  return dtype == VTD_FP8 ? VTD_BF16 : dtype == VTD_BF16X3 ? VTD_F32 : dtype;
}
size_t es_of(int dtype) { return act_dtype(dtype) == VTD_BF16 ? 2 : 4; }
// GEMM A operands (patches, LayerNorm out, MLP / head activations): bytes per logical element
// (VTD_BF16X3: the two bf16 pieces [hi | lo]) and the stored width of a K-wide logical row;
// opk: the GEMM's K (and the weights' row width) for it (VTD_BF16X3: K' = 3 K)
size_t eop_of(int dtype) { return dtype == VTD_BF16X3 ? 4 : es_of(dtype); }
int opa(int dtype, int k) { return dtype == VTD_BF16X3 ? 2 * k : k; }
int opk(int dtype, int k) { return dtype == VTD_BF16X3 ? 3 * k : k; }
// dtype of the residual stream x: bf16 in the bf16 / fp8 modes (the stream the GEMM
// epilogues add into and the LayerNorms read), f32 in the f32 mode.  VTD_RESID_F32=1
// keeps an f32 stream in the bf16 modes (A/B diagnostic; costs ~7 % at C2).
int resid_dtype(int dtype) {
  static const bool f32 = [] {
    const char* v = getenv("VTD_RESID_F32");
    return v && atoi(v) != 0;
  }();
  return act_dtype(dtype) == VTD_BF16 && !f32 ? VTD_BF16 : VTD_F32;
}
int k8_of(int k) { return (int)round_up(k, 128); }
// Encoder rows of a micro-batch part: a part's batch x tokens rounded up to whole 256-row
// tiles (pad), so that every encoder GEMM of the part runs full tiles -- the fast epilogues
// and the producer-side LayerNorm partial statistics -- instead of a last partial row tile
// on the generic epilogue (C2 at B = 64 in two parts of 32 images: 6272 rows -> 6400).  The
// pad rows start from zero patches; rows never mix in a GEMM, LayerNorm or the attention
// (which reads the real images' rows only), and the head reads the real rows only.
int64_t gemm_rows(const vtd_dims& d, bool pad) { return pad ? round_up(d.rows, 256) : d.rows; }
// whether the parts of a split forward pad their rows (VTD_SPLIT_PAD=0: not, A/B only)
bool split_pad() {
  static const bool on = [] {
    const char* v = getenv("VTD_SPLIT_PAD");
    return !v || atoi(v) != 0;
  }();
  return on;
}
// pad: the encoder runs on rows rounded up to whole 256-row GEMM tiles (gemm_rows)
// nparts: the micro-batch parts running concurrently (each part's encoder rows are padded
// when > 1, split_pad; its head's split-K launches target 256 / nparts workgroups, since the
// parts' head launches co-run: +0.2 % at C2 B = 256, +0.9 % at B = 64,
// profiles/r05_splitk_target_ab.log)
int splitk_target(int nparts) { return 256 / std::max(nparts, 1); }
// Split-K count of an encoder Dense layer (M x N, K-steps of 64): the count minimising a model
// of its time -- rounds of the part's 256 / nparts workgroups x K-steps per split x ~1.5 us,
// plus the fp32 partials written and read at ~4 TB/s -- if it saves >= 10 % over no split.
// Few-tile, long-K layers of small batches split (C2 B = 8: mlp2 42 tiles x 48 K-steps);
// a layer that already fills a round does not (C2 B = 32: splitting mlp2 / mlp3 cost 6 %,
// profiles/r06_enc_splitk_ab.log).  Only counts whose partials fit max_bytes (the plan's
// kEncSplitBytes: a batch-independent reserve, so the workspace stays monotonic in the batch).
// 1 = no split.
constexpr size_t kEncSplitBytes = size_t(64) << 20;
int enc_splitk_choice(int64_t M, int N, int K, int nparts, int dtype, size_t max_bytes) {
  if ((dtype != VTD_BF16 && dtype != VTD_BF16X3) || M <= 0 || N <= 64 || N % 4 != 0 || K % 64 != 0 || knob(VTD_KNOB_SPLITK) == 0) return 1;
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int nk = K / 64, cus = 256 / std::max(nparts, 1);
  auto rounds = [&](int64_t wgs) { return (double)((wgs + cus - 1) / cus); };
  const double t1 = rounds(tiles) * nk * 1.5;
  double best = 0.9 * t1;
  int bs = 1;
  for (int sp = 2; sp <= std::min(16, nk / 4); ++sp) {
    const int nks = (nk + sp - 1) / sp;
    if ((sp - 1) * nks >= nk) continue;                   // every split non-empty
    if ((size_t)sp * M * N * 4 > max_bytes) break;
    const double t = rounds(tiles * sp) * nks * 1.5 + 2.0 * sp * (double)M * N * 4 / 4e6;
    if (t < best) {
      best = t;
      bs = sp;
    }
  }
  return bs;
}
Plan make_plan(const vtd_config* c, const vtd_dims& d, int nparts = 1) {
  const bool pad = nparts > 1 && split_pad();
  Plan p{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) / 256 * 256;
    return o;
  };
  const size_t es = es_of(c->dtype), eop = eop_of(c->dtype);
  const size_t R = (size_t)gemm_rows(d, pad), HR = (size_t)d.head_rows;
  int mlp_max = 0, head_max = 0;
  for (int j = 0; j < c->mlp_quantities; ++j) mlp_max = std::max(mlp_max, d.mlp_units_p[j]);
  for (int j = 0; j < d.n_head; ++j) head_max = std::max(head_max, d.head_units_p[j]);
  p.patches = take(R * d.patch_dim_p * eop);
  p.x = take(R * d.d_p * 4);
  p.xb = take(act_dtype(c->dtype) == VTD_BF16 ? R * d.d_p * 2 : 0);
  p.h = take(R * d.d_p * eop);
  p.stat = take(R * 8);                 // LayerNorm (mean, rstd) per row, fold path
  p.pstat = take(R * (d.d_p / 64) * 8);  // producer partial (sum, sumsq) per 64 columns
  p.qkv = take(R * d.qkv_p * es);
  // the attention output; VTD_BF16X3: written by the attention kernel as the split-bf16
  // operand of attention_output (attn3), no f32 copy
  p.attn = take(c->dtype == VTD_BF16X3 ? 0 : R * d.inner_p * es);
  p.attn3 = take(c->dtype == VTD_BF16X3 ? R * d.inner_p * eop : 0);
  p.mlp0 = take(R * mlp_max * eop);
  p.mlp1 = take(R * mlp_max * eop);
  p.u = take(HR * d.tokens_p * eop);
  p.head0 = take(HR * head_max * eop);
  p.head1 = take(HR * head_max * eop);
  // fp32 split-K partials of the head's few-tile, long-K Dense layers (gemm_splitk_choice)
  size_t sk = 0;
  for (int j = 0, k = d.tokens_p; j < d.n_head; k = d.head_units_p[j], ++j) {
    const int s = gemm_splitk_choice((int)HR, d.head_units_p[j], opk(c->dtype, k),
                                     c->dtype == VTD_BF16X3 ? VTD_BF16X3 : act_dtype(c->dtype),
                                     splitk_target(nparts));
    if (s > 1) sk = std::max(sk, (size_t)s * HR * d.head_units_p[j] * 4);
  }
  // and of the encoder's few-tile Dense layers (small batches, enc_gemm; bf16 operands): a
  // fixed reserve, whose size bounds their split counts (enc_splitk_choice)
  if (c->dtype == VTD_BF16 || c->dtype == VTD_BF16X3) sk = std::max(sk, kEncSplitBytes);
  p.splitk_bytes = sk;
  p.splitk = take(sk);
  // VTD_FP8: one MX-fp8 copy of the current encoder GEMM's A operand + its scales
  p.k8_max = 0;
  p.s8_rows = round_up((int64_t)R, 4);
  if (c->dtype == VTD_FP8) {
    p.k8_max = std::max(k8_of(d.d_p), k8_of(d.inner_p));
    for (int j = 0; j + 1 < c->mlp_quantities; ++j) p.k8_max = std::max(p.k8_max, k8_of(d.mlp_units_p[j]));
  }
  // two MX-fp8 operand buffers: an MLP GEMM reads one and writes the next one's operand
  p.q8 = take(R * p.k8_max);
  p.s8 = take((size_t)p.s8_rows * p.k8_max / 32);
  p.q8b = take(R * p.k8_max);
  p.s8b = take((size_t)p.s8_rows * p.k8_max / 32);
  p.total = off;
  return p;
}
// Two-stream micro-batching of vtd_forward: the images are independent, so a large
// batch is run as two halves on the caller's stream and an internal second stream.  The
// halves' kernels co-run, so the last partial round of one half's GEMM tiles (e.g. 588
// tiles of an N = 768 layer = 2.3 rounds of 256 CUs) runs beside the other half's work
// instead of leaving CUs idle.  VTD_STREAMS=1 disables it; so does per-kernel profiling
// (vtd_profile_enable): each profiled launch then runs alone and its events time it.
constexpr int kMaxSplit = 4;   // VTD_STREAMS is clamped to [1, kMaxSplit]
// fewest 256-row tiles per part (VTD_SPLIT_MIN_TILES; C2 at B = 256, 2 parts: 98 each; at
// B = 64, 2 parts of 24.5 tiles padded to 25: +15 % over one stream since round 5, once the
// parts' 75-tile layers run the 256-tile kernels, profiles/r05_b64_split_ab.log)
int split_min_tiles() {
  static const int t = [] {
    const char* v = getenv("VTD_SPLIT_MIN_TILES");
    return v ? std::max(1, atoi(v)) : 24;
  }();
  return t;
}
int split_parts(const vtd_config* c, const vtd_dims& d) {
  static const int streams = [] {
    const char* v = getenv("VTD_STREAMS");
    return v ? atoi(v) : 2;
  }();
  int ns = std::min(std::max(streams, 1), (int)kMaxSplit);
  while (ns > 1 && (c->batch < ns || d.rows < (int64_t)ns * split_min_tiles() * 256)) --ns;
  return ns;
}
int split_count(const vtd_config* c, const vtd_dims& d) {
  return prof().enabled ? 1 : split_parts(c, d);
}
vtd_config sub_config(const vtd_config* c, int part, int nsplit) {
  vtd_config s = *c;
  const int b0 = c->batch / nsplit;
  s.batch = part == nsplit - 1 ? c->batch - b0 * (nsplit - 1) : b0;
  return s;
}
// workspace of either form (profiling can toggle between them)
size_t split_workspace(const vtd_config* c, const vtd_dims& d) {
  const size_t whole = make_plan(c, d).total;
  vtd_dims dd;
  if (derive(c, &dd) != VTD_OK) return 0;
  const int ns = split_parts(c, dd);
  if (ns == 1) return whole;
  size_t total = 0;
  for (int i = 0; i < ns; ++i) {
    const vtd_config sc = sub_config(c, i, ns);
    vtd_dims sd;
    if (derive(&sc, &sd) != VTD_OK) return 0;
    total += make_plan(&sc, sd, ns).total;
  }
  return std::max(total, whole);
}
// The side streams and the fork / join events are shared by every caller on a device, so
// a split forward holds `mu` from its fork record to its join wait (calls are
// re-entrant across host threads on distinct streams).  hipStreamWaitEvent orders the
// waiting stream behind the event's latest record at the time of the wait call: another
// thread's record in between would order this call's halves behind THAT caller's stream
// position instead; and a side stream joined to a graph capture must carry nothing else
// until its join.  The lock covers host-side enqueueing only (~1 ms per forward at C2).
struct SideStream {
  int device = -1;
  std::mutex mu;
  hipStream_t s[kMaxSplit - 1] = {};
  hipEvent_t fork = nullptr, join[kMaxSplit - 1] = {};
};
// per-device side stream + fork/join events, created on the first eager call (never
// during a HIP-graph capture: a captured first call runs unsplit)
SideStream* side_stream(hipStream_t st) {
  static std::mutex mu;
  static SideStream per_dev[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  SideStream& ss = per_dev[dev];
  if (ss.device == dev) return &ss;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
    return nullptr;
  if (hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming) != hipSuccess) return nullptr;
  for (int i = 0; i < kMaxSplit - 1; ++i)
    if (hipStreamCreateWithFlags(&ss.s[i], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ss.join[i], hipEventDisableTiming) != hipSuccess)
      return nullptr;
  ss.device = dev;
  return &ss;
}

// Stages of one forward: 0 = patches + linear projection, 1..L = encoder layer s - 1,
// L + 1 = head + decode.  forward_impl runs stages [s_lo, s_hi); `partials` carries
// "the GEMM that last wrote x emitted LayerNorm partials" from one stage to the next.
// nparts: the micro-batch parts of the forward (workspace plan, row padding, head split-K);
// nconc: how many of them run concurrently (nparts, or 1 when they run one after another on
// the caller's stream: a first call under graph capture) -- the persistent attention's grid
int forward_impl(const vtd_config* cfg, const vtd_weights* w, const float* images,
                 float* logits, float* dets, char* ws, hipStream_t st, int s_lo, int s_hi,
                 bool& partials, int nparts, int nconc);
}  // namespace

}  // namespace vtd

using namespace vtd;

extern "C" {

int vtd_abi_version(void) { return VTD_ABI_VERSION; }

int vtd_set_knob(int k, int value) {
  VTD_CHECK_ARG(k >= 0 && k < VTD_KNOB_COUNT, "vtd_set_knob: unknown knob");
  knob_init();
  return g_knob[k].exchange(value, std::memory_order_relaxed);
}
int vtd_get_knob(int k) {
  VTD_CHECK_ARG(k >= 0 && k < VTD_KNOB_COUNT, "vtd_get_knob: unknown knob");
  return knob(k);
}
const char* vtd_last_error(void) { return g_last_error.c_str(); }

int vtd_derive_dims(const vtd_config* cfg, vtd_dims* out) { return derive(cfg, out); }

int vtd_workspace_bytes(const vtd_config* cfg, size_t* bytes) {
  VTD_CHECK_ARG(bytes, "null bytes pointer");
  vtd_dims d;
  int rc = derive(cfg, &d);
  if (rc) return rc;
  *bytes = split_workspace(cfg, d);
  return *bytes ? VTD_OK : fail(VTD_ERR_INVALID_ARG, "workspace: bad split config");
}

int vtd_forward(const vtd_config* cfg, const vtd_weights* w, const float* images,
                float* logits, float* dets, void* workspace, size_t workspace_bytes,
                void* stream_) {
  vtd_dims d;
  int rc = derive(cfg, &d);
  if (rc) return rc;
  VTD_CHECK_ARG(w && images && logits && workspace, "forward: null pointer");
  VTD_CHECK_ARG(w->layers, "forward: weights.layers is null");
  const size_t need = split_workspace(cfg, d);
  if (workspace_bytes < need)
    return fail(VTD_ERR_WORKSPACE, "forward: workspace too small (need " +
                                       std::to_string(need) + " bytes)");
  hipStream_t st = static_cast<hipStream_t>(stream_);
  char* ws = static_cast<char*>(workspace);
  const int ns = split_count(cfg, d);
  SideStream* side = ns > 1 ? side_stream(st) : nullptr;
  const int n_stages = cfg->repeat_times + 2;
  if (!side) {
    bool partials = false;
    if (ns == 1)
      return forward_impl(cfg, w, images, logits, dets, ws, st, 0, n_stages, partials, 1, 1);
    // no side stream (first call under capture): the halves run in order on `st`
  }
  const size_t img = (size_t)cfg->image_h * cfg->image_w * cfg->channels;
  // one caller at a time per device from the fork record to the join wait (SideStream)
  std::unique_lock<std::mutex> side_lock;
  if (side) side_lock = std::unique_lock<std::mutex>(side->mu);
  // fork: one record, every side stream waits on it.  Knob VTD_KNOB_STAGGER = k > 0: the
  // record follows the caller-stream part's first k stages, so the other parts run k
  // stages behind (their kernels then pair with different kernels of the first part)
  // default: one stage behind for small parts (<= 32 row tiles: C2 at B = 64, +1.5 %), in
  // phase otherwise (B = 96 / 128 / 256: 0 to -1.5 % with a stagger; profiles/r05_b64_split_ab.log)
  const int ks = knob(VTD_KNOB_STAGGER);
  const int part_tiles = (int)((d.rows / ns + 255) / 256);
  const int stagger =
      side ? std::min(ks >= 0 ? ks : (part_tiles <= 32 ? 1 : 0), n_stages) : 0;
  auto fork = [&]() -> int {
    VTD_HIP(hipEventRecord(side->fork, st));
    for (int part = 1; part < ns; ++part) VTD_HIP(hipStreamWaitEvent(side->s[part - 1], side->fork, 0));
    return VTD_OK;
  };
  if (side && stagger == 0 && (rc = fork())) return rc;
  struct Part {
    vtd_config cfg;
    const float* images;
    float* logits;
    float* dets;
    char* ws;
    hipStream_t st;
    bool partials;
  } parts[kMaxSplit];
  int64_t b0 = 0;
  size_t ws_off = 0;
  for (int part = 0; part < ns; ++part) {
    Part& P = parts[part];
    P.cfg = sub_config(cfg, part, ns);
    vtd_dims dp;
    rc = derive(&P.cfg, &dp);
    if (rc) return rc;
    P.st = side && part > 0 ? side->s[part - 1] : st;
    const size_t out_off = (size_t)b0 * VTD_MAX_DETECT * 6;
    P.images = images + b0 * img;
    P.logits = logits + out_off;
    P.dets = dets ? dets + out_off : nullptr;
    P.ws = ws + ws_off;
    P.partials = false;
    b0 += P.cfg.batch;
    ws_off += make_plan(&P.cfg, dp, ns).total;
  }
  // Launches are interleaved part by part, one stage (encoder layer) at a time: issuing
  // all of one part's ~110 launches before the next part's first one left the second
  // stream idle for the host's whole enqueue time of the first (~0.7 ms at C2, B = 256).
  for (int t = 0; t < n_stages + stagger; ++t) {
    // stagger k: the fork is recorded once part 0 has issued stages 0 .. k - 1, before it
    // issues stage k, so the other parts run exactly k stages behind
    if (side && stagger > 0 && t == stagger && (rc = fork())) return rc;
    for (int part = 0; part < ns; ++part) {
      Part& P = parts[part];
      const int s = part == 0 ? t : t - stagger;
      if (s < 0 || s >= n_stages) continue;
      rc = forward_impl(&P.cfg, w, P.images, P.logits, P.dets, P.ws, P.st, s, s + 1, P.partials,
                        ns, side ? ns : 1);
      if (rc) return rc;
    }
  }
  if (side) {                       // join: each side stream's record and the caller's wait
    for (int part = 1; part < ns; ++part) {
      VTD_HIP(hipEventRecord(side->join[part - 1], side->s[part - 1]));
      VTD_HIP(hipStreamWaitEvent(st, side->join[part - 1], 0));
    }
  }
  return VTD_OK;
}
}  // extern "C"

namespace vtd {
namespace {
int forward_impl(const vtd_config* cfg, const vtd_weights* w, const float* images,
                 float* logits, float* dets, char* ws, hipStream_t st, int s_lo, int s_hi,
                 bool& partials, int nparts, int nconc) {
  vtd_dims d;
  int rc = derive(cfg, &d);
  if (rc) return rc;
  const Plan P = make_plan(cfg, d, nparts);
  const bool pad = nparts > 1 && split_pad();
  const bool fp8 = cfg->dtype == VTD_FP8;
  const int dt = act_dtype(cfg->dtype);
  // VTD_BF16X3: every GEMM runs on split-bf16 operands (bf16 kernels over K' = 3 K_p, A rows
  // stored [hi | lo], 2 K_p wide: ka), whose A operands the producers write directly (odt);
  // qkv / attention / x stay f32
  const bool x3 = cfg->dtype == VTD_BF16X3;
  const int gdt = x3 ? VTD_BF16X3 : dt, odt = x3 ? VTD_BF16X3 : dt;
  auto kk = [&](int k) { return opk(cfg->dtype, k); };
  auto ka = [&](int k) { return opa(cfg->dtype, k); };
  const int B = cfg->batch, N = d.tokens, D = d.d, Dp = d.d_p;
  // R: the encoder's rows (the real batch x tokens, or whole 256-row tiles of a part: pad)
  const int64_t R = gemm_rows(d, pad);
  VTD_CHECK_ARG(R < (int64_t)1 << 31, "forward: batch*tokens too large");
  const int M = (int)R;
  void* patches = ws + P.patches;
  const int rdt = resid_dtype(cfg->dtype);
  float* stat = reinterpret_cast<float*>(ws + P.stat);
  void* x = ws + P.x;
  float* pstat = reinterpret_cast<float*>(ws + P.pstat);
  const int nslot = Dp / 64;
  // fold path: the GEMM writing x emits partial row statistics when it can (full tiles on
  // the bf16 fast epilogues); the LayerNorm point then only finalizes them (`partials`)
  static const bool partials_on = [] {       // VTD_LN_PARTIALS=0: row-statistics pass
    const char* v = getenv("VTD_LN_PARTIALS");
    return !v || atoi(v) != 0;
  }();
  auto emit_stats = [&](vtd_epilogue& e, bool next_fold) {
    partials = false;
    // centred per-block partials need every 64-column block full of valid columns
    if (!next_fold || fp8 || dt != VTD_BF16 || !partials_on || D != Dp) return;
    e.statout = pstat; e.stat_ld = (int)R;       // slot-major planes of R rows
    partials = gemm_emits_stats(M, Dp, dt, &e);
    if (!partials) { e.statout = nullptr; e.stat_ld = 0; }
  };
#ifndef VTD_DIAG
#define VTD_DIAG 0
#endif
  // VTD_DIAG builds only (timing diagnostics, WRONG outputs): VTD_DIAG_NOFIN skips the
  // LayerNorm finalize launches, VTD_DIAG_NOATTN the attention launches, VTD_DIAG_NOHEAD
  // the detection head
  // (VTD_DIAG_NOFIN=n: after the first n finalize launches, so the consumers keep applying
  // the last real row statistics: activations stay realistic, MFMA power and clock with them)
  static const int diag_nofin = VTD_DIAG && getenv("VTD_DIAG_NOFIN") ? atoi(getenv("VTD_DIAG_NOFIN")) : -1;
  static std::atomic<int> diag_fin_count{0};
  static const bool diag_noattn = VTD_DIAG && getenv("VTD_DIAG_NOATTN");
  auto row_stats = [&]() -> int {
    if (diag_nofin >= 0 && partials && diag_fin_count.fetch_add(1) >= diag_nofin) return VTD_OK;
    return partials ? ln_stats_finalize_launch(pstat, R, nslot, D, 1e-3f, stat, st)
                    : ln_stats_launch(x, rdt, R, D, Dp, 1e-3f, stat, st);
  };
  void* xb = ws + P.xb;
  void* h = ws + P.h;
  void* qkv = ws + P.qkv;
  void* attn = ws + P.attn;
  void* mlp[2] = {ws + P.mlp0, ws + P.mlp1};
  void* u = ws + P.u;
  void* head[2] = {ws + P.head0, ws + P.head1};
  const int act = cfg->use_mish ? VTD_ACT_MISH : VTD_ACT_GELU_TANH;
  const double fR = (double)d.rows;             // algorithmic FLOPs: the real rows
  uint8_t* q8 = reinterpret_cast<uint8_t*>(ws + P.q8);
  uint8_t* s8 = reinterpret_cast<uint8_t*>(ws + P.s8);
  // encoder Dense layer (query/key/value, attention_output, MLP): bf16/f32 GEMM, or in
  // VTD_FP8 mode MX-fp8 quantization of the bf16 A operand + the block-scaled MFMA GEMM
  // against the MX-fp8 weights (W [Np][K8], S [K8/128][Np][4])
  auto enc_gemm = [&](int Np, int K, const void* a, const void* W, const uint8_t* S,
                      const vtd_epilogue* e, double flops) -> int {
    if (!fp8) {
      // few-tile, long-K layers (small batches) split K (enc_splitk_choice);
      // not with partial statistics, which the split-K epilogue does not write
      static const bool enc_split = [] {      // VTD_ENC_SPLITK=0: off (A/B)
        const char* v = getenv("VTD_ENC_SPLITK");
        return !v || atoi(v) != 0;
      }();
      const int ks = !enc_split || e->statout
                         ? 1 : enc_splitk_choice(M, Np, kk(K), nparts, gdt, P.splitk_bytes);
      if (ks > 1)
        return gemm_splitk_launch(M, Np, kk(K), a, ka(K), W, kk(K), gdt, e,
                                  reinterpret_cast<float*>(ws + P.splitk), ks, st, flops);
      return gemm_launch(M, Np, kk(K), a, ka(K), W, kk(K), gdt, e, st, flops);
    }
    const int K8 = k8_of(K);
    int r = quantize_mx8_launch(a, VTD_BF16, R, K, K, K8, q8, K8, s8, P.s8_rows, st);
    if (r) return r;
    return gemm_mx8_launch(M, Np, K8, q8, K8, s8, P.s8_rows, static_cast<const uint8_t*>(W), K8,
                           S, Np, e, st, flops);
  };
  // VTD_FP8: the GEMM on an operand a producer already wrote as MX-fp8 (q, s)
  uint8_t* q8b = reinterpret_cast<uint8_t*>(ws + P.q8b);
  uint8_t* s8b = reinterpret_cast<uint8_t*>(ws + P.s8b);
  auto mx_gemm = [&](int Np, int K, const uint8_t* qa, const uint8_t* sa, const void* W,
                     const uint8_t* S, const vtd_epilogue* e, double flops) -> int {
    const int K8 = k8_of(K);
    return gemm_mx8_launch(M, Np, K8, qa, K8, sa, P.s8_rows, static_cast<const uint8_t*>(W), K8,
                           S, Np, e, st, flops);
  };
  // VTD_FP8 LayerNorm straight into the MX-fp8 operand buffer q8 / s8
  auto ln_mx8 = [&](const float* g, const float* b) -> int {
    return layernorm_mx8_launch(x, rdt, R, D, Dp, g, b, 1e-3f, q8, k8_of(Dp), k8_of(Dp), s8,
                                P.s8_rows, st);
  };

  const int n_stages = cfg->repeat_times + 2;
  if (s_lo <= 0 && 0 < s_hi) {
  // ---- ExtractImagePatches + flatten (vtd.py:271-280)
  rc = patches_launch(images, B, cfg->image_h, cfg->image_w, cfg->channels,
                      cfg->patch_size, patches, ka(d.patch_dim_p), odt, st);
  if (rc) return rc;
  if (R > d.rows) {                                   // pad rows: zero patches
    const size_t row_bytes = (size_t)d.patch_dim_p * eop_of(cfg->dtype);
    VTD_HIP(hipMemsetAsync(static_cast<char*>(patches) + (size_t)d.rows * row_bytes, 0,
                           (size_t)(R - d.rows) * row_bytes, st));
    // and the attention output's pad rows, which the attention never writes
    const size_t attn_row = (size_t)d.inner_p * (x3 ? eop_of(cfg->dtype) : es_of(cfg->dtype));
    VTD_HIP(hipMemsetAsync(static_cast<char*>(x3 ? ws + P.attn3 : attn) + (size_t)d.rows * attn_row,
                           0, (size_t)(R - d.rows) * attn_row, st));
  }
  // ---- linear_projection + position embedding add (vtd.py:291-307)
  {
    vtd_epilogue e{};
    e.bias = w->b_patch;
    e.rowadd = w->pos_embedding; e.rowadd_period = N; e.rowadd_ncols = D;
    e.act = VTD_ACT_NONE;
    e.out = x; e.ldo = Dp; e.out_dtype = rdt;
    emit_stats(e, cfg->repeat_times > 0 && w->layers[0].ln1_colsum);
    rc = gemm_launch(M, Dp, kk(d.patch_dim_p), patches, ka(d.patch_dim_p), w->w_patch,
                     kk(d.patch_dim_p), gdt, &e, st, 2.0 * fR * D * d.patch_dim);
    if (rc) return rc;
  }
  }
  const int q = cfg->mlp_quantities;
  const float scale = 1.0f / std::sqrt((float)cfg->key_dim);
  const int i_lo = std::max(s_lo - 1, 0), i_hi = std::min(s_hi - 1, cfg->repeat_times);
  for (int i = i_lo; i < i_hi; ++i) {                  // vtd.py:350-412
    const vtd_layer_weights& L = w->layers[i];
    if ((fp8 || x3) && (L.ln1_colsum || L.ln2_colsum))
      return fail(VTD_ERR_UNSUPPORTED, "forward: LayerNorm fold (ln*_colsum) is not supported in "
                                       "the VTD_FP8 / VTD_BF16X3 modes");
    // the folded GEMMs take the residual stream x itself as their A operand (read in dt)
    if (rdt != dt && (L.ln1_colsum || L.ln2_colsum))
      return fail(VTD_ERR_UNSUPPORTED, "forward: LayerNorm fold (ln*_colsum) needs the residual "
                                       "stream in the compute dtype (unset VTD_RESID_F32)");
    // LayerNorm 1: its own pass into h, or folded into the query/key/value GEMM
    const void* a1 = h;
    if (L.ln1_colsum) {
      rc = row_stats();
      a1 = x;
    } else if (fp8) {
      rc = ln_mx8(L.ln1_gamma, L.ln1_beta);       // LayerNorm + MX quantization, one pass
    } else {
      rc = layernorm_launch(x, rdt, R, D, Dp, L.ln1_gamma, L.ln1_beta, 1e-3f, h, ka(Dp), odt, st);
    }
    if (rc) return rc;
    {
      vtd_epilogue e{};
      e.bias = L.b_qkv; e.act = VTD_ACT_NONE;
      e.out = qkv; e.ldo = d.qkv_p; e.out_dtype = dt;
      if (L.ln1_colsum) { e.lnstat = stat; e.colsum = L.ln1_colsum; }
      const double fl = 2.0 * fR * D * 3.0 * cfg->num_heads * cfg->key_dim;
      rc = fp8 ? mx_gemm(d.qkv_p, Dp, q8, s8, L.w_qkv, L.s_qkv, &e, fl)
               : enc_gemm(d.qkv_p, Dp, a1, L.w_qkv, L.s_qkv, &e, fl);
      if (rc) return rc;
    }
    // VTD_FP8 with whole MX K-steps: attention writes the output GEMM's MX-fp8 operand
    const bool attn_mx8 = fp8 && d.inner_p % 128 == 0 && k8_of(d.inner_p) == d.inner_p;
    const double attn_flops = 4.0 * B * cfg->num_heads * (double)N * N * cfg->key_dim;
    rc = diag_noattn ? VTD_OK
         : attn_mx8 ? attention_mx8_launch(qkv, B, N, cfg->num_heads, d.key_dim_p, d.qkv_p, scale,
                                         q8, d.inner_p, s8, P.s8_rows, st, attn_flops)
         : x3 ? attention_launch(qkv, B, N, cfg->num_heads, d.key_dim_p, d.qkv_p, scale,
                                 ws + P.attn3, ka(d.inner_p), VTD_BF16X3, st, attn_flops, nconc)
                  : attention_launch(qkv, B, N, cfg->num_heads, d.key_dim_p, d.qkv_p, scale,
                                     attn, d.inner_p, dt, st, attn_flops, nconc);
    if (rc) return rc;
    // VTD_BF16X3: the attention wrote the attention_output GEMM's split-bf16 operand itself
    const void* attn_op = x3 ? ws + P.attn3 : attn;
    {
      vtd_epilogue e{};
      e.bias = L.b_out; e.act = VTD_ACT_NONE;
      e.resid = x; e.ldr = Dp;
      e.out = x; e.ldo = Dp; e.out_dtype = rdt;
      emit_stats(e, L.ln2_colsum != nullptr);
      const double fl = 2.0 * fR * cfg->num_heads * cfg->key_dim * D;
      rc = attn_mx8 ? mx_gemm(Dp, d.inner_p, q8, s8, L.w_out, L.s_out, &e, fl)
                    : enc_gemm(Dp, d.inner_p, attn_op, L.w_out, L.s_out, &e, fl);
      if (rc) return rc;
    }
    const void* a = h;
    // VTD_FP8: the current MLP operand as MX-fp8 (aq, as), written by its producer
    const uint8_t* aq = nullptr;
    const uint8_t* as = nullptr;
    if (L.ln2_colsum) {
      rc = row_stats();
      a = x;
    } else if (fp8) {
      rc = ln_mx8(L.ln2_gamma, L.ln2_beta);
      aq = q8; as = s8;
    } else {
      rc = layernorm_launch(x, rdt, R, D, Dp, L.ln2_gamma, L.ln2_beta, 1e-3f, h, ka(Dp), odt, st);
    }
    if (rc) return rc;
    int k = Dp, kv = D;
    for (int j = 0; j < q; ++j) {
      const bool last = j == q - 1;
      vtd_epilogue e{};
      e.bias = L.b_mlp[j]; e.act = act;
      if (j == 0 && L.ln2_colsum) { e.lnstat = stat; e.colsum = L.ln2_colsum; }
      if (last) {
        e.resid = x; e.ldr = Dp;
        e.out = x; e.ldo = Dp; e.out_dtype = rdt;
        if (i == cfg->repeat_times - 1 && dt == VTD_BF16 && rdt == VTD_F32) {
          e.out2 = xb; e.ldo2 = Dp;           // bf16 copy of an f32 stream for the head
        }
        emit_stats(e, i + 1 < cfg->repeat_times && w->layers[i + 1].ln1_colsum);
      } else {
        e.out = mlp[j & 1]; e.ldo = ka(d.mlp_units_p[j]); e.out_dtype = odt;
      }
      // VTD_FP8: an inner MLP layer writes the next layer's MX-fp8 operand itself (into the
      // operand buffer it is not reading) when every tile takes the fast epilogue
      uint8_t* nq = nullptr;
      uint8_t* ns = nullptr;
      if (fp8 && !last) {
        nq = aq == q8b ? q8 : q8b;        // (enc_gemm quantizes into q8)
        ns = aq == q8b ? s8 : s8b;
        vtd_epilogue ef = e;
        ef.out = nq; ef.ldo = k8_of(d.mlp_units_p[j]); ef.out_dtype = VTD_FP8;
        ef.scale_out = ns; ef.scale_rows = P.s8_rows;
        if (gemm_mx8_emits_fp8(M, d.mlp_units_p[j], &ef)) e = ef;
        else nq = ns = nullptr;
      }
      const double fl = 2.0 * fR * kv * d.mlp_units[j];
      rc = aq ? mx_gemm(d.mlp_units_p[j], k, aq, as, L.w_mlp[j], L.s_mlp[j], &e, fl)
              : enc_gemm(d.mlp_units_p[j], k, a, L.w_mlp[j], L.s_mlp[j], &e, fl);
      if (rc) return rc;
      a = mlp[j & 1];
      aq = nq;
      as = ns;
      k = d.mlp_units_p[j];
      kv = d.mlp_units[j];
    }
  }
  if (!(s_lo <= n_stages - 1 && n_stages - 1 < s_hi)) return VTD_OK;
  static const bool diag_nohead = VTD_DIAG && getenv("VTD_DIAG_NOHEAD");
  if (diag_nohead) return VTD_OK;
  // ---- mlp_head: Dense(17) + Reshape((17, -1)) as a scatter epilogue (vtd.py:454-463)
  {
    VTD_HIP(hipMemsetAsync(u, 0, (size_t)d.head_rows * d.tokens_p * eop_of(cfg->dtype), st));
    vtd_epilogue e{};
    e.bias = w->b_det; e.act = VTD_ACT_NONE;
    e.out = u; e.ldo = ka(d.tokens_p); e.out_dtype = odt;
    e.scatter_tokens = N;
    const void* a = dt == rdt ? x : xb;
    if (x3) {                        // the f32 stream x as the split-bf16 operand (h is free)
      rc = split_bf16x3_launch(static_cast<const float*>(x), R, Dp, Dp, h, ka(Dp), 0, st);
      if (rc) return rc;
      a = h;
    }
    // the real rows only (the scatter addresses images by row)
    rc = gemm_launch((int)d.rows, VTD_MAX_DETECT, kk(Dp), a, ka(Dp), w->w_det, kk(Dp), gdt, &e,
                     st, 2.0 * fR * D * VTD_MAX_DETECT);
    if (rc) return rc;
  }
  const int HR = (int)d.head_rows;
  const void* a = u;
  int k = d.tokens_p, kv = N;
  for (int j = 0; j < d.n_head; ++j) {                // vtd.py:468-486
    vtd_epilogue e{};
    e.bias = w->b_head[j]; e.act = act;
    e.out = head[j & 1]; e.ldo = ka(d.head_units_p[j]); e.out_dtype = odt;
    const double fl = 2.0 * HR * (double)kv * d.head_units[j];
    const int ks = gemm_splitk_choice(HR, d.head_units_p[j], kk(k), gdt, splitk_target(nparts));
    rc = ks > 1 ? gemm_splitk_launch(HR, d.head_units_p[j], kk(k), a, ka(k), w->w_head[j], kk(k),
                                     gdt, &e, reinterpret_cast<float*>(ws + P.splitk), ks, st, fl)
                : gemm_launch(HR, d.head_units_p[j], kk(k), a, ka(k), w->w_head[j], kk(k), gdt,
                              &e, st, fl);
    if (rc) return rc;
    a = head[j & 1];
    k = d.head_units_p[j];
    kv = d.head_units[j];
  }
  {                                                   // MLP_Head_no_Sigmoid vtd.py:489-493
    vtd_epilogue e{};
    e.bias = w->b_final; e.act = VTD_ACT_NONE;
    e.out = logits; e.ldo = 6; e.out_dtype = VTD_F32;
    e.detections = dets;                              // transform_predictions, fused
    rc = gemm_launch(HR, 6, kk(k), a, ka(k), w->w_final, kk(k), gdt, &e, st,
                     2.0 * HR * (double)kv * 6);
    if (rc) return rc;
  }
  return VTD_OK;
}
}  // namespace
}  // namespace vtd

extern "C" {

int vtd_profile_enable(int enable) {
  ProfState& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  p.enabled = enable != 0;
  return VTD_OK;
}

int vtd_profile_reset(void) {
  ProfState& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  for (auto& r : p.pending) (void)hipEventSynchronize(p.events[r.ev1]);
  p.pending.clear();
  p.next_event = 0;
  for (int i = 0; i < VTD_PROF_CLASSES; ++i) p.ms[i] = 0, p.launches[i] = 0, p.flops[i] = 0;
  return VTD_OK;
}

int vtd_profile_read(double* ms, int64_t* launches, double* flops, int n_classes) {
  ProfState& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  for (auto& r : p.pending) {
    hipError_t e = hipEventSynchronize(p.events[r.ev1]);
    if (e != hipSuccess) return fail(VTD_ERR_HIP, std::string("profile: ") + hipGetErrorString(e));
    float t = 0.f;
    (void)hipEventElapsedTime(&t, p.events[r.ev0], p.events[r.ev1]);
    p.ms[r.cls] += t;
    p.launches[r.cls] += 1;
    p.flops[r.cls] += r.flops;
  }
  p.pending.clear();
  p.next_event = 0;
  for (int i = 0; i < n_classes && i < VTD_PROF_CLASSES; ++i) {
    if (ms) ms[i] = p.ms[i];
    if (launches) launches[i] = p.launches[i];
    if (flops) flops[i] = p.flops[i];
  }
  return VTD_OK;
}

}  // extern "C"
