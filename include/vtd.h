/*
 * vtd.h — C-ABI of libvtd.so, the MI355X (gfx950) forward path of the Vision
 * Transformer detector of westlake-moonlight/vision_transformer_detector.
 *
 * The reference has no FFI: its forward is a Keras graph whose arithmetic runs in
 * TensorFlow 2.9.1's own kernels.  Each entry point below replaces one layer class
 * of that graph (cited as vtd.py:N = /root/reference/vision_transformer_detector.py);
 * `vtd_forward` replaces the whole `model(images, training=False)` call.
 *
 * Conventions
 *  - Every pointer argument named *_dev is DEVICE memory owned by the caller.  The
 *    library never allocates or frees memory inside a compute call and keeps no
 *    pointer after it returns.  `stream` is a hipStream_t (NULL = default stream).
 *  - Calls are asynchronous on `stream`, perform no host synchronisation and no
 *    allocation, and are therefore HIP-graph capturable.
 *  - Return value: VTD_OK (0) or a negative vtd_status; `vtd_last_error()` returns a
 *    thread-local message for the last failure on the calling thread.
 *  - "Padded" widths: every activation/weight row is padded with zeros to a multiple
 *    of VTD_KALIGN elements (see vtd_dims); pad columns are guaranteed zero on output.
 */
#ifndef VTD_H_
#define VTD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VTD_ABI_VERSION 16
#define VTD_KALIGN 64          /* K / row padding granule, elements              */
#define VTD_MAX_MLP 16         /* max encoder_mlp_quantities                     */
#define VTD_MAX_HEAD 64        /* max mlp_head layers * repeats                   */
#define VTD_MAX_DETECT 17      /* Constants.MAX_DETECT_OBJECTS_QUANTITY vtd.py:28 */

typedef enum vtd_status {
  VTD_OK = 0,
  VTD_ERR_INVALID_ARG = -1,    /* bad shape / null pointer / unsupported combo  */
  VTD_ERR_UNSUPPORTED = -2,    /* dtype or size not supported by this build     */
  VTD_ERR_HIP = -3,            /* a HIP runtime call failed (message has code)  */
  VTD_ERR_WORKSPACE = -4       /* workspace too small                           */
} vtd_status;

typedef enum vtd_dtype {       /* compute (GEMM operand) dtype                   */
  VTD_F32 = 0,                 /* parity mode: f32 operands, f32 MFMA            */
  VTD_BF16 = 1,                /* throughput mode: bf16 operands, f32 accumulate */
  VTD_FP8 = 2,                 /* forward mode only (vtd_config.dtype): encoder  */
                               /* Dense layers in MX-fp8 (vtd_gemm_mx8), the rest */
                               /* as VTD_BF16                                     */
  VTD_BF16X3 = 3               /* split-bf16 parity mode: every Dense layer as    */
                               /* three bf16 MFMA products with f32 accumulation, */
                               /* the rest fp32 (see "Split-bf16 operands")       */
} vtd_dtype;

/* Split-bf16 operands (VTD_BF16X3).  An f32 value v is held as hi = bf16(v) (round to
 * nearest even) and lo = bf16(v - hi): hi + lo carries 16 significand bits, and
 * hi_a hi_b + lo_a hi_b + hi_a lo_b leaves out only lo_a lo_b (<= 2^-18 |a b|).  A K-wide
 * f32 row is stored as a bf16 row of P-wide pieces (P >= K, P % 64 == 0 for a GEMM, the
 * columns [K, P) of every piece zero):
 *   A operand (activations, role 0):  [ hi | lo ]        (row stride >= 2 P)
 *   B operand (weights W^T, role 1):  [ hi | hi | lo ]   (row stride >= 3 P)
 * and vtd_gemm with dtype VTD_BF16X3, K = 3 P, reads each A row as [hi | lo | hi] (its K loop
 * returns to A's column 0 after 2 P) against the B row: one bf16 GEMM whose fp32
 * accumulators sum the three products.  Producers write the A form directly:
 * vtd_epilogue.out_dtype = VTD_BF16X3, vtd_layernorm / vtd_extract_patches / vtd_attention
 * with dtype = VTD_BF16X3 (ldo / ldy = 2 P); vtd_split_bf16x3 converts any f32 matrix. */

typedef enum vtd_act {         /* activation fused in a GEMM epilogue            */
  VTD_ACT_NONE = 0,
  VTD_ACT_GELU_TANH = 1,       /* tfa.layers.GELU() approximate=True vtd.py:402 */
  VTD_ACT_MISH = 2             /* MishActivation vtd.py:119-129                  */
} vtd_act;

/* create_vision_transformer_detector(...) kwargs, vtd.py:498-506.  dropout,
 * max_weight and clip_weight only act on training (Keras Dropout / MHA dropout are the
 * identity at inference; constraints apply after optimizer steps): no fields here. */
typedef struct vtd_config {
  int batch;
  int image_h, image_w, channels;     /* input_shape                              */
  int patch_size;
  int embedding_dim;
  int num_heads;                      /* encoder_num_heads                        */
  int key_dim;                        /* encoder_key_dim                          */
  int mlp_quantities;                 /* encoder_mlp_quantities                   */
  int repeat_times;                   /* encoder_repeat_times                     */
  int head_last_units;                /* mlp_head_last_units                      */
  int head_layers;                    /* mlp_head_dense_layers_quantity           */
  int head_repeats;                   /* mlp_head_dense_mish_block_repeats        */
  int use_mish;                       /* 1 = Mish, 0 = GELU(tanh)                 */
  int dtype;                          /* vtd_dtype                                */
} vtd_config;

/* Derived sizes (elements).  Fill with vtd_derive_dims. */
typedef struct vtd_dims {
  int grid_h, grid_w;                 /* ceil(H/p), ceil(W/p)  (SAME padding)     */
  int tokens;                         /* N = grid_h*grid_w                        */
  int pad_top, pad_left;              /* SAME pad_before                          */
  int patch_dim, patch_dim_p;         /* P = p*p*C and padded                     */
  int d, d_p;                         /* embedding_dim and padded                 */
  int key_dim_p;                      /* per-head padded key dim (32/64/128)      */
  int inner_p;                        /* num_heads * key_dim_p                    */
  int qkv_p;                          /* padded 3*inner_p                         */
  int mlp_units[VTD_MAX_MLP];         /* encoder MLP widths                       */
  int mlp_units_p[VTD_MAX_MLP];
  int n_head;                         /* head Dense layers (excl. dense & final)  */
  int head_units[VTD_MAX_HEAD];
  int head_units_p[VTD_MAX_HEAD];
  int tokens_p;                       /* head input width (Reshape) padded        */
  int64_t rows;                       /* batch * tokens                           */
  int64_t head_rows;                  /* batch * 17                               */
} vtd_dims;

/* Device pointers of one encoder block, packed by vtd_pack_dense / vtd_pack_vector.
 * Matrices: dtype = cfg.dtype, layout W^T [N_p][K_p] (row = output unit).
 * Vectors: fp32, padded with zeros.
 * VTD_FP8: w_qkv / w_out / w_mlp are MX-fp8 e4m3 [N_p][K8] (K8 = K_p rounded up to 128,
 * vtd_quantize_mx8 of the packed fp32 matrix) and s_* their scales [K8/128][N_p][4];
 * the s_* fields are ignored in the other modes.
 * LayerNorm fold (VTD_BF16 only): when ln1_colsum is non-NULL, w_qkv / b_qkv hold
 * vtd_fold_layernorm's W * diag(ln1_gamma) and b + W ln1_beta, ln1_colsum its column
 * sums, and the forward applies LayerNorm 1 in the query/key/value GEMM's epilogue
 * (vtd_epilogue.lnstat) instead of a LayerNorm pass; ln2_colsum likewise for LayerNorm 2
 * and w_mlp[0] / b_mlp[0].  NULL: the LayerNorm kernels run (ln*_gamma / beta used). */
typedef struct vtd_layer_weights {
  const float* ln1_gamma; const float* ln1_beta;        /* [d_p]                  */
  const void* w_qkv; const float* b_qkv;                /* [qkv_p][d_p], [qkv_p]  */
  const void* w_out; const float* b_out;                /* [d_p][inner_p], [d_p]  */
  const float* ln2_gamma; const float* ln2_beta;        /* [d_p]                  */
  const void* w_mlp[VTD_MAX_MLP]; const float* b_mlp[VTD_MAX_MLP];
  const uint8_t* s_qkv; const uint8_t* s_out;          /* VTD_FP8 block scales   */
  const uint8_t* s_mlp[VTD_MAX_MLP];
  const float* ln1_colsum; const float* ln2_colsum;     /* LN fold, or NULL        */
} vtd_layer_weights;

typedef struct vtd_weights {
  const void* w_patch; const float* b_patch;            /* [d_p][patch_dim_p]     */
  const float* pos_embedding;                           /* [tokens] fp32          */
  const vtd_layer_weights* layers;                      /* HOST array [repeat_times] */
  const void* w_det; const float* b_det;                /* Dense(17): [64][d_p]   */
  const void* w_head[VTD_MAX_HEAD]; const float* b_head[VTD_MAX_HEAD];
  const void* w_final; const float* b_final;            /* Dense(6): [64][136_p]  */
} vtd_weights;

/* ---------------------------------------------------------------- library ------ */
int vtd_abi_version(void);
const char* vtd_last_error(void);

/* Shapes of the graph built by create_vision_transformer_detector (vtd.py:498-583). */
int vtd_derive_dims(const vtd_config* cfg, vtd_dims* out);

/* Bytes of scratch `vtd_forward` needs for this config (256-B aligned buffers). */
int vtd_workspace_bytes(const vtd_config* cfg, size_t* bytes);

/* ---------------------------------------------------------------- weights ------ */
/* Pack a Keras Dense/EinsumDense kernel (fp32, row-major [K][N], device) into the
 * transposed, zero-padded compute layout dst[n_row_offset + n'][k'] (dtype), where
 * k' = (k / k_group) * k_group_p + k % k_group   (per-head K padding, attention_output)
 * n' = (n / n_group) * n_group_p + n % n_group   (per-head N padding, query/key/value).
 * Pass k_group = k_group_p = K (resp. N) for no grouping.  dst must be pre-zeroed. */
int vtd_pack_dense(const float* src_dev, int K, int N, int k_group, int k_group_p,
                   int n_group, int n_group_p, void* dst_dev, int ld_dst,
                   int n_row_offset, int dtype, void* stream);
/* Same re-indexing for a bias / LN vector (fp32 -> fp32). */
int vtd_pack_vector(const float* src_dev, int N, int n_group, int n_group_p,
                    float* dst_dev, int offset, void* stream);

/* f32 x [rows][ldx] (first K columns) -> split-bf16 y [rows][ldy], P >= K wide pieces
 * (columns [K, P) of each piece written as zero): role 0 the A operand [hi | lo], P = ldy / 2
 * (ldy % 2 == 0); role 1 the B operand [hi | hi | lo], P = ldy / 3 (ldy % 3 == 0). */
int vtd_split_bf16x3(const float* x_dev, int64_t rows, int K, int ldx, void* y_dev, int ldy,
                     int role, void* stream);

/* ---------------------------------------------------------------- per-op ------- */
/* ExtractImagePatches (vtd.py:177-206) + Reshape flatten_patches (vtd.py:279-280):
 * images NHWC fp32 [B][H][W][C] -> patches [B*N][ld_out] (dtype), SAME zero pad,
 * (kh, kw, c) order; columns [P, ld_out) written as zero.  dtype VTD_BF16X3: the split-bf16
 * A operand, two ld_out / 2 wide pieces (ld_out % 16 == 0). */
int vtd_extract_patches(const float* images_dev, int B, int H, int W, int C, int p,
                        void* out_dev, int ld_out, int dtype, void* stream);

/* Dense + activation (vtd.py:297, 389-403, 454, 472-483, 489):
 * C[m][n] = act(sum_k A[m][k] * Bt[n][k] + bias[n] + rowadd[m % rowadd_period]
 *               (rowadd only for n < rowadd_ncols)) + resid[m][n]
 * for m < M, n < N.  A, Bt in `dtype`; K % VTD_KALIGN == 0; lda, ldb % 8 == 0.
 * dtype VTD_BF16X3: bf16 operands, A the split-bf16 A operand [hi | lo] (lda >= 2 K / 3), Bt
 * the B operand [hi | hi | lo] (ldb >= K; its two hi pieces must be equal, as
 * vtd_split_bf16x3 role 1 writes them: a kernel may read either), K = 3 P with P % 64 == 0
 * (see "Split-bf16 operands").
 * out: fp32 (out_dtype 0), bf16 (1) or split-bf16 (VTD_BF16X3: the next GEMM's A operand
 * [hi | lo], two ldo / 2 wide pieces, ldo % 2 == 0, ldo / 2 >= N; bf16 / split-bf16
 * operands only); out2 (nullable) a second bf16 copy.
 * scatter_tokens > 0 selects the head Reshape epilogue (vtd.py:461-463): element
 * (m = b*T + t, n < 17) is stored at out[(b*17 + f / T) * ldo + f % T], f = t*17 + n. */
typedef struct vtd_epilogue {
  const float* bias;            /* [N] or NULL                                    */
  const float* rowadd;          /* position embedding per row, or NULL            */
  int rowadd_period, rowadd_ncols;
  int act;                      /* vtd_act                                         */
  const void* resid; int ldr;   /* residual in out_dtype (may alias out), or NULL  */
  void* out; int ldo; int out_dtype;
  void* out2; int ldo2;         /* optional bf16 copy                              */
  int scatter_tokens;
  /* LayerNorm folded into the GEMM (A = the raw rows x, Bt = W * diag(gamma) as stored,
   * bias = b + W beta): lnstat[2m], lnstat[2m+1] = mean, rstd of row m
   * (vtd_layernorm_stats) and colsum[n] = sum_k Bt[n][k]; the accumulator becomes
   * (acc - mean * colsum[n]) * rstd before bias / act.  Both NULL: no fold. */
  const float* lnstat; const float* colsum;
  /* Partial LayerNorm statistics of the output (the fold path's producer side): for row m
   * and 64-column block b, statout[2 (b stat_ld + m)] = mean and [.. + 1] = sum of squared
   * deviations from that mean, of the block's 64 stored bf16 values (centred partials:
   * exact whatever |mean| / std).  Slot-major: one plane of stat_ld >= M rows per block.
   * Only on full 256 x 256 tiles of the bf16 fast epilogues -- dtype VTD_BF16, M % 256 ==
   * N % 256 == 0 and at least 64 tiles (else vtd_gemm returns VTD_ERR_UNSUPPORTED); NULL: none. */
  float* statout; int stat_ld;
  /* out_dtype VTD_FP8 (vtd_gemm_mx8 only, every tile full: M % 256 == N % 256 == 0): the
   * output is written as the next GEMM's MX-fp8 A operand, byte for byte what
   * vtd_quantize_mx8 makes of the bf16-rounded output: e4m3 out[m * ldo + n] and
   * scale_out[n/128][scale_rows][4]. */
  uint8_t* scale_out; int64_t scale_rows;
  /* transform_predictions (vtd.py:586-647) fused into the final Dense(6) (SURVEY §8b
   * vtd_head_decode): with N == 6, an fp32 output and no scatter, detections[m * 6 + n] =
   * sigmoid(C[m][n]), clipped to [0, 1] for n >= 2, times (1, 79, 608, 608, 608, 608) --
   * what vtd_decode computes from the stored logits, bit for bit.  NULL: none. */
  float* detections;
} vtd_epilogue;
int vtd_gemm(int M, int N, int K, const void* A_dev, int lda, const void* Bt_dev,
             int ldb, int dtype, const vtd_epilogue* epi, void* stream);
/* Split-K form of vtd_gemm (dtype VTD_BF16 or VTD_BF16X3; what vtd_forward runs for the
 * detection head's few-tile, long-K Dense layers, vtd.py:468-486): `ksplit` K ranges of
 * K / 64 / ksplit
 * K-steps each write fp32 partial sums into part_dev ([ksplit][M][N] floats,
 * part_bytes >= ksplit * M * N * 4), then one pass sums them in split order and applies
 * the epilogue (the LayerNorm fold included; no partial statistics).  K % 64 == 0, N % 4 == 0,
 * 2 <= ksplit <= K / 64 with every split non-empty.  vtd_gemm_splitk_choice returns the
 * split count vtd_forward uses for (M, N, K, dtype) (1 = no split). */
int vtd_gemm_splitk(int M, int N, int K, const void* A_dev, int lda, const void* Bt_dev,
                    int ldb, int dtype, const vtd_epilogue* epi, float* part_dev,
                    size_t part_bytes, int ksplit, void* stream);
int vtd_gemm_splitk_choice(int M, int N, int K, int dtype);

/* MX-fp8 operands (OCP MX: e4m3 elements, one E8M0 scale byte e = 2^(e-127) per 32
 * consecutive K elements).  vtd_quantize_mx8: x [rows][ldx] (x_dtype F32 or BF16), first
 * K columns -> q [rows][ldq] e4m3 bytes with Kq columns (Kq % 128 == 0, columns [K, Kq)
 * zero) and scales s[Kq/128][s_rows][4] (s_rows >= rows; the 4 scales of one 128-wide
 * K-step of a row are one dword).  Block scale: the least 2^E with amax <= 448 * 2^E,
 * E in [-126, 126]; elements round to nearest even (oracle/mx8.py restates both).
 * vtd_gemm_mx8: as vtd_gemm (same epilogue) with A [M][lda], Bt [N][ldb] in that format,
 * K % 128 == 0, lda/ldb % 16 == 0, sa_rows >= M, sb_rows >= N, both % 4 == 0;
 * D = sum_k dec(A) dec(Bt) accumulated in fp32 by v_mfma_scale_f32_16x16x128_f8f6f4. */
int vtd_quantize_mx8(const void* x_dev, int x_dtype, int64_t rows, int K, int ldx, int Kq,
                     uint8_t* q_dev, int ldq, uint8_t* s_dev, int64_t s_rows, void* stream);
/* vtd_layernorm with the output quantized as vtd_quantize_mx8 does the bf16-rounded
 * LayerNorm output (Kq % 128 == 0 >= D columns, ldq % 16 == 0): LN + quantize in one pass. */
int vtd_layernorm_mx8(const void* x_dev, int x_dtype, int64_t rows, int D, int ldx,
                      const float* gamma_dev, const float* beta_dev, float eps, uint8_t* q_dev,
                      int ldq, int Kq, uint8_t* s_dev, int64_t s_rows, void* stream);
int vtd_gemm_mx8(int M, int N, int K, const uint8_t* A_dev, int lda, const uint8_t* sA_dev,
                 int64_t sa_rows, const uint8_t* Bt_dev, int ldb, const uint8_t* sB_dev,
                 int64_t sb_rows, const vtd_epilogue* epi, void* stream);

/* keras LayerNormalization(axis=-1, epsilon) (vtd.py:353-357, 375-379):
 * x (x_dtype: fp32, or the bf16 residual stream) [rows][ldx] -> y (dtype) [rows][ldy];
 * fp32 statistics over the first D columns; columns [D, ldy) of y written as zero.
 * dtype VTD_BF16X3: y is the split-bf16 A operand, two ldy / 2 wide pieces. */
int vtd_layernorm(const void* x_dev, int x_dtype, int64_t rows, int D, int ldx,
                  const float* gamma_dev, const float* beta_dev, float eps,
                  void* y_dev, int ldy, int dtype, void* stream);

/* Row statistics of keras LayerNormalization (the same two-pass fp32 mean / biased
 * variance as vtd_layernorm): stat[2r] = mean, stat[2r+1] = 1 / sqrt(var + eps) of the
 * first D columns of row r of x (x_dtype F32 or BF16). */
int vtd_layernorm_stats(const void* x_dev, int x_dtype, int64_t rows, int D, int ldx,
                        float eps, float* stat_dev, void* stream);

/* (mean, rstd) per row from the centred partials a producer GEMM wrote
 * (vtd_epilogue.statout with stat_ld == rows: `slots` planes of `rows` (mean, M2) pairs,
 * D == 64 * slots): Chan's merge of the block (mean, M2) pairs in fp32, no one-pass
 * sum(x^2) - mean^2 cancellation. */
int vtd_layernorm_stats_finalize(const float* partial_dev, int64_t rows, int slots, int D,
                                 float eps, float* stat_dev, void* stream);

/* Folds LayerNorm(gamma, beta) into the Dense layer that consumes it: w32 fp32 packed
 * W^T [N][ldw] (first K columns used) -> w_out (dtype) [N][ldo] = W^T[n][k] * gamma[k]
 * (columns [K, ldo) zero), bias_out[n] = bias_in[n] + sum_k W^T[n][k] beta[k] and
 * colsum[n] = sum_k w_out[n][k] (of the stored, rounded values); fp64 sums.
 * LN(x) W + b == (x W' - mean * colsum) * rstd + bias_out, exactly in real arithmetic. */
int vtd_fold_layernorm(const float* w32_dev, int N, int K, int ldw, const float* gamma_dev,
                       const float* beta_dev, const float* bias_in_dev, void* w_out_dev,
                       int ldo, int dtype, float* bias_out_dev, float* colsum_dev,
                       void* stream);

/* keras MultiHeadAttention core (vtd.py:364-369): per batch b, head h,
 * O = softmax(scale * Q K^T) V with Q, K, V read from qkv [B*N][ldqkv] at column
 * offsets h*dkp, inner + h*dkp, 2*inner + h*dkp (inner = heads*dkp); O written to
 * out [B*N][ldo] at column h*dkp.  dkp in {32, 64, 128}; scale = 1/sqrt(key_dim).
 * dtype VTD_BF16X3 (the split-bf16 parity mode): qkv is fp32, every product runs as three
 * bf16 MFMA products (hi.hi + lo.hi + hi.lo, fp32 softmax statistics), and out is the
 * split-bf16 A operand of the attention-output Dense, [hi | lo] in two ldo / 2 wide pieces
 * (ldo % 2 == 0, ldo / 2 >= heads*dkp; columns [heads*dkp, ldo / 2) not written). */
int vtd_attention(const void* qkv_dev, int B, int N, int heads, int dkp, int ldqkv,
                  float scale, void* out_dev, int ldo, int dtype, void* stream);

/* vtd_attention (bf16 operands) with the output written as the MX-fp8 A operand of the
 * attention-output Dense (VTD_FP8 mode): q_dev [B*N][ldq] e4m3 bytes, s_dev
 * [heads*dkp/128][s_rows][4] E8M0 scales (the vtd_quantize_mx8 layout); byte-identical to
 * vtd_attention (bf16 out) followed by vtd_quantize_mx8. heads*dkp % 128 == 0, ldq % 16 == 0,
 * s_rows >= B*N. */
int vtd_attention_mx8(const void* qkv_dev, int B, int N, int heads, int dkp, int ldqkv,
                      float scale, uint8_t* q_dev, int ldq, uint8_t* s_dev, int64_t s_rows,
                      void* stream);

/* transform_predictions (vtd.py:586-647): logits fp32 [n][6] -> detections fp32
 * [sigmoid, sigmoid*79, clip(sigmoid)*608 x4]. */
int vtd_decode(const float* logits_dev, int64_t n, float* dets_dev, void* stream);

/* transform_predictions + the detection test of MeanAveragePrecision.update_state
 * (vtd.py:1359-1384), per slot: dets as vtd_decode; category = round-half-even of the
 * decoded class (tf.round); class confidence = (0.5 - |cls - category|) / 0.5;
 * valid = objectness > obj_threshold && confidence > cls_threshold
 * (Constants.OBJECTNESS_THRESHOLD / CLASSIFICATION_CONFIDENCE_THRESHOLD = 0.5).
 * category_dev (int32) and valid_dev (uint8) may be NULL. */
int vtd_decode_detections(const float* logits_dev, int64_t n, float* dets_dev,
                          int32_t* category_dev, uint8_t* valid_dev, float obj_threshold,
                          float cls_threshold, void* stream);

/* ---------------------------------------------------------------- input ------- */
/* _get_image_tensor_coco after decode (vision_transformer_utilities.py:418-449):
 * tf.image.resize_with_pad(image, target_h, target_w) (bilinear, half-pixel centers, no
 * antialias; TF 2.9 float32 geometry: ratio = max(w/tw, h/th), resized = floor(side/ratio),
 * pad_before = floor((target - side/ratio)/2)) -> clip [0, 255] -> /127.5 -> -1.
 * pixels_dev: B decoded uint8 HWC (C = 3) images, image b at byte offset offsets_dev[b];
 * sizes_dev: int32 [B][2] = (height, width). out_dev: fp32 NHWC [B][target_h][target_w][3]
 * in [-1, 1] (pad = -1), i.e. the `images` argument of vtd_forward. Images whose resized
 * side would be 0 (TF raises for them) must be rejected by the caller: the kernel writes
 * the pad value for them. Replaces the tf.image / tf.clip_by_value / arithmetic ops at
 * vision_transformer_utilities.py:438-447. */
int vtd_resize_with_pad(const uint8_t* pixels_dev, const int64_t* offsets_dev,
                        const int32_t* sizes_dev, int B, int target_h, int target_w,
                        float* out_dev, void* stream);

/* JPEG decode on the device, tf.image.decode_image(file, channels=3)
 * (vision_transformer_utilities.py:431) for baseline / extended sequential and progressive
 * Huffman JPEG: 8-bit, 1, 3 or 4 (CMYK / YCCK) components, 4:4:4 / 4:2:2 / 4:2:0, restart
 * intervals.  libjpeg-turbo's decode path (what TF uses): ISLOW IDCT, fancy upsampling,
 * YCbCr -> RGB; gray -> RGB replicated; CMYK (YCCK -> CMYK as jdcolor.c) -> RGB as TF's
 * jpeg_mem.cc (Adobe marker: R = K C / 255, else (255 - K)(255 - C) / 255).  Other JPEGs
 * (arithmetic-coded, lossless, 12-bit, 4:4:0, ...) return VTD_ERR_UNSUPPORTED with the reason.
 * vtd_jpeg_info: header only (host).  The images are HOST buffers; their marker segments are
 * parsed on the host, the entropy-coded data + derived tables copied to the workspace on
 * `stream` (through a pinned staging buffer the library reuses), image i written as RGB
 * uint8 HWC at out_dev + out_offsets[i] (host array). */
int vtd_jpeg_info(const uint8_t* jpeg, size_t len, int* h, int* w, int* comps);
int vtd_jpeg_workspace_bytes(const uint8_t* const* jpegs, const size_t* lens, int n,
                             int32_t* dims /* nullable: 2n ints, (h, w) per image */,
                             size_t* bytes);
int vtd_jpeg_decode(const uint8_t* const* jpegs, const size_t* lens, int n, uint8_t* out_dev,
                    const int64_t* out_offsets, void* workspace_dev, size_t workspace_bytes,
                    void* stream);

/* PNG decode, tf.image.decode_image(file, channels=3) for PNG (vision_transformer_utilities.py
 * :431) as TF's libpng path does it: every colour type and bit depth (1-16), Adam7
 * interlacing; palette -> RGB, gray -> RGB, alpha / tRNS dropped, 16-bit -> high byte.  The
 * chunk walk (critical-chunk CRCs checked) and the zlib inflate run on the host over a few
 * threads; a row filter byte above 4 is an error (libpng's "bad adaptive filter value"); the
 * filtered scanlines are copied to the workspace on `stream` (pinned staging the library
 * reuses) and un-filtered + converted on the device (rows of up to 16 KiB of filtered bytes
 * through LDS, wider ones in place in the workspace: no width limit beyond w * h <= 2^28),
 * image i written as RGB uint8 HWC at out_dev + out_offsets[i].  Same calling convention as
 * the JPEG entry points; vtd_png_info's comps = samples per pixel of the file (1-4).
 * vtd_png_inflate: the host half alone for one file (chunk walk, inflate, filter-byte check)
 * into a caller HOST buffer; *need = the filtered scanline bytes of all passes (out == NULL:
 * only *need). */
int vtd_png_info(const uint8_t* png, size_t len, int* h, int* w, int* comps);
int vtd_png_workspace_bytes(const uint8_t* const* pngs, const size_t* lens, int n,
                            int32_t* dims, size_t* bytes);
int vtd_png_decode(const uint8_t* const* pngs, const size_t* lens, int n, uint8_t* out_dev,
                   const int64_t* out_offsets, void* workspace_dev, size_t workspace_bytes,
                   void* stream);
int vtd_png_inflate(const uint8_t* png, size_t len, uint8_t* out, size_t out_bytes, size_t* need);

/* BMP decode, tf.image.decode_image(file, channels=3) for BMP as TF 2.x's DecodeImageV2 does it
 * (decode_image_op.cc): the file's channels = bits-per-pixel / 8 in {1, 3, 4}, rows bottom-up
 * (top-down for a negative height) padded to 4 bytes; 24-bit BGR -> RGB, 32-bit BGRA -> RGB
 * (alpha dropped), 8-bit -> the stored byte replicated (TF applies no palette).  Other bit
 * depths and any compression but BI_RGB / BI_BITFIELDS (RLE, BI_JPEG, BI_PNG: bytes TF would
 * misread as pixels) return VTD_ERR_UNSUPPORTED.  Same
 * calling convention as the PNG / JPEG entry points; comps = 3. */
int vtd_bmp_info(const uint8_t* bmp, size_t len, int* h, int* w, int* comps);
int vtd_bmp_workspace_bytes(const uint8_t* const* bmps, const size_t* lens, int n,
                            int32_t* dims, size_t* bytes);
int vtd_bmp_decode(const uint8_t* const* bmps, const size_t* lens, int n, uint8_t* out_dev,
                   const int64_t* out_offsets, void* workspace_dev, size_t workspace_bytes,
                   void* stream);

/* ---------------------------------------------------------------- forward ------ */
/* model(images, training=False) (vtd.py:579-581, ipynb:836):
 * images NHWC fp32 [B][H][W][C] in [-1, 1] -> logits fp32 [B][17][6] (pre-sigmoid),
 * and, if dets_dev != NULL, transform_predictions(logits) fp32 [B][17][6]. */
int vtd_forward(const vtd_config* cfg, const vtd_weights* w, const float* images_dev,
                float* logits_dev, float* dets_dev, void* workspace_dev,
                size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- metric ------- */
/* iou_calculator (vtd.py:761-875), elementwise over n box pairs.  Each box is the last
 * 4 floats (x, y, height, width) of a row of `stride` floats (stride 4: bare boxes;
 * stride 6: detection rows).  iou_dev: n floats.  Intersections follow the reference's
 * strict-inequality overlap test; IoU = inter / (union + 1e-8). */
int vtd_iou(const float* label_bbox_dev, const float* pred_bbox_dev, int64_t n, int stride,
            float* iou_dev, void* stream);

/* MeanAveragePrecision (vtd.py:1268-2060).  The state is the reference's three
 * Variables, caller-allocated in device memory:
 *   latest_positive_bboxes    float [VTD_MAP_CLASSES][VTD_MAP_LATEST][VTD_MAP_PER_IMAGE][2]
 *   labels_quantity_per_image float [VTD_MAP_CLASSES][VTD_MAP_LATEST]
 *   showed_up_classes         uint8 [VTD_MAP_CLASSES]
 * vtd_map_update = update_state(y_true, y_pred, use_transform_predictions=False)
 * (vtd.py:1310-1862): y_true / y_pred fp32 [batch][boxes][6] rows (objectness, class,
 * x, y, height, width); labels mark empty rows with class -8; y_pred is DECODED (run
 * vtd_decode first for raw logits).  One launch per batch, stream-ordered.
 * vtd_map_result = result() (vtd.py:1865-2049): out_dev fp32 [11] = the AP at IoU
 * thresholds linspace(0.5, 0.95, 10), then the mAP (their mean). */
#define VTD_MAP_CLASSES 80        /* Constants.CLASSES vtd.py:20 */
#define VTD_MAP_LATEST 3          /* Constants.LATEST_RELATED_IMAGES vtd.py:32 */
#define VTD_MAP_PER_IMAGE 14      /* Constants.BBOXES_PER_IMAGE vtd.py:37 */
#define VTD_MAP_MAX_BOXES 64      /* boxes per image accepted by vtd_map_update */
int vtd_map_reset(float* latest_positive_bboxes, float* labels_quantity_per_image,
                  uint8_t* showed_up_classes, void* stream);
int vtd_map_update(float* latest_positive_bboxes, float* labels_quantity_per_image,
                   uint8_t* showed_up_classes, const float* y_true_dev,
                   const float* y_pred_dev, int batch, int boxes, void* stream);
int vtd_map_result(const float* latest_positive_bboxes, const float* labels_quantity_per_image,
                   const uint8_t* showed_up_classes, float* out_dev, void* stream);

/* Optional per-kernel timing of vtd_forward (hipEvents on `stream`, recorded around
 * every launch while enabled).  vtd_profile_read returns per-class totals in ms
 * summed over the forwards since the last reset; classes: 0 gemm, 1 attention,
 * 2 layernorm, 3 patches, 4 other. Also returns per-class launch counts and FLOPs. */
#define VTD_PROF_CLASSES 5
int vtd_profile_enable(int enable);
int vtd_profile_reset(void);
int vtd_profile_read(double* ms, int64_t* launches, double* flops, int n_classes);

/* Run-time switches (kernel-variant A/B knobs).  Each is read ONCE per process from its
 * environment variable at the first use of any knob; vtd_set_knob overrides one for the
 * rest of the process (returns the previous value) so tests compare variants in one
 * process.  -1 = unset: the library's default.
 *   VTD_KNOB_ATTN_VARIANT (VTD_ATTN_VARIANT): bf16 attention kernel, 4 = persistent short-
 *     sequence kernel where it applies (default), 2 = streaming, 3 = streaming 8-wave,
 *     1 = the register-staged first kernel.
 *   VTD_KNOB_ATTN_GRID (VTD_ATTN_GRID): persistent attention workgroups (default: CUs).
 *   VTD_KNOB_GEMM_NGW (VTD_GEMM_NGW): GEMM tile-order group width (0 = row-major).
 *   VTD_KNOB_SPLITK (VTD_SPLITK): 0 disables split-K (the head's and, at small batches, the
 *     encoder's), a value >= 64 sets the head's workgroup target per launch (default 256);
 *     both change the workspace size.
 *   VTD_KNOB_JPEG_CHUNK_BITS (VTD_JPEG_CHUNK_BITS): Huffman chunk length of vtd_jpeg_decode.
 *   VTD_KNOB_SKINNY (VTD_SKINNY): 0 keeps the head's narrow bf16 layers (N <= 320) on the
 *     128 x 128 kernel instead of the skinny one; a value >= 64 sets the N threshold (such
 *     layers are then not split-K).
 *   VTD_KNOB_F32_PP2 (VTD_F32_PP2): 0 keeps large fp32-mode GEMMs on the 128 x 128 kernel
 *     instead of the 256-tile f32 one.
 *   VTD_KNOB_STAGGER (VTD_STAGGER): the two-stream split's second micro-batch starts k stages
 *     (patch embedding, encoder layers) behind the first (default: 1 for parts of at most 32
 *     row tiles of 256 -- C2 at B = 64 -- else 0, in phase).
 *   VTD_KNOB_GEMM_TR (VTD_GEMM_TR): 256-tile bf16 GEMM accumulator layout, 1 = transposed
 *     (register-direct epilogue) for every layer, 0 = for none (default: activation layers).
 *   VTD_KNOB_FIN_WGS (VTD_FIN_WGS): LayerNorm-statistics finalize as n grid-stride
 *     workgroups of 1024 threads (default: one 256-thread workgroup per 256 rows).
 *   VTD_KNOB_GEMM_TPW (VTD_GEMM_TPW): consecutive 256 x 256 output tiles per bf16 GEMM
 *     workgroup (default 1); with more, the next tile's first K-stage loads during the
 *     current tile's epilogue. */
enum {
  VTD_KNOB_ATTN_VARIANT = 0,
  VTD_KNOB_ATTN_GRID = 1,
  VTD_KNOB_GEMM_NGW = 2,
  VTD_KNOB_SPLITK = 3,
  VTD_KNOB_JPEG_CHUNK_BITS = 4,
  VTD_KNOB_SKINNY = 5,
  VTD_KNOB_F32_PP2 = 6,
  VTD_KNOB_STAGGER = 7,
  VTD_KNOB_GEMM_TR = 8,
  VTD_KNOB_FIN_WGS = 9,
  VTD_KNOB_GEMM_TPW = 10,
  VTD_KNOB_COUNT = 11
};
int vtd_set_knob(int knob, int value);
int vtd_get_knob(int knob);

#ifdef __cplusplus
}
#endif
#endif /* VTD_H_ */
