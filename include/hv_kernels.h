/*
 * hv_kernels.h -- C ABI of the MI355X (gfx950) HybridVision hot-path library (libhvs.so).
 *
 * The reference (nazimurahman/humanoid-vision-system) has no FFI layer: its hot path is
 * stock PyTorch ops called from the src/models nn.Modules.  These entry points are what
 * those modules bind to instead (the Python side is humanoid-vision-system_amd/hv_amd,
 * see INTEGRATION.md).  Each entry point names the reference function it replaces.
 *
 * Conventions
 *   - plain device pointers + sizes; no torch types.  Activations are token-major
 *     (NHWC / [tokens, channels]) and either fp32 or bf16 (raw 16-bit storage).
 *   - the caller owns every buffer (PyTorch caching allocator); kernels never allocate.
 *   - every call is asynchronous on `stream`, performs no host synchronisation and is
 *     hipGraph-capturable.
 *   - return value: 0 on success, a hipError_t (>0) from the launch, or a negative
 *     argument-error code (HV_EINVAL / HV_EUNSUPPORTED).
 */
#ifndef HV_KERNELS_H
#define HV_KERNELS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* hv_stream_t; /* == hipStream_t */

enum { HV_F32 = 0, HV_BF16 = 1, HV_F16 = 2 /* preprocess output only */ };
enum { HV_ACT_NONE = 0, HV_ACT_RELU = 1, HV_ACT_SILU = 2, HV_ACT_GELU = 3,
       HV_ACT_LEAKY = 4 /* slope 0.1 */, HV_ACT_SIGMOID = 5 };
enum { HV_OK = 0, HV_EINVAL = -1, HV_EUNSUPPORTED = -2 };

/* ABI version: 2 since hv_adamw gained `steps` and `active`, hv_grad_norms `active`, the dropout
 * entry points and hv_gemm_desc a device `seed_offset`, hv_mhc_fused_supported gained `variant`,
 * hv_mhc_fused_args grew by 8 bytes and the hv_gemm_set_* / hv_mhc_fused_set_* setters were
 * removed; 3 since hv_gemm_desc gained `colsum_part` and hv_mhc_fused_args `split_work` /
 * `split_count` (appended); 4 since hv_nms / hv_nms_work_bytes take `max_cells` (any candidate count,
 * any max_det).  Bindings compare it with the version they were written against. */
#define HV_ABI_VERSION 4
int hv_abi_version(void);
/* build provenance: a hash of the sources (the .hip / .h files of csrc, the include headers, the Makefile) the
 * library was compiled from; the Python loader recomputes it and refuses a stale build */
const char* hv_build_id(void);
/* lets bindings verify their struct mirrors */
void hv_struct_sizes(int* out5);  /* sizeof of the 5 ABI structs, in declaration order */

/* ------------------------------------------------------------------------------------
 * Sinkhorn-Knopp projection, grouped.
 * Replaces SinkhornKnoppProjection.forward (reference src/models/manifold_layers.py:32-93,
 * called from ManifoldHyperConnection.constrained_matrices :205-221).
 * M = softmax(raw / tau, -1) * m, then `iters` x (row-normalise, column-normalise) with
 * eps; history[t] = |mean(row sums at iteration t) - 1|.  All matrices of a table run in
 * the same 2*iters+2 launches.  The table lives in device memory (hv_sinkhorn_entry[count]);
 * row_block_start / col_start are exclusive prefix sums filled by the host.
 * ------------------------------------------------------------------------------------ */
typedef struct hv_sinkhorn_entry {
  const float* raw;   /* [batch, n, m] fp32 */
  float* out;         /* [batch, n, m] fp32 (also holds the softmax kernel K during the run) */
  float* history;     /* [iters] or NULL */
  float* work;        /* hv_sinkhorn_work_floats(batch, n, m, iters) floats */
  int batch, n, m, iters;
  float eps, tau;
  int row_block_start; /* prefix over entries of batch*ceil(n/16) */
  int col_start;       /* prefix over entries of batch*m */
  int row_start;       /* prefix over entries of batch*n */
  int pad_;
} hv_sinkhorn_entry;

size_t hv_sinkhorn_work_floats(int batch, int n, int m, int iters);
int hv_sinkhorn_group_forward(const hv_sinkhorn_entry* dev_table, int count,
                              int total_rows, int total_row_blocks, int total_cols,
                              int max_iters, hv_stream_t stream);
/* The same, split for two streams (a captured graph's parallel branches): part 1 = the small
   entries (<= 256 x 256: one workgroup each, all iterations inside one launch), part 2 = the
   large ones (grouped row / column passes), 0 = both on `stream`.  Parts 1 and 2 touch
   disjoint entries. */
int hv_sinkhorn_group_forward_part(const hv_sinkhorn_entry* tab, int count, int total_rows,
                                   int total_row_blocks, int total_cols, int max_iters, int part,
                                   hv_stream_t stream);
/* The single-workgroup kernel keeps the per-iteration row-sum history in LDS: up to this many
   iterations.  Beyond it part 0 runs every entry through the grouped passes (any iteration
   count, as the reference accepts) and part 1 returns HV_EUNSUPPORTED. */
int hv_sinkhorn_small_max_iters(void);

/* ------------------------------------------------------------------------------------
 * MFMA GEMM with fused prologue/epilogue:  C[M,N] = epi( A'[M,K] . B[N,K]^T )
 * Replaces the conv2d / linear / matmul calls of the reference hot path
 * (vision_backbone.py:42-49,112-114; feature_fusion.py:33-49,65; yolo_head.py:120-127,139;
 *  manifold_layers.py:253-263; vit_encoder_decoder.py:94-97,146-152).
 * A' = A (dense), LayerNorm-normalised A (a_mean/a_rstd per row), an implicit im2col of an
 * NHWC image (conv_k > 0), or the K-concatenation [A | A2] (a2 != NULL, split at k1).
 * epi: v = acc*alpha; v *= scale[n]; v += bias[n]; v = act(v); v += residual[m, n]; store.
 * ------------------------------------------------------------------------------------ */
typedef struct hv_gemm_desc {
  int dtype;          /* HV_F32 or HV_BF16: storage type of A, A2 and B (fp32 accumulate) */
  int M, N, K;
  const void* A; long lda;
  const void* A2; long lda2; int k1;   /* optional second K segment */
  const void* B; long ldb;             /* [N, K], K contiguous */
  void* C; long ldc; int c_dtype;      /* output storage type */
  const float* a_mean;                 /* LN prologue (optional) */
  const float* a_rstd;
  const float* scale;                  /* [N] optional */
  const float* bias;                   /* [N] optional */
  int act;
  float alpha;
  const void* residual; long ldr; int r_dtype;  /* optional */
  int r_mod;          /* > 0: residual row index = m % r_mod (broadcast over images) */
  /* implicit-GEMM convolution: A is an NHWC image [conv_n, conv_h, conv_w, conv_c];
     K = conv_k*conv_k*conv_c ordered (kh, kw, c); M = conv_n*conv_oh*conv_ow */
  int conv_n, conv_h, conv_w, conv_c, conv_k, conv_stride, conv_pad, conv_oh, conv_ow;
  /* with a_mean/a_rstd: b_colsum[n] = sum_k B[n,k] lets the LDS-DMA kernel apply the
     LayerNorm after the product, rstd (acc - mean colsum) (exact); NULL: LN on load */
  const float* b_colsum;
  /* ---- training-step extensions ----
     epi_mode 0: as above.
     epi_mode 1 (forward, saves the pre-activation): aux[m, n] = pre-act value (aux_dtype),
                then v = dropout(act(v)) with drop_p / drop_seed.
     epi_mode 2 (gradient): v = acc * alpha * keep(m, n) / (1 - drop_p) * act'(aux[m, n])
                (+ residual) -- the backward of act + dropout fused into the dgrad GEMM.
     keep(m, n) = hv_drop_keep(drop_seed, m * N + n, drop_p), identical in every kernel. */
  void* aux; long ld_aux; int aux_dtype;
  int epi_mode;
  float drop_p;
  unsigned int drop_seed;
  /* dgrad of a convolution: A is the output-gradient image [conv_n, conv_h, conv_w, conv_c]
     (conv_h/conv_w = forward OUTPUT size, conv_c = forward cout), rows are the pixels of the
     forward INPUT [conv_n, conv_oh, conv_ow]; B = W^T [cin, kh, kw, cout]; tap (kh, kw) of
     input pixel (ih, iw) reads output pixel ((ih + pad - kh) / stride, ...) when divisible. */
  int conv_transposed;
  /* per-call kernel selection, 0 = automatic (the product default).  Bit fields HV_GV_* below;
     tests and A/B tools pin a kernel variant per launch -- there is no process-global switch,
     so concurrent callers (engine worker threads, streams) never see each other's choice. */
  int variant;
  /* split-K for small output grids (inference epilogues, epi_mode 0, bf16, LDS-DMA kernel):
     splitk > 1 splits the K-tiles of every output tile over `splitk` workgroups, each writing
     its fp32 partial product to splitk_work [splitk][M][N] and bumping the tile's arrival
     counter; the LAST workgroup to arrive sums the partials in slice order (deterministic,
     independent of arrival order) and runs the epilogue above.  0 or 1 = off.  The caller owns
     the workspace (splitk * M * N floats) and the counters (HV_SPLITK_MAX_TILES ints, zero
     before the first use; every launch leaves them zero again). */
  float* splitk_work;
  int* splitk_count;
  int splitk;
  int pad2_;
  /* dropout seed offset (device, may be NULL): the epilogues' keep(m, n) uses drop_seed +
     *seed_offset, so a graph-captured training step draws new masks on every replay by
     advancing one device word (the seed arguments baked into the graph stay constant) */
  const unsigned int* seed_offset;
  /* gradient epilogue (epi_mode 2) only, may be NULL: column sums of C as stored, per 64-row
     block -- colsum_part[b * N + n] = sum of C[m, n] over m in [64 b, 64 b + 64) (fp32; a
     workgroup owning a taller tile writes its sum into its first block and zeros into the
     others).  ceil(M / 128) * 2 blocks must be allocated; hv_colsum_final reduces the first
     ceil(M / 64).  The bias gradient of the layer whose activation backward this launch fuses,
     without a second pass over C (replaces hv_colsum on it).  HV_EUNSUPPORTED when the call
     does not take the LDS-DMA kernel's staged gradient epilogue; nothing is launched then.  It
     takes: epi_mode 2, bf16, no split-K, no transposed conv, not the Cin = 32 3x3 conv, C 16-B
     aligned with ldc % 8 == 0 (the residual likewise), no variant forcing another path, and the
     operands the LDS-DMA kernel accepts: dense K % 8 == 0 (K-tails of a 64-deep k-tile are
     zero-filled) or an implicit conv with Cin % 8 == 0. */
  float* colsum_part;
} hv_gemm_desc;

#define HV_SPLITK_MAX_TILES 4096
#define HV_GV_TILE_MASK    0x7     /* force: 1 128x128, 2 64x128, 3 128x64, 4 64x64 (LDS-DMA ring),
                                      5 256x256 ping-pong, 6 persistent small-K */
#define HV_GV_REGSTAGE     0x8     /* register-staged kernel only (no LDS-DMA path) */
#define HV_GV_NO_BIG       0x10    /* never the 256x256 ping-pong kernel */
#define HV_GV_BIG_ALWAYS   0x20    /* the 256x256 kernel whenever eligible */
#define HV_GV_NO_SMALL     0x40    /* no 64x64 tiles for small grids */
#define HV_GV_TRAIN128     0x80    /* 128x128 tiles for the training epilogues */
#define HV_GV_FLAT_EPI     0x100   /* fragment-layout (not LDS-staged) inference epilogue */
#define HV_GV_FLAT_TRAIN   0x200   /* fragment-layout training epilogue */
#define HV_GV_SHALLOW      0x400   /* 2-buffer rings for the 64x64 / 64x128 / 128x64 tiles */
#define HV_GV_CONV_KTAIL   0x800   /* convolutions with K % 64 != 0 on the LDS-DMA kernel */
#define HV_GV_NO_SMALLK    0x1000  /* no persistent small-K kernel */
#define HV_GV_SK_DIAG1     0x2000  /* small-K kernel diagnostics (tools/k256_probe2.py; outputs
                                      garbage): skip the stores */
#define HV_GV_SK_DIAG2     0x4000  /* ... skip the k-loop */
#define HV_GV_SK_RES3      0x8000  /* small-K kernel: B-resident column-stationary form (K 192 / 256, no
                                      residual), 3-stage A ring */
#define HV_GV_SK_RES4      0x10000 /* ... 4-stage A ring */
#define HV_GV_TRAIN_BIG    0x20000 /* training epilogues (epi_mode 1 / 2) may take the 256x256 ping-pong kernel
                                      (measured +1.2 % train-step time at B=16, so opt-in) */
#define HV_GV_DEEP8        0x40000 /* 64x64 tiles on the 8-stage ring (inference epilogues; measured no gain) */
#define HV_GV_NO_DEEP8     0x80000 /* (kept for the A/B tools: the 8-stage ring is never automatic) */
#define HV_GV_TRAIN_NOPF   0x100000 /* gradient epilogue (epi_mode 2) loads each pass's aux rows after the previous
                                      pass's stores (the pre-round-4 form; default: one pass ahead) */
int hv_gemm(const hv_gemm_desc* d, hv_stream_t stream);
/* ------------------------------------------------------------------------------------
 * Row statistics / normalisation (manifold_layers.py:250,267 LayerNorm eps 1e-5;
 * RMSNorm :449-456 eps 1e-8).
 * ------------------------------------------------------------------------------------ */
int hv_row_stats(int dtype, const void* x, long ldx, int rows, int cols, float eps,
                 float* mean, float* rstd, hv_stream_t stream);
/* y = LN(x [+ res_in]) * gamma + beta [+ res_out];  x may be fp32 or bf16 */
int hv_layernorm(int x_dtype, const void* x, int rows, int cols, float eps,
                 const float* gamma, const float* beta,
                 int y_dtype, void* y, const void* res_out, int res_dtype, hv_stream_t stream);
int hv_rmsnorm(int dtype, const void* x, int rows, int cols, float eps, const float* scale,
               void* y, hv_stream_t stream);

/* ------------------------------------------------------------------------------------
 * mHC coefficient preparation (parameter-only; manifold_layers.py:205-221 + the algebraic
 * fold documented in DESIGN.md): writes fp32
 *   gc[D, Hd]   = (gamma_pre (.) sigmoid(H_pre_raw)) centred over the input index
 *                 (stored [Hd, D] when gc_transposed)
 *   u[Hd]       = beta_pre . sigmoid(H_pre_raw)
 *   wct[D, D+Hd]= [H_res - rowmean | 2 sigmoid(H_post_raw) - rowmean]^T
 * ------------------------------------------------------------------------------------ */
int hv_mhc_prep(int D, int Hd, const float* h_pre_raw, const float* h_post_raw,
                const float* h_res, const float* gamma_pre, const float* beta_pre,
                float* gc, int gc_transposed /* 1: gc is [Hd, D] */, float* u, float* wct,
                float* row_mean_ws, hv_stream_t stream);

/* conv weight [cout, cin, k, k] fp32 -> implicit-GEMM operand [cout, k, k, cin] (fp32|bf16),
   optionally scaled per output channel */
int hv_conv_weight_prep(const float* w, int cout, int cin, int k, const float* scale,
                        int y_dtype, void* y, hv_stream_t stream);
/* eval BatchNorm (+ conv bias) -> per-channel scale/bias (gamma == NULL: bias passthrough) */
int hv_bn_fold(int c, const float* gamma, const float* beta, const float* mean, const float* var,
               const float* conv_bias, float eps, float* scale_out, float* bias_out,
               hv_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Fused mHC token chain (ManifoldHyperConnection.forward, manifold_layers.py:223-280) for
 * the small-D backbone sites: LN_pre, folded GEMM1 + GELU, GEMM2 + GELU, [x|h2] Wc, LN_post
 * in one launch, intermediates on chip.  bf16 only;
 * (D, Hd) in {(32,128), (64,256), (128,512), (256,512)}.
 * Operands are the folded coefficients of hv_mhc_prep + the fold GEMM.
 * ------------------------------------------------------------------------------------ */
typedef struct hv_mhc_fused_args {
  int dtype, D, Hd, T;
  const void* x;        /* [T, D] */
  const void* a1t;      /* [2Hd, D]  = W1 Gc^T */
  const float* c1;      /* [2Hd]     = W1 u + b1 */
  const void* w2;       /* [Hd, 2Hd] */
  const float* b2;      /* [Hd] */
  const void* wct;      /* [D, D+Hd] centred [H_res ; H_post]^T */
  const float* g_post;  /* [D] */
  const float* b_post;  /* [D] */
  const void* residual; /* optional [T, D], added after LN_post (transformer residual stream) */
  void* out;            /* [T, D] */
  int variant;          /* per-call kernel selection, 0 = automatic; HV_MV_* below */
  int pad_;
  /* HV_MV_TOKSPLIT2 / 4 only (read from the first site of a group): fp32 workspace of
     n_sites * ceil(T / 16) * NSPL * 16 * D floats, and n_sites * ceil(T / 16) int arrival
     counters that are zero before the launch (every launch leaves them zero) */
  float* split_work;
  int* split_count;
} hv_mhc_fused_args;
#define HV_MV_SHAPE_MASK  0xff   /* workgroup shape: 1 three 4-wave groups per CU, 2 one 8-wave group,
                                    5 (D = 128) the per-wave 4-wave kernel instead of split-hidden,
                                    6 (D = 64) the per-wave 4-wave kernel instead of split-hidden,
                                    7 (D = 32/64) per-wave kernel with unmerged fragment reads,
                                    8 / 9 (D = 32/64) the software-pipelined per-wave kernel
                                    (9: unmerged fragment reads), 10 (D = 32/64) the per-wave
                                    kernel without pipelining, 12 (D = 128 / 256 split-hidden) the
                                    chunk loop waits for the A1^T half of the next-next chunk only */
#define HV_MV_WIDE        0x100  /* also run (256, 512) fused, per-wave kernel (slower than the GEMM chain; tests) */
#define HV_MV_SPLIT256    0x200  /* (256, 512) on the split-hidden kernel */
#define HV_MV_TOK         0x400  /* token-tile kernel (hv_mhc_tok.hip): 32 (or 16) tokens per workgroup,
                                    weights streamed L2 -> registers; (D, Hd) in {(128, 512), (256, 512),
                                    (256, 1024)} -- small token counts (ViT, B=1) */
#define HV_MV_TOK16       0x800  /* with HV_MV_TOK: 16-token tiles (Hd = 1024 always uses 16) */
#define HV_MV_TOKSPLIT2   0x1000 /* with HV_MV_TOK, D = 256, Hd 512 / 1024: 16-token tiles shared by 2 / 4 workgroups, each */
#define HV_MV_TOKSPLIT4   0x2000 /* owning Hd / NSPL of the h2 units; the last to finish reduces (split_work) */
#define HV_MV_TOKSPLIT_SC1 0x4000 /* ignored since ABI 4 (round 6): the write-through hand-off was
                                     removed; the fenced release / acquire hand-off is the only one */
#define HV_MV_ABLATE_SHIFT 16    /* diagnostics (tools/mhc_ablate*.py; outputs garbage) */
/* 1 when (D, Hd, dtype) has a fused kernel under `variant` */
int hv_mhc_fused_supported(int D, int Hd, int dtype, int variant);
int hv_mhc_fused(const hv_mhc_fused_args* args, hv_stream_t stream);
/* n <= 3 sites with equal (dtype, D, Hd, T, variant) in ONE launch of the token-tile kernel (the
   attention's q / k / v projections, which read the same x: MultiHeadManifoldAttention.forward,
   manifold_layers.py:386-398); variant must include HV_MV_TOK */
int hv_mhc_fused_group(const hv_mhc_fused_args* sites, int n, hv_stream_t stream);

/* y[N] = W[N, K] x[K] + b  (fp32; folded mHC bias c1 = W1 u + b1) */
int hv_gemv(const float* W, const float* x, const float* b, int N, int K, float* y, hv_stream_t stream);

/* elementwise cast fp32 -> (fp32|bf16) */
int hv_cast(const float* x, long n, int y_dtype, void* y, hv_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Grouped per-forward coefficient preparation (every mHC site of a model in 3 launches).
 * Replaces ManifoldHyperConnection.constrained_matrices (manifold_layers.py:205-221) plus
 * the fold of H_pre into the first MLP Linear (:253-256) for all sites at once:
 *   phase 1: column partials of g.s(H_pre_raw), b.s(H_pre_raw); row means of H_res, H_post
 *   phase 2: Gc (fp32 scratch [D,Hd] when folding; Gc^T [Hd,D] in dtype otherwise), u, Wc^T
 *   phase 3 (fold sites): A1^T = W1 Gc^T [2Hd, D] (MFMA, dtype) and c1 = W1 u + b1 (fp32)
 *   phase 4: cs = row sums of a1 as stored (hv_gemm_desc.b_colsum of the first GEMM)
 * Unfolded sites get c1 = u.  blk[] are exclusive per-phase block prefixes filled by the
 * host with hv_mhc_prep_blocks(); totals are the sums.
 * ------------------------------------------------------------------------------------ */
typedef struct hv_mhc_prep_entry {
  const float* h_pre_raw;   /* [D, Hd] */
  const float* h_post_raw;  /* [Hd, D] */
  const float* h_res;       /* [D, D] Sinkhorn output */
  const float* gamma_pre;   /* [D] */
  const float* beta_pre;    /* [D] */
  const float* w1;          /* [2Hd, Hd] mlp[0].weight (fold sites) */
  const float* b1;          /* [2Hd] mlp[0].bias (fold sites) */
  void* a1;                 /* fold: A1^T [2Hd, D]; else Gc^T [Hd, D]  (dtype) */
  float* c1;                /* fold: [2Hd]; else u [Hd] */
  void* wct;                /* [D, D+Hd] (dtype) */
  float* scratch;           /* hv_mhc_prep_scratch_floats(D, Hd) */
  float* cs;                /* [rows of a1] fp32 row sums of a1 as stored (LN-after-GEMM) */
  int D, Hd, fold, pad_;
  int blk[4];
} hv_mhc_prep_entry;

size_t hv_mhc_prep_scratch_floats(int D, int Hd);
/* blocks of each phase for one entry (out4[0..3]) */
void hv_mhc_prep_blocks(int D, int Hd, int fold, int* out4);
int hv_mhc_prep_group(const hv_mhc_prep_entry* dev_table, int count, int dtype,
                      const int* totals4 /* host */, hv_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Grouped weight preparation: fp32 parameters -> GEMM operands in one launch.
 *   kind 0 (cast):  dst[i] = src[i], i < n
 *   kind 1 (conv):  dst[co, (kh*k+kw)*cin + ci] = w[co, ci, kh, kw], zero-padded to ldk
 *                   columns; the per-channel scale/bias of eval BatchNorm (+ conv bias),
 *                   computed exactly as hv_bn_fold (gamma == NULL: s = 1, bias = conv bias
 *                   or 0), go to scale_out / bias_out (when non-NULL) for the GEMM epilogue.
 * Replaces the per-forward weight casts of autocast and the BN folding of the reference's
 * Conv-BN pairs (vision_backbone.py:113, feature_fusion.py:44, yolo_head.py:122).
 * ------------------------------------------------------------------------------------ */
typedef struct hv_wprep_entry {
  const float* src;
  void* dst;
  const float* gamma;
  const float* beta;
  const float* mean;
  const float* var;
  const float* cbias;
  float* scale_out;
  float* bias_out;
  long n;                   /* cast: elements; conv: cout */
  int kind, dtype, cin, k, ldk, blk;
  float eps;
  int pad_;
} hv_wprep_entry;

int hv_wprep_blocks(int kind, long n, int cin, int k);
int hv_wprep_group(const hv_wprep_entry* dev_table, int count, int total_blocks, hv_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Pointwise / layout kernels of the CNN + FPN path (NHWC).
 * ------------------------------------------------------------------------------------ */
/* NCHW fp32 image -> NHWC (fp32|bf16) */
int hv_nchw_to_nhwc(const float* x, int n, int c, int h, int w, int y_dtype, void* y,
                    hv_stream_t stream);
/* Direct 3x3 stem convolution (vision_backbone.py:230: Conv2d(3, C, 3, stride, pad) + folded BN
 * affine + act, the first ConvMHCLayer's conv) from the image: x_nhwc = 0 -> x is the NCHW fp32
 * batch (rounded to `dtype` on load, as hv_nchw_to_nhwc would store it); x_nhwc = 1 -> x is NHWC
 * in `dtype` (the engine's preprocessed input).  y NHWC [n, oh, ow, cout] in `dtype`, weights
 * [cout, ldw] as from hv_conv_weight_prep (K order kh, kw, cin).  cin == 3, k == 3,
 * cout in {32, 64}; HV_EUNSUPPORTED otherwise (callers use hv_gemm's implicit-GEMM conv). */
int hv_conv_stem(int dtype, const void* x, int x_nhwc, int n, int cin, int h, int w, int k, int stride,
                 int pad, const void* wt, int ldw, int cout, const float* scale, const float* bias, int act,
                 void* y, hv_stream_t stream);
/* MaxPool2d(2, 2) (vision_backbone.py:248) */
int hv_maxpool2x2(int dtype, const void* x, int n, int h, int w, int c, void* y,
                  hv_stream_t stream);
/* SE gate then MaxPool2d(2, 2): y = maxpool(x * gate[n, c]) in one pass (the stem's last
 * ConvMHCLayer gate followed by vision_backbone.py:248's pool; gate NULL = plain pool).
 * c % 8 == 0, 16-B aligned x / y / gate.  Bitwise equal to hv_scale_residual + hv_maxpool2x2. */
int hv_scale_maxpool2x2(int dtype, const void* x, const float* gate, int n, int h, int w, int c,
                        void* y, hv_stream_t stream);
/* global average pool over H*W -> fp32 [n, c]  (vision_backbone.py:78; hybrid_vision.py:387) */
size_t hv_channel_mean_work_floats(int n, int hw, int c);
int hv_channel_mean(int dtype, const void* x, int n, int hw, int c, float* out, float* work,
                    hv_stream_t stream);
/* squeeze-excite MLP: s = sigmoid(W2 silu(W1 pooled + b1) + b2)  (vision_backbone.py:77-83) */
int hv_se_mlp(const float* pooled, int n, int c, int cr, const float* w1, const float* b1,
              const float* w2, const float* b2, float* gate, hv_stream_t stream);
/* same with caller scratch hidden[n, cr] fp32: n <= 4 then runs as two batched stages over many
 * workgroups (one wave per output unit, coalesced weight rows) instead of one workgroup per image */
int hv_se_mlp2(const float* pooled, int n, int c, int cr, const float* w1, const float* b1,
               const float* w2, const float* b2, float* hidden, float* gate, hv_stream_t stream);
/* whole SE gate of an NHWC map in one call: hv_channel_mean into `gate`, then hv_se_mlp2 in place
 * (bitwise equal to that pair).  work: hv_channel_mean_work_floats(n, hw, c) floats; hidden as
 * hv_se_mlp2.  (vision_backbone.py:77-83) */
int hv_se_gate(int dtype, const void* x, int n, int hw, int c, int cr, const float* w1, const float* b1,
               const float* w2, const float* b2, float* work, float* hidden, float* gate, hv_stream_t stream);
/* y = x * gate[n, c] (+ identity)  (vision_backbone.py:126-132) */
int hv_scale_residual(int dtype, const void* x, const float* gate, const void* identity,
                      int n, int hw, int c, void* y, hv_stream_t stream);
/* y = a + nearest_upsample(b) with integer factor (feature_fusion.py:116-146) */
int hv_upsample_add(int dtype, const void* a, const void* b, int n, int h, int w, int c,
                    int hb, int wb, void* y, hv_stream_t stream);
/* y = (a + b) * alpha  (hybrid_vision.py:256-258) */
int hv_add_scaled(int dtype, const void* a, const void* b, long count, float alpha, void* y,
                  hv_stream_t stream);
/* y[n, p, c] = x[n, p, c] + v[n, c]  (broadcast per image; vit_encoder_decoder.py:175-183) */
int hv_add_rowvec(int dtype, const void* x, const float* v, int n, int p, int c, void* y,
                  hv_stream_t stream);
/* linear interpolation of a [L, D] table to [Lout, D] (F.interpolate mode='linear') */
int hv_interp_linear(const float* src, int L, int D, int Lout, float* dst, hv_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Transformer pieces (vit_encoder_decoder.py:77-108, manifold_layers.py:404-427)
 * ------------------------------------------------------------------------------------ */
/* y[b, 0] = cls + pos[0]; y[b, 1+i] = x[b, i] + pos[1+i];  then RMSNorm(scale) */
int hv_vit_tokens(int dtype, const void* x, const float* cls, const float* pos, const float* scale,
                  int n, int tokens, int d, void* y, hv_stream_t stream);
/* out = softmax(q k^T * sm_scale) v per (batch, head); q/k/v/out token-major [n, L, heads*hd] */
int hv_attention(int dtype, const void* q, const void* k, const void* v, void* out,
                 int n, int L, int heads, int hd, float sm_scale, hv_stream_t stream);
/* bf16 MFMA attention for hd == 32 (flash-style online softmax, P rounded to bf16 as the
   MFMA operand).  vt_work: hv_attention_work_elems() bf16 elements (V transposed per head,
   keys zero-padded to a multiple of 32). */
size_t hv_attention_work_elems(int n, int L, int heads, int hd);
int hv_attention_mfma(const void* q, const void* k, const void* v, void* vt_work, void* out,
                      int n, int L, int heads, int hd, float sm_scale, hv_stream_t stream);
/* y[b, c] = x[b, 0, c]  (strided row gather) */
int hv_gather_rows(int dtype, const void* x, long stride_rows, int n, int c, void* y,
                   hv_stream_t stream);

/* General MultiHeadManifoldAttention core (manifold_layers.py:404-427): q [n, Lq, heads*hd],
   k / v [n, Lk, heads*hd] (cross-attention allowed), optional key_padding_mask [n, Lk] (1 =
   masked, -inf before the softmax), optional weights [n, heads, Lq, Lk] fp32 (need_weights).
   hd in {16, 32, 64}.  Rows with every key masked are NaN, as in the reference. */
int hv_attention_general(int dtype, const void* q, const void* k, const void* v,
                         const unsigned char* key_padding_mask, void* out, float* weights, int n,
                         int Lq, int Lk, int heads, int hd, float sm_scale, hv_stream_t stream);

/* Batched device-to-device copy of `count` byte ranges in one launch per 24 ranges (the
   engine's owned copies of a graph replay's outputs: InferenceEngine.infer returns fresh
   tensors per call, engine.py:251-317, while a replay rewrites the captured buffers). */
typedef struct hv_copy_segment {
  const void* src;
  void* dst;
  long long bytes;
} hv_copy_segment;
int hv_copy_segments(const hv_copy_segment* segs /* host array */, int count, hv_stream_t stream);
/* n host bytes -> device `dst`, stream-ordered, carried in kernel arguments (1 KiB per launch):
   usable inside a graph capture, where pinning host memory for an async copy is refused; the
   host buffer may be reused as soon as the call returns. */
int hv_write_bytes(void* dst, const void* src, long long n, hv_stream_t stream);

/* ------------------------------------------------------------------------------------
 * YOLO decode (yolo_head.py:196-201 permute + YOLODecoder.forward :220-294, shims S4/S5).
 * logits: NHWC [n, h, w, A*(5+nc)] (fp32|bf16).  Writes fp32 predictions [n, A, h, w, 5+nc],
 * boxes [n, A, h, w, 4] (xyxy, normalised), scores [.., nc], class_scores, objectness,
 * int64 class_indices.
 * ------------------------------------------------------------------------------------ */
int hv_yolo_decode(int dtype, const void* logits, int n, int h, int w, int A, int nc,
                   const float* anchor_wh /* [A, 2] */, float* predictions, float* boxes,
                   float* scores, float* class_scores, int64_t* class_indices,
                   float* objectness,
                   float* detections /* optional [n, A, h, w, 5+nc]: xyxy box, objectness,
                                        sigmoid class probabilities (the per-scale layout
                                        DetectionPostprocessor reads, postprocessing.py:234-244) */,
                   hv_stream_t stream);



/* ------------------------------------------------------------------------------------
 * Detection post-processing: YOLODetectionHead.post_process +
 * non_max_suppression (yolo_head.py:571-731) for a whole batch in two launches.
 * Per (image, scale): class_score > conf_thr, greedy NMS (keep IoU < iou_thr, best first,
 * at most max_det); then per image the same NMS over the concatenated per-scale survivors.
 * No candidate cap: segments with more than 8192 candidates, and cross-scale passes with more
 * than 8192 survivors, sort in the workspace (hv_nms_work_bytes sizes it from max_cells, which
 * must be >= every scale's `cells`).  Outputs [batch, max_det] (+ count[batch]); rows at and past
 * count[b] are written as zeros.  Bit-exact with the reference for any input; max_det >= 1
 * (the reference keeps one box at max_detections = 0; that case is refused here).
 * hv_nms_work_bytes returns 0 for arguments hv_nms refuses.
 * ------------------------------------------------------------------------------------ */
typedef struct hv_nms_scale {
  const float* boxes;          /* [batch, cells, 4] xyxy (decoder output [B, A, H, W, 4]) */
  const float* class_scores;   /* [batch, cells] */
  const int64_t* class_indices;/* [batch, cells] */
  long cells;                  /* A * H * W */
} hv_nms_scale;
size_t hv_nms_work_bytes(int batch, int nscales, int max_det, long max_cells);
int hv_nms(const hv_nms_scale* dev_scales, int nscales, int batch, float conf_thr, float iou_thr,
           int max_det, long max_cells, float* boxes, float* scores, int64_t* labels, int* count,
           void* work, hv_stream_t stream);
/* The sort inside it, on its own: out_idx = torch.sort(vals, descending=True).indices of the CPU
 * reference (libstdc++ introsort over (value, index) pairs, NOT stable on ties), exactly, for
 * vals[n] without NaNs.  depth_limit < 0: std::sort's own 2*floor(log2 n); >= 0 forces it (the
 * heap-sort fallback).  One workgroup; work: hv_sort_desc_exact_work_bytes(n) bytes. */
size_t hv_sort_desc_exact_work_bytes(int n);
int hv_sort_desc_exact(const float* vals, int n, int depth_limit, int* out_idx, void* work, hv_stream_t stream);


/* ------------------------------------------------------------------------------------
 * Image preprocessing (ImagePreprocessor.process, inference/preprocessing.py:
 * 181-276): uint8 HWC frames [n, h, w, 3] (BGR when swap_rb) -> bilinear resize
 * (F.interpolate align_corners=False) -> /255 -> (v - mean) / std, written as NHWC
 * (nhwc = 1, the model's token layout) or NCHW, in fp32 / bf16 / fp16.  One launch per batch.
 * ------------------------------------------------------------------------------------ */
int hv_preprocess(const uint8_t* img, int n, int h, int w, int swap_rb, int out_h, int out_w,
                  const float* mean_std /* host [6] */, int out_dtype, int nhwc, void* out,
                  hv_stream_t stream);
/* The reference's default (torchvision on PIL, preprocessing.py:104-131,268-274; kornia is not
   in requirements.txt) = Pillow Image.resize(BILINEAR), reproduced bit-exactly: antialiased
   triangle filter, 22-bit fixed-point taps, uint8-rounded horizontal then vertical pass; then
   (u / 255 - mean) / std in fp32.  The resample table is built on the HOST
   (hv_pil_resample_tables, hv_pil_table_ints int32 entries) and uploaded by the caller. */
size_t hv_pil_table_ints(int in_h, int in_w, int out_h, int out_w);
int hv_pil_resample_tables(int in_h, int in_w, int out_h, int out_w, int* table_host);
int hv_preprocess_pil(const uint8_t* img, int n, int h, int w, int swap_rb, int out_h, int out_w,
                      const int* table_dev, const float* mean_std /* host [6] */, int out_dtype, int nhwc,
                      void* out, hv_stream_t stream);

/* ====================================================================================
 * Training step: backward kernels, BatchNorm batch statistics,
 * dropout, YOLOLoss, clipping and AdamW.  Same conventions as above (caller-owned
 * buffers, asynchronous, graph-capturable); gradients of parameters are fp32.
 * Dropout masks are never stored: keep(idx) is regenerated from (seed, element index)
 * by the forward and the backward kernels alike (hv_common.h hv_drop_scale).  Every dropout
 * entry point also takes `seed_offset` (device word, may be NULL): the effective seed is
 * seed + *seed_offset, read by the kernel -- a captured training graph advances it per replay.
 * ==================================================================================== */

/* Weight-gradient GEMM C[N1, N2] (+)= sum_p A[p, n1] * B[p, n2]  (both token-major).
   B may be an implicit im2col of an NHWC image (conv_k > 0; columns ordered (kh, kw, ci),
   rows = output pixels), i.e. dW = dY^T im2col(X) of a convolution, or dW = dY^T X of a
   Linear / mHC coefficient matrix.  Split-K partials go to `work`
   (hv_wgrad_work_floats), reduced in a fixed order.  Autograd of the conv/linear/matmul
   calls listed at hv_gemm. */
typedef struct hv_wgrad_desc {
  int dtype;                 /* storage type of A and B */
  int P, N1, N2;
  const void* A; long lda;
  const void* B; long ldb;
  float* C; long ldc;
  int accumulate;            /* 1: C += result */
  int variant;               /* 0 = automatic; HV_WV_* below (A/B selections) */
  float* work;
  int conv_n, conv_h, conv_w, conv_c, conv_k, conv_stride, conv_pad, conv_oh, conv_ow;
  int pad2_;
} hv_wgrad_desc;
#define HV_WV_K64    0x1       /* bf16: 64 pixel rows per LDS stage (bitwise the default result) */
#define HV_WV_CAP64  0x2       /* at most 64 pixel splits (the round-4 plan) */
/* upper bound over every variant's plan */
size_t hv_wgrad_work_floats(int dtype, int P, int N1, int N2);
int hv_wgrad(const hv_wgrad_desc* d, hv_stream_t stream);

/* dgrad operand of a conv weight: w [cout, cin, k, k] fp32 -> y [cin, k, k, cout]
   (flip: taps reversed, for the stride-1 dgrad as a plain convolution) */
int hv_dgrad_weight_prep(const float* w, int cout, int cin, int k, int flip, int y_dtype, void* y,
                         hv_stream_t stream);
/* y[cols, rows] = x[rows, cols]^T  (fp32 -> y_dtype) */
int hv_transpose_cast(const float* x, int rows, int cols, int y_dtype, void* y, hv_stream_t stream);
/* Grouped transposes / casts of parameter-sized matrices in ONE launch (the training step's
   per-forward operand layouts of every mHC site: A1, Wc, W2^T, Gc^T, W1^T, the W2 cast).  Entry:
   x [rows, cols] (x_dtype) -> y [cols, rows] when transpose, else [rows, cols] (y_dtype); blk = the
   entry's first block (exclusive prefix of hv_transpose_blocks over the table). */
typedef struct hv_transpose_entry {
  const void* x;
  void* y;
  int rows, cols, x_dtype, y_dtype, transpose, blk;
} hv_transpose_entry;
int hv_transpose_blocks(int rows, int cols);
int hv_transpose_group(const hv_transpose_entry* tab, int count, int total_blocks, hv_stream_t stream);
/* conv weight gradient [cout, (kh, kw, cin)] -> parameter layout [cout, cin, kh, kw] (fp32) */
int hv_conv_grad_reorder(const float* g, int cout, int cin, int k, float* y, hv_stream_t stream);
/* out[c] (+)= sum_r x[r, c]  (bias gradients); deterministic two-pass */
size_t hv_colsum_work_floats(int rows, int cols);
int hv_colsum(int dtype, const void* x, long ldx, int rows, int cols, float* out, int accumulate,
              float* work, hv_stream_t stream);
/* out[c] (+)= sum_b part[b * cols + c] over b < nblk, fixed order (the second pass of hv_colsum;
   reduces hv_gemm_desc.colsum_part) */
int hv_colsum_final(const float* part, int nblk, int cols, float* out, int accumulate, hv_stream_t stream);

/* BatchNorm2d in training mode over NHWC rows (vision_backbone.py:113, feature_fusion.py:44,
   yolo_head.py:122): batch mean / biased var -> rstd; running stats updated with momentum
   and the unbiased variance (torch semantics). */
size_t hv_bn_work_floats(int rows, int c);
int hv_bn_stats(int dtype, const void* x, int rows, int c, float eps, float momentum,
                float* mean, float* rstd, float* running_mean, float* running_var, float* work,
                hv_stream_t stream);
/* y = act((x - mean) rstd gamma + beta) */
int hv_bn_apply(int dtype, const void* x, int rows, int c, const float* mean, const float* rstd,
                const float* gamma, const float* beta, int act, void* y, hv_stream_t stream);
/* backward of act(BN_train(x)): dx, dgamma, dbeta (work: hv_bn_work_floats) */
int hv_bn_backward(int dtype, const void* x, const void* dy, int rows, int c, const float* mean,
                   const float* rstd, const float* gamma, const float* beta, int act, void* dx,
                   float* dgamma, float* dbeta, float* work, hv_stream_t stream);

/* Row-norm training kernels.  mode 0 = LayerNorm (eps), 1 = RMSNorm (x / sqrt(mean x^2 + eps)).
   forward: y = dropout(norm(x) * gamma + beta) (+ residual); saves mean (LN) and rstd. */
int hv_rownorm_train(int mode, int x_dtype, const void* x, int rows, int cols, float eps,
                     const float* gamma, const float* beta, float drop_p, unsigned int seed,
                     const unsigned int* seed_offset, int y_dtype, void* y, const void* residual, float* mean,
                     float* rstd, hv_stream_t stream);
/* backward: g = dy * keep; dx = norm'(x)^T (g * gamma) (+ dx_add); dgamma/dbeta (may be NULL)
   = column sums of g * xhat / g.  gamma == NULL: no affine (the folded mHC LN_pre). */
size_t hv_rownorm_work_floats(int rows, int cols);
int hv_rownorm_backward(int mode, int x_dtype, const void* x, int dy_dtype, const void* dy, int rows,
                        int cols, const float* mean, const float* rstd, const float* gamma,
                        float drop_p, unsigned int seed, const unsigned int* seed_offset, int dx_dtype, void* dx,
                        const void* dx_add, float* dgamma, float* dbeta, float* work, hv_stream_t stream);
/* Coefficient backward of one mHC site (autograd of constrained_matrices, manifold_layers.py:
   205-221, through the fold of DESIGN.md §2): from dGc [D, Hd] (gradient of the centred gate),
   du [Hd], dWc_x [D, D] and dWc_h [Hd, D] (gradients of the centred output coefficients):
   dH_pre_raw, dgamma_pre, dbeta_pre, dH_res (-> Sinkhorn backward) and dH_post_raw. fp32. */
size_t hv_mhc_param_backward_work_floats(int D, int Hd);
int hv_mhc_param_backward(int D, int Hd, const float* dgc, const float* du, const float* h_pre_raw,
                          const float* gamma_pre, const float* beta_pre, const float* dwc_x,
                          const float* dwc_h, const float* h_post_raw, float* dh_pre_raw, float* dgamma,
                          float* dbeta, float* dh_res, float* dh_post_raw, float* work, hv_stream_t stream);
/* dpre[i] = dy[i] * keep(i) * act'(pre[i])  (elementwise; dy/pre/dpre share dtype) */
int hv_act_backward(int dtype, const void* dy, const void* pre, long n, int act, float drop_p,
                    unsigned int seed, const unsigned int* seed_offset, void* dpre, hv_stream_t stream);
/* y = dropout(x) (elementwise, idx = element index) */
int hv_dropout(int dtype, const void* x, long n, float drop_p, unsigned int seed,
               const unsigned int* seed_offset, void* y, hv_stream_t stream);

/* Sinkhorn backward through every iteration, grouped (autograd of manifold_layers.py:56-73).
   Uses the a_t / b_t scaling vectors the forward left in each entry's `work`; recomputes K
   from raw.  draw = dL/draw for dL/dM = dout.  bwork: hv_sinkhorn_bwd_work_floats. */
typedef struct hv_sinkhorn_bwd_entry {
  hv_sinkhorn_entry fwd;
  const float* dout;   /* [batch, n, m] */
  float* draw;         /* [batch, n, m] */
  float* bwork;
} hv_sinkhorn_bwd_entry;
size_t hv_sinkhorn_bwd_work_floats(int batch, int n, int m);
int hv_sinkhorn_group_backward(const hv_sinkhorn_bwd_entry* dev_table, int count, int total_rows,
                               int total_row_blocks, int total_cols, int max_iters,
                               hv_stream_t stream);

/* squeeze-excite backward (vision_backbone.py:76-85,126-128):
   dgate[n, c] = sum_hw dout * y (b == NULL: sum_hw a) -> chan_dot;
   MLP backward per image -> dpooled, parameter grads; dy = dout * gate + dpooled / hw */
size_t hv_chan_dot_work_floats(int n, int hw, int c);
int hv_chan_dot(int dtype, const void* a, const void* b, int n, int hw, int c, float* out, float* work,
                hv_stream_t stream);
int hv_se_mlp_backward(const float* pooled, const float* dgate, int n, int c, int cr, const float* w1,
                       const float* b1, const float* w2, const float* b2, float* dpooled, float* dw1,
                       float* db1, float* dw2, float* db2, float* work, hv_stream_t stream);
int hv_se_backward_apply(int dtype, const void* dout, const float* gate, const float* dpooled, int n,
                         int hw, int c, void* dy, hv_stream_t stream);
/* MaxPool2d(2,2) backward (first maximum in scan order receives the gradient) */
int hv_maxpool2x2_backward(int dtype, const void* x, const void* dy, int n, int h, int w, int c,
                           void* dx, hv_stream_t stream);
/* nearest-upsample backward: db[n, hb, wb, c] = sum of dy over each (h/hb x w/wb) block */
int hv_upsample_backward(int dtype, const void* dy, int n, int h, int w, int c, int hb, int wb,
                         void* db, hv_stream_t stream);
/* z[b, 0] = cls + pos[0]; z[b, 1+i] = x[b, i] + pos[1+i]  (no norm; training form) */
int hv_vit_assemble(int dtype, const void* x, const float* cls, const float* pos, int n, int tokens,
                    int d, void* z, hv_stream_t stream);
/* its backward: dx = dz[:, 1:], dcls = sum_b dz[b, 0], dpos = sum_b dz[b] (fp32) */
int hv_vit_assemble_backward(int dtype, const void* dz, int n, int tokens, int d, void* dx, float* dcls,
                             float* dpos, hv_stream_t stream);
/* dx[b * stride_rows + r] = (r == 0) ? dy[b] : 0 */
int hv_scatter_rows(int dtype, const void* dy, long stride_rows, int n, int c, void* dx,
                    hv_stream_t stream);

/* attention with dropout on the probabilities (manifold_layers.py:404-427, train mode):
   forward writes o and lse [n, heads, L] (log-sum-exp of the scaled scores);
   backward recomputes P from lse:  dq, dk, dv. */
int hv_attention_train(int dtype, const void* q, const void* k, const void* v, void* o, float* lse,
                       int n, int L, int heads, int hd, float sm_scale, float drop_p, unsigned int seed,
                       const unsigned int* seed_offset, hv_stream_t stream);
/* work: n * heads * L floats (row dots dout . o) */
int hv_attention_backward(int dtype, const void* q, const void* k, const void* v, const void* o,
                          const void* dout, const float* lse, int n, int L, int heads, int hd,
                          float sm_scale, float drop_p, unsigned int seed, const unsigned int* seed_offset,
                          void* dq, void* dk, void* dv, float* work, hv_stream_t stream);
/* The same two operations on the matrix cores (bf16, head_dim 32): identical dropout keep(i, j)
   and lse convention, so the forward and backward of either path pair.  vt_work /  work hold
   transposed zero-padded [n*heads, 32, Lp] operand copies (hv_attention_train_mfma_work_elems
   bf16 elements each; the backward needs 3 of them followed by n*heads*L floats). */
size_t hv_attention_train_mfma_work_elems(int n, int L, int heads);
int hv_attention_train_mfma(const void* q, const void* k, const void* v, void* o, float* lse, int n, int L,
                            int heads, float sm_scale, float drop_p, unsigned int seed,
                            const unsigned int* seed_offset, void* vt_work, hv_stream_t stream);
int hv_attention_backward_mfma(const void* q, const void* k, const void* v, const void* o, const void* dout,
                               const float* lse, int n, int L, int heads, float sm_scale, float drop_p,
                               unsigned int seed, const unsigned int* seed_offset, void* dq, void* dk, void* dv,
                               void* work, hv_stream_t stream);

/* YOLOLoss for one scale (yolo_head.py:374-465): logits NHWC [n, h, w, A*P], targets
   [n, A, h, w, P] fp32.  Writes sums[0..3] = raw coord / obj / noobj / cls sums, sums[4] =
   this scale's contribution to total_loss, sums[5] = #objects, and dlogits (NHWC, d_dtype) =
   d total_loss / d logits (all zero when the scale has no object, like the reference's
   `continue`).  work: hv_yolo_loss_work_floats. */
size_t hv_yolo_loss_work_floats(int n, int h, int w, int A);
int hv_yolo_loss(int dtype, const void* logits, const float* targets, int n, int h, int w, int A, int P,
                 float l_coord, float l_obj, float l_noobj, float l_cls, float* sums, int d_dtype,
                 void* dlogits, float* work, hv_stream_t stream);

/* Gradient clipping + AdamW over a device table of parameters (mhc_trainer.py:342-383 and
   optimizer.py:131-191, i.e. torch.nn.utils.clip_grad_norm_ per group then AdamW). */
typedef struct hv_param_entry {
  float* param; float* grad; float* exp_avg; float* exp_avg_sq;
  long n;
  int group;          /* clipping group 0..3 */
  int blk;            /* first block of this entry (prefix over entries) */
} hv_param_entry;
int hv_param_blocks(long n);
/* norms[g] = ||grads of group g||_2 ; coefs[g] = min(1, max_norm[g] / (norms[g] + 1e-6));
   work: 2 * total_blocks floats.  active (device [count], may be NULL): entries with active[i] == 0
   received no gradient this step (torch.optim's grad-is-None) and are skipped -- a data-parallel
   step decides this on the device (flags all-reduced over ranks), with no host round trip. */
int hv_grad_norms(const hv_param_entry* dev_table, int count, int total_blocks, int groups,
                  const float* max_norm /* host [groups] */, float* norms, float* coefs, float* work,
                  const int* active, hv_stream_t stream);
/* AdamW step with the clip coefficient of each parameter's group (coefs may be NULL).  Bias
   correction 1 - beta^t uses each parameter's own step count steps[i] (device [count], the
   torch.optim.AdamW per-parameter state['step']; a parameter that skipped steps keeps its own
   count) or, with steps == NULL, `step` for every parameter. */
int hv_adamw(const hv_param_entry* dev_table, int count, int total_blocks, const float* coefs,
             float lr, float beta1, float beta2, float eps, float weight_decay, int step,
             const int* steps, const int* active /* as hv_grad_norms */, hv_stream_t stream);
/* the same step with the hyper-parameters read from DEVICE memory, hyper = {lr, beta1, beta2,
   eps, weight_decay} (fp32): a captured graph replays with whatever the host last wrote there,
   so a learning-rate scheduler does not force a re-capture.  Per-parameter `steps` required. */
int hv_adamw_dev(const hv_param_entry* dev_table, int count, int total_blocks, const float* coefs,
                 const float* hyper, const int* steps, const int* active, hv_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Stability monitor (ManifoldHyperConnection._monitor_stability, reference
 * src/models/manifold_layers.py:282-316), device-side and grouped over all mHC sites.
 * hv_symeig_group: eig = ascending eigenvalues of (h + h^T)/2 for every entry (the
 * torch.linalg.eigvalsh call, :288-290): fp64 Householder tridiagonalisation + Sturm
 * bisection.  Entries sorted by n descending (host_n[] = their n, same order, n <= 2048);
 * row_start = exclusive prefix of n over the table.  2*(max n - 2) + 3 launches, no host sync.
 * ------------------------------------------------------------------------------------ */
typedef struct hv_symeig_entry {
  const float* h;      /* [n, n] fp32 row-major */
  float* eig;          /* [n] */
  double* work;        /* hv_symeig_work_doubles(n) */
  int n;
  int row_start;
} hv_symeig_entry;
size_t hv_symeig_work_doubles(int n);
int hv_symeig_group(const hv_symeig_entry* dev_table, const int* host_n, int count, hv_stream_t stream);
/* signal ratio mean_r|x_out[r]| / (mean_r|x_in[r]| + 1e-8) (:296-298) and the row/column-sum
   errors |sum(h)/n - 1| (:306-315) -> out3[3]; history[slot] = ratio when history != NULL
   (:300-303).  x_in/x_out: [rows, D] of `dtype`; h: [n, n] fp32; work: hv_stability_work_floats. */
size_t hv_stability_work_floats(int rows);
int hv_stability_stats(int dtype, const void* x_in, const void* x_out, int rows, int D, const float* h, int n,
                       float* work, float* history, int slot, float* out3, hv_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* HV_KERNELS_H */
