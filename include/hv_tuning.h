/* HybridVision MI355X kernels -- tuning and diagnostics interface (NOT the drop-in ABI).
 *
 * Process-global knobs used by the A/B tools (the tools/ scripts) and by tests that pin every kernel
 * variant against the default one.  The product path (the hv_amd package) never calls them; they are
 * relaxed atomics, so flipping one while another thread launches is race-free but changes
 * which kernel that thread's next launch picks -- use only in single-threaded benchmarks.
 *
 * The launch counters count host-side launches per kernel family (every launch through the C
 * ABI, graph capture included), so a test can prove which kernels a model forward ran.
 */
#ifndef HV_TUNING_H
#define HV_TUNING_H

#ifdef __cplusplus
extern "C" {
#endif

/* GEMM path selection: 1 = register-staged kernel only, 0 = default (LDS-DMA when eligible) */
void hv_gemm_set_path(int regstage_only);
/* 256x256 ping-pong LDS-DMA kernel selection: 0 off, 1 by shape (default), 2 whenever eligible */
void hv_gemm_set_big_tile(int mode);
/* 64x64-tile LDS-DMA kernel for small grids: 1 on (default), 0 off */
void hv_gemm_set_small_tile(int mode);
/* 128x128 tiles for the training epilogues (epi_mode 1/2): 0 = 64x128 only (default), 1 on */
void hv_gemm_set_train128(int on);
/* LDS-staged coalesced epilogue for the LDS-DMA kernels (inference modes): 1 on (default), 0 off */
void hv_gemm_set_staged_epilogue(int on);
/* LDS-staged epilogue for the training modes (epi_mode 1/2) of the LDS-DMA kernels: 1 on (default), 0 off */
void hv_gemm_set_staged_train(int on);
/* deeper LDS-DMA rings (4 / 3 buffers) for the 64x64 / 64x128 / 128x64 tiles: 1 on (default), 0 = 2 */
void hv_gemm_set_deep_ring(int on);
/* force the LDS-DMA tile: 0 auto (default), 1 128x128, 2 64x128, 3 128x64, 4 64x64, 5 256x256 ping-pong */
void hv_gemm_set_force_tile(int code);
/* convolutions with K % 64 != 0 (channels % 8 == 0) on the LDS-DMA kernel: 0 off (default), 1 on */
void hv_gemm_set_conv_ktail(int on);
/* persistent small-K (K <= 512) GEMM kernel: 1 on (default), 0 off */
void hv_gemm_set_smallk(int on);
/* fused mHC: 1 also dispatches (256, 512) to the fused kernel (off by default: slower) */
void hv_mhc_fused_enable_wide(int on);
/* fused mHC workgroup shape: 0 default (4-wave groups), 1 three groups per CU, 2 one 8-wave group */
void hv_mhc_fused_set_variant(int v);

/* kernel families counted by hv_diag_launch_counts */
enum hv_kernel_family {
  HV_KF_GEMM_PP256 = 0,      /* gemm_pp256_kernel (256x256 ping-pong LDS-DMA) */
  HV_KF_GEMM_GLDS_128x128 = 1,
  HV_KF_GEMM_GLDS_64x128 = 2,
  HV_KF_GEMM_GLDS_128x64 = 3,
  HV_KF_GEMM_GLDS_64x64 = 4,
  HV_KF_GEMM_REGSTAGE = 5,   /* gemm_kernel (register-staged; fp32 parity mode and fallbacks) */
  HV_KF_MHC_FUSED = 6,       /* mhc_fused_kernel */
  HV_KF_ATTN_MFMA = 7,       /* k_attention_mfma */
  HV_KF_ATTN_SCALAR = 8,     /* k_attention (fp32 / other head dims) */
  HV_KF_SINKHORN_GROUP = 9,  /* one grouped Sinkhorn forward (all its passes) */
  HV_KF_ATTN_GENERAL = 10,   /* hv_attention_general (cross / masked / weights / CLS-row queries) */
  HV_KF_GEMM_SMALLK = 11,    /* gemm_sk_kernel (persistent small-K, register epilogue) */
  HV_KF_GEMM_SPLITK = 12,    /* split-K LDS-DMA GEMM (64x64 tiles) + its reduce launch */
  HV_KF_COUNT = 16
};
/* copies the HV_KF_COUNT launch counters into out[] */
void hv_diag_launch_counts(long long* out);
void hv_diag_reset_counts(void);

#ifdef __cplusplus
}
#endif
#endif
