/* HybridVision MI355X kernels -- diagnostics interface (NOT the drop-in ABI).
 *
 * Kernel-variant selection is per call (hv_gemm_desc.variant, hv_mhc_fused_args.variant in
 * hv_kernels.h); there are no process-global tuning switches.
 *
 * The launch counters count host-side launches per kernel family (every launch through the C
 * ABI, graph capture included), so a test can prove which kernels a model forward ran.
 */
#ifndef HV_TUNING_H
#define HV_TUNING_H

#ifdef __cplusplus
extern "C" {
#endif

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
