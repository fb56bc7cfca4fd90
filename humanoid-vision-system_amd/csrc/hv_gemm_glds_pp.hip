// 256x256 ping-pong kernel and the split-K 64x64 kernel (instantiations of hv_gemm_glds.h).
#include "hv_gemm_glds.h"

int hv_glds_launch_splitk(const hv_gemm_desc& d, hipStream_t s) {
  const unsigned tiles = hv_cdiv(d.M, 64) * hv_cdiv(d.N, 64);
  hv_diag_count(HV_KF_GEMM_SPLITK);
  const dim3 grid(tiles, d.splitk);
  if (d.conv_k > 0) gemm_glds_kernel<64, 64, true, false, false, 4, true><<<grid, 256, 0, s>>>(d);
  else gemm_glds_kernel<64, 64, false, false, false, 4, true><<<grid, 256, 0, s>>>(d);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

// LDS-staged epilogues (inference: +25-35 % at K <= 512; training modes too) unless the call
// asks for the fragment-layout one (HV_GV_FLAT_EPI / HV_GV_FLAT_TRAIN)

int hv_glds_launch256(const hv_gemm_desc& d, hipStream_t s) {
  const unsigned grid = hv_cdiv(d.M, 256) * hv_cdiv(d.N, 256);
  hv_diag_count(HV_KF_GEMM_PP256);
  // fragment-layout epilogue here: the staged one measured 1.3x slower on this kernel (K >= 1024,
  // where the output stream is a small part of the work)
  if (d.epi_mode) {
    // training epilogues (store the pre-activation / apply the activation backward) on the
    // fragment-layout epilogue
    if (d.conv_k > 0) gemm_pp256_kernel<true, false, true><<<grid, 512, 0, s>>>(d);
    else gemm_pp256_kernel<false, false, true><<<grid, 512, 0, s>>>(d);
  } else if (d.conv_k > 0) {
    gemm_pp256_kernel<true, false><<<grid, 512, 0, s>>>(d);
  } else {
    gemm_pp256_kernel<false, false><<<grid, 512, 0, s>>>(d);
  }
  HV_CHECK_LAUNCH();
  return HV_OK;
}
