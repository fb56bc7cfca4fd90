// LDS-DMA ring GEMM instantiation (hv_gemm_glds.h): infer 32x64 -- the small-M, long-K GEMMs of
// the B=1 frame (M ~ 400 tokens / pixels, K >= 1,024), where 64x64 tiles leave one workgroup per CU.
#include "hv_gemm_glds.h"

int hv_glds_infer_32x64(const hv_gemm_desc& d, hipStream_t s) { return launch_infer<32, 64>(d, s); }
