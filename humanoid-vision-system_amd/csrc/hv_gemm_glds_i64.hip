// LDS-DMA ring GEMM instantiations (hv_gemm_glds.h): infer 64x64, infer 64x128.
#include "hv_gemm_glds.h"

int hv_glds_infer_64x64(const hv_gemm_desc& d, hipStream_t s) { return launch_infer<64, 64>(d, s); }
int hv_glds_infer_64x128(const hv_gemm_desc& d, hipStream_t s) { return launch_infer<64, 128>(d, s); }
