// LDS-DMA ring GEMM instantiations (hv_gemm_glds.h): train 64x64, train 64x128.
#include "hv_gemm_glds.h"

int hv_glds_train_64x64(const hv_gemm_desc& d, hipStream_t s) { return launch_train<64, 64>(d, s); }
int hv_glds_train_64x128(const hv_gemm_desc& d, hipStream_t s) { return launch_train<64, 128>(d, s); }
