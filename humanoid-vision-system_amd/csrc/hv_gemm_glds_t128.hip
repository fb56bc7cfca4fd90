// LDS-DMA ring GEMM instantiations (hv_gemm_glds.h): train 128x64, train 128x128.
#include "hv_gemm_glds.h"

int hv_glds_train_128x64(const hv_gemm_desc& d, hipStream_t s) { return launch_train<128, 64>(d, s); }
int hv_glds_train_128x128(const hv_gemm_desc& d, hipStream_t s) { return launch_train<128, 128>(d, s); }
