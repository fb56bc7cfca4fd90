// Build provenance of libhvs.so: HV_SRC_HASH is computed by the Makefile over the exact source
// set this library is compiled from (hv_amd/_lib.py recomputes it at load time and refuses a
// library whose sources changed since it was built).
#include "hv_common.h"

#ifndef HV_SRC_HASH
#define HV_SRC_HASH "unknown"
#endif

extern "C" const char* hv_build_id(void) { return HV_SRC_HASH; }
