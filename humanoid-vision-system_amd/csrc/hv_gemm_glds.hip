// Kernel selection of the LDS-DMA GEMM family (hv_gemm_glds.h); the instantiations live in
// hv_gemm_glds_{i64,i128,t64,t128,pp}.hip.
#include "hv_gemm_glds.h"

namespace {
template <int BM, int BN>
int launch(const hv_gemm_desc& d, hipStream_t s) {
  if (d.epi_mode) {
    if constexpr (BM == 64 && BN == 64) return hv_glds_train_64x64(d, s);
    else if constexpr (BM == 64) return hv_glds_train_64x128(d, s);
    else if constexpr (BN == 64) return hv_glds_train_128x64(d, s);
    else return hv_glds_train_128x128(d, s);
  }
  if constexpr (BM == 64 && BN == 64) return hv_glds_infer_64x64(d, s);
  else if constexpr (BM == 64) return hv_glds_infer_64x128(d, s);
  else if constexpr (BN == 64) return hv_glds_infer_128x64(d, s);
  else return hv_glds_infer_128x128(d, s);
}
}  // namespace

int hv_gemm_smallk(const hv_gemm_desc& d, hipStream_t s, bool force);   // hv_gemm_sk.hip
// Per-call variants (hv_gemm_desc.variant, HV_GV_*): measured-off choices stay selectable for the
// A/B tools -- 128x128 training tiles (199 vs 182 ms/step), the LDS-DMA kernel for convs with
// K % 64 != 0 (in-model 23.73 vs 23.59 ms).

// Returns HV_EUNSUPPORTED when the shape/mode is not covered (caller falls back).
int hv_gemm_glds(const hv_gemm_desc& d, hipStream_t s) {
  // K % 64 != 0 only for convolutions (channels a multiple of 8): the last K-tile's tail reads the
  // zero line for both operands (e.g. 3x3 convs with 32 input channels, K = 288)
  if (d.dtype != HV_BF16 || d.conv_transposed) return HV_EUNSUPPORTED;
  // dense K % 8 == 0 tails as well (e.g. the stem-stage mHC GEMMs, K = 32, M = 1.6 M rows: ~1 ms
  // each on the register-staged kernel); not with an LN prologue (the zero tail would normalise to
  // non-zero) or a second A operand
  const bool dense_tail = d.conv_k == 0 && !d.A2 && !d.a_mean && d.K % 8 == 0 &&
                          !(d.variant & HV_GV_NO_DENSE_KTAIL);
  if (d.K % 64 && !((d.variant & HV_GV_CONV_KTAIL) && d.conv_k > 0 && d.K % 8 == 0) && !dense_tail)
    return HV_EUNSUPPORTED;
  if (d.a_mean && (!d.b_colsum || d.A2 || d.conv_k > 0)) return HV_EUNSUPPORTED;
  if (d.conv_k > 0 ? (d.conv_c % 8) : (d.lda % 8)) return HV_EUNSUPPORTED;
  if (d.A2 && (d.k1 % 64 || d.lda2 % 8)) return HV_EUNSUPPORTED;
  if (d.ldb % 8) return HV_EUNSUPPORTED;
  if (d.splitk > 1) {
    // caller-requested split-K (small output grids, long K): inference epilogues only
    if (d.K % 64) return HV_EUNSUPPORTED;
    if (d.epi_mode || !d.splitk_work || !d.splitk_count || d.splitk > 64 ||
        (long)hv_cdiv(d.M, 64) * hv_cdiv(d.N, 64) > HV_SPLITK_MAX_TILES)
      return HV_EINVAL;
    return hv_glds_launch_splitk(d, s);
  }
  const long t128 = (long)hv_cdiv(d.M, 128) * hv_cdiv(d.N, 128);
  const long t256 = (long)hv_cdiv(d.M, 256) * hv_cdiv(d.N, 256);
  switch (d.variant & HV_GV_TILE_MASK) {
    case 1: return launch<128, 128>(d, s);
    case 2: return launch<64, 128>(d, s);
    case 3: return launch<128, 64>(d, s);
    case 4: return launch<64, 64>(d, s);
    case 5: if (d.K % 64 == 0 && d.conv_c % 64 == 0) return hv_glds_launch256(d, s); break;
    case 6: return hv_gemm_smallk(d, s, true);
    default: {
      const int rc = hv_gemm_smallk(d, s, false);             // persistent small-K kernel (hv_gemm_sk.hip)
      if (rc != HV_EUNSUPPORTED) return rc;
      break;
    }
  }
  // 256x256 ping-pong kernel: long contractions with wide outputs on grids that still fill most
  // CUs.  Measured in the model (tools/gemm_breakdown.py, cold operands): wins for N >= 1024
  // (25600x1024x2048, 6400x2048x4096: -5..11 %); loses to the 128x128 ring for N <= 512 and for
  // the implicit-im2col convolutions (+3..29 %); K = 256 loses everywhere (prologue-bound)
  if ((!d.epi_mode || (d.variant & HV_GV_TRAIN_BIG)) && d.K % 64 == 0 && d.conv_c % 64 == 0 &&
      !(d.variant & HV_GV_NO_BIG) &&
      ((d.variant & HV_GV_BIG_ALWAYS) || (d.conv_k == 0 && d.K >= 1024 && d.N >= 1024 && t256 >= 160)))
    return hv_glds_launch256(d, s);
  if (d.N <= 64) return launch<128, 64>(d, s);
  // small grids (the ViT / head mHC GEMMs: M = 16 x 401 tokens): 64x64 tiles fill the 256 CUs
  const long t64x128 = (long)hv_cdiv(d.M, 64) * hv_cdiv(d.N, 128);
  if (!(d.variant & HV_GV_NO_SMALL) && t64x128 < 320) {
    // long K on a grid of < 256 64x64 tiles (B=1: M ~ 400): 32-row tiles give each CU two or
    // more workgroups whose barrier / LDS-read / MFMA chains overlap (a lone workgroup's chain
    // sets the per-K-tile time, profiles/r04/deep8_rejected.txt).  HV_GLDS32=0 turns it off.
    static const bool t32 = [] {
      const char* e = getenv("HV_GLDS32");
      return !(e && e[0] == '0');
    }();
    // K >= 256 for M > 64 (the ViT's 401-token MLP GEMMs gain too), K >= 1,024 for the
    // 1-16-row final-fusion GEMMs; HV_GLDS32_K forces one threshold for every M (A/B)
    static const int t32k = [] {
      const char* e = getenv("HV_GLDS32_K");
      return e ? atoi(e) : 0;
    }();
    static const int t32t = [] {
      const char* e = getenv("HV_GLDS32_TILES");
      return e ? atoi(e) : 256;
    }();
    const int kmin = t32k > 0 ? t32k : (d.M > 64 ? 256 : 1024);
    const long t64 = (long)hv_cdiv(d.M, 64) * hv_cdiv(d.N, 64);
    if (t32 && !d.epi_mode && d.K >= kmin && t64 < t32t) return hv_glds_infer_32x64(d, s);
    return launch<64, 64>(d, s);
  }
  if (d.M <= 64 || t128 < 256 || (d.epi_mode && !(d.variant & HV_GV_TRAIN128))) return launch<64, 128>(d, s);
  return launch<128, 128>(d, s);
}
