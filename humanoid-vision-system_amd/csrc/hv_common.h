// Shared device helpers for the HybridVision gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/hv_kernels.h"
#include "../../include/hv_tuning.h"

// host-side launch counter (hv_diag.hip); relaxed atomic increment
void hv_diag_count(int family);

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

#define HV_WAVE 64

__device__ __forceinline__ float bf2f(unsigned short v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// Round-to-nearest-even through the hardware convert (v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ unsigned short f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}

// Storage-type adaptors: activations are either fp32 or bf16 (raw ushort bits).
template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float load(const float* p, size_t i) { return p[i]; }
  static __device__ __forceinline__ void store(float* p, size_t i, float v) { p[i] = v; }
};
template <> struct Elem<unsigned short> {
  static __device__ __forceinline__ float load(const unsigned short* p, size_t i) { return bf2f(p[i]); }
  static __device__ __forceinline__ void store(unsigned short* p, size_t i, float v) { p[i] = f2bf(v); }
};

__device__ __forceinline__ float hv_gelu(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
// GELU for bf16 outputs: x * sigmoid(x * p(x^2)) with p fitted (minimax over all x, x^2
// clamped at 64) to |err| <= 2.6e-5 against the exact erf GELU -- far below bf16 resolution --
// in 9 VALU instructions (2 transcendental) instead of ~15 for an erf evaluation.
__device__ __forceinline__ float hv_gelu_fast(float x) {
  const float x2 = fminf(x * x, 64.f);
  const float p = fmaf(fmaf(1.0142630839702301e-3f, x2, -0.10677572552514955f), x2, -2.3011213415186913f);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * p));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// two floats -> two RNE bf16 in one dword (v_cvt_pk_bf16_f32), low half = a
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

__device__ __forceinline__ float hv_sigmoid(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float hv_silu(float x) { return x / (1.0f + __expf(-x)); }

__device__ __forceinline__ float hv_act(float v, int act) {
  switch (act) {
    case HV_ACT_RELU: return v > 0.f ? v : 0.f;
    case HV_ACT_SILU: return hv_silu(v);
    case HV_ACT_GELU: return hv_gelu(v);
    case HV_ACT_LEAKY: return v > 0.f ? v : 0.1f * v;
    case HV_ACT_SIGMOID: return hv_sigmoid(v);
    default: return v;
  }
}

// Derivative of hv_act at the pre-activation z (training backward).
__device__ __forceinline__ float hv_act_grad(float z, int act) {
  switch (act) {
    case HV_ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case HV_ACT_SILU: { const float s = hv_sigmoid(z); return s * (1.f + z * (1.f - s)); }
    case HV_ACT_GELU:
      return 0.5f * (1.0f + erff(z * 0.70710678118654752f)) + z * 0.3989422804014327f * __expf(-0.5f * z * z);
    case HV_ACT_LEAKY: return z > 0.f ? 1.f : 0.1f;
    case HV_ACT_SIGMOID: { const float s = hv_sigmoid(z); return s * (1.f - s); }
    default: return 1.f;
  }
}

// Derivative of hv_gelu_fast, the GELU a bf16 training forward applies (its backward then
// differentiates the function it ran): with s = 1 / (1 + 2^(x p(x^2))),
// d/dx [x s] = s - x s (1 - s) ln2 (p + 2 x^2 p'(x^2))  (p' = 0 where x^2 is clamped)
__device__ __forceinline__ float hv_gelu_grad_fast(float x) {
  const float x2r = x * x;
  const float x2 = fminf(x2r, 64.f);
  const float p = fmaf(fmaf(1.0142630839702301e-3f, x2, -0.10677572552514955f), x2, -2.3011213415186913f);
  const float dp = x2r < 64.f ? fmaf(2.0285261679404602e-3f, x2, -0.10677572552514955f) : 0.f;
  const float sg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * p));
  return sg - x * sg * (1.f - sg) * 0.6931471805599453f * fmaf(2.f * x2, dp, p);
}

// Dropout keep mask shared by every training kernel: element idx of a tensor dropped with
// probability p under `seed` (counter-based, so the backward regenerates it instead of storing).
__device__ __forceinline__ uint32_t hv_hash32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ float hv_drop_scale(uint32_t seed, unsigned long long idx, float p) {
  if (p <= 0.f) return 1.f;
  uint32_t h = hv_hash32((uint32_t)idx * 0x9E3779B1u + seed);
  h = hv_hash32(h ^ ((uint32_t)(idx >> 32) * 0x85EBCA77u) ^ (seed * 0x27d4eb2fu));
  const float u = (float)(h >> 8) * (1.0f / 16777216.0f);
  return u >= p ? 1.0f / (1.0f - p) : 0.f;
}

// effective dropout seed of a call: its seed argument plus the optional device offset word
// (hv_kernels.h seed_offset; a captured training graph advances it on every replay)
__device__ __forceinline__ uint32_t hv_seed(uint32_t seed, const unsigned int* off) { return off ? seed + *off : seed; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `scratch` needs 16 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

// Device-side bounds checks of the debug build (`make debug` -> libhvs_debug.so, -DHV_DEBUG):
// a violation prints its file:line and condition; no trap (a trapping wave faults the device
// for every process on it).  Release builds compile them out.
#ifdef HV_DEBUG
#define HV_DCHECK(cond) \
  do { if (!(cond)) printf("HV_DCHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); } while (0)
#else
#define HV_DCHECK(cond) do {} while (0)
#endif

#define HV_CHECK_LAUNCH() \
  do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return (int)e_; } while (0)

// Instantiate KERNEL_CALL with T = storage type of dtype code dt (returns HV_EINVAL otherwise).
#define HV_DISPATCH(dt, KERNEL_CALL)                                     \
  do {                                                                   \
    if ((dt) == HV_BF16) { using T = unsigned short; KERNEL_CALL; }      \
    else if ((dt) == HV_F32) { using T = float; KERNEL_CALL; }           \
    else return HV_EINVAL;                                               \
  } while (0)

static inline unsigned hv_cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }
