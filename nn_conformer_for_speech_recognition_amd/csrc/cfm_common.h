// Common device/host helpers for the Conformer-on-MI355X (gfx950, CDNA4) kernels.
//
// Everything here is written for gfx950 only: 64-lane wavefronts, MFMA 32x32x16 bf16 /
// 32x32x2 f32, ds_read_b64_tr_b16 transposed LDS reads.  No CUDA shims, no dual paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/cfm.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CFM_LDS(p) ((__attribute__((address_space(3))) void*)(p))

// ----------------------------------------------------------------------------- errors (host)
namespace cfm {
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);
// out[n] (+)= sum_p part[p*ldp + n]  (deterministic, block = 16 waves x 64 columns; ldp 0 -> N)
void colreduce(const float* part, int nparts, long N, float* out, int accumulate, hipStream_t s, long ldp = 0);
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace cfm

#define CFM_EXPORT extern "C" __attribute__((visibility("default")))

#define CFM_REQUIRE(cond, code, msg)                                  \
  do {                                                                \
    if (!(cond)) return cfm::fail((code), std::string(__func__) + ": " + (msg)); \
  } while (0)

// ----------------------------------------------------------------------------- conversions
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// load a float from a pointer whose element type is given at run time (wave-uniform)
__device__ __forceinline__ float ld_dyn(const void* p, int dtype, long idx) {
  return dtype == CFM_BF16 ? (float)((const bf16*)p)[idx] : ((const float*)p)[idx];
}
__device__ __forceinline__ void st_dyn(void* p, int dtype, long idx, float v) {
  if (dtype == CFM_BF16) ((bf16*)p)[idx] = (bf16)v;
  else ((float*)p)[idx] = v;
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float silu_grad_f(float x) {
  float s = 1.f / (1.f + __expf(-x));
  return s * (1.f + x * (1.f - s));
}
__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + __expf(-x)); }

// ----------------------------------------------------------------------------- dropout RNG
// Counter-based: keep(seed, idx) is a pure function, so backward regenerates the mask.
__device__ __forceinline__ uint32_t cfm_hash(uint64_t seed, uint64_t idx) {
  uint64_t z = idx * 0x9E3779B97F4A7C15ull + seed;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}
// returns scale (1/(1-p)) if kept, 0 if dropped
__device__ __forceinline__ float dropout_scale(float p, uint64_t seed, uint64_t idx) {
  if (p <= 0.f) return 1.f;
  float u = (float)(cfm_hash(seed, idx) >> 8) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

// ----------------------------------------------------------------------------- reductions
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

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
