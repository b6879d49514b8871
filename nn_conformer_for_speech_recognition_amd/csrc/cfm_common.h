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
// the same sums written as bf16 (rounded as cfm_cast; may use part's first row as scratch)
void colreduce_bf16(float* part, int nparts, long N, bf16* out, hipStream_t s, long ldp = 0);
// out{A,B}[n] = sum_p part{A,B}[p * ldp + n]: two reductions, one launch (bit-identical to two colreduce calls;
// ldp 0 -> N)
void colreduce_pair(const float* partA, const float* partB, int nparts, long N, float* outA, float* outB,
                    hipStream_t s, long ldp = 0);
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
// device step counter bound by cfm_rng_bind (nullptr: seeds are used as passed); read by every
// dropout kernel at run time so one captured HIP graph replays with fresh masks each step
extern const uint64_t* g_rng_salt;
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

// sigmoid via the hardware reciprocal (v_rcp_f32, 1 ulp) instead of an IEEE division (~10 VALU ops):
// these run per element in GEMM epilogues.  exp(-x) = inf gives rcp = 0 (silu(-inf side) = -0).
// workgroup barrier for LDS hand-offs only: this wave's LDS operations complete, then s_barrier.  __syncthreads()
// is also a workgroup release fence, which makes every wave wait for ALL its outstanding vector-memory operations
// (s_waitcnt vmcnt(0)) -- global stores included, whose acknowledgements a loop that streams results out (the
// rel-pos dK/dV kernel's dS rows, the CTC recursion's alpha / beta rows) then pays once per tile or frame, and
// loads issued ahead as a prefetch, which it turns into a stall.  Only for barriers whose consumers read LDS, never for
// global data written before the barrier and read after it by another wave.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float sigmoid_f(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float silu_f(float x) { return x * sigmoid_f(x); }
__device__ __forceinline__ float silu_grad_f(float x) {
  const float s = sigmoid_f(x);
  return s * (1.f + x * (1.f - s));
}

// 8 consecutive elements (16-B aligned) of a bf16 or f32 array, as f32
__device__ __forceinline__ void ld8_dyn(const void* p, int dt, long idx, float (&o)[8]) {
  if (dt == CFM_BF16) {
    const uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p) + idx);
    const bf16x8 b = __builtin_bit_cast(bf16x8, u);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (float)b[e];
  } else {
    const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + idx);
    const float4 c = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + idx + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = c.x; o[5] = c.y; o[6] = c.z; o[7] = c.w;
  }
}
__device__ __forceinline__ void st8_dyn(void* p, int dt, long idx, const float (&v)[8]) {
  if (dt == CFM_BF16) {
    bf16x8 b;
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = (bf16)v[e];
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p) + idx) = __builtin_bit_cast(uint4, b);
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + idx) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + idx + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// ----------------------------------------------------------------------------- dropout RNG
// Counter-based dropout: element idx of a call keyed by `seed` draws 16 uniform bits; elements
// 2j and 2j+1 share one 32-bit hash of j + key (attn_mix below: two full-rate 24-bit multiply-adds; the key itself
// comes from lowbias32), so the mask costs a few VALU ops per element and is regenerated bit-identically in the
// backward kernels.
__device__ __forceinline__ uint32_t cfm_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// The dropout element hash (every dropout: attention probabilities, GEMM epilogues, scale_dropout, the LayerNorm
// backward's g2): two full-rate 24-bit multiply-adds (v_mad_u32_u24) in place of lowbias32's two 32-bit
// multiplies (v_mul_lo_u32, quarter rate) -- the attention kernels hash one pair per two scores and were
// VALU-bound on it.  Each round x += lo24(x) * C with C even is lo24 * (C + 1) + (hi8 << 24): C + 1 odd makes
// it a bijection of the 32-bit word (two inputs with equal images have equal lo24, since C + 1 is invertible
// mod 2^24, hence equal hi8), so the whole hash is one-to-one and distinct element pairs never share bits by
// construction.  (Round 4's form multiplied lo24 alone and dropped the high byte: x and x ^ (d * 0x01000100)
// collided.)
// The key is ADDED to the pair index (not xor-ed, as for lowbias32), so a lane's base + key folds into one
// register and each pair costs one add.
// Over the attention and GEMM-epilogue index patterns its keep rate and lag-1..8 / diagonal correlations of the
// keep decisions match lowbias32's to within sampling noise (tests/test_dropout_hash_cpu.py).
__device__ __forceinline__ uint32_t attn_mix(uint32_t x) {
  x ^= x >> 16;
  x += (x & 0xFFFFFFu) * 0x9E3778u;
  x ^= x >> 15;
  x += (x & 0xFFFFFFu) * 0x85EBCAu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_key(uint64_t seed, uint32_t jhi) {
  return cfm_mix32(jhi ^ (uint32_t)seed ^ cfm_mix32((uint32_t)(seed >> 32) + 0x9E3779B9u));
}
__device__ __forceinline__ uint32_t drop_bits(uint64_t seed, uint64_t idx) {
  const uint64_t j = idx >> 1;
  const uint32_t h = attn_mix((uint32_t)j + drop_key(seed, (uint32_t)(j >> 32)));
  return (idx & 1) ? (h >> 16) : (h & 0xFFFFu);
}
// dropped iff the 16 bits fall below round(p * 65536); kept elements scale by the exact inverse
// keep probability
__device__ __forceinline__ uint32_t drop_thr(float p) { return (uint32_t)(p * 65536.f + 0.5f); }
__device__ __forceinline__ float drop_keep_scale(uint32_t thr) { return 65536.f / (float)(65536u - thr); }
// the seed a kernel actually uses: the caller's seed offset by the bound device step counter
__device__ __forceinline__ uint64_t salted_seed(uint64_t seed, const uint64_t* salt) {
  return salt ? seed + salt[0] * 0x9E3779B97F4A7C15ull : seed;
}
// timing probe of a launch (cfm_gemm_desc.probe): first workgroup start / last workgroup end
__device__ __forceinline__ void probe_begin(unsigned long long* slot) {
  if (slot && threadIdx.x == 0) atomicMin(slot, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void probe_end(unsigned long long* slot) {
  if (slot) {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(slot + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}
// returns the keep scale if kept, 0 if dropped
__device__ __forceinline__ float dropout_scale(float p, uint64_t seed, uint64_t idx) {
  if (p <= 0.f) return 1.f;
  const uint32_t thr = drop_thr(p);
  return drop_bits(seed, idx) >= thr ? drop_keep_scale(thr) : 0.f;
}
// the attention-dropout keep scale of element idx (the SIMT attention kernels): the same element hash
__device__ __forceinline__ float attn_dropout_scale(float p, uint64_t seed, uint64_t idx) {
  return dropout_scale(p, seed, idx);
}
// attn_dropout_scale with the per-seed key hoisted (valid for idx < 2^33, where drop_key's high word is 0):
// bit-identical masks at one mix per element pair (MFMA attention kernels: key = drop_key(seed, 0))
__device__ __forceinline__ float dropout_keyed(uint32_t thr, float keep, uint32_t key, uint64_t idx) {
  const uint32_t h = attn_mix((uint32_t)(idx >> 1) + key);
  const uint32_t bits = (idx & 1) ? (h >> 16) : (h & 0xFFFFu);
  return bits >= thr ? keep : 0.f;
}
// the same mask for the 8 consecutive elements base .. base+7 (5 hashes instead of 8 x 2)
__device__ __forceinline__ void dropout_scale8(float p, uint64_t seed, uint64_t base, float (&s)[8]) {
  const uint32_t thr = drop_thr(p);
  const float keep = drop_keep_scale(thr);
  const uint64_t j0 = base >> 1;
  const uint32_t lo0 = (uint32_t)j0;
  if (lo0 <= 0xFFFFFFFBu) {
    const uint32_t key = drop_key(seed, (uint32_t)(j0 >> 32));
    uint32_t h[5];
    const int odd = (int)(base & 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) h[q] = attn_mix(lo0 + q + key);
    h[4] = odd ? attn_mix(lo0 + 4 + key) : 0u;   // (an even base needs 4 pair hashes)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = (odd + e) >> 1;
      const uint32_t b = ((odd + e) & 1) ? (h[q] >> 16) : (h[q] & 0xFFFFu);
      s[e] = b >= thr ? keep : 0.f;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = drop_bits(seed, base + e) >= thr ? keep : 0.f;
  }
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

__host__ __device__ static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
