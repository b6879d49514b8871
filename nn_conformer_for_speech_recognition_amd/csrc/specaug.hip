// specaug.hip — SpecAugment apply: composed time-warp gather + freq/time masks in one HBM pass.
//
// Reference: lib/standard/asrnn.py:91-192.  The draws are made on the host with python
// `random` in the reference's order (see specaugment.py); this kernel evaluates the warp
// table Wt_b(t) of asrnn.py:109-115 per element with the same arithmetic (float64 true
// division + truncation for t <= w0, integer floor division otherwise), so the gathered
// indices are bit-identical to the reference's.
// HBM-bound: one fp32 read + one fp32 write per element; threads run along t (coalesced).
#include "cfm_common.h"

namespace {

__device__ __forceinline__ int warp_index(int t, int w, int w0, int tau) {
  if (t >= tau) return t;                                        // asrnn.py:115 identity tail
  if (t <= w0) return (int)((((double)(w0 + w)) / (double)w0) * (double)t);   // :111
  const long num = (long)(tau - 1 - w0 - w) * t + (long)(tau - 1) * w;         // :113
  const long den = (long)(tau - 1 - w0);
  long q = num / den;
  if ((num % den != 0) && ((num < 0) != (den < 0))) --q;        // floor semantics
  return (int)q;
}

__global__ void specaug_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int F, int T,
                               const int32_t* __restrict__ prm, int intended, float mask_value) {
  const int nw = prm[0], nf = prm[1], nt = prm[2];
  const int32_t* warps = prm + 4;
  const int32_t* freqs = warps + 3 * nw * B;
  const int32_t* times = freqs + 2 * nf;
  const long total = (long)B * F * T;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int t = (int)(i % T);
    const long bf = i / T;
    const int f = (int)(bf % F);
    const int b = (int)(bf / F);
    int src = t;
    for (int p = nw - 1; p >= 0; --p) {             // x_n[t] = x_{n-1}[Wt_n(t)]: apply last pass first
      const int32_t* q = warps + 3 * (p * B + b);
      src = warp_index(src, q[0], q[1], q[2]);
    }
    float v = x[bf * T + src];
    if (intended) {
      for (int k = 0; k < nf; ++k) {
        const int f0 = freqs[2 * k], fw = freqs[2 * k + 1];
        if (f >= f0 && f < f0 + fw) v = mask_value;
      }
      for (int k = 0; k < nt; ++k) {
        const int t0 = times[2 * (k * B + b)], tw = times[2 * (k * B + b) + 1];
        if (t >= t0 && t < t0 + tw) v = mask_value;
      }
    }
    y[i] = v;
  }
}

}  // namespace

CFM_EXPORT int cfm_specaug_apply(const float* x, float* y, int B, int F, int T, const int32_t* params,
                                 int n_params, int intended, float mask_value, void* stream) {
  CFM_REQUIRE(x && y && params, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(x != y, CFM_ERR_ARG, "x and y must not alias");
  CFM_REQUIRE(B >= 0 && F >= 0 && T >= 0 && n_params >= 4, CFM_ERR_SHAPE, "bad shape");
  const long total = (long)B * F * T;
  if (total == 0) return CFM_OK;
  long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(specaug_kernel, dim3((unsigned)blocks), dim3(256), 0, cfm::as_stream(stream), x, y, B,
                     F, T, params, intended, mask_value);
  return cfm::check_launch("cfm_specaug_apply");
}
