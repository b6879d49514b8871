// convsub.hip — first subsampling convolution (lib/convsubsampling.py:21, Conv2d(1 -> C1, 7x7,
// stride 2, no padding)) forward and weight-gradient.
//
// The input has ONE channel, so this is 49 MACs per output: HBM-write-bound (C1 = 512 outputs
// per input pixel pair).  Output is NHWC (B, F1, T1, C1) in the compute dtype so that the
// second convolution (implicit GEMM in gemm.hip) reads 16-byte channel chunks.
// Forward: one workgroup per (b, f1, 32-frame tile); the 7 x 69 input patch sits in LDS (all
// lanes read the same pixel: LDS broadcast), each thread owns up to 2 channels with their 49
// taps in registers; stores are 1 KiB-coalesced channel rows.  (VALU-bound: 49 FMAs per output;
// an MFMA im2col form is the next step.)  The weight-gradient stages the block's [32][C1] dh1 rows
// (one contiguous run in NHWC) in LDS with 16-byte loads and keeps the 7x7 input window in registers.
// Weight-gradient: a persistent grid sweeps (b, f1) rows; each thread accumulates 49 tap sums +
// the bias sum for its channels in registers; per-workgroup partials are reduced by a second
// kernel (deterministic).
#include "cfm_common.h"

namespace {
constexpr int KK = 7, ST = 2, TW = 32;   // kernel, stride, output frames per workgroup
constexpr int PW = (TW - 1) * ST + KK;   // 69 input columns per patch
constexpr int CMAX = 512;                // channels supported (2 per thread)

// the 7x7 input window of output frame tt slides by 2 columns per frame: keep it in registers
// (fully unrolled frame loop -> the shifts are register renames) so each frame costs 14 LDS
// broadcast reads for 98 FMAs instead of 49
template <typename TO>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, TO* __restrict__ h1, int F,
                                                        int T, int C1, int F1, int T1) {
  __shared__ float patch[KK][PW + 1];
  const int tid = threadIdx.x;
  const int t10 = blockIdx.x * TW, f1 = blockIdx.y, b = blockIdx.z;
  const float* xb = x + (long)b * F * T;
  for (int i = tid; i < KK * PW; i += 256) {
    const int r = i / PW, cc = i % PW;
    const int fr = ST * f1 + r, tc = ST * t10 + cc;
    patch[r][cc] = (tc < T) ? xb[(long)fr * T + tc] : 0.f;
  }
  float wr[2][KK * KK], bb[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int c = tid + 256 * q;
#pragma unroll
    for (int k = 0; k < KK * KK; ++k) wr[q][k] = c < C1 ? w[c * KK * KK + k] : 0.f;
    bb[q] = c < C1 ? bias[c] : 0.f;
  }
  __syncthreads();
  const int nt = min(TW, T1 - t10);
  for (int tt = 0; tt < nt; ++tt) {
    float a0 = bb[0], a1 = bb[1];
#pragma unroll
    for (int kh = 0; kh < KK; ++kh)
#pragma unroll
      for (int kw = 0; kw < KK; ++kw) {
        const float v = patch[kh][ST * tt + kw];
        a0 += wr[0][kh * KK + kw] * v;
        a1 += wr[1][kh * KK + kw] * v;
      }
    TO* row = h1 + (((long)b * F1 + f1) * T1 + t10 + tt) * C1;
    if (tid < C1) row[tid] = from_f32<TO>(a0);
    if (tid + 256 < C1) row[tid + 256] = from_f32<TO>(a1);
  }
}

// partial dW: ws[blk][c][50] (49 taps + bias)
template <typename TI>
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(const TI* __restrict__ dh1, const float* __restrict__ x,
                                                          int B, int F, int T, int C1, int F1, int T1,
                                                          float* __restrict__ ws) {
  __shared__ float patch[KK][PW + 1];
  __shared__ __attribute__((aligned(16))) TI stage[TW * CMAX];   // the block's [nt][C1] dh1 rows
  const int tid = threadIdx.x;
  float acc[2][KK * KK + 1];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int k = 0; k <= KK * KK; ++k) acc[q][k] = 0.f;
  const int ntile = (T1 + TW - 1) / TW;
  const long nwork = (long)B * F1 * ntile;
  for (long wi = blockIdx.x; wi < nwork; wi += gridDim.x) {
    const int tile = (int)(wi % ntile);
    const long bf = wi / ntile;
    const int f1 = (int)(bf % F1), b = (int)(bf / F1);
    const int t10 = tile * TW;
    __syncthreads();
    const float* xb = x + (long)b * F * T;
    for (int i = tid; i < KK * PW; i += 256) {
      const int r = i / PW, cc = i % PW;
      const int tc = ST * t10 + cc;
      patch[r][cc] = (tc < T) ? xb[(long)(ST * f1 + r) * T + tc] : 0.f;
    }
    const int nt = min(TW, T1 - t10);
    {
      const TI* src = dh1 + (((long)b * F1 + f1) * T1 + t10) * C1;
      const long n = (long)nt * C1;
      constexpr int V = 16 / sizeof(TI);
      if ((C1 % V) == 0 && ((uintptr_t)src % 16) == 0) {
        for (long i = (long)tid * V; i < n; i += 256 * V)
          *reinterpret_cast<uint4*>(stage + i) = *reinterpret_cast<const uint4*>(src + i);
      } else {
        for (long i = tid; i < n; i += 256) stage[i] = src[i];
      }
    }
    __syncthreads();
    float win[KK][KK];
#pragma unroll
    for (int r = 0; r < KK; ++r)
#pragma unroll
      for (int q = 0; q < KK; ++q) win[r][q] = patch[r][q];
#pragma unroll
    for (int tt = 0; tt < TW; ++tt) {
      if (tt >= nt) break;
      if (tt > 0) {
#pragma unroll
        for (int r = 0; r < KK; ++r) {
#pragma unroll
          for (int q = 0; q < KK - ST; ++q) win[r][q] = win[r][q + ST];
          win[r][KK - 2] = patch[r][ST * tt + KK - 2];
          win[r][KK - 1] = patch[r][ST * tt + KK - 1];
        }
      }
      const float g0 = 2 * tid < C1 ? to_f32(stage[tt * C1 + 2 * tid]) : 0.f;
      const float g1 = 2 * tid + 1 < C1 ? to_f32(stage[tt * C1 + 2 * tid + 1]) : 0.f;
#pragma unroll
      for (int kh = 0; kh < KK; ++kh)
#pragma unroll
        for (int kw = 0; kw < KK; ++kw) {
          acc[0][kh * KK + kw] += g0 * win[kh][kw];
          acc[1][kh * KK + kw] += g1 * win[kh][kw];
        }
      acc[0][KK * KK] += g0;
      acc[1][KK * KK] += g1;
    }
  }
  float* out = ws + (long)blockIdx.x * C1 * (KK * KK + 1);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int c = 2 * tid + q;
    if (c < C1)
#pragma unroll
      for (int k = 0; k <= KK * KK; ++k) out[(long)c * (KK * KK + 1) + k] = acc[q][k];
  }
}

__global__ void conv1_wgrad_reduce(const float* __restrict__ ws, int nblk, int C1, float* __restrict__ dw,
                                   float* __restrict__ db) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int per = KK * KK + 1;
  if (i >= C1 * per) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += ws[(long)b * C1 * per + i];
  const int c = i / per, k = i % per;
  if (k < KK * KK) dw[c * KK * KK + k] = (float)s;
  else if (db) db[c] = (float)s;
}

constexpr int WGRAD_BLOCKS = 512;   // 2 workgroups per CU (174 VGPRs)
}  // namespace

CFM_EXPORT int cfm_conv1_fwd(const float* x, const float* w1, const float* b1, void* h1, int dtype_h, int B, int F,
                             int T, int C1, void* stream) {
  CFM_REQUIRE(x && w1 && b1 && h1, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(C1 > 0 && C1 <= CMAX, CFM_ERR_UNSUPPORTED, "conv1 supports up to 512 channels");
  CFM_REQUIRE(F >= KK && T >= KK && B > 0, CFM_ERR_SHAPE, "input smaller than the 7x7 kernel");
  const int F1 = (F - KK) / ST + 1, T1 = (T - KK) / ST + 1;
  CFM_REQUIRE(F1 <= 65535, CFM_ERR_SHAPE, "too many mel bins");
  dim3 grid(cdiv(T1, TW), F1, B);
  hipStream_t s = cfm::as_stream(stream);
  if (dtype_h == CFM_BF16)
    hipLaunchKernelGGL(conv1_fwd_kernel<bf16>, grid, dim3(256), 0, s, x, w1, b1, (bf16*)h1, F, T, C1, F1, T1);
  else
    hipLaunchKernelGGL(conv1_fwd_kernel<float>, grid, dim3(256), 0, s, x, w1, b1, (float*)h1, F, T, C1, F1, T1);
  return cfm::check_launch("cfm_conv1_fwd");
}

CFM_EXPORT size_t cfm_conv1_bwd_ws_bytes(int B, int F, int T, int C1) {
  (void)B; (void)F; (void)T;
  return (size_t)WGRAD_BLOCKS * C1 * (KK * KK + 1) * sizeof(float);
}

CFM_EXPORT int cfm_conv1_bwd_weight(const void* dh1, int dtype_h, const float* x, float* dw1, float* db1, int B, int F,
                                    int T, int C1, float* ws, void* stream) {
  CFM_REQUIRE(dh1 && x && dw1 && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(C1 > 0 && C1 <= CMAX, CFM_ERR_UNSUPPORTED, "conv1 supports up to 512 channels");
  const int F1 = (F - KK) / ST + 1, T1 = (T - KK) / ST + 1;
  const long nwork = (long)B * F1 * cdiv(T1, TW);
  const int nblk = (int)(nwork < WGRAD_BLOCKS ? nwork : WGRAD_BLOCKS);
  hipStream_t s = cfm::as_stream(stream);
  if (dtype_h == CFM_BF16)
    hipLaunchKernelGGL(conv1_wgrad_kernel<bf16>, dim3(nblk), dim3(256), 0, s, (const bf16*)dh1, x, B, F, T, C1, F1,
                       T1, ws);
  else
    hipLaunchKernelGGL(conv1_wgrad_kernel<float>, dim3(nblk), dim3(256), 0, s, (const float*)dh1, x, B, F, T, C1, F1,
                       T1, ws);
  hipLaunchKernelGGL(conv1_wgrad_reduce, dim3(cdiv((long)C1 * (KK * KK + 1), 256)), dim3(256), 0, s, ws, nblk, C1,
                     dw1, db1);
  return cfm::check_launch("cfm_conv1_bwd_weight");
}
