// convmod.hip — the HBM-bound middle of torchaudio's _ConvolutionModule:
//   GLU(dim=channel) -> depthwise Conv1d(K, 'same' zero padding, bias) -> BatchNorm1d -> SiLU
// and its backward, plus the generic BatchNorm1d of the projection block.
// Token-major layout (row = b*T + t, channel contiguous) so every load is coalesced across
// channels; each workgroup owns a 64-channel x TT-frame tile of one utterance and stages the GLU
// output (or dy) with its (K-1)/2 halo in LDS.  The kernel size is a template parameter for the
// sizes the configs use (31, 33, ...) so the tap loops unroll.
// BatchNorm batch statistics (train mode) are per-channel sums over all B*T rows, INCLUDING
// padded frames — exactly what torchaudio/transformers do (padding is not masked there).
// Per-workgroup partial sums go to a workspace and are combined by cfm::colreduce
// (deterministic two-level reduction; no atomics).
#include <cstdlib>

#include "cfm_common.h"

namespace {
constexpr int CT = 64;    // channels per workgroup (one per lane)
constexpr int TT = 64;    // frames per workgroup
constexpr int KMAX = 63;  // largest supported depthwise kernel
constexpr int BN_PARTS = 256;

__device__ __forceinline__ float glu_at(const void* a, int dta, long row, int C, int c) {
  const float x = ld_dyn(a, dta, row * 2 * C + c);
  const float g = ld_dyn(a, dta, row * 2 * C + C + c);
  return x * sigmoid_f(g);
}

// grid: (ceil(C/CT), ceil(T/TT), B), block 256 = 4 waves; lane = channel, wave strides time.
// part: [2][nparts][C] (sum, sumsq) with part index b*gridDim.y + blockIdx.y.
template <int KT, typename TA>
__global__ __launch_bounds__(256) void glu_dwconv_fwd_kernel(const void* __restrict__ a, int dta,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias, float* __restrict__ y,
                                                             int T, int C, int Krt, float* __restrict__ part) {
  const int K = KT > 0 ? KT : Krt;
  extern __shared__ float sg[];                  // [(TT+K-1)][CT]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * CT + lane;
  const int t0 = blockIdx.y * TT, b = blockIdx.z;
  const int pad = (K - 1) / 2;
  const int rows = TT + K - 1;
  if constexpr (KT > 0) {
    // every load of the wave's rows in flight before the first use (latency, not bandwidth, bound)
    // unconditional loads at clamped addresses (a select around each load makes hipcc branch and
    // wait vmcnt(0) per element); out-of-range rows are zeroed after the fact
    constexpr int NR = (TT + KT - 1 + 3) / 4;
    const TA* ap = reinterpret_cast<const TA*>(a) + (c < C ? c : C - 1);
    float xv[NR], gv[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int t = min(max(t0 - pad + wv + 4 * i, 0), T - 1);
      const long row = (long)b * T + t;
      xv[i] = to_f32(ap[row * 2 * C]);
      gv[i] = to_f32(ap[row * 2 * C + C]);
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int r = wv + 4 * i, t = t0 - pad + r;
      const bool ok = c < C && t >= 0 && t < T;
      if (r < rows) sg[r * CT + lane] = ok ? xv[i] * sigmoid_f(gv[i]) : 0.f;
    }
  } else {
    for (int r = wv; r < rows; r += 4) {
      const int t = t0 - pad + r;
      float v = 0.f;
      if (c < C && t >= 0 && t < T) v = glu_at(a, dta, (long)b * T + t, C, c);
      sg[r * CT + lane] = v;
    }
  }
  __syncthreads();
  constexpr int KR = KT > 0 ? KT : KMAX;
  float wr[KR];
  const int cw = c < C ? c : C - 1;
#pragma unroll
  for (int k = 0; k < KR; ++k) wr[k] = w[cw * K + (k < K ? k : 0)];
#pragma unroll
  for (int k = 0; k < KR; ++k) wr[k] = (c < C && k < K) ? wr[k] : 0.f;
  const float bb = c < C ? bias[cw] : 0.f;
  float s1 = 0.f, s2 = 0.f;
  if constexpr (KT > 0) {
    // wave w: frames 16w .. 16w+15 with the 16+K-1 GLU values they touch held in registers
    constexpr int FB = TT / 4, WN = FB + KT - 1;
    const int tb = wv * FB;
    float win[WN];
#pragma unroll
    for (int j = 0; j < WN; ++j) win[j] = sg[(tb + j) * CT + lane];
#pragma unroll
    for (int f = 0; f < FB; ++f) {
      const int t = t0 + tb + f;
      float acc = bb;
#pragma unroll
      for (int k = 0; k < KT; ++k) acc += wr[k] * win[f + k];
      if (c < C && t < T) {
        y[((long)b * T + t) * C + c] = acc;
        s1 += acc;
        s2 += acc * acc;
      }
    }
  } else {
    for (int tt = wv; tt < TT; tt += 4) {
      const int t = t0 + tt;
      if (t >= T) break;
      float acc = bb;
#pragma unroll
      for (int k = 0; k < KR; ++k)
        if (k < K) acc += wr[k] * sg[(tt + k) * CT + lane];
      if (c < C) {
        y[((long)b * T + t) * C + c] = acc;
        s1 += acc;
        s2 += acc * acc;
      }
    }
  }
  __syncthreads();
  sg[wv * CT + lane] = s1;
  sg[(4 + wv) * CT + lane] = s2;
  __syncthreads();
  if (wv == 0 && c < C) {
    const float a1 = sg[lane] + sg[CT + lane] + sg[2 * CT + lane] + sg[3 * CT + lane];
    const float a2 = sg[4 * CT + lane] + sg[5 * CT + lane] + sg[6 * CT + lane] + sg[7 * CT + lane];
    const long part_idx = (long)b * gridDim.y + blockIdx.y;
    const long nparts = (long)gridDim.z * gridDim.y;
    part[part_idx * C + c] = a1;
    part[(nparts + part_idx) * C + c] = a2;
  }
}

// Vectorised forward (bf16 a, C % 4 == 0, compiled K): staging loads and the y stores move 4 channels per lane
// (8- / 16-byte accesses) through LDS; the taps run lane = channel as above.  Same partial-sum layout.
// (Packed-fp32 taps as in the backward measured slower here: 17.2 -> 20.0 us, 94 -> 195 VGPRs, occupancy 5 -> 2.)
template <int KT>
__global__ __launch_bounds__(256) void glu_dwconv_fwd_vec_kernel(const bf16* __restrict__ a,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ bias,
                                                                 float* __restrict__ y, int T, int C,
                                                                 float* __restrict__ part) {
  constexpr int PAD = (KT - 1) / 2, ROWS = TT + KT - 1, NP = (ROWS + 15) / 16;
  constexpr int FB = TT / 4, WN = FB + KT - 1;
  constexpr int L_OUT = TT * CT + 8 * CT;
  __shared__ __attribute__((aligned(16))) float sm[ROWS * CT > L_OUT ? ROWS * CT : L_OUT];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int q = tid & 15, rs = tid >> 4;
  const int c0 = blockIdx.x * CT, t0 = blockIdx.y * TT, b = blockIdx.z;
  const int cq = c0 + 4 * q;
  const bool cok = cq < C;
  const int cqc = cok ? cq : C - 4;
  const int c = c0 + lane, cw = c < C ? c : C - 1;
  float wr[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) wr[k] = w[cw * KT + k];
  const float bb = bias[cw];
  bf16x4 x4[NP], g4[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int t = min(max(t0 - PAD + rs + 16 * p, 0), T - 1);
    const long row = (long)b * T + t;
    x4[p] = *reinterpret_cast<const bf16x4*>(a + row * 2 * C + cqc);
    g4[p] = *reinterpret_cast<const bf16x4*>(a + row * 2 * C + C + cqc);
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int r = rs + 16 * p, t = t0 - PAD + r;
    if (r < ROWS) {
      const bool ok = cok && t >= 0 && t < T;
      f32x4 g;
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = ok ? (float)x4[p][j] * sigmoid_f((float)g4[p][j]) : 0.f;
      *reinterpret_cast<f32x4*>(sm + r * CT + 4 * q) = g;
    }
  }
  __syncthreads();
  const int tb = wv * FB;
  float win[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j) win[j] = sm[(tb + j) * CT + lane];
  float acc[FB], s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int f = 0; f < FB; ++f) {
    float v = bb;
#pragma unroll
    for (int k = 0; k < KT; ++k) v += wr[k] * win[f + k];
    acc[f] = v;
    if (c < C && t0 + tb + f < T) {
      s1 += v;
      s2 += v * v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int f = 0; f < FB; ++f) sm[(tb + f) * CT + lane] = acc[f];
  sm[TT * CT + wv * CT + lane] = s1;
  sm[TT * CT + (4 + wv) * CT + lane] = s2;
  __syncthreads();
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int f = rs + 16 * p - PAD, t = t0 + f;
    if (f >= 0 && f < TT && t < T && cok)
      *reinterpret_cast<f32x4*>(y + ((long)b * T + t) * C + cq) = *reinterpret_cast<const f32x4*>(sm + f * CT + 4 * q);
  }
  if (wv == 0 && c < C) {
    const float* r = sm + TT * CT;
    const float a1 = r[lane] + r[CT + lane] + r[2 * CT + lane] + r[3 * CT + lane];
    const float a2 = r[4 * CT + lane] + r[5 * CT + lane] + r[6 * CT + lane] + r[7 * CT + lane];
    const long part_idx = (long)b * gridDim.y + blockIdx.y;
    const long nparts = (long)gridDim.z * gridDim.y;
    part[part_idx * C + c] = a1;
    part[(nparts + part_idx) * C + c] = a2;
  }
}

// the column sums of the (sum, sumsq) partial rows and the batch stats + running-stat update in one launch
// (round 4: cfm::colreduce_pair then bn_finalize_kernel, two ~5 us launches per BatchNorm forward): per 64
// channels, 16 waves sum parts wv, wv + 16, ... of both arrays in the colreduce2 order, wave 0 adds the 16 wave
// sums in order and finalises -- bit-identical to the two-launch form
__global__ __launch_bounds__(1024) void bn_stats_kernel(const float* __restrict__ partA, const float* __restrict__ partB,
                                                        int nparts, long M, int C, float* __restrict__ mean,
                                                        float* __restrict__ invstd, float* __restrict__ rmean,
                                                        float* __restrict__ rvar, float momentum, float eps) {
  __shared__ float red[2][16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float sa = 0.f, sb = 0.f;
  if (c < C) {
    for (int p0 = wv; p0 < nparts; p0 += 16 * 8) {
      float va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool ok = p0 + 16 * u < nparts;
        va[u] = ok ? partA[(long)(p0 + 16 * u) * C + c] : 0.f;
        vb[u] = ok ? partB[(long)(p0 + 16 * u) * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        sa += va[u];
        sb += vb[u];
      }
    }
  }
  red[0][wv][lane] = sa;
  red[1][wv][lane] = sb;
  __syncthreads();
  if (wv != 0 || c >= C) return;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    s1 += red[0][q][lane];
    s2 += red[1][q][lane];
  }
  const double mu = (double)s1 / (double)M;
  double var = (double)s2 / (double)M - mu * mu;
  if (var < 0.0) var = 0.0;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mu;
  if (rvar)
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)(M > 1 ? var * (double)M / (double)(M - 1) : var);
}

// batch stats from column sums s1 (sum) and s2 (sum of squares) + running-stat update.
__global__ void bn_finalize_kernel(const float* __restrict__ s1, const float* __restrict__ s2, long M, int C,
                                   float* __restrict__ mean, float* __restrict__ invstd,
                                   float* __restrict__ rmean, float* __restrict__ rvar, float momentum, float eps) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const double mu = (double)s1[c] / (double)M;
  double var = (double)s2[c] / (double)M - mu * mu;
  if (var < 0.0) var = 0.0;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mu;
  if (rvar)
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)(M > 1 ? var * (double)M / (double)(M - 1) : var);
}

__global__ void bn_eval_stats_kernel(const float* __restrict__ rmean, const float* __restrict__ rvar, int C,
                                     float eps, float* __restrict__ mean, float* __restrict__ invstd) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  mean[c] = rmean[c];
  invstd[c] = rsqrtf(rvar[c] + eps);
}

__global__ void bn_apply_kernel(const float* __restrict__ y, const float* __restrict__ gamma,
                                const float* __restrict__ beta, const float* __restrict__ mean,
                                const float* __restrict__ invstd, void* __restrict__ z, int dtz, long M, int C,
                                int act) {
  const long n = M * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float u = (y[i] - mean[c]) * invstd[c] * gamma[c] + beta[c];
    st_dyn(z, dtz, i, act ? silu_f(u) : u);
  }
}

// 8 consecutive elements per thread, one pass (C % 8 == 0, 16-B aligned): the grid-stride kernel above runs ~3
// iterations per thread whose loads each wait behind the previous iteration's store (one in-order vmcnt queue)
template <int DTZ>
__global__ __launch_bounds__(256) void bn_apply_vec8(const float* __restrict__ y, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, const float* __restrict__ mean,
                                                     const float* __restrict__ invstd, void* __restrict__ z, long M,
                                                     int C, int act) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= M * C) return;
  const int c = (int)(i % C);
  float v[8];
  ld8_dyn(y, CFM_F32, i, v);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float u = (v[e] - mean[c + e]) * invstd[c + e] * gamma[c + e] + beta[c + e];
    v[e] = act ? silu_f(u) : u;
  }
  st8_dyn(z, DTZ, i, v);
}

// row-chunk partial sums (sum, sumsq) of y over (M, C); grid (ceil(C/64), nparts), 4 waves per block
__global__ __launch_bounds__(256) void bn_stats_rows_kernel(const float* __restrict__ y, long M, int C,
                                                            long rows_per, float* __restrict__ part) {
  __shared__ float red[2][4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const long r0 = (long)blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float s1 = 0.f, s2 = 0.f;
  if (c < C)
    for (long r = r0 + wv; r < r1; r += 4) {
      const float v = y[r * C + c];
      s1 += v;
      s2 += v * v;
    }
  red[0][wv][lane] = s1;
  red[1][wv][lane] = s2;
  __syncthreads();
  if (wv == 0 && c < C) {
    part[(long)blockIdx.y * C + c] = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
    part[(long)(gridDim.y + blockIdx.y) * C + c] =
        red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
  }
}

// row-chunk partials (sum du, sum du*yhat) for the BN backward; same geometry
__global__ __launch_bounds__(256) void bn_bwd_rows_kernel(const void* __restrict__ dz, int dtdz,
                                                          const float* __restrict__ y, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, long M, int C,
                                                          long rows_per, float* __restrict__ part, int act) {
  __shared__ float red[2][4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const long r0 = (long)blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float sd = 0.f, sdx = 0.f;
  if (c < C) {
    const float mu = mean[c], is = invstd[c], g = gamma[c], bt = beta[c];
    for (long r = r0 + wv; r < r1; r += 4) {
      const long i = r * C + c;
      const float yh = (y[i] - mu) * is;
      const float du = ld_dyn(dz, dtdz, i) * (act ? silu_grad_f(yh * g + bt) : 1.f);
      sd += du;
      sdx += du * yh;
    }
  }
  red[0][wv][lane] = sd;
  red[1][wv][lane] = sdx;
  __syncthreads();
  if (wv == 0 && c < C) {
    part[(long)blockIdx.y * C + c] = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
    part[(long)(gridDim.y + blockIdx.y) * C + c] =
        red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
  }
}

__global__ void bn_bwd_apply_kernel(const void* __restrict__ dz, int dtdz, const float* __restrict__ y,
                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                    const float* __restrict__ mean, const float* __restrict__ invstd,
                                    const float* __restrict__ dgamma, const float* __restrict__ dbeta, int training,
                                    float* __restrict__ dy, long M, int C, int act) {
  const long n = M * C;
  const float invM = 1.f / (float)M;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float is = invstd[c], g = gamma[c];
    const float yh = (y[i] - mean[c]) * is;
    const float du = ld_dyn(dz, dtdz, i) * (act ? silu_grad_f(yh * g + beta[c]) : 1.f);
    float v = du;
    if (training) v = du - dbeta[c] * invM - yh * dgamma[c] * invM;
    dy[i] = g * is * v;
  }
}

// SyncBatchNorm input gradient: the sums are over M_total rows of all replicas (invM = 1 / M_total)
__global__ void bn_bwd_apply_total_kernel(const void* __restrict__ dz, int dtdz, const float* __restrict__ y,
                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                          const float* __restrict__ mean, const float* __restrict__ invstd,
                                          const float* __restrict__ dgamma, const float* __restrict__ dbeta,
                                          float* __restrict__ dy, long M, int C, float invM) {
  const long n = M * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float is = invstd[c], g = gamma[c];
    const float yh = (y[i] - mean[c]) * is;
    const float du = ld_dyn(dz, dtdz, i) * silu_grad_f(yh * g + beta[c]);
    dy[i] = g * is * (du - dbeta[c] * invM - yh * dgamma[c] * invM);
  }
}

// BatchNorm1d + SiLU backward folded into the depthwise-conv backward (BN=true): the kernel reads dz (the
// pointwise-conv-2 data gradient) and the BN input y and forms the BN input gradient
//   dy = gamma * invstd * (du - dbeta / M - yhat * dgamma / M)   (train; eval: gamma * invstd * du)
//   du = dz * silu'(yhat * gamma + beta),  yhat = (y - mean) * invstd
// on the fly, so the fp32 dy never goes through HBM (one write + one read of B*T*C floats and a launch saved).
struct BnBwd {
  const void* dz; int dtdz;
  const float* y;
  const float *gamma, *beta, *mean, *invstd, *dgamma, *dbeta;
  float invM;
  int training;
};

// backward of y = dwconv(GLU(a)).  grid (ceil(C/CT), ceil(T/TT), B)
// part: [nparts][K+1][C] per-block partial dw (K taps) and db (tap K).
template <int KT, typename TA, bool BN = false>
__global__ __launch_bounds__(256) void glu_dwconv_bwd_kernel(const float* __restrict__ dy,
                                                             const void* __restrict__ a, int dta,
                                                             const float* __restrict__ w, void* __restrict__ da,
                                                             int dtda, int T, int C, int Krt,
                                                             float* __restrict__ part, BnBwd bn) {
  const int K = KT > 0 ? KT : Krt;
  extern __shared__ float sm[];                  // sdy [(TT+K-1)][CT], sg [(TT+K-1)][CT]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * CT + lane;
  const int t0 = blockIdx.y * TT, b = blockIdx.z;
  const int pad = (K - 1) / 2;
  const int rows = TT + K - 1;
  float* sdy = sm;
  float* sg = sm + rows * CT;
  if constexpr (KT > 0) {
    constexpr int NR = (TT + KT - 1 + 3) / 4;
    const int cc = c < C ? c : C - 1;
    const TA* ap = reinterpret_cast<const TA*>(a) + cc;
    float dv[NR], xv[NR], gv[NR];
    float bg = 0.f, bis = 0.f, bmu = 0.f, bbt = 0.f, bk1 = 0.f, bk2 = 0.f;
    if constexpr (BN) {
      bg = bn.gamma[cc]; bis = bn.invstd[cc]; bmu = bn.mean[cc]; bbt = bn.beta[cc];
      bk1 = bn.training ? bn.dbeta[cc] * bn.invM : 0.f;
      bk2 = bn.training ? bn.dgamma[cc] * bn.invM : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int t = min(max(t0 - pad + wv + 4 * i, 0), T - 1);
      const long row = (long)b * T + t;
      if constexpr (BN) {
        const float yh = (bn.y[row * C + cc] - bmu) * bis;
        const float du = ld_dyn(bn.dz, bn.dtdz, row * C + cc) * silu_grad_f(yh * bg + bbt);
        dv[i] = bg * bis * (du - bk1 - yh * bk2);
      } else {
        dv[i] = dy[row * C + cc];
      }
      xv[i] = to_f32(ap[row * 2 * C]);
      gv[i] = to_f32(ap[row * 2 * C + C]);
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int r = wv + 4 * i, t = t0 - pad + r;
      const bool ok = c < C && t >= 0 && t < T;
      if (r < rows) {
        sdy[r * CT + lane] = ok ? dv[i] : 0.f;
        sg[r * CT + lane] = ok ? xv[i] * sigmoid_f(gv[i]) : 0.f;
      }
    }
  } else {
    static_assert(!BN || KT > 0, "BN folding: compiled kernel sizes only");
    for (int r = wv; r < rows; r += 4) {
      const int t = t0 - pad + r;
      float vd = 0.f, vg = 0.f;
      if (c < C && t >= 0 && t < T) {
        const long row = (long)b * T + t;
        vd = dy[row * C + c];
        vg = glu_at(a, dta, row, C, c);
      }
      sdy[r * CT + lane] = vd;
      sg[r * CT + lane] = vg;
    }
  }
  __syncthreads();
  constexpr int KR = KT > 0 ? KT : KMAX;
  float wr[KR], dw[KR];
  const int cw = c < C ? c : C - 1;
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    wr[k] = w[cw * K + (k < K ? k : 0)];
    dw[k] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < KR; ++k) wr[k] = (c < C && k < K) ? wr[k] : 0.f;
  float db = 0.f;
  // y[t] = sum_k w[k] g[t+k-pad]  =>  dg[t] = sum_k w[k] dy[t-k+pad];  sdy[r] = dy[t0-pad+r]
  // dw[k] += dy[t] * g[t+k-pad]  (sg[r] = g[t0-pad+r] -> r = tt + k)
  auto emit = [&](int t, float dg) {
    const long row = (long)b * T + t;
    const float x = to_f32(reinterpret_cast<const TA*>(a)[row * 2 * C + c]);
    const float s = sigmoid_f(to_f32(reinterpret_cast<const TA*>(a)[row * 2 * C + C + c]));
    st_dyn(da, dtda, row * 2 * C + c, dg * s);
    st_dyn(da, dtda, row * 2 * C + C + c, dg * x * s * (1.f - s));
  };
  if constexpr (KT > 0) {
    // wave w: frames 16w .. 16w+15; the dy and GLU values they touch (16+K-1 each) in registers
    constexpr int FB = TT / 4, WN = FB + KT - 1;
    const int tb = wv * FB;
    float wd[WN], wg[WN];
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      wd[j] = sdy[(tb + j) * CT + lane];     // dy rows tb .. tb+WN-1  (frame f, tap k: row tb+f-k+2pad)
      wg[j] = sg[(tb + j) * CT + lane];      // g rows tb .. tb+WN-1   (frame f, tap k: row tb+f+k)
    }
    // the GLU inputs of the wave's frames, loaded unconditionally (clamped) ahead of the math
    const int cc2 = c < C ? c : C - 1;
    float xa[FB], ga[FB];
#pragma unroll
    for (int f = 0; f < FB; ++f) {
      const long row = (long)b * T + min(t0 + tb + f, T - 1);
      xa[f] = to_f32(reinterpret_cast<const TA*>(a)[row * 2 * C + cc2]);
      ga[f] = to_f32(reinterpret_cast<const TA*>(a)[row * 2 * C + C + cc2]);
    }
#pragma unroll
    for (int f = 0; f < FB; ++f) {
      const int t = t0 + tb + f;
      float dg = 0.f;
#pragma unroll
      for (int k = 0; k < KT; ++k) dg += wr[k] * wd[f - k + 2 * ((KT - 1) / 2)];
      const float dyt = wd[f + (KT - 1) / 2];
#pragma unroll
      for (int k = 0; k < KT; ++k) dw[k] += dyt * wg[f + k];
      db += dyt;
      if (c < C && t < T) {
        const long row = (long)b * T + t;
        const float sg1 = sigmoid_f(ga[f]);
        if constexpr (sizeof(TA) == 2) {
          if (dtda == CFM_BF16) {
            reinterpret_cast<bf16*>(da)[row * 2 * C + c] = (bf16)(dg * sg1);
            reinterpret_cast<bf16*>(da)[row * 2 * C + C + c] = (bf16)(dg * xa[f] * sg1 * (1.f - sg1));
            continue;
          }
        }
        st_dyn(da, dtda, row * 2 * C + c, dg * sg1);
        st_dyn(da, dtda, row * 2 * C + C + c, dg * xa[f] * sg1 * (1.f - sg1));
      }
    }
  } else {
    for (int tt = wv; tt < TT; tt += 4) {
      const int t = t0 + tt;
      if (t >= T) break;
      float dg = 0.f;
#pragma unroll
      for (int k = 0; k < KR; ++k)
        if (k < K) dg += wr[k] * sdy[(tt - k + 2 * pad) * CT + lane];
      const float dyt = sdy[(tt + pad) * CT + lane];
#pragma unroll
      for (int k = 0; k < KR; ++k)
        if (k < K) dw[k] += dyt * sg[(tt + k) * CT + lane];
      db += dyt;
      if (c < C) emit(t, dg);
    }
  }
  __syncthreads();
  float* red = sm;   // [4 waves][K+1][CT]
#pragma unroll
  for (int k = 0; k < KR; ++k)
    if (KT > 0 || k < K) red[(wv * (K + 1) + k) * CT + lane] = dw[k];
  red[(wv * (K + 1) + K) * CT + lane] = db;
  __syncthreads();
  const long part_idx = (long)b * gridDim.y + blockIdx.y;
  for (int i = threadIdx.x; i < (K + 1) * CT; i += 256) {
    const int k = i / CT, l = i % CT;
    const int cc = blockIdx.x * CT + l;
    if (cc < C) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) s += red[(q * (K + 1) + k) * CT + l];
      part[(part_idx * (K + 1) + k) * C + cc] = s;
    }
  }
}

// Vectorised backward (bf16 a / da, C % 4 == 0, compiled K): the staging loads and the da stores move 4 channels
// per lane (8- and 16-byte accesses: the scalar kernel above issues one 2-byte load per lane per row) while the
// depthwise math stays lane = channel out of LDS.  The GLU-input gradient goes back through LDS so the lane that
// staged a row's GLU inputs also writes that row's da from its registers (no second read of a).
// Staging map: thread = (row group rs = tid / 16, channel quad q = tid % 16); pass p covers rows rs + 16 p.
template <int KT, bool BN, bool DZ16>
__global__ __launch_bounds__(256) void glu_dwconv_bwd_vec_kernel(const float* __restrict__ dy,
                                                                 const bf16* __restrict__ a,
                                                                 const float* __restrict__ w, bf16* __restrict__ da,
                                                                 int T, int C, float* __restrict__ part, BnBwd bn) {
  constexpr int PAD = (KT - 1) / 2, ROWS = TT + KT - 1, NP = (ROWS + 15) / 16;
  constexpr int FB = TT / 4, WN = FB + KT - 1;
  constexpr int L_STAGE = 2 * ROWS * CT, L_OUT = TT * CT + 4 * (KT + 1) * CT;
  __shared__ __attribute__((aligned(16))) float sm[L_STAGE > L_OUT ? L_STAGE : L_OUT];
  float* sdy = sm;                 // [ROWS][CT] dy (staging)      | [TT][CT] dg (output)
  float* sg = sm + ROWS * CT;      // [ROWS][CT] GLU output        | red [4][KT+1][CT] after TT*CT
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int q = tid & 15, rs = tid >> 4;
  const int c0 = blockIdx.x * CT, t0 = blockIdx.y * TT, b = blockIdx.z;
  const int cq = c0 + 4 * q;
  const bool cok = cq < C;
  const int cqc = cok ? cq : C - 4;
  const int c = c0 + lane, cw = c < C ? c : C - 1;
  float wr[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) wr[k] = w[cw * KT + k];
  f32x4 bg, bis, bmu, bbt, bk1, bk2;
  if constexpr (BN) {
    bg = *reinterpret_cast<const f32x4*>(bn.gamma + cqc);
    bis = *reinterpret_cast<const f32x4*>(bn.invstd + cqc);
    bmu = *reinterpret_cast<const f32x4*>(bn.mean + cqc);
    bbt = *reinterpret_cast<const f32x4*>(bn.beta + cqc);
    if (bn.training) {
      bk1 = *reinterpret_cast<const f32x4*>(bn.dbeta + cqc) * bn.invM;
      bk2 = *reinterpret_cast<const f32x4*>(bn.dgamma + cqc) * bn.invM;
    } else {
      bk1 = f32x4{0.f, 0.f, 0.f, 0.f};
      bk2 = bk1;
    }
  }
  f32x4 v4[NP];
  bf16x4 z4[NP];
  bf16x4 x4[NP], g4[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int t = min(max(t0 - PAD + rs + 16 * p, 0), T - 1);
    const long row = (long)b * T + t;
    if constexpr (BN) {
      v4[p] = *reinterpret_cast<const f32x4*>(bn.y + row * C + cqc);
      if constexpr (DZ16) z4[p] = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(bn.dz) + row * C + cqc);
    } else {
      v4[p] = *reinterpret_cast<const f32x4*>(dy + row * C + cqc);
    }
    x4[p] = *reinterpret_cast<const bf16x4*>(a + row * 2 * C + cqc);
    g4[p] = *reinterpret_cast<const bf16x4*>(a + row * 2 * C + C + cqc);
  }
  f32x4 zf[NP];
  if constexpr (BN && !DZ16) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int t = min(max(t0 - PAD + rs + 16 * p, 0), T - 1);
      zf[p] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(bn.dz) + ((long)b * T + t) * C + cqc);
    }
  }
  // per-element BN + SiLU backward and GLU on packed FP32 pairs (v_pk_fma / v_pk_mul / v_pk_add: the transcendental
  // exp / rcp stay scalar); the gate sigmoid of the tile's own rows is kept for the da stores (sg4: computed once --
  // the stores recomputed it); same operations per element as the scalar form, up to FMA contraction
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 gi2[2], nmi2[2], bg2[2], bbt2[2], bk1_2[2], bk2_2[2];
  if constexpr (BN) {
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      gi2[h2] = f2{bg[2 * h2] * bis[2 * h2], bg[2 * h2 + 1] * bis[2 * h2 + 1]};
      nmi2[h2] = f2{-bmu[2 * h2] * bis[2 * h2], -bmu[2 * h2 + 1] * bis[2 * h2 + 1]};
      bg2[h2] = f2{bg[2 * h2], bg[2 * h2 + 1]};
      bbt2[h2] = f2{bbt[2 * h2], bbt[2 * h2 + 1]};
      bk1_2[h2] = f2{bk1[2 * h2], bk1[2 * h2 + 1]};
      bk2_2[h2] = f2{bk2[2 * h2], bk2[2 * h2 + 1]};
    }
  }
  f32x4 sg4[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int r = rs + 16 * p, t = t0 - PAD + r;
    if (r < ROWS) {
      const bool ok = cok && t >= 0 && t < T;
      f32x4 d, g;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        f2 dv;
        if constexpr (BN) {
          const f2 v = {v4[p][2 * h2], v4[p][2 * h2 + 1]};
          const f2 yh = __builtin_elementwise_fma(v, f2{bis[2 * h2], bis[2 * h2 + 1]}, nmi2[h2]);
          const f2 pre = __builtin_elementwise_fma(yh, bg2[h2], bbt2[h2]);
          const f2 sgm = {sigmoid_f(pre.x), sigmoid_f(pre.y)};
          // silu'(x) = s (1 + x (1 - s))
          const f2 sgr = __builtin_elementwise_fma(sgm, pre * (f2{1.f, 1.f} - sgm), sgm);
          f2 dz;
          if constexpr (DZ16) dz = f2{(float)z4[p][2 * h2], (float)z4[p][2 * h2 + 1]};
          else dz = f2{zf[p][2 * h2], zf[p][2 * h2 + 1]};
          const f2 du = dz * sgr;
          dv = gi2[h2] * (__builtin_elementwise_fma(-yh, bk2_2[h2], du) - bk1_2[h2]);
        } else {
          dv = f2{v4[p][2 * h2], v4[p][2 * h2 + 1]};
        }
        const f2 sgg = {sigmoid_f((float)g4[p][2 * h2]), sigmoid_f((float)g4[p][2 * h2 + 1])};
        const f2 gv = f2{(float)x4[p][2 * h2], (float)x4[p][2 * h2 + 1]} * sgg;
        sg4[p][2 * h2] = sgg.x;
        sg4[p][2 * h2 + 1] = sgg.y;
        d[2 * h2] = ok ? dv.x : 0.f;
        d[2 * h2 + 1] = ok ? dv.y : 0.f;
        g[2 * h2] = ok ? gv.x : 0.f;
        g[2 * h2 + 1] = ok ? gv.y : 0.f;
      }
      *reinterpret_cast<f32x4*>(sdy + r * CT + 4 * q) = d;
      *reinterpret_cast<f32x4*>(sg + r * CT + 4 * q) = g;
    }
  }
  __syncthreads();
  // wave w: frames 16w .. 16w+15; the dy and GLU values they touch (16+K-1 each) in registers
  const int tb = wv * FB;
  float wd[WN], wg[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    wd[j] = sdy[(tb + j) * CT + lane];
    wg[j] = sg[(tb + j) * CT + lane];
  }
  // packed fp32 FMAs (v_pk_fma_f32, two per lane per instruction): dg over frame pairs (f, f+1), dw over tap
  // pairs (k, k+1) -- every output keeps the scalar loop's accumulation order (dg[f] over k, dw[k] over f),
  // so the results are bit-identical
  typedef float f2 __attribute__((ext_vector_type(2)));
  float dw[KT + 1], dg[FB];
#pragma unroll
  for (int k = 0; k <= KT; ++k) dw[k] = 0.f;
#pragma unroll
  for (int f = 0; f < FB; f += 2) {
    f2 s = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const f2 x = {wd[f - k + 2 * PAD], wd[f + 1 - k + 2 * PAD]};
      const f2 w = {wr[k], wr[k]};
      s = __builtin_elementwise_fma(w, x, s);
    }
    dg[f] = s.x;
    dg[f + 1] = s.y;
  }
#pragma unroll
  for (int f = 0; f < FB; ++f) {
    const float dyt = wd[f + PAD];
    const f2 d2 = {dyt, dyt};
#pragma unroll
    for (int k = 0; k + 1 < KT; k += 2) {
      f2 a = {dw[k], dw[k + 1]};
      const f2 x = {wg[f + k], wg[f + k + 1]};
      a = __builtin_elementwise_fma(d2, x, a);
      dw[k] = a.x;
      dw[k + 1] = a.y;
    }
    if constexpr (KT & 1) dw[KT - 1] += dyt * wg[f + KT - 1];
    dw[KT] += dyt;
  }
  __syncthreads();
#pragma unroll
  for (int f = 0; f < FB; ++f) sm[(tb + f) * CT + lane] = dg[f];
  float* red = sm + TT * CT;
#pragma unroll
  for (int k = 0; k <= KT; ++k) red[(wv * (KT + 1) + k) * CT + lane] = dw[k];
  __syncthreads();
  // da of the tile's own rows, from the staging registers of the thread that loaded them
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int r = rs + 16 * p, f = r - PAD, t = t0 + f;
    if (f >= 0 && f < TT && t < T && cok) {
      const f32x4 d = *reinterpret_cast<const f32x4*>(sm + f * CT + 4 * q);
      bf16x4 o1, o2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float sg1 = sg4[p][j];
        o1[j] = (bf16)(d[j] * sg1);
        o2[j] = (bf16)(d[j] * (float)x4[p][j] * sg1 * (1.f - sg1));
      }
      const long row = (long)b * T + t;
      *reinterpret_cast<bf16x4*>(da + row * 2 * C + cq) = o1;
      *reinterpret_cast<bf16x4*>(da + row * 2 * C + C + cq) = o2;
    }
  }
  const long part_idx = (long)b * gridDim.y + blockIdx.y;
  for (int i = tid; i < (KT + 1) * CT; i += 256) {
    const int k = i / CT, l = i % CT;
    const int cc = c0 + l;
    if (cc < C)
      part[(part_idx * (KT + 1) + k) * C + cc] =
          red[k * CT + l] + red[((KT + 1) + k) * CT + l] + red[(2 * (KT + 1) + k) * CT + l] +
          red[(3 * (KT + 1) + k) * CT + l];
  }
}

// sums[k][c] (k <= K) -> dw[c][k], db[c]
__global__ void dwconv_scatter_kernel(const float* __restrict__ sums, int C, int K, float* __restrict__ dw,
                                      float* __restrict__ db) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= C * (K + 1)) return;
  const int k = i / C, c = i % C;
  if (k < K) dw[c * K + k] = sums[i];
  else if (db) db[c] = sums[i];
}

int ew_grid(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

void bn_apply(const float* y, const float* gamma, const float* beta, const float* mean, const float* invstd, void* z,
              int dtz, long M, int C, int act, hipStream_t s) {
  const bool vec = C % 8 == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)z & 15) == 0 &&
                   (dtz == CFM_BF16 || dtz == CFM_F32) && M * C / 8 / 256 < (1L << 31);
  if (vec) {
    const unsigned nb = (unsigned)((M * C / 8 + 255) / 256);
    if (dtz == CFM_BF16)
      hipLaunchKernelGGL(bn_apply_vec8<CFM_BF16>, dim3(nb), dim3(256), 0, s, y, gamma, beta, mean, invstd, z, M, C, act);
    else
      hipLaunchKernelGGL(bn_apply_vec8<CFM_F32>, dim3(nb), dim3(256), 0, s, y, gamma, beta, mean, invstd, z, M, C, act);
    return;
  }
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_grid(M * C)), dim3(256), 0, s, y, gamma, beta, mean, invstd, z, dtz, M, C,
                     act);
}

long conv_nparts(int B, int T) { return (long)B * ((T + TT - 1) / TT); }

// fwd stats from [2][nparts][C] partials at ws; scratch (2C) right after them
void bn_stats_finalize(const float* ws, int nparts, long M, int C, float* mean, float* invstd, float* rm, float* rv,
                       float mom, float eps, hipStream_t s) {
  hipLaunchKernelGGL(bn_stats_kernel, dim3(cdiv(C, 64)), dim3(1024), 0, s, ws, ws + (long)nparts * C, nparts, M, C,
                     mean, invstd, rm, rv, mom, eps);
}

int bn_bwd_impl(const void* dz, int dtdz, const float* y, const float* gamma, const float* beta, const float* mean,
                const float* invstd, int training, int act, float* dy, float* dgamma, float* dbeta, long M, int C,
                float* ws, hipStream_t s) {
  const long rows_per = (M + BN_PARTS - 1) / BN_PARTS;
  hipLaunchKernelGGL(bn_bwd_rows_kernel, dim3(cdiv(C, 64), BN_PARTS), dim3(256), 0, s, dz, dtdz, y, gamma, beta, mean,
                     invstd, M, C, rows_per > 0 ? rows_per : 1, ws, act);
  cfm::colreduce_pair(ws, ws + (long)BN_PARTS * C, BN_PARTS, C, dbeta, dgamma, s);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ew_grid(M * C)), dim3(256), 0, s, dz, dtdz, y, gamma, beta, mean,
                     invstd, dgamma, dbeta, training, dy, M, C, act);
  return CFM_OK;
}

#define CFM_K_CASES(X) X(3) X(5) X(7) X(15) X(31) X(33)
bool g_dwconv_scalar = getenv("CFM_DWCONV_SCALAR") != nullptr;   // A/B: the one-channel-per-lane kernels
}  // namespace

CFM_EXPORT size_t cfm_convmod_ws_bytes(int B, int T, int C, int K) {
  const long np = conv_nparts(B, T);
  const long fwd = 2 * np * C + 2L * C;
  const long bwd = np * (long)C * (K + 1) + (long)C * (K + 1);
  const long bn = 2L * BN_PARTS * C;
  long m = fwd > bwd ? fwd : bwd;
  if (bn > m) m = bn;
  return (size_t)m * sizeof(float);
}

// partial-sum rows of the depthwise conv's weight-gradient partials (for a deferred cfm_colreduce_group task)
CFM_EXPORT long cfm_convmod_nparts(int B, int T) { return conv_nparts(B, T); }

CFM_EXPORT size_t cfm_bn_ws_bytes(int C) { return (size_t)(2L * BN_PARTS * C + 2L * C) * sizeof(float); }

CFM_EXPORT int cfm_glu_dwconv_fwd(const void* a, int dta, const float* w, const float* bias, float* y, int B,
                                  int T, int C, int K, float* ws, void* stream) {
  CFM_REQUIRE(a && w && bias && y && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(K >= 1 && K <= KMAX && (K % 2) == 1, CFM_ERR_UNSUPPORTED, "depthwise kernel must be odd and <= 63");
  CFM_REQUIRE(B > 0 && T > 0 && C > 0, CFM_ERR_SHAPE, "bad shape");
  dim3 grid(cdiv(C, CT), cdiv(T, TT), B);
  const size_t lds = (size_t)(TT + K - 1) * CT * sizeof(float);
  hipStream_t s = cfm::as_stream(stream);
  if (dta == CFM_BF16 && (C % 4) == 0 && !g_dwconv_scalar) {
    switch (K) {
#define X(k) case k: hipLaunchKernelGGL((glu_dwconv_fwd_vec_kernel<k>), grid, dim3(256), 0, s, reinterpret_cast<const bf16*>(a), w, bias, y, T, C, ws); \
                     return cfm::check_launch("cfm_glu_dwconv_fwd");
      CFM_K_CASES(X)
#undef X
      default: break;
    }
  }
  switch (K) {
#define X(k) case k: if (dta == CFM_BF16) hipLaunchKernelGGL((glu_dwconv_fwd_kernel<k, bf16>), grid, dim3(256), lds, s, a, dta, w, bias, y, T, C, K, ws); \
                    else hipLaunchKernelGGL((glu_dwconv_fwd_kernel<k, float>), grid, dim3(256), lds, s, a, dta, w, bias, y, T, C, K, ws); break;
    CFM_K_CASES(X)
#undef X
    default:
      if (dta == CFM_BF16) hipLaunchKernelGGL((glu_dwconv_fwd_kernel<0, bf16>), grid, dim3(256), lds, s, a, dta, w, bias, y, T, C, K, ws);
      else hipLaunchKernelGGL((glu_dwconv_fwd_kernel<0, float>), grid, dim3(256), lds, s, a, dta, w, bias, y, T, C, K, ws);
  }
  return cfm::check_launch("cfm_glu_dwconv_fwd");
}

CFM_EXPORT int cfm_bn_silu_fwd(const float* y, const float* gamma, const float* beta, float* running_mean,
                               float* running_var, float momentum, float eps, int training, float* mean,
                               float* invstd, void* z, int dtz, int B, int T, int C, const float* ws,
                               void* stream) {
  CFM_REQUIRE(y && gamma && beta && mean && invstd && z, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(B > 0 && T > 0 && C > 0, CFM_ERR_SHAPE, "bad shape");
  hipStream_t s = cfm::as_stream(stream);
  const long M = (long)B * T;
  if (training) {
    CFM_REQUIRE(ws, CFM_ERR_ARG, "training mode needs the partial sums of cfm_glu_dwconv_fwd");
    bn_stats_finalize(ws, (int)conv_nparts(B, T), M, C, mean, invstd, running_mean, running_var, momentum, eps, s);
  } else {
    CFM_REQUIRE(running_mean && running_var, CFM_ERR_ARG, "eval mode needs running stats");
    hipLaunchKernelGGL(bn_eval_stats_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, running_mean, running_var, C,
                       eps, mean, invstd);
  }
  bn_apply(y, gamma, beta, mean, invstd, z, dtz, M, C, 1, s);
  return cfm::check_launch("cfm_bn_silu_fwd");
}

CFM_EXPORT int cfm_bn_silu_bwd(const void* dz, int dtdz, const float* y, const float* gamma, const float* beta,
                               const float* mean, const float* invstd, int training, float* dy, float* dgamma,
                               float* dbeta, long M, int C, float* ws, void* stream) {
  CFM_REQUIRE(dz && y && gamma && beta && mean && invstd && dy && dgamma && dbeta && ws, CFM_ERR_ARG,
              "null pointer");
  bn_bwd_impl(dz, dtdz, y, gamma, beta, mean, invstd, training, 1, dy, dgamma, dbeta, M, C, ws,
              cfm::as_stream(stream));
  return cfm::check_launch("cfm_bn_silu_bwd");
}

CFM_EXPORT int cfm_bn_fwd(const float* y, const float* gamma, const float* beta, float* running_mean,
                          float* running_var, float momentum, float eps, int training, float* mean, float* invstd,
                          void* z, int dtz, long M, int C, int act, float* ws, void* stream) {
  CFM_REQUIRE(y && gamma && beta && mean && invstd && z && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(M > 0 && C > 0, CFM_ERR_SHAPE, "bad shape");
  hipStream_t s = cfm::as_stream(stream);
  if (training) {
    const long rows_per = (M + BN_PARTS - 1) / BN_PARTS;
    hipLaunchKernelGGL(bn_stats_rows_kernel, dim3(cdiv(C, 64), BN_PARTS), dim3(256), 0, s, y, M, C,
                       rows_per > 0 ? rows_per : 1, ws);
    bn_stats_finalize(ws, BN_PARTS, M, C, mean, invstd, running_mean, running_var, momentum, eps, s);
  } else {
    CFM_REQUIRE(running_mean && running_var, CFM_ERR_ARG, "eval mode needs running stats");
    hipLaunchKernelGGL(bn_eval_stats_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, running_mean, running_var, C,
                       eps, mean, invstd);
  }
  bn_apply(y, gamma, beta, mean, invstd, z, dtz, M, C, act, s);
  return cfm::check_launch("cfm_bn_fwd");
}

CFM_EXPORT int cfm_bn_bwd(const void* dz, int dtdz, const float* y, const float* gamma, const float* beta,
                          const float* mean, const float* invstd, int training, int act, float* dy, float* dgamma,
                          float* dbeta, long M, int C, float* ws, void* stream) {
  CFM_REQUIRE(dz && y && gamma && beta && mean && invstd && dy && dgamma && dbeta && ws, CFM_ERR_ARG,
              "null pointer");
  bn_bwd_impl(dz, dtdz, y, gamma, beta, mean, invstd, training, act, dy, dgamma, dbeta, M, C, ws,
              cfm::as_stream(stream));
  return cfm::check_launch("cfm_bn_bwd");
}

namespace {

// the vectorised backward for bf16 a/da, C % 4 == 0 and a compiled K; false if not eligible
bool dwconv_bwd_vec(const float* dy, const void* a, int dta, const float* w, void* da, int dtda, int B, int T, int C,
                    int K, float* ws, const BnBwd& bn, bool use_bn, hipStream_t s) {
  if (g_dwconv_scalar || dta != CFM_BF16 || dtda != CFM_BF16 || (C % 4) != 0) return false;
  const bool dz16 = use_bn && bn.dtdz == CFM_BF16;
  dim3 grid(cdiv(C, CT), cdiv(T, TT), B);
  const bf16* ab = reinterpret_cast<const bf16*>(a);
  bf16* dab = reinterpret_cast<bf16*>(da);
  switch (K) {
#define X(k) case k:                                                                                             \
    if (!use_bn) hipLaunchKernelGGL((glu_dwconv_bwd_vec_kernel<k, false, false>), grid, dim3(256), 0, s, dy, ab, w, dab, T, C, ws, bn); \
    else if (dz16) hipLaunchKernelGGL((glu_dwconv_bwd_vec_kernel<k, true, true>), grid, dim3(256), 0, s, dy, ab, w, dab, T, C, ws, bn); \
    else hipLaunchKernelGGL((glu_dwconv_bwd_vec_kernel<k, true, false>), grid, dim3(256), 0, s, dy, ab, w, dab, T, C, ws, bn); \
    return true;
    CFM_K_CASES(X)
#undef X
    default: return false;
  }
}
}  // namespace

CFM_EXPORT int cfm_glu_dwconv_bwd(const float* dy, const void* a, int dta, const float* w, void* da, int dtda,
                                  float* dw, float* db, int B, int T, int C, int K, float* ws, void* stream) {
  CFM_REQUIRE(dy && a && w && da && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(K >= 1 && K <= KMAX && (K % 2) == 1, CFM_ERR_UNSUPPORTED, "depthwise kernel must be odd and <= 63");
  CFM_REQUIRE(B > 0 && T > 0 && C > 0, CFM_ERR_SHAPE, "bad shape");
  dim3 grid(cdiv(C, CT), cdiv(T, TT), B);
  size_t lds = (size_t)2 * (TT + K - 1) * CT * sizeof(float);
  const size_t red = (size_t)4 * (K + 1) * CT * sizeof(float);
  if (red > lds) lds = red;
  hipStream_t s = cfm::as_stream(stream);
  if (!dwconv_bwd_vec(dy, a, dta, w, da, dtda, B, T, C, K, ws, BnBwd{}, false, s)) switch (K) {
#define X(k) case k: if (dta == CFM_BF16) hipLaunchKernelGGL((glu_dwconv_bwd_kernel<k, bf16>), grid, dim3(256), lds, s, dy, a, dta, w, da, dtda, T, C, K, ws, BnBwd{}); \
                    else hipLaunchKernelGGL((glu_dwconv_bwd_kernel<k, float>), grid, dim3(256), lds, s, dy, a, dta, w, da, dtda, T, C, K, ws, BnBwd{}); break;
    CFM_K_CASES(X)
#undef X
    default:
      if (dta == CFM_BF16) hipLaunchKernelGGL((glu_dwconv_bwd_kernel<0, bf16>), grid, dim3(256), lds, s, dy, a, dta, w, da, dtda, T, C, K, ws, BnBwd{});
      else hipLaunchKernelGGL((glu_dwconv_bwd_kernel<0, float>), grid, dim3(256), lds, s, dy, a, dta, w, da, dtda, T, C, K, ws, BnBwd{});
  }
  if (!dw) return cfm::check_launch("cfm_glu_dwconv_bwd");   // weight grads later: cfm_glu_dwconv_bwd_wgrad
  const long np = conv_nparts(B, T);
  float* sums = ws + np * (long)C * (K + 1);
  cfm::colreduce(ws, (int)np, (long)C * (K + 1), sums, 0, s);
  hipLaunchKernelGGL(dwconv_scatter_kernel, dim3(cdiv((long)C * (K + 1), 256)), dim3(256), 0, s, sums, C, K, dw, db);
  return cfm::check_launch("cfm_glu_dwconv_bwd");
}

// the BatchNorm1d + SiLU input gradient folded into the depthwise-conv backward (BnBwd above); dbeta / dgamma are
// the BN parameter gradients of this pass (cfm_bn_silu_bwd_sums, or their all-reduced totals under SyncBN, with
// invM = 1 / rows summed over).  Weight partials as cfm_glu_dwconv_bwd (dw == NULL: deferred).
CFM_EXPORT int cfm_glu_dwconv_bwd_bn(const void* dz, int dtdz, const float* y, const float* gamma, const float* beta,
                                     const float* mean, const float* invstd, const float* dbeta, const float* dgamma,
                                     float invM, int training, const void* a, int dta, const float* w, void* da,
                                     int dtda, float* dw, float* db, int B, int T, int C, int K, float* ws,
                                     void* stream) {
  CFM_REQUIRE(dz && y && gamma && beta && mean && invstd && a && w && da && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(!training || (dbeta && dgamma), CFM_ERR_ARG, "training mode needs dbeta / dgamma");
  CFM_REQUIRE(K >= 1 && K <= KMAX && (K % 2) == 1, CFM_ERR_UNSUPPORTED, "depthwise kernel must be odd and <= 63");
  CFM_REQUIRE(B > 0 && T > 0 && C > 0, CFM_ERR_SHAPE, "bad shape");
  dim3 grid(cdiv(C, CT), cdiv(T, TT), B);
  size_t lds = (size_t)2 * (TT + K - 1) * CT * sizeof(float);
  const size_t red = (size_t)4 * (K + 1) * CT * sizeof(float);
  if (red > lds) lds = red;
  hipStream_t s = cfm::as_stream(stream);
  const BnBwd bn{dz, dtdz, y, gamma, beta, mean, invstd, dgamma, dbeta, invM, training};
  if (!dwconv_bwd_vec(nullptr, a, dta, w, da, dtda, B, T, C, K, ws, bn, true, s)) switch (K) {
#define X(k) case k: if (dta == CFM_BF16) hipLaunchKernelGGL((glu_dwconv_bwd_kernel<k, bf16, true>), grid, dim3(256), lds, s, nullptr, a, dta, w, da, dtda, T, C, K, ws, bn); \
                    else hipLaunchKernelGGL((glu_dwconv_bwd_kernel<k, float, true>), grid, dim3(256), lds, s, nullptr, a, dta, w, da, dtda, T, C, K, ws, bn); break;
    CFM_K_CASES(X)
#undef X
    default:
      return cfm::fail(CFM_ERR_UNSUPPORTED, "cfm_glu_dwconv_bwd_bn: kernel size without a compiled variant");
  }
  if (!dw) return cfm::check_launch("cfm_glu_dwconv_bwd_bn");
  const long np = conv_nparts(B, T);
  float* sums = ws + np * (long)C * (K + 1);
  cfm::colreduce(ws, (int)np, (long)C * (K + 1), sums, 0, s);
  hipLaunchKernelGGL(dwconv_scatter_kernel, dim3(cdiv((long)C * (K + 1), 256)), dim3(256), 0, s, sums, C, K, dw, db);
  return cfm::check_launch("cfm_glu_dwconv_bwd_bn");
}

CFM_EXPORT int cfm_glu_dwconv_bwd_wgrad(float* ws, int B, int T, int C, int K, float* dw, float* db, void* stream) {
  CFM_REQUIRE(ws && dw, CFM_ERR_ARG, "null pointer");
  hipStream_t s = cfm::as_stream(stream);
  const long np = conv_nparts(B, T);
  float* sums = ws + np * (long)C * (K + 1);
  cfm::colreduce(ws, (int)np, (long)C * (K + 1), sums, 0, s);
  hipLaunchKernelGGL(dwconv_scatter_kernel, dim3(cdiv((long)C * (K + 1), 256)), dim3(256), 0, s, sums, C, K, dw, db);
  return cfm::check_launch("cfm_glu_dwconv_bwd_wgrad");
}

// ----------------------------------------------------------------------------- SyncBatchNorm split
// Cross-replica BatchNorm (the ConvModule BN under data parallelism, SURVEY.md §8e caveat): the host
// all-reduces the per-channel sums between the two halves of each pass.
//   fwd: cfm_bn_silu_fwd_sums (sum, sumsq of this rank's rows, from cfm_glu_dwconv_fwd's partials)
//        -> all-reduce -> cfm_bn_silu_fwd_apply (batch stats over M_total rows, running stats, z)
//   bwd: cfm_bn_silu_bwd_sums (sum du, sum du*yhat: this rank's dbeta, dgamma)
//        -> all-reduce a copy -> cfm_bn_silu_bwd_apply (dy with the global sums over M_total rows)
CFM_EXPORT int cfm_bn_silu_fwd_sums(const float* ws, int B, int T, int C, float* sums, void* stream) {
  CFM_REQUIRE(ws && sums && B > 0 && T > 0 && C > 0, CFM_ERR_ARG, "bad args");
  const long np = conv_nparts(B, T);
  cfm::colreduce_pair(ws, ws + np * C, (int)np, C, sums, sums + C, cfm::as_stream(stream));
  return cfm::check_launch("cfm_bn_silu_fwd_sums");
}

CFM_EXPORT int cfm_bn_silu_fwd_apply(const float* y, const float* gamma, const float* beta, float* running_mean,
                                     float* running_var, float momentum, float eps, const float* sums, long M_total,
                                     float* mean, float* invstd, void* z, int dtz, long M, int C, void* stream) {
  CFM_REQUIRE(y && gamma && beta && sums && mean && invstd && z && M_total > 0 && M > 0 && C > 0, CFM_ERR_ARG,
              "bad args");
  hipStream_t s = cfm::as_stream(stream);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, sums, sums + C, M_total, C, mean,
                     invstd, running_mean, running_var, momentum, eps);
  bn_apply(y, gamma, beta, mean, invstd, z, dtz, M, C, 1, s);
  return cfm::check_launch("cfm_bn_silu_fwd_apply");
}

CFM_EXPORT int cfm_bn_silu_bwd_sums(const void* dz, int dtdz, const float* y, const float* gamma, const float* beta,
                                    const float* mean, const float* invstd, long M, int C, float* ws, float* dbeta,
                                    float* dgamma, void* stream) {
  CFM_REQUIRE(dz && y && gamma && beta && mean && invstd && ws && dbeta && dgamma && M > 0 && C > 0, CFM_ERR_ARG,
              "bad args");
  hipStream_t s = cfm::as_stream(stream);
  const long rows_per = (M + BN_PARTS - 1) / BN_PARTS;
  hipLaunchKernelGGL(bn_bwd_rows_kernel, dim3(cdiv(C, 64), BN_PARTS), dim3(256), 0, s, dz, dtdz, y, gamma, beta, mean,
                     invstd, M, C, rows_per > 0 ? rows_per : 1, ws, 1);
  cfm::colreduce_pair(ws, ws + (long)BN_PARTS * C, BN_PARTS, C, dbeta, dgamma, s);
  return cfm::check_launch("cfm_bn_silu_bwd_sums");
}

CFM_EXPORT int cfm_bn_silu_bwd_apply(const void* dz, int dtdz, const float* y, const float* gamma, const float* beta,
                                     const float* mean, const float* invstd, const float* dbeta_total,
                                     const float* dgamma_total, long M_total, float* dy, long M, int C, void* stream) {
  CFM_REQUIRE(dz && y && gamma && beta && mean && invstd && dbeta_total && dgamma_total && dy && M_total > 0,
              CFM_ERR_ARG, "bad args");
  hipLaunchKernelGGL(bn_bwd_apply_total_kernel, dim3(ew_grid(M * C)), dim3(256), 0, cfm::as_stream(stream), dz, dtdz,
                     y, gamma, beta, mean, invstd, dgamma_total, dbeta_total, dy, M, C, 1.f / (float)M_total);
  return cfm::check_launch("cfm_bn_silu_bwd_apply");
}
