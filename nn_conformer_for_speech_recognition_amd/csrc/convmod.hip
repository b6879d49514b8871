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

// backward of y = dwconv(GLU(a)).  grid (ceil(C/CT), ceil(T/TT), B)
// part: [nparts][K+1][C] per-block partial dw (K taps) and db (tap K).
template <int KT, typename TA>
__global__ __launch_bounds__(256) void glu_dwconv_bwd_kernel(const float* __restrict__ dy,
                                                             const void* __restrict__ a, int dta,
                                                             const float* __restrict__ w, void* __restrict__ da,
                                                             int dtda, int T, int C, int Krt,
                                                             float* __restrict__ part) {
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
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int t = min(max(t0 - pad + wv + 4 * i, 0), T - 1);
      const long row = (long)b * T + t;
      dv[i] = dy[row * C + cc];
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

long conv_nparts(int B, int T) { return (long)B * ((T + TT - 1) / TT); }

// fwd stats from [2][nparts][C] partials at ws; scratch (2C) right after them
void bn_stats_finalize(const float* ws, int nparts, long M, int C, float* mean, float* invstd, float* rm, float* rv,
                       float mom, float eps, hipStream_t s) {
  float* sums = const_cast<float*>(ws) + 2L * nparts * C;
  cfm::colreduce_pair(ws, ws + (long)nparts * C, nparts, C, sums, sums + C, s);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, sums, sums + C, M, C, mean, invstd,
                     rm, rv, mom, eps);
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
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_grid(M * C)), dim3(256), 0, s, y, gamma, beta, mean, invstd, z, dtz,
                     M, C, 1);
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
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_grid(M * C)), dim3(256), 0, s, y, gamma, beta, mean, invstd, z, dtz,
                     M, C, act);
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
  switch (K) {
#define X(k) case k: if (dta == CFM_BF16) hipLaunchKernelGGL((glu_dwconv_bwd_kernel<k, bf16>), grid, dim3(256), lds, s, dy, a, dta, w, da, dtda, T, C, K, ws); \
                    else hipLaunchKernelGGL((glu_dwconv_bwd_kernel<k, float>), grid, dim3(256), lds, s, dy, a, dta, w, da, dtda, T, C, K, ws); break;
    CFM_K_CASES(X)
#undef X
    default:
      if (dta == CFM_BF16) hipLaunchKernelGGL((glu_dwconv_bwd_kernel<0, bf16>), grid, dim3(256), lds, s, dy, a, dta, w, da, dtda, T, C, K, ws);
      else hipLaunchKernelGGL((glu_dwconv_bwd_kernel<0, float>), grid, dim3(256), lds, s, dy, a, dta, w, da, dtda, T, C, K, ws);
  }
  if (!dw) return cfm::check_launch("cfm_glu_dwconv_bwd");   // weight grads later: cfm_glu_dwconv_bwd_wgrad
  const long np = conv_nparts(B, T);
  float* sums = ws + np * (long)C * (K + 1);
  cfm::colreduce(ws, (int)np, (long)C * (K + 1), sums, 0, s);
  hipLaunchKernelGGL(dwconv_scatter_kernel, dim3(cdiv((long)C * (K + 1), 256)), dim3(256), 0, s, sums, C, K, dw, db);
  return cfm::check_launch("cfm_glu_dwconv_bwd");
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
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_grid(M * C)), dim3(256), 0, s, y, gamma, beta, mean, invstd, z, dtz,
                     M, C, 1);
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
