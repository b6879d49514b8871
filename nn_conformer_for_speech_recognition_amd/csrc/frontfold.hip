// frontfold.hip — the 'frame'-mode front-end (ConvSubSampling -> per-frame Linear) as ONE linear map.
//
// lib/convsubsampling.py:41-43 applies conv_sub_1 then conv_sub_2 with no activation, no padding and no
// dropout between them, and the 'frame' projection (the standard_linear of asrnn.py:28,208, applied to
// every subsampled frame; dropout comes after it) is linear too.  Their composition is a Ke x Ke conv of
// stride Se (Ke = k1 + (k2-1) s1 = 11, Se = s1 s2 = 4 for the reference's 7x7/s2 + 3x3/s2) followed by the
// per-frame Linear, i.e. one map from an (Ke frames x F mel rows) window to D outputs:
//   W_eff[c2][e][f] = sum_{c1,a,b} W2[c2][c1][a][b] W1[c1][e - s1 a][f - s1 b]        b_eff = b2 + W2 . b1
//   Wfull[o][f][r]  = sum_{f2,c2} Wp[o][f2 C2 + c2] W_eff[c2][r - Se f2][f]            bfull = bp + Wp . b_eff
// (e, r along the mel axis, f along time).  The step then runs ONE GEMM over a strided view of the packed
// input (cfm.h, cfm_ffold_*) instead of conv1 (HBM-bound, 907 MB of h1), conv2 (253 GFLOP) and the
// projection (28 GFLOP), and the backward ONE weight-gradient-shaped GEMM H = G^T X; every parameter
// gradient follows from H and S = colsum(G):
//   dW_eff[c2][e][f] = sum_{o,f2} Wp[o][f2 C2 + c2] H[o][f][Se f2 + e]      db_eff = sum_{o,f2} Wp S
//   dWp[o][f2 C2 + c2] = sum_{e,f} W_eff[c2][e][f] H[o][f][Se f2 + e] + b_eff[c2] S[o]        dbp = S
//   dW2[c2][c1][a][b] = sum_{kh,kw} W1[c1][kh][kw] dW_eff[c2][s1 a + kh][s1 b + kw] + b1[c1] db_eff[c2]
//   dW1[c1][kh][kw]   = sum_{c2,a,b} W2[c2][c1][a][b] dW_eff[c2][s1 a + kh][s1 b + kw]
//   db1[c1] = sum_{c2,a,b} W2[c2][c1][a][b] db_eff[c2]                                          db2 = db_eff
// These contractions are 0.03-0.2 GMAC each: plain fp32 SIMT kernels with LDS-staged operands, every
// reduction done in a fixed order (deterministic, no atomics).
#include "cfm_common.h"

namespace {

struct FG {   // device copy of the geometry
  int B, F, T, C1, C2, D, k1, s1, k2, s2;
  int F2, T2, Ke, Se, Fp, Cx, Kp, nh, Tslot, Ke2;
};

FG dev_geo(const cfm_ffold_geo& g) {
  return FG{g.B, g.F, g.T, g.C1, g.C2, g.D, g.k1, g.s1, g.k2, g.s2, g.F2, g.T2, g.Ke, g.Se, g.Fp, g.Cx, g.Kp,
            g.Cx / g.Fp, g.Tslot, g.Ke * g.Ke};
}

// ------------------------------------------------------------------------------------------- pack
// 32 frames per block: the (F x 32) slab of x is read along time (coalesced), transposed through LDS and
// written as 32 contiguous rows of Cx channels (hi rows of Fp, then lo rows for the bf16 hi/lo split)
constexpr int PF = 32;
template <typename TO>
__global__ __launch_bounds__(256) void ffold_pack_kernel(const float* __restrict__ x, TO* __restrict__ xt, FG g,
                                                         long nframes) {
  extern __shared__ float tile[];   // [PF][F + 1]
  const long f0 = (long)blockIdx.x * PF;
  for (int i = threadIdx.x; i < PF * g.F; i += 256) {
    const int tt = i % PF, r = i / PF;
    const long gt = f0 + tt;
    const long b = gt / g.Tslot, t = gt - b * g.Tslot;
    tile[tt * (g.F + 1) + r] = (b < g.B && t < g.T) ? x[((long)b * g.F + r) * g.T + t] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < PF * g.Cx; i += 256) {
    const int tt = i / g.Cx, c = i - tt * g.Cx;
    const long gt = f0 + tt;
    if (gt >= nframes) continue;
    const int h = c / g.Fp, r = c - h * g.Fp;
    const float v = r < g.F ? tile[tt * (g.F + 1) + r] : 0.f;
    float o = v;
    if constexpr (sizeof(TO) == 2) o = h == 0 ? v : v - (float)(bf16)v;   // lo row: the residual of the hi row
    xt[gt * g.Cx + c] = from_f32<TO>(o);
  }
}

// ------------------------------------------------------------------------------------------- compose
// W_eff partials over 64-channel chunks of conv1: grid (C2, ceil(C1/64)); thread j < Ke^2 -> tap (e, f),
// thread Ke^2 -> the b1 term of b_eff
constexpr int CCH = 64;
__global__ __launch_bounds__(256) void ffold_weff_part_kernel(const float* __restrict__ w1, const float* __restrict__ b1,
                                                              const float* __restrict__ w2, float* __restrict__ part,
                                                              FG g) {
  extern __shared__ float sm[];
  const int k1k1 = g.k1 * g.k1, k2k2 = g.k2 * g.k2;
  float* w2s = sm;                      // [CCH][k2k2]
  float* w1s = w2s + CCH * k2k2;        // [CCH][k1k1]
  float* b1s = w1s + CCH * k1k1;        // [CCH]
  const int c2 = blockIdx.x, c10 = blockIdx.y * CCH, nc = min(CCH, g.C1 - c10);
  for (int i = threadIdx.x; i < nc * k2k2; i += blockDim.x) w2s[i] = w2[((long)c2 * g.C1 + c10) * k2k2 + i];
  for (int i = threadIdx.x; i < nc * k1k1; i += blockDim.x) w1s[i] = w1[(long)c10 * k1k1 + i];
  for (int i = threadIdx.x; i < nc; i += blockDim.x) b1s[i] = b1[c10 + i];
  __syncthreads();
  const int j = threadIdx.x;
  if (j > g.Ke2) return;
  float acc = 0.f;
  if (j < g.Ke2) {
    const int e = j / g.Ke, f = j - e * g.Ke;
    for (int c = 0; c < nc; ++c)
      for (int a = 0; a < g.k2; ++a) {
        const int kh = e - g.s1 * a;
        if (kh < 0 || kh >= g.k1) continue;
        for (int bb = 0; bb < g.k2; ++bb) {
          const int kw = f - g.s1 * bb;
          if (kw < 0 || kw >= g.k1) continue;
          acc += w2s[c * k2k2 + a * g.k2 + bb] * w1s[c * k1k1 + kh * g.k1 + kw];
        }
      }
  } else {
    for (int c = 0; c < nc; ++c) {
      float s = 0.f;
      for (int q = 0; q < k2k2; ++q) s += w2s[c * k2k2 + q];
      acc += s * b1s[c];
    }
  }
  part[((long)blockIdx.y * g.C2 + c2) * (g.Ke2 + 1) + j] = acc;
}

// out[i] = sum_p part[p n + i] in order (+ add[i / (Ke^2+1)] on the bias slots)
__global__ __launch_bounds__(256) void ffold_reduce_kernel(const float* __restrict__ part, int np, int n,
                                                           const float* __restrict__ add, int row,
                                                           float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int p = 0; p < np; ++p) s += part[(long)p * n + i];
  if (add && i % row == row - 1) s += add[i / row];
  out[i] = s;
}

// Wfull / bfull: two output rows o per block; W_eff (+ b_eff column) and the two Wp rows in LDS.  Output
// (f, r): the (f2, e = r - Se f2) pairs with 0 <= e < Ke are f2 = r/Se - jj, jj < ceil(Ke/Se) (a uniform
// trip count; invalid pairs read a clamped address and are discarded)
template <typename TW>
__global__ __launch_bounds__(256) void ffold_wfull_kernel(const float* __restrict__ wp, const float* __restrict__ bp,
                                                          const float* __restrict__ weff, TW* __restrict__ wfull,
                                                          float* __restrict__ bfull, FG g) {
  extern __shared__ float sm[];
  const int R = g.Ke2 + 1, NF = g.F2 * g.C2;
  float* ws = sm;               // [C2][Ke^2 + 1]
  float* wps = ws + g.C2 * R;   // [2][F2 * C2]
  __shared__ float red[2][4];
  const int o0 = blockIdx.x * 2;
  const int nro = min(2, g.D - o0);
  for (int i = threadIdx.x; i < g.C2 * R; i += 256) ws[i] = weff[i];
  for (int i = threadIdx.x; i < 2 * NF; i += 256) {
    const int q = i / NF;
    wps[i] = q < nro ? wp[(long)(o0 + q) * NF + (i - q * NF)] : 0.f;
  }
  __syncthreads();
  const int JJ = (g.Ke + g.Se - 1) / g.Se;
  for (int idx = threadIdx.x; idx < g.Ke * g.Fp; idx += 256) {
    const int f = idx / g.Fp, r = idx - f * g.Fp;
    float a0 = 0.f, a1 = 0.f;
    for (int jj = 0; jj < JJ; ++jj) {
      const int f2 = r / g.Se - jj, e = r - g.Se * f2;
      const bool ok = f2 >= 0 && f2 < g.F2 && e < g.Ke && r < g.F;
      const int f2c = ok ? f2 : 0, ec = ok ? e : 0;
      const float* wcol = ws + ec * g.Ke + f;
      const float* p0 = wps + f2c * g.C2;
      const float* p1 = p0 + NF;
      float t0 = 0.f, t1 = 0.f;
      for (int c2 = 0; c2 < g.C2; ++c2) {
        const float w = wcol[c2 * R];
        t0 += p0[c2] * w;
        t1 += p1[c2] * w;
      }
      if (ok) { a0 += t0; a1 += t1; }
    }
    for (int q = 0; q < nro; ++q)
      for (int h = 0; h < g.nh; ++h)
        wfull[(long)(o0 + q) * g.Kp + f * g.Cx + h * g.Fp + r] = from_f32<TW>(q ? a1 : a0);
  }
  for (int c = g.Ke * g.Cx + threadIdx.x; c < g.Kp; c += 256)
    for (int q = 0; q < nro; ++q) wfull[(long)(o0 + q) * g.Kp + c] = from_f32<TW>(0.f);
  // bfull[o] = bp[o] + sum_{f2,c2} Wp[o][f2 C2 + c2] b_eff[c2]
  float s0 = 0.f, s1 = 0.f;
  for (int i = threadIdx.x; i < NF; i += 256) {
    const float be = ws[(i % g.C2) * R + g.Ke2];
    s0 += wps[i] * be;
    s1 += wps[NF + i] * be;
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) { red[0][wv] = s0; red[1][wv] = s1; }
  __syncthreads();
  if (threadIdx.x < nro) {
    const int q = threadIdx.x;
    bfull[o0 + q] = bp[o0 + q] + ((red[q][0] + red[q][1]) + (red[q][2] + red[q][3]));
  }
}

// ------------------------------------------------------------------------------------------- backward
// H row o as Hs[f * F + r] = sum_h H[o][f Cx + h Fp + r]
__device__ __forceinline__ void load_hrow(const float* __restrict__ H, const FG& g, int o, float* hs, int tid, int nt) {
  for (int i = tid; i < g.Ke * g.F; i += nt) {
    const int f = i / g.F, r = i - f * g.F;
    float v = 0.f;
    if (o < g.D)
      for (int h = 0; h < g.nh; ++h) v += H[(long)o * g.Kp + f * g.Cx + h * g.Fp + r];
    hs[i] = v;
  }
}

// dW_eff / db_eff partials over 16-row chunks of o: grid (ceil(D/16), ceil(C2/16))
constexpr int OB = 16, CB = 16;
__global__ __launch_bounds__(256) void ffold_bwd_part_kernel(const float* __restrict__ H, const float* __restrict__ S,
                                                             const float* __restrict__ wp, float* __restrict__ part,
                                                             FG g) {
  extern __shared__ float sm[];
  const int KF = g.Ke * g.F, R = g.Ke2 + 1, NF = g.F2 * g.C2;
  float* hs = sm;                     // [OB][Ke * F]
  float* wps = hs + OB * KF;          // [OB][F2][CB]
  float* ss = wps + OB * g.F2 * CB;   // [OB]
  const int o0 = blockIdx.x * OB, c0 = blockIdx.y * CB;
  for (int q = 0; q < OB; ++q) load_hrow(H, g, o0 + q, hs + q * KF, threadIdx.x, 256);
  for (int i = threadIdx.x; i < OB * g.F2 * CB; i += 256) {
    const int q = i / (g.F2 * CB), rem = i - q * g.F2 * CB, f2 = rem / CB, cl = rem - f2 * CB;
    const int o = o0 + q, c2 = c0 + cl;
    wps[i] = (o < g.D && c2 < g.C2) ? wp[(long)o * NF + f2 * g.C2 + c2] : 0.f;
  }
  for (int i = threadIdx.x; i < OB; i += 256) ss[i] = o0 + i < g.D ? S[o0 + i] : 0.f;
  __syncthreads();
  for (int idx = threadIdx.x; idx < CB * R; idx += 256) {
    const int cl = idx / R, j = idx - cl * R, c2 = c0 + cl;
    if (c2 >= g.C2) continue;
    float acc = 0.f;
    if (j < g.Ke2) {
      const int e = j / g.Ke, f = j - e * g.Ke;
      for (int q = 0; q < OB; ++q) {
        const float* hrow = hs + q * KF + f * g.F + e;
        const float* wrow = wps + q * g.F2 * CB + cl;
        for (int f2 = 0; f2 < g.F2; ++f2) acc += wrow[f2 * CB] * hrow[g.Se * f2];
      }
    } else {
      for (int q = 0; q < OB; ++q) {
        float t = 0.f;
        for (int f2 = 0; f2 < g.F2; ++f2) t += wps[q * g.F2 * CB + f2 * CB + cl];
        acc += t * ss[q];
      }
    }
    part[((long)blockIdx.x * g.C2 + c2) * R + j] = acc;
  }
}

// dWp rows o0, o0+1 per block (W_eff and the two H rows in LDS); dWp[o][f2 C2 + c2]
__global__ __launch_bounds__(256) void ffold_bwd_wp_kernel(const float* __restrict__ H, const float* __restrict__ S,
                                                           const float* __restrict__ weff, float* __restrict__ dwp,
                                                           FG g) {
  extern __shared__ float sm[];
  const int KF = g.Ke * g.F, R = g.Ke2 + 1, NF = g.F2 * g.C2;
  float* ws = sm;               // [C2][R]
  float* hs = ws + g.C2 * R;    // [2][Ke * F]
  const int o0 = blockIdx.x * 2, nro = min(2, g.D - o0);
  for (int i = threadIdx.x; i < g.C2 * R; i += 256) ws[i] = weff[i];
  load_hrow(H, g, o0, hs, threadIdx.x, 256);
  load_hrow(H, g, o0 + 1, hs + KF, threadIdx.x, 256);
  __syncthreads();
  const float S0 = S[o0], S1 = nro > 1 ? S[o0 + 1] : 0.f;
  for (int idx = threadIdx.x; idx < NF; idx += 256) {
    const int f2 = idx / g.C2, c2 = idx - f2 * g.C2;
    const float* wrow = ws + c2 * R;
    float a0 = 0.f, a1 = 0.f;
    for (int e = 0; e < g.Ke; ++e) {
      const float* h0 = hs + g.Se * f2 + e;
      for (int f = 0; f < g.Ke; ++f) {
        const float w = wrow[e * g.Ke + f];
        a0 += w * h0[f * g.F];
        a1 += w * h0[KF + f * g.F];
      }
    }
    const float be = wrow[g.Ke2];
    dwp[(long)o0 * NF + idx] = a0 + be * S0;
    if (nro > 1) dwp[(long)(o0 + 1) * NF + idx] = a1 + be * S1;
  }
}

// dW2 / db2: one block per c2 (dW_eff row in LDS)
__global__ __launch_bounds__(256) void ffold_bwd_w2_kernel(const float* __restrict__ w1, const float* __restrict__ b1,
                                                           const float* __restrict__ dweff, float* __restrict__ dw2,
                                                           float* __restrict__ db2, FG g) {
  __shared__ float dws[256];
  const int R = g.Ke2 + 1, c2 = blockIdx.x, k1k1 = g.k1 * g.k1, k2k2 = g.k2 * g.k2;
  for (int i = threadIdx.x; i < R; i += 256) dws[i] = dweff[(long)c2 * R + i];
  __syncthreads();
  const float dbe = dws[g.Ke2];
  if (threadIdx.x == 0) db2[c2] = dbe;
  for (int idx = threadIdx.x; idx < g.C1 * k2k2; idx += 256) {
    const int c1 = idx / k2k2, ab = idx - c1 * k2k2, a = ab / g.k2, bb = ab - a * g.k2;
    const float* w1r = w1 + (long)c1 * k1k1;
    float acc = 0.f;
    for (int kh = 0; kh < g.k1; ++kh)
      for (int kw = 0; kw < g.k1; ++kw)
        acc += w1r[kh * g.k1 + kw] * dws[(g.s1 * a + kh) * g.Ke + g.s1 * bb + kw];
    dw2[((long)c2 * g.C1 + c1) * k2k2 + ab] = acc + b1[c1] * dbe;
  }
}

// dW1 / db1: four conv1 channels per block (one wave each); all of dW_eff and the four channels' W2 taps in LDS
__global__ __launch_bounds__(256) void ffold_bwd_w1_kernel(const float* __restrict__ w2, const float* __restrict__ dweff,
                                                           float* __restrict__ dw1, float* __restrict__ db1, FG g) {
  extern __shared__ float sm[];
  const int R = g.Ke2 + 1, k1k1 = g.k1 * g.k1, k2k2 = g.k2 * g.k2;
  float* dws = sm;              // [C2][R]
  float* w2s = dws + g.C2 * R;  // [4][C2][k2k2]
  const int c10 = blockIdx.x * 4;
  for (int i = threadIdx.x; i < g.C2 * R; i += 256) dws[i] = dweff[i];
  for (int i = threadIdx.x; i < 4 * g.C2 * k2k2; i += 256) {
    const int q = i / (g.C2 * k2k2), rem = i - q * g.C2 * k2k2, c2 = rem / k2k2, ab = rem - c2 * k2k2;
    const int c1 = c10 + q;
    w2s[i] = c1 < g.C1 ? w2[((long)c2 * g.C1 + c1) * k2k2 + ab] : 0.f;
  }
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, c1 = c10 + wv;
  if (c1 >= g.C1 || lane > k1k1) return;
  const float* w2c = w2s + wv * g.C2 * k2k2;
  float acc = 0.f;
  if (lane < k1k1) {
    const int kh = lane / g.k1, kw = lane - kh * g.k1;
    for (int c2 = 0; c2 < g.C2; ++c2)
      for (int a = 0; a < g.k2; ++a)
        for (int bb = 0; bb < g.k2; ++bb)
          acc += w2c[c2 * k2k2 + a * g.k2 + bb] * dws[c2 * R + (g.s1 * a + kh) * g.Ke + g.s1 * bb + kw];
    dw1[(long)c1 * k1k1 + lane] = acc;
  } else {
    for (int c2 = 0; c2 < g.C2; ++c2) {
      float t = 0.f;
      for (int q = 0; q < k2k2; ++q) t += w2c[c2 * k2k2 + q];
      acc += t * dws[c2 * R + g.Ke2];
    }
    db1[c1] = acc;
  }
}

constexpr size_t LDS_MAX = 160 * 1024;

size_t wfull_lds(const cfm_ffold_geo& g) { return ((size_t)g.C2 * (g.Ke * g.Ke + 1) + 2 * (size_t)g.F2 * g.C2) * 4; }
size_t part_lds(const cfm_ffold_geo& g) {
  return ((size_t)OB * g.Ke * g.F + (size_t)OB * g.F2 * CB + OB) * 4;
}
size_t wp_lds(const cfm_ffold_geo& g) { return ((size_t)g.C2 * (g.Ke * g.Ke + 1) + 2 * (size_t)g.Ke * g.F) * 4; }
size_t w1_lds(const cfm_ffold_geo& g) {
  return ((size_t)g.C2 * (g.Ke * g.Ke + 1) + 4 * (size_t)g.C2 * g.k2 * g.k2) * 4;
}
int nparts(const cfm_ffold_geo& g) { return cdiv(g.C1, CCH) > cdiv(g.D, OB) ? cdiv(g.C1, CCH) : cdiv(g.D, OB); }

}  // namespace

CFM_EXPORT int cfm_ffold_geometry(cfm_ffold_geo* g) {
  CFM_REQUIRE(g != nullptr, CFM_ERR_ARG, "null geometry");
  CFM_REQUIRE(g->B > 0 && g->F > 0 && g->T > 0 && g->C1 > 0 && g->C2 > 0 && g->D > 0, CFM_ERR_SHAPE, "bad sizes");
  CFM_REQUIRE(g->k1 > 0 && g->s1 > 0 && g->k2 > 0 && g->s2 > 0, CFM_ERR_SHAPE, "bad kernels / strides");
  CFM_REQUIRE(g->dtype == CFM_BF16 || g->dtype == CFM_F32, CFM_ERR_DTYPE, "dtype");
  const int F1 = (g->F - g->k1) / g->s1 + 1, T1 = (g->T - g->k1) / g->s1 + 1;
  CFM_REQUIRE(g->F >= g->k1 && g->T >= g->k1 && F1 >= g->k2 && T1 >= g->k2, CFM_ERR_SHAPE, "input smaller than the kernels");
  g->F2 = (F1 - g->k2) / g->s2 + 1;
  g->T2 = (T1 - g->k2) / g->s2 + 1;
  g->Ke = g->k1 + (g->k2 - 1) * g->s1;
  g->Se = g->s1 * g->s2;
  CFM_REQUIRE(g->Ke * g->Ke + 1 <= 256 && g->k1 * g->k1 + 1 <= 64, CFM_ERR_UNSUPPORTED, "kernel too large");
  const int nh = (g->dtype == CFM_BF16 && g->hilo) ? 2 : 1;
  g->Fp = (g->F + 7) / 8 * 8;
  g->Cx = nh * g->Fp;
  g->Kp = g->dtype == CFM_BF16 ? (g->Ke * g->Cx + 63) / 64 * 64 : g->Ke * g->Cx;
  g->lda = g->Se * g->Cx;
  g->T2p = g->T2 - 1 + (g->Kp + g->lda - 1) / g->lda;
  g->Tslot = g->Se * g->T2p;
  const long slack = (g->Kp + g->Cx - 1) / g->Cx;
  g->xt_elems = ((long)g->B * g->Tslot + slack) * g->Cx;
  const long R = (long)g->C2 * (g->Ke * g->Ke + 1);
  g->ws_floats = R * (2 + nparts(*g));
  CFM_REQUIRE(wfull_lds(*g) <= LDS_MAX && part_lds(*g) <= LDS_MAX && wp_lds(*g) <= LDS_MAX && w1_lds(*g) <= LDS_MAX,
              CFM_ERR_UNSUPPORTED, "front-end fold: LDS staging exceeds 160 KiB");
  CFM_REQUIRE((long)g->B * g->Tslot * g->Cx * (g->dtype == CFM_BF16 ? 2 : 4) < (1L << 31), CFM_ERR_SHAPE,
              "packed input >= 2 GiB");
  return CFM_OK;
}

CFM_EXPORT int cfm_ffold_pack(const float* x, void* xt, const cfm_ffold_geo* g, void* stream) {
  CFM_REQUIRE(x && xt && g, CFM_ERR_ARG, "null pointer");
  const FG d = dev_geo(*g);
  const long nframes = g->xt_elems / g->Cx;
  const dim3 grid((unsigned)((nframes + PF - 1) / PF));
  const size_t lds = (size_t)PF * (g->F + 1) * 4;
  hipStream_t s = cfm::as_stream(stream);
  if (g->dtype == CFM_BF16)
    hipLaunchKernelGGL(ffold_pack_kernel<bf16>, grid, dim3(256), lds, s, x, (bf16*)xt, d, nframes);
  else
    hipLaunchKernelGGL(ffold_pack_kernel<float>, grid, dim3(256), lds, s, x, (float*)xt, d, nframes);
  return cfm::check_launch("cfm_ffold_pack");
}

CFM_EXPORT int cfm_ffold_compose(const float* w1, const float* b1, const float* w2, const float* b2, const float* wp,
                                 const float* bp, void* wfull, float* bfull, float* ws, const cfm_ffold_geo* g,
                                 void* stream) {
  CFM_REQUIRE(w1 && b1 && w2 && b2 && wp && bp && wfull && bfull && ws && g, CFM_ERR_ARG, "null pointer");
  const FG d = dev_geo(*g);
  hipStream_t s = cfm::as_stream(stream);
  const int R = g->Ke * g->Ke + 1, n = g->C2 * R;
  float* weff = ws;
  float* part = ws + 2 * (long)n;
  const int ns = cdiv(g->C1, CCH);
  const size_t lds1 = ((size_t)CCH * (g->k2 * g->k2 + g->k1 * g->k1) + CCH) * 4;
  hipLaunchKernelGGL(ffold_weff_part_kernel, dim3(g->C2, ns), dim3(R <= 128 ? 128 : 256), lds1, s, w1, b1, w2, part, d);
  hipLaunchKernelGGL(ffold_reduce_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, part, ns, n, b2, R, weff);
  if (g->dtype == CFM_BF16)
    hipLaunchKernelGGL(ffold_wfull_kernel<bf16>, dim3(cdiv(g->D, 2)), dim3(256), wfull_lds(*g), s, wp, bp, weff,
                       (bf16*)wfull, bfull, d);
  else
    hipLaunchKernelGGL(ffold_wfull_kernel<float>, dim3(cdiv(g->D, 2)), dim3(256), wfull_lds(*g), s, wp, bp, weff,
                       (float*)wfull, bfull, d);
  return cfm::check_launch("cfm_ffold_compose");
}

CFM_EXPORT int cfm_ffold_bwd_weights(const float* H, const float* S, const float* w1, const float* b1, const float* w2,
                                     const float* wp, float* ws, float* dw1, float* db1, float* dw2, float* db2,
                                     float* dwp, const cfm_ffold_geo* g, void* stream) {
  CFM_REQUIRE(H && S && w1 && b1 && w2 && wp && ws && dw1 && db1 && dw2 && db2 && dwp && g, CFM_ERR_ARG,
              "null pointer");
  const FG d = dev_geo(*g);
  hipStream_t s = cfm::as_stream(stream);
  const int R = g->Ke * g->Ke + 1, n = g->C2 * R;
  const float* weff = ws;
  float* dweff = ws + n;
  float* part = ws + 2 * (long)n;
  const int nob = cdiv(g->D, OB);
  hipLaunchKernelGGL(ffold_bwd_part_kernel, dim3(nob, cdiv(g->C2, CB)), dim3(256), part_lds(*g), s, H, S, wp, part, d);
  hipLaunchKernelGGL(ffold_reduce_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, part, nob, n, nullptr, R, dweff);
  hipLaunchKernelGGL(ffold_bwd_wp_kernel, dim3(cdiv(g->D, 2)), dim3(256), wp_lds(*g), s, H, S, weff, dwp, d);
  hipLaunchKernelGGL(ffold_bwd_w2_kernel, dim3(g->C2), dim3(256), 0, s, w1, b1, dweff, dw2, db2, d);
  hipLaunchKernelGGL(ffold_bwd_w1_kernel, dim3(cdiv(g->C1, 4)), dim3(256), w1_lds(*g), s, w2, dweff, dw1, db1, d);
  return cfm::check_launch("cfm_ffold_bwd_weights");
}
