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
// These contractions are 0.03-0.2 GMAC each: fp32 GEMMs on cfm_gemm's exact-f32 MFMA path (deterministic
// split-K slabs, no atomics) over re-indexed views, with elementwise gathers between them.
#include "cfm_common.h"

namespace {

struct FG {   // device copy of the geometry
  int B, F, T, C1, C2, D, k1, s1, k2, s2;
  int F2, T2, Ke, Se, Fp, Cx, Kp, nh, Tslot, Ke2;
  int n1, n2;   // padded row lengths (multiples of 4) of the tap + bias tables: k1^2 + 1 -> n1, Ke^2 + 1 -> n2
};
inline int pad4(int n) { return (n + 3) / 4 * 4; }

FG dev_geo(const cfm_ffold_geo& g) {
  return FG{g.B, g.F, g.T, g.C1, g.C2, g.D, g.k1, g.s1, g.k2, g.s2, g.F2, g.T2, g.Ke, g.Se, g.Fp, g.Cx, g.Kp,
            g.Cx / g.Fp, g.Tslot, g.Ke * g.Ke, pad4(g.k1 * g.k1 + 1), pad4(g.Ke * g.Ke + 1)};
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
// The contractions run as fp32 GEMMs on the exact-f32 MFMA path of cfm_gemm over re-indexed views, with
// elementwise gathers between them (n1 = 52 columns: the k1^2 = 49 conv1 taps, the bias, zero padding to a
// multiple of 4 for the split-K reduction; n2 = 124: the Ke^2 = 121 taps, the bias, padding):
//   P    (C2*k2^2 x n1)    = W2t^T W1e            W2t = W2 as (C1 x C2 k2^2), W1e = [W1 | b1] (C1 x n1)
//   Weff (C2 x n2)         = gather(P) (+ b2)     the conv composition; column Ke^2 = b_eff
//   Q    (D*F2 x n2)       = Wp' Weff^T            Wp' = Wp viewed as (D F2 x C2)
//   Wfull, bfull           = gather(Q) (+ bp)
// backward:
//   Hg   (D*F2 x n2)       = gather(H) | S        Hg[(o,f2)][(e,f)] = H[o][f][Se f2 + e], column Ke^2 = S[o]
//   dWeff (C2 x n2)        = Wp'^T Hg             (split-K slabs; column Ke^2 = db_eff)
//   dWp  (D*F2 x C2)       = Hg Weff^T            (= dWp (D x F2 C2) in its own layout)
//   Gd   (C2*k2^2 x n1)    = gather(dWeff)        Gd[(c2,a,b)][(kh,kw)] = dWeff[c2][s1 a + kh][s1 b + kw], | db_eff
//   dW2  (C2 x C1 x k2^2)  = per c2: W1e Gd_c2^T  (written in the reference layout)
//   W1o  (C1 x n1)         = W2t Gd               -> dW1 = W1o[:, :49], db1 = W1o[:, 49]

// W2 (C2, C1, k2^2) -> W2t (C1, C2 k2^2); W1 (C1, k1^2), b1 -> W1e (C1, n1)
__global__ __launch_bounds__(256) void ffold_prep_kernel(const float* __restrict__ w1, const float* __restrict__ b1,
                                                         const float* __restrict__ w2, float* __restrict__ w2t,
                                                         float* __restrict__ w1e, FG g) {
  const int k1k1 = g.k1 * g.k1, k2k2 = g.k2 * g.k2, n1 = g.n1, n2t = g.C2 * k2k2;
  const long nt = (long)g.C1 * n2t, ne = (long)g.C1 * n1;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nt + ne; i += (long)gridDim.x * 256) {
    if (i < nt) {
      const int c1 = (int)(i / n2t), rem = (int)(i - (long)c1 * n2t), c2 = rem / k2k2, ab = rem - c2 * k2k2;
      w2t[i] = w2[((long)c2 * g.C1 + c1) * k2k2 + ab];
    } else {
      const long j = i - nt;
      const int c1 = (int)(j / n1), t = (int)(j - (long)c1 * n1);
      w1e[j] = t < k1k1 ? w1[(long)c1 * k1k1 + t] : (t == k1k1 ? b1[c1] : 0.f);
    }
  }
}

// Weff[c2][(e,f)] = sum_{a,b valid} P[(c2,a,b)][(e - s1 a) k1 + f - s1 b];  Weff[c2][Ke^2] = b2 + sum_ab P[.][k1^2]
__global__ __launch_bounds__(256) void ffold_weff_kernel(const float* __restrict__ P, const float* __restrict__ b2,
                                                         float* __restrict__ weff, FG g) {
  const int n1 = g.n1, n2 = g.n2, k2k2 = g.k2 * g.k2, k1k1 = g.k1 * g.k1;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= g.C2 * n2) return;
  const int c2 = i / n2, j = i - c2 * n2;
  const float* pc = P + (long)c2 * k2k2 * n1;
  float acc = 0.f;
  if (j < g.Ke2) {
    const int e = j / g.Ke, f = j - e * g.Ke;
    for (int a = 0; a < g.k2; ++a) {
      const int kh = e - g.s1 * a;
      if (kh < 0 || kh >= g.k1) continue;
      for (int bb = 0; bb < g.k2; ++bb) {
        const int kw = f - g.s1 * bb;
        if (kw >= 0 && kw < g.k1) acc += pc[(a * g.k2 + bb) * n1 + kh * g.k1 + kw];
      }
    }
  } else if (j == g.Ke2) {
    acc = b2[c2];
    for (int ab = 0; ab < k2k2; ++ab) acc += pc[ab * n1 + k1k1];
  }
  weff[i] = acc;
}

// Wfull[o][f Cx + h Fp + r] = sum_{f2: 0 <= r - Se f2 < Ke} Q[(o,f2)][(r - Se f2) Ke + f] (zero past Ke Cx);
// bfull[o] = bp[o] + sum_f2 Q[(o,f2)][Ke^2].  One thread per (o, column < Kp)
template <typename TW>
__global__ __launch_bounds__(256) void ffold_wfull_kernel(const float* __restrict__ Q, const float* __restrict__ bp,
                                                          TW* __restrict__ wfull, float* __restrict__ bfull, FG g) {
  const int n2 = g.n2;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)g.D * g.Kp) return;
  const int o = (int)(i / g.Kp), col = (int)(i - (long)o * g.Kp);
  const float* qo = Q + (long)o * g.F2 * n2;
  if (col == 0) {
    float s = bp[o];
    for (int f2 = 0; f2 < g.F2; ++f2) s += qo[f2 * n2 + g.Ke2];
    bfull[o] = s;
  }
  float acc = 0.f;
  if (col < g.Ke * g.Cx) {
    const int f = col / g.Cx, r = (col - f * g.Cx) % g.Fp;
    if (r < g.F) {
      const int f2hi = min(r / g.Se, g.F2 - 1);
      for (int f2 = f2hi; f2 >= 0 && r - g.Se * f2 < g.Ke; --f2) acc += qo[f2 * n2 + (r - g.Se * f2) * g.Ke + f];
    }
  }
  wfull[i] = from_f32<TW>(acc);
}

// ------------------------------------------------------------------------------------------- backward gathers
// Hg[(o,f2)][(e,f)] = sum_h H[o][f Cx + h Fp + Se f2 + e];  Hg[(o,f2)][Ke^2] = S[o]
__global__ __launch_bounds__(256) void ffold_hg_kernel(const float* __restrict__ H, const float* __restrict__ S,
                                                       float* __restrict__ hg, FG g) {
  const int n2 = g.n2;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)g.D * g.F2 * n2) return;
  const int row = (int)(i / n2), j = (int)(i - (long)row * n2), o = row / g.F2, f2 = row - o * g.F2;
  float v;
  if (j < g.Ke2) {
    const int e = j / g.Ke, f = j - e * g.Ke;
    const float* h = H + (long)o * g.Kp + f * g.Cx + g.Se * f2 + e;
    v = 0.f;
    for (int q = 0; q < g.nh; ++q) v += h[q * g.Fp];
  } else {
    v = j == g.Ke2 ? S[o] : 0.f;
  }
  hg[i] = v;
}

// Gd[(c2,a,b)][(kh,kw)] = dWeff[c2][(s1 a + kh) Ke + s1 b + kw];  Gd[.][k1^2] = db_eff[c2] (= db2)
__global__ __launch_bounds__(256) void ffold_gd_kernel(const float* __restrict__ dweff, float* __restrict__ gd,
                                                       float* __restrict__ db2, FG g) {
  const int n1 = g.n1, n2 = g.n2, k2k2 = g.k2 * g.k2, k1k1 = g.k1 * g.k1;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= g.C2 * k2k2 * n1) return;
  const int row = i / n1, t = i - row * n1, c2 = row / k2k2, ab = row - c2 * k2k2, a = ab / g.k2, bb = ab - a * g.k2;
  const float* dw = dweff + (long)c2 * n2;
  if (t < k1k1) {
    const int kh = t / g.k1, kw = t - kh * g.k1;
    gd[i] = dw[(g.s1 * a + kh) * g.Ke + g.s1 * bb + kw];
  } else if (t == k1k1) {
    gd[i] = dw[g.Ke2];
    if (ab == 0) db2[c2] = dw[g.Ke2];
  } else {
    gd[i] = 0.f;
  }
}

// dW2[c2][c1][ab] = dW2t[c1][c2 k2^2 + ab]
__global__ __launch_bounds__(256) void ffold_dw2_kernel(const float* __restrict__ w2g, float* __restrict__ dw2, FG g) {
  const int k2k2 = g.k2 * g.k2;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)g.C1 * g.C2 * k2k2) return;
  const int c2 = (int)(i / ((long)g.C1 * k2k2)), rem = (int)(i - (long)c2 * g.C1 * k2k2), c1 = rem / k2k2,
            ab = rem - c1 * k2k2;
  dw2[i] = w2g[(long)c1 * g.C2 * k2k2 + c2 * k2k2 + ab];
}

// W1o (C1 x n1) -> dw1 (C1 x k1^2), db1 (C1)
__global__ __launch_bounds__(256) void ffold_w1_split_kernel(const float* __restrict__ w1o, float* __restrict__ dw1,
                                                             float* __restrict__ db1, FG g) {
  const int n1 = g.n1, k1k1 = g.k1 * g.k1;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= g.C1 * n1) return;
  const int c1 = i / n1, t = i - c1 * n1;
  if (t < k1k1) dw1[(long)c1 * k1k1 + t] = w1o[i];
  else if (t == k1k1) db1[c1] = w1o[i];
}

// workspace layout (floats), shared by compose and the backward (W2t, W1e and Weff persist in between)
struct WsLayout {
  long w2t, w1e, P, weff, Q, dweff, gd, w1o, w2g, slab, total;
};
WsLayout ws_layout(const cfm_ffold_geo& g) {
  const long n1 = pad4(g.k1 * g.k1 + 1), n2 = pad4(g.Ke * g.Ke + 1), k2k2 = (long)g.k2 * g.k2;
  WsLayout L;
  long o = 0;
  auto take = [&](long n) { const long r = o; o += (n + 63) / 64 * 64; return r; };
  L.w2t = take((long)g.C1 * g.C2 * k2k2);
  L.w1e = take((long)g.C1 * n1);
  L.P = take((long)g.C2 * k2k2 * n1);
  L.weff = take((long)g.C2 * n2);
  L.Q = take((long)g.D * g.F2 * n2);            // forward Q / backward Hg
  L.dweff = take((long)g.C2 * n2);
  L.gd = take((long)g.C2 * k2k2 * n1);
  L.w1o = take((long)g.C1 * n1);
  L.w2g = take((long)g.C1 * g.C2 * k2k2);
  const long sC = 64L * g.C2 * n2, sF = 16L * g.C1 * n1, sP = 8L * g.C2 * k2k2 * n1;
  L.slab = take(std::max(sC, std::max(sF, sP)));
  L.total = o;
  return L;
}

// fp32 GEMM through the C ABI (exact-f32 MFMA path)
int f32gemm(int M, int N, int K, const float* A, long lda, int akm, const float* B, long ldb, int bkm, float* C,
            long ldc, int batch, long sa, long sb, long sc, int split, float* slab, hipStream_t s) {
  cfm_gemm_desc d{};
  d.M = M; d.N = N; d.K = K; d.batch = batch; d.dtype_ab = CFM_F32;
  d.A = A; d.lda = lda; d.stride_a = sa; d.a_kmajor = akm;
  d.B = B; d.ldb = ldb; d.stride_b = sb; d.b_kmajor = bkm;
  d.C = C; d.ldc = ldc; d.stride_c = sc; d.dtype_c = CFM_F32;
  d.alpha = 1.f; d.out_scale = 1.f; d.ldr = N; d.dtype_pre = CFM_F32; d.dtype_r = CFM_F32;
  d.split_k = split; d.workspace = split > 1 ? slab : nullptr;
  return cfm_gemm(&d, (void*)s);
}

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
  g->ws_floats = ws_layout(*g).total;
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
  const WsLayout L = ws_layout(*g);
  const int n1 = d.n1, n2 = d.n2, k2k2 = g->k2 * g->k2;
  const long nprep = (long)g->C1 * (g->C2 * k2k2 + n1);
  hipLaunchKernelGGL(ffold_prep_kernel, dim3((unsigned)std::min<long>(cdiv(nprep, 256), 2048)), dim3(256), 0, s, w1,
                     b1, w2, ws + L.w2t, ws + L.w1e, d);
  // P (C2 k2^2 x n1) = sum_c1 W2t[c1][(c2,ab)] W1e[c1][t]: A, B MN-major over k = c1
  const int splitP = std::max(1, std::min(8, g->C1 / 64));
  int rc = f32gemm(g->C2 * k2k2, n1, g->C1, ws + L.w2t, (long)g->C2 * k2k2, 0, ws + L.w1e, n1, 0, ws + L.P, n1, 1, 0,
                   0, 0, splitP, ws + L.slab, s);
  if (rc != CFM_OK) return rc;
  hipLaunchKernelGGL(ffold_weff_kernel, dim3(cdiv(g->C2 * n2, 256)), dim3(256), 0, s, ws + L.P, b2, ws + L.weff, d);
  // Q (D F2 x n2) = Wp' (D F2 x C2, K-major) Weff (C2 x n2: MN-major B over k = c2)
  rc = f32gemm(g->D * g->F2, n2, g->C2, wp, g->C2, 1, ws + L.weff, n2, 0, ws + L.Q, n2, 1, 0, 0, 0, 1, nullptr, s);
  if (rc != CFM_OK) return rc;
  const long nw = (long)g->D * g->Kp;
  if (g->dtype == CFM_BF16)
    hipLaunchKernelGGL(ffold_wfull_kernel<bf16>, dim3((unsigned)cdiv(nw, 256)), dim3(256), 0, s, ws + L.Q, bp,
                       (bf16*)wfull, bfull, d);
  else
    hipLaunchKernelGGL(ffold_wfull_kernel<float>, dim3((unsigned)cdiv(nw, 256)), dim3(256), 0, s, ws + L.Q, bp,
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
  const WsLayout L = ws_layout(*g);
  const int n1 = d.n1, n2 = d.n2, k2k2 = g->k2 * g->k2;
  const long nhg = (long)g->D * g->F2 * n2;
  float* hg = ws + L.Q;
  hipLaunchKernelGGL(ffold_hg_kernel, dim3((unsigned)cdiv(nhg, 256)), dim3(256), 0, s, H, S, hg, d);
  // dWeff (C2 x n2) = sum_{(o,f2)} Wp'[(o,f2)][c2] Hg[(o,f2)][n]: both MN-major over k = (o, f2), split-K slabs
  const int KC = g->D * g->F2;
  const int splitC = std::max(1, std::min(64, KC / 256));
  int rc = f32gemm(g->C2, n2, KC, wp, g->C2, 0, hg, n2, 0, ws + L.dweff, n2, 1, 0, 0, 0, splitC, ws + L.slab, s);
  if (rc != CFM_OK) return rc;
  // dWp (D F2 x C2) = Hg (K-major, k = n) Weff^T (K-major)
  rc = f32gemm(KC, g->C2, n2, hg, n2, 1, ws + L.weff, n2, 1, dwp, g->C2, 1, 0, 0, 0, 1, nullptr, s);
  if (rc != CFM_OK) return rc;
  hipLaunchKernelGGL(ffold_gd_kernel, dim3(cdiv(g->C2 * k2k2 * n1, 256)), dim3(256), 0, s, ws + L.dweff, ws + L.gd,
                     db2, d);
  // dW2t (C1 x C2 k2^2) = W1e (C1 x n1, K-major) Gd^T (Gd: (C2 k2^2) x n1, K-major); then dW2 = its permute
  rc = f32gemm(g->C1, g->C2 * k2k2, n1, ws + L.w1e, n1, 1, ws + L.gd, n1, 1, ws + L.w2g, (long)g->C2 * k2k2, 1, 0, 0,
               0, 1, nullptr, s);
  if (rc != CFM_OK) return rc;
  hipLaunchKernelGGL(ffold_dw2_kernel, dim3(cdiv((long)g->C1 * g->C2 * k2k2, 256)), dim3(256), 0, s, ws + L.w2g, dw2, d);
  // W1o (C1 x n1) = W2t (C1 x C2 k2^2, K-major) Gd ((C2 k2^2) x n1: MN-major B over k = (c2, ab))
  const int KF = g->C2 * k2k2;
  const int splitF = std::max(1, std::min(16, KF / 64));
  rc = f32gemm(g->C1, n1, KF, ws + L.w2t, KF, 1, ws + L.gd, n1, 0, ws + L.w1o, n1, 1, 0, 0, 0, splitF, ws + L.slab, s);
  if (rc != CFM_OK) return rc;
  hipLaunchKernelGGL(ffold_w1_split_kernel, dim3(cdiv(g->C1 * n1, 256)), dim3(256), 0, s, ws + L.w1o, dw1, db1, d);
  return cfm::check_launch("cfm_ffold_bwd_weights");
}
