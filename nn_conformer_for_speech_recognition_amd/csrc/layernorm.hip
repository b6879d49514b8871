// layernorm.hip — nn.LayerNorm(D) forward/backward over token rows (one wave per row).
//
// Used by every LayerNorm of the torchaudio ConformerLayer (ffn*.sequential.0,
// self_attn_layer_norm, conv_module.layer_norm, final_layer_norm).  The residual stream is
// fp32; the normalised output feeds the next GEMM in the compute dtype (bf16 or fp32).
// Backward fuses the residual-gradient add (dx = LN'(dy) + dres) and produces dgamma/dbeta
// through per-workgroup partial rows reduced by cfm::colreduce (deterministic, no atomics).
// Fast path (D = 64*V, fp32 residual stream): each lane owns V contiguous features, so every
// load/store is a 16-B vector; other shapes/dtypes take the generic strided path.
#include "cfm_common.h"

namespace {
constexpr int MAXJ = 16;   // D <= 1024

// ---------------------------------------------------------------- vector helpers (V per lane)
template <int V> __device__ __forceinline__ void ldv(const float* p, float (&o)[V]) {
  if constexpr (V % 4 == 0) {
#pragma unroll
    for (int i = 0; i < V / 4; ++i) {
      const float4 a = reinterpret_cast<const float4*>(p)[i];
      o[4 * i] = a.x; o[4 * i + 1] = a.y; o[4 * i + 2] = a.z; o[4 * i + 3] = a.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = p[i];
  }
}
template <int V> __device__ __forceinline__ void ldv(const bf16* p, float (&o)[V]) {
  if constexpr (V % 8 == 0) {
#pragma unroll
    for (int i = 0; i < V / 8; ++i) {
      const bf16x8 b = __builtin_bit_cast(bf16x8, reinterpret_cast<const uint4*>(p)[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[8 * i + e] = (float)b[e];
    }
  } else if constexpr (V == 4) {
    const bf16x4 b = __builtin_bit_cast(bf16x4, *reinterpret_cast<const uint2*>(p));
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (float)b[e];
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = (float)p[i];
  }
}
template <int V> __device__ __forceinline__ void stv(float* p, const float (&v)[V]) {
  if constexpr (V % 4 == 0) {
#pragma unroll
    for (int i = 0; i < V / 4; ++i)
      reinterpret_cast<float4*>(p)[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) p[i] = v[i];
  }
}
template <int V> __device__ __forceinline__ void stv(bf16* p, const float (&v)[V]) {
  if constexpr (V % 8 == 0) {
#pragma unroll
    for (int i = 0; i < V / 8; ++i) {
      bf16x8 b;
#pragma unroll
      for (int e = 0; e < 8; ++e) b[e] = (bf16)v[8 * i + e];
      reinterpret_cast<uint4*>(p)[i] = __builtin_bit_cast(uint4, b);
    }
  } else if constexpr (V == 4) {
    bf16x4 b;
#pragma unroll
    for (int e = 0; e < 4; ++e) b[e] = (bf16)v[e];
    *reinterpret_cast<uint2*>(p) = __builtin_bit_cast(uint2, b);
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) p[i] = (bf16)v[i];
  }
}

// ---------------------------------------------------------------- vectorised kernels
// LN_FWD_ROWS rows per wave: every row's load is issued before the first reduction, so a wave keeps
// that many 2-KB row reads in flight (one row per wave left the kernel latency-bound at ~50 % of HBM)
constexpr int LN_FWD_ROWS = 2;
// MX: a second output of the bf16 y -- its MX e4m3 copy (cfm_quant_mx's bytes and block scales of the bf16 values,
// for the fp8 forward GEMM that consumes it): the 32 / V lanes of a 32-feature block exchange their maxima by xor
// shuffles, so the copy costs its 1.03 bytes per element of stores instead of a separate 3-byte pass.
struct LnMx {
  uint8_t* y8;    // M x D e4m3
  uint8_t* s8;    // M x D/32 e8m0
};
__device__ __forceinline__ int ln_mx_k(float a) {   // = fp8.hip mx_k
  if (!(a > 0.f) || !(a < INFINITY)) return 0;
  int e;
  const float m = 2.f * frexpf(a, &e);
  const int k = (m <= 1.75f ? 8 : 7) - (e - 1);
  return k < 126 ? (k > -126 ? k : -126) : 126;
}
template <int V>
__device__ __forceinline__ void ln_store_mx(const LnMx& mx, long row, int D, int lane, const float (&v)[V]) {
  constexpr int LPB = 32 / V;       // lanes per 32-feature block
  float q[V], m = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    q[i] = (float)(bf16)v[i];       // the bf16 value the GEMM would otherwise read
    m = fmaxf(m, fabsf(q[i]));
  }
#pragma unroll
  for (int o = 1; o < LPB; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const int k = ln_mx_k(m);
  const float sc = ldexpf(1.f, k);
  uint8_t* yp = mx.y8 + row * D + lane * V;
#pragma unroll
  for (int i = 0; i < V; i += 4) {
    int w = 0;
    w = __builtin_amdgcn_cvt_pk_fp8_f32(q[i] * sc, q[i + 1] * sc, w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(q[i + 2] * sc, q[i + 3] * sc, w, true);
    *reinterpret_cast<int*>(yp + i) = w;
  }
  if (lane % LPB == 0) mx.s8[row * (D / 32) + lane / LPB] = (uint8_t)(127 - k);
}

// RS: the residual add of the module before this LayerNorm moved in here (cfm_layernorm_fwd_res): the row is
// x + delta (delta: that module's bf16 output -- bias, dropout and out_scale applied by its GEMM's epilogue), stored
// to xo (the fp32 residual stream the backward reads) and normalised.  The GEMM then writes 2 B per element instead of
// reading and writing the 4-B stream in an epilogue nothing overlaps; the bytes move into this streaming pass.
struct LnRes {
  const bf16* d;   // M x D delta
  float* xo;       // M x D: x + delta
};

template <int V, typename TY, bool MX = false, typename TX = float, bool RS = false>
__global__ __launch_bounds__(256) void ln_fwd_vec(const TX* __restrict__ x, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, TY* __restrict__ y,
                                                  float* __restrict__ mean_out, float* __restrict__ rstd_out, long M,
                                                  float eps, LnMx mx = {}, LnRes rs = {}) {
  constexpr int D = 64 * V, R = LN_FWD_ROWS;
  const int lane = threadIdx.x & 63;
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= M) return;
  float v[R][V], g[V], b[V];
  [[maybe_unused]] float dl[RS ? R : 1][RS ? V : 1];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (row0 + r < M) {
      ldv<V>(x + (row0 + r) * D + lane * V, v[r]);
      if constexpr (RS) ldv<V>(rs.d + (row0 + r) * D + lane * V, dl[r]);
    } else {
#pragma unroll
      for (int i = 0; i < V; ++i) v[r][i] = 0.f;
      if constexpr (RS) {
#pragma unroll
        for (int i = 0; i < V; ++i) dl[r][i] = 0.f;
      }
    }
  }
  if constexpr (RS) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int i = 0; i < V; ++i) v[r][i] += dl[r][i];
      if (row0 + r < M) stv<V>(rs.xo + (row0 + r) * D + lane * V, v[r]);
    }
  }
  ldv<V>(gamma + lane * V, g);
  ldv<V>(beta + lane * V, b);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) s += v[r][i];
    const float mean = wave_sum(s) * (1.f / D);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      v[r][i] -= mean;
      q += v[r][i] * v[r][i];
    }
    const float rstd = rsqrtf(wave_sum(q) * (1.f / D) + eps);
    if (row0 + r < M) {    // wave-uniform
#pragma unroll
      for (int i = 0; i < V; ++i) v[r][i] = v[r][i] * rstd * g[i] + b[i];
      stv<V>(y + (row0 + r) * D + lane * V, v[r]);
      if constexpr (MX) ln_store_mx<V>(mx, row0 + r, D, lane, v[r]);
      if (lane == 0) {
        mean_out[row0 + r] = mean;
        rstd_out[row0 + r] = rstd;
      }
    }
  }
}

// optional fused second output of the vectorised backward: g2 = bf16(dx * scale * dropout(p, seed))
struct LnDrop {
  void* g2;
  float scale, p;
  uint64_t seed;
  const uint64_t* salt;
};

template <int V, typename TDY, typename TX = float>
__global__ __launch_bounds__(256) void ln_bwd_vec(const TDY* __restrict__ dy, const TX* __restrict__ x,
                                                  const float* __restrict__ gamma, const float* __restrict__ mean_in,
                                                  const float* __restrict__ rstd_in, const float* __restrict__ dres,
                                                  float* __restrict__ dx, float* __restrict__ ws, long M, LnDrop dr) {
  if (dr.g2 && dr.p > 0.f) dr.seed = salted_seed(dr.seed, dr.salt);
  constexpr int D = 64 * V;
  __shared__ float red[4][2 * D];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wglob = blockIdx.x * 4 + wv;
  const int nwaves = gridDim.x * 4;
  float gm[V], pg[V], pb[V];
  ldv<V>(gamma + lane * V, gm);
#pragma unroll
  for (int i = 0; i < V; ++i) pg[i] = pb[i] = 0.f;
  for (long row = wglob; row < M; row += nwaves) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float d[V], xh[V], g[V];
    ldv<V>(dy + row * D + lane * V, d);
    ldv<V>(x + row * D + lane * V, xh);
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      xh[i] = (xh[i] - mean) * rstd;
      g[i] = d[i] * gm[i];
      pg[i] += d[i] * xh[i];
      pb[i] += d[i];
      sg += g[i];
      sgx += g[i] * xh[i];
    }
    sg = wave_sum(sg) * (1.f / D);
    sgx = wave_sum(sgx) * (1.f / D);
    float o[V];
    if (dres) ldv<V>(dres + row * D + lane * V, o);
    else {
#pragma unroll
      for (int i = 0; i < V; ++i) o[i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] += rstd * (g[i] - sg - xh[i] * sgx);
    stv<V>(dx + row * D + lane * V, o);
    if constexpr (V == 8) {
      if (dr.g2) {   // the next module's input gradient: bf16(dx * scale * dropout mask), as cfm_scale_dropout
        float sc[8];
        if (dr.p > 0.f) dropout_scale8(dr.p, dr.seed, (uint64_t)(row * D + lane * V), sc);
#pragma unroll
        for (int i = 0; i < 8; ++i) sc[i] = dr.p > 0.f ? dr.scale * sc[i] : dr.scale;
        float q[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] = o[i] * sc[i];
        st8_dyn(dr.g2, CFM_BF16, row * D + lane * V, q);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) {
    red[wv][lane * V + i] = pg[i];
    red[wv][D + lane * V + i] = pb[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += 256)
    ws[(long)blockIdx.x * 2 * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

// ---------------------------------------------------------------- lane-group kernels (D % 8 == 0, D <= 8 G)
// Widths that are not 64 * V (Conformer-S: D = 144) on 16-B vectors: a group of G lanes owns one row, 8 contiguous
// features per lane (lanes 8 j >= D idle), 64 / G rows per wave, the row sums over the group by xor shuffles inside
// it.  (The strided generic kernels below moved 4-B elements with per-element dtype branches: 20 us per D-144
// backward where the bytes take ~5.)
template <int G> __device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int G, typename TY, typename TX = float, bool RS = false>
__global__ __launch_bounds__(256) void ln_fwd_grp(const TX* __restrict__ x, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, TY* __restrict__ y,
                                                  float* __restrict__ mean_out, float* __restrict__ rstd_out, long M,
                                                  int D, float eps, LnRes rs = {}) {
  constexpr int RPW = 64 / G, R = LN_FWD_ROWS;
  const int lane = threadIdx.x & 63, j = lane % G, c = 8 * j;
  const bool act = c < D;
  const long row0 = (((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / G) * R;
  float v[R][8], g[8], b[8];
  [[maybe_unused]] float dl[RS ? R : 1][8];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (act && row0 + r < M) {
      ldv<8>(x + (row0 + r) * D + c, v[r]);
      if constexpr (RS) ldv<8>(rs.d + (row0 + r) * D + c, dl[r]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[r][i] = 0.f;
      if constexpr (RS) {
#pragma unroll
        for (int i = 0; i < 8; ++i) dl[r][i] = 0.f;
      }
    }
  }
  if constexpr (RS) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[r][i] += dl[r][i];
      if (act && row0 + r < M) stv<8>(rs.xo + (row0 + r) * D + c, v[r]);
    }
  }
  if (act) {
    ldv<8>(gamma + c, g);
    ldv<8>(beta + c, b);
  }
  const float invd = 1.f / (float)D;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[r][i];
    const float mean = group_sum<G>(s) * invd;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      v[r][i] = act ? v[r][i] - mean : 0.f;
      q += v[r][i] * v[r][i];
    }
    const float rstd = rsqrtf(group_sum<G>(q) * invd + eps);
    if (row0 + r < M) {
      if (act) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[r][i] = v[r][i] * rstd * g[i] + b[i];
        stv<8>(y + (row0 + r) * D + c, v[r]);
      }
      if (j == 0) {
        mean_out[row0 + r] = mean;
        rstd_out[row0 + r] = rstd;
      }
    }
  }
}

template <int G, typename TDY, typename TX = float>
__global__ __launch_bounds__(256) void ln_bwd_grp(const TDY* __restrict__ dy, const TX* __restrict__ x,
                                                  const float* __restrict__ gamma, const float* __restrict__ mean_in,
                                                  const float* __restrict__ rstd_in, const float* __restrict__ dres,
                                                  float* __restrict__ dx, float* __restrict__ ws, long M, int D,
                                                  LnDrop dr) {
  if (dr.g2 && dr.p > 0.f) dr.seed = salted_seed(dr.seed, dr.salt);
  constexpr int RPW = 64 / G;
  __shared__ float red[4][2 * 8 * G];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, j = lane % G, c = 8 * j;
  const bool act = c < D;
  const long slot = ((long)blockIdx.x * 4 + wv) * RPW + lane / G;
  const long nslots = (long)gridDim.x * 4 * RPW;
  float gm[8], pg[8], pb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) gm[i] = pg[i] = pb[i] = 0.f;
  if (act) ldv<8>(gamma + c, gm);
  const float invd = 1.f / (float)D;
  // every group of the wave runs the same trip count (the shuffles span the wave); rows past M are masked.  Two rows
  // per group and iteration, all their loads issued before the first reduction (one row at a time left the kernel
  // latency-bound: 9.4 us per D-144 backward for ~28 MB)
  const long nrow_iter = (M + nslots - 1) / nslots;
  for (long it = 0; it < nrow_iter; it += 2) {
    long row[2];
    bool live[2];
    float mean[2], rstd[2], d[2][8], xh[2][8], o[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      row[u] = slot + (it + u) * nslots;
      live[u] = act && row[u] < M;
      mean[u] = row[u] < M ? mean_in[row[u]] : 0.f;
      rstd[u] = row[u] < M ? rstd_in[row[u]] : 0.f;
      if (live[u]) {
        ldv<8>(dy + row[u] * D + c, d[u]);
        ldv<8>(x + row[u] * D + c, xh[u]);
        if (dres) ldv<8>(dres + row[u] * D + c, o[u]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (!live[u]) d[u][i] = xh[u][i] = 0.f;
        if (!live[u] || !dres) o[u][i] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float g[8], sg = 0.f, sgx = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xh[u][i] = live[u] ? (xh[u][i] - mean[u]) * rstd[u] : 0.f;
        g[i] = d[u][i] * gm[i];
        pg[i] += d[u][i] * xh[u][i];
        pb[i] += d[u][i];
        sg += g[i];
        sgx += g[i] * xh[u][i];
      }
      sg = group_sum<G>(sg) * invd;
      sgx = group_sum<G>(sgx) * invd;
      if (live[u]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[u][i] += rstd[u] * (g[i] - sg - xh[u][i] * sgx);
        stv<8>(dx + row[u] * D + c, o[u]);
        if (dr.g2) {   // the next module's input gradient: bf16(dx * scale * dropout mask), as cfm_scale_dropout
          float sc[8];
          if (dr.p > 0.f) dropout_scale8(dr.p, dr.seed, (uint64_t)(row[u] * D + c), sc);
#pragma unroll
          for (int i = 0; i < 8; ++i) sc[i] = dr.p > 0.f ? dr.scale * sc[i] : dr.scale;
          float q[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) q[i] = o[u][i] * sc[i];
          st8_dyn(dr.g2, CFM_BF16, row[u] * D + c, q);
        }
      }
    }
  }
  // the groups of a wave hold the same columns: fold them (xor over the group index bits), then group 0 writes
#pragma unroll
  for (int o = G; o < 64; o <<= 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      pg[i] += __shfl_xor(pg[i], o, 64);
      pb[i] += __shfl_xor(pb[i], o, 64);
    }
  }
  if (lane < G) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[wv][c + i] = pg[i];
      red[wv][8 * G + c + i] = pb[i];
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < 2 * D; q += 256) {
    const int k = q < D ? q : 8 * G + (q - D);
    ws[(long)blockIdx.x * 2 * D + q] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  }
}

// ---------------------------------------------------------------- generic kernels (any D <= 1024)
__global__ __launch_bounds__(256) void ln_fwd_kernel(const void* __restrict__ x, int dtx,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, void* __restrict__ y,
                                                     int dty, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, long M, int D, float eps,
                                                     const void* __restrict__ delta = nullptr, int dtd = 0,
                                                     float* __restrict__ xo = nullptr) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[MAXJ];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < D ? ld_dyn(x, dtx, row * D + c) : 0.f;
    if (delta && c < D) {   // (cfm_layernorm_fwd_res: x + delta, stored to xo)
      v[j] += ld_dyn(delta, dtd, row * D + c);
      xo[row * D + c] = v[j];
    }
    s += v[j];
  }
  const float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = lane + 64 * j;
    const float d = c < D ? v[j] - mean : 0.f;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = lane + 64 * j;
    if (c < D) st_dyn(y, dty, row * D + c, (v[j] - mean) * rstd * gamma[c] + beta[c]);
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

__global__ __launch_bounds__(256) void ln_bwd_kernel(const void* __restrict__ dy, int dtdy,
                                                     const void* __restrict__ x, int dtx,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in,
                                                     const void* __restrict__ dres, int dtres,
                                                     void* __restrict__ dx, int dtdx, float* __restrict__ ws,
                                                     long M, int D) {
  const int lane = threadIdx.x & 63;
  const int wglob = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  float pg[MAXJ], pb[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) pg[j] = pb[j] = 0.f;
  for (long row = wglob; row < M; row += nwaves) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[MAXJ], g[MAXJ];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c = lane + 64 * j;
      if (c < D) {
        const float d = ld_dyn(dy, dtdy, row * D + c);
        xh[j] = (ld_dyn(x, dtx, row * D + c) - mean) * rstd;
        g[j] = d * gamma[c];
        pg[j] += d * xh[j];
        pb[j] += d;
      } else {
        xh[j] = g[j] = 0.f;
      }
      sg += g[j];
      sgx += g[j] * xh[j];
    }
    sg = wave_sum(sg) / D;
    sgx = wave_sum(sgx) / D;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c = lane + 64 * j;
      if (c < D) {
        float v = rstd * (g[j] - sg - xh[j] * sgx);
        if (dres) v += ld_dyn(dres, dtres, row * D + c);
        st_dyn(dx, dtdx, row * D + c, v);
      }
    }
  }
  __shared__ float red[4][2 * 64 * MAXJ];
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = lane + 64 * j;
    if (c < D) {
      red[wv][c] = pg[j];
      red[wv][D + c] = pb[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += 256)
    ws[(long)blockIdx.x * 2 * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

int ln_bwd_blocks(long M) {
  long b = (M + 15) / 16;     // ~4 rows per wave
  return (int)(b < 1024 ? (b < 1 ? 1 : b) : 1024);
}

bool aligned16(const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; }

template <int V>
bool ln_fwd_fast(const void* x, int dtx, const float* gamma, const float* beta, void* y, int dty, float* mean,
                 float* rstd, long M, int D, float eps, hipStream_t s, LnMx mx = {}, LnRes rs = {}) {
  // x: the fp32 residual stream, or bf16 (the bf16 mode's residual stream, conformer.py RES_BF16)
  if (D != 64 * V || (dtx != CFM_F32 && dtx != CFM_BF16) || !aligned16(x) || !aligned16(y) || !aligned16(gamma) ||
      !aligned16(beta))
    return false;
  dim3 g((unsigned)((M + 4 * LN_FWD_ROWS - 1) / (4 * LN_FWD_ROWS)));
  if (rs.d) {   // fp32 x + bf16 delta (cfm_layernorm_fwd_res)
    if (dtx != CFM_F32 || !aligned16(rs.d) || !aligned16(rs.xo) || (V < 4 && ((uintptr_t)rs.d & 15)))
      return false;
    if (mx.y8) {
      if constexpr (V >= 4) {
        if (dty != CFM_BF16) return false;
        hipLaunchKernelGGL((ln_fwd_vec<V, bf16, true, float, true>), g, dim3(256), 0, s, (const float*)x, gamma, beta,
                           (bf16*)y, mean, rstd, M, eps, mx, rs);
        return true;
      }
      return false;
    }
    if (dty == CFM_BF16)
      hipLaunchKernelGGL((ln_fwd_vec<V, bf16, false, float, true>), g, dim3(256), 0, s, (const float*)x, gamma, beta,
                         (bf16*)y, mean, rstd, M, eps, LnMx{}, rs);
    else
      hipLaunchKernelGGL((ln_fwd_vec<V, float, false, float, true>), g, dim3(256), 0, s, (const float*)x, gamma, beta,
                         (float*)y, mean, rstd, M, eps, LnMx{}, rs);
    return true;
  }
  auto go = [&](auto xt) {
    typedef decltype(xt) TX;
    if (mx.y8) {
      if constexpr (V >= 4) {
        if (dty != CFM_BF16) return false;
        hipLaunchKernelGGL((ln_fwd_vec<V, bf16, true, TX>), g, dim3(256), 0, s, (const TX*)x, gamma, beta, (bf16*)y,
                           mean, rstd, M, eps, mx);
        return true;
      }
      return false;
    }
    if (dty == CFM_BF16)
      hipLaunchKernelGGL((ln_fwd_vec<V, bf16, false, TX>), g, dim3(256), 0, s, (const TX*)x, gamma, beta, (bf16*)y, mean,
                         rstd, M, eps, LnMx{});
    else
      hipLaunchKernelGGL((ln_fwd_vec<V, float, false, TX>), g, dim3(256), 0, s, (const TX*)x, gamma, beta, (float*)y,
                         mean, rstd, M, eps, LnMx{});
    return true;
  };
  return dtx == CFM_BF16 ? go(bf16{}) : go(float{});
}

template <int V>
bool ln_bwd_fast(const void* dy, int dtdy, const void* x, int dtx, const float* gamma, const float* mean,
                 const float* rstd, const void* dres, int dtres, void* dx, int dtdx, float* ws, long M, int D, int nb,
                 hipStream_t s, LnDrop dr) {
  if (D != 64 * V || (dtx != CFM_F32 && dtx != CFM_BF16) || dtdx != CFM_F32 || (dres && dtres != CFM_F32))
    return false;
  if (!aligned16(dy) || !aligned16(x) || !aligned16(dres) || !aligned16(dx) || !aligned16(gamma)) return false;
  if (dr.g2 && (V != 8 || !aligned16(dr.g2))) return false;
  auto go = [&](auto xt) {
    typedef decltype(xt) TX;
    if (dtdy == CFM_BF16)
      hipLaunchKernelGGL((ln_bwd_vec<V, bf16, TX>), dim3(nb), dim3(256), 0, s, (const bf16*)dy, (const TX*)x, gamma,
                         mean, rstd, (const float*)dres, (float*)dx, ws, M, dr);
    else
      hipLaunchKernelGGL((ln_bwd_vec<V, float, TX>), dim3(nb), dim3(256), 0, s, (const float*)dy, (const TX*)x, gamma,
                         mean, rstd, (const float*)dres, (float*)dx, ws, M, dr);
  };
  if (dtx == CFM_BF16) go(bf16{});
  else go(float{});
  return true;
}
// D % 8 == 0 widths below 512 that are not 64 * V: the lane-group kernels (G = next power of two >= D / 8)
int ln_group(int D) {
  if (D % 8 || D > 512) return 0;
  const int n = D / 8;
  return n <= 16 ? 16 : n <= 32 ? 32 : 64;
}

bool ln_fwd_grouped(const void* x, int dtx, const float* gamma, const float* beta, void* y, int dty, float* mean,
                    float* rstd, long M, int D, float eps, hipStream_t s, LnRes rs = {}) {
  const int G = ln_group(D);
  if (!G || (dtx != CFM_F32 && dtx != CFM_BF16) || (dty != CFM_F32 && dty != CFM_BF16) || !aligned16(x) ||
      !aligned16(y) || !aligned16(gamma) || !aligned16(beta))
    return false;
  if (rs.d && (dtx != CFM_F32 || !aligned16(rs.d) || !aligned16(rs.xo))) return false;
  const long rows_per_block = 4L * (64 / G) * LN_FWD_ROWS;
  const dim3 g((unsigned)((M + rows_per_block - 1) / rows_per_block));
  auto go = [&](auto gt) {
    constexpr int GG = decltype(gt)::value;
    if (rs.d) {
      if (dty == CFM_BF16)
        hipLaunchKernelGGL((ln_fwd_grp<GG, bf16, float, true>), g, dim3(256), 0, s, (const float*)x, gamma, beta,
                           (bf16*)y, mean, rstd, M, D, eps, rs);
      else
        hipLaunchKernelGGL((ln_fwd_grp<GG, float, float, true>), g, dim3(256), 0, s, (const float*)x, gamma, beta,
                           (float*)y, mean, rstd, M, D, eps, rs);
      return;
    }
    auto go2 = [&](auto xt) {
      typedef decltype(xt) TX;
      if (dty == CFM_BF16)
        hipLaunchKernelGGL((ln_fwd_grp<GG, bf16, TX>), g, dim3(256), 0, s, (const TX*)x, gamma, beta, (bf16*)y, mean,
                           rstd, M, D, eps);
      else
        hipLaunchKernelGGL((ln_fwd_grp<GG, float, TX>), g, dim3(256), 0, s, (const TX*)x, gamma, beta, (float*)y,
                           mean, rstd, M, D, eps);
    };
    if (dtx == CFM_BF16) go2(bf16{});
    else go2(float{});
  };
  if (G == 16) go(std::integral_constant<int, 16>{});
  else if (G == 32) go(std::integral_constant<int, 32>{});
  else go(std::integral_constant<int, 64>{});
  return true;
}

bool ln_bwd_grouped(const void* dy, int dtdy, const void* x, int dtx, const float* gamma, const float* mean,
                    const float* rstd, const void* dres, int dtres, void* dx, int dtdx, float* ws, long M, int D,
                    int nb, hipStream_t s, LnDrop dr) {
  const int G = ln_group(D);
  if (!G || (dtx != CFM_F32 && dtx != CFM_BF16) || dtdx != CFM_F32 || (dres && dtres != CFM_F32)) return false;
  if (dtdy != CFM_BF16 && dtdy != CFM_F32) return false;
  if (!aligned16(dy) || !aligned16(x) || !aligned16(dres) || !aligned16(dx) || !aligned16(gamma)) return false;
  if (dr.g2 && !aligned16(dr.g2)) return false;
  auto go = [&](auto gt) {
    constexpr int GG = decltype(gt)::value;
    auto go2 = [&](auto xt) {
      typedef decltype(xt) TX;
      if (dtdy == CFM_BF16)
        hipLaunchKernelGGL((ln_bwd_grp<GG, bf16, TX>), dim3(nb), dim3(256), 0, s, (const bf16*)dy, (const TX*)x, gamma,
                           mean, rstd, (const float*)dres, (float*)dx, ws, M, D, dr);
      else
        hipLaunchKernelGGL((ln_bwd_grp<GG, float, TX>), dim3(nb), dim3(256), 0, s, (const float*)dy, (const TX*)x,
                           gamma, mean, rstd, (const float*)dres, (float*)dx, ws, M, D, dr);
    };
    if (dtx == CFM_BF16) go2(bf16{});
    else go2(float{});
  };
  if (G == 16) go(std::integral_constant<int, 16>{});
  else if (G == 32) go(std::integral_constant<int, 32>{});
  else go(std::integral_constant<int, 64>{});
  return true;
}
}  // namespace

CFM_EXPORT int cfm_layernorm_fwd(const void* x, int dtx, const float* gamma, const float* beta, void* y, int dty,
                                 float* mean, float* rstd, long M, int D, float eps, void* stream) {
  CFM_REQUIRE(x && gamma && beta && y && mean && rstd, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(D > 0 && D <= 64 * MAXJ && M >= 0, CFM_ERR_SHAPE, "D must be in (0, 1024]");
  if (M == 0) return CFM_OK;
  hipStream_t s = cfm::as_stream(stream);
  const bool fast = ln_fwd_fast<2>(x, dtx, gamma, beta, y, dty, mean, rstd, M, D, eps, s) ||
                    ln_fwd_fast<4>(x, dtx, gamma, beta, y, dty, mean, rstd, M, D, eps, s) ||
                    ln_fwd_fast<8>(x, dtx, gamma, beta, y, dty, mean, rstd, M, D, eps, s) ||
                    ln_fwd_fast<16>(x, dtx, gamma, beta, y, dty, mean, rstd, M, D, eps, s) ||
                    ln_fwd_grouped(x, dtx, gamma, beta, y, dty, mean, rstd, M, D, eps, s);
  if (!fast)
    hipLaunchKernelGGL(ln_fwd_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, x, dtx, gamma, beta, y, dty,
                       mean, rstd, M, D, eps);
  return cfm::check_launch("cfm_layernorm_fwd");
}

CFM_EXPORT int cfm_layernorm_fwd_mx_ex(const void* x, int dtx, const float* gamma, const float* beta, void* y, void* y8,
                                       uint8_t* s8, float* mean, float* rstd, long M, int D, float eps, void* stream) {
  CFM_REQUIRE(x && gamma && beta && y && y8 && s8 && mean && rstd, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(dtx == CFM_F32 || dtx == CFM_BF16, CFM_ERR_DTYPE, "x: f32 or bf16");
  CFM_REQUIRE((D == 256 || D == 512 || D == 1024) && M >= 0, CFM_ERR_SHAPE, "D in {256, 512, 1024}");
  CFM_REQUIRE((uintptr_t)y8 % 8 == 0, CFM_ERR_ALIGN, "8-B aligned y8");
  if (M == 0) return CFM_OK;
  hipStream_t s = cfm::as_stream(stream);
  const LnMx mx{(uint8_t*)y8, s8};
  const bool ok = ln_fwd_fast<4>(x, dtx, gamma, beta, y, CFM_BF16, mean, rstd, M, D, eps, s, mx) ||
                  ln_fwd_fast<8>(x, dtx, gamma, beta, y, CFM_BF16, mean, rstd, M, D, eps, s, mx) ||
                  ln_fwd_fast<16>(x, dtx, gamma, beta, y, CFM_BF16, mean, rstd, M, D, eps, s, mx);
  CFM_REQUIRE(ok, CFM_ERR_ALIGN, "16-B aligned x / y / gamma / beta");
  return cfm::check_launch("cfm_layernorm_fwd_mx");
}

CFM_EXPORT int cfm_layernorm_fwd_res(const float* x, const void* delta, int dtd, float* xout, const float* gamma,
                                     const float* beta, void* y, int dty, void* y8, uint8_t* s8, float* mean,
                                     float* rstd, long M, int D, float eps, void* stream) {
  CFM_REQUIRE(x && delta && xout && gamma && beta && y && mean && rstd, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE((const void*)x != (const void*)xout && delta != (const void*)xout, CFM_ERR_ARG,
              "xout must not alias x or delta");
  CFM_REQUIRE(dtd == CFM_F32 || dtd == CFM_BF16, CFM_ERR_DTYPE, "delta: f32 or bf16");
  CFM_REQUIRE(dty == CFM_F32 || dty == CFM_BF16, CFM_ERR_DTYPE, "y: f32 or bf16");
  CFM_REQUIRE(D > 0 && D <= 64 * MAXJ && M >= 0, CFM_ERR_SHAPE, "D must be in (0, 1024]");
  CFM_REQUIRE(!y8 || (s8 && dty == CFM_BF16 && (D == 256 || D == 512 || D == 1024) && (uintptr_t)y8 % 8 == 0),
              CFM_ERR_SHAPE, "MX copy: bf16 y, D in {256, 512, 1024}, 8-B aligned y8, s8");
  if (M == 0) return CFM_OK;
  hipStream_t s = cfm::as_stream(stream);
  const LnMx mx{(uint8_t*)y8, s8};
  const LnRes rs{dtd == CFM_BF16 ? (const bf16*)delta : nullptr, xout};
  bool fast = false;
  if (rs.d) {
    fast = ln_fwd_fast<2>(x, CFM_F32, gamma, beta, y, dty, mean, rstd, M, D, eps, s, mx, rs) ||
           ln_fwd_fast<4>(x, CFM_F32, gamma, beta, y, dty, mean, rstd, M, D, eps, s, mx, rs) ||
           ln_fwd_fast<8>(x, CFM_F32, gamma, beta, y, dty, mean, rstd, M, D, eps, s, mx, rs) ||
           ln_fwd_fast<16>(x, CFM_F32, gamma, beta, y, dty, mean, rstd, M, D, eps, s, mx, rs) ||
           (!y8 && ln_fwd_grouped(x, CFM_F32, gamma, beta, y, dty, mean, rstd, M, D, eps, s, rs));
  }
  if (!fast) {
    CFM_REQUIRE(!y8, CFM_ERR_ALIGN, "MX copy: 16-B aligned x / delta / xout / y / gamma / beta");
    hipLaunchKernelGGL(ln_fwd_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, (const void*)x, (int)CFM_F32,
                       gamma, beta, y, dty, mean, rstd, M, D, eps, delta, dtd, xout);
  }
  return cfm::check_launch("cfm_layernorm_fwd_res");
}

CFM_EXPORT int cfm_layernorm_fwd_mx(const float* x, const float* gamma, const float* beta, void* y, void* y8,
                                    uint8_t* s8, float* mean, float* rstd, long M, int D, float eps, void* stream) {
  return cfm_layernorm_fwd_mx_ex(x, CFM_F32, gamma, beta, y, y8, s8, mean, rstd, M, D, eps, stream);
}

CFM_EXPORT size_t cfm_layernorm_ws_bytes(long M, int D) {
  return (size_t)ln_bwd_blocks(M) * 2 * D * sizeof(float) + 2 * D * sizeof(float);
}

CFM_EXPORT int cfm_scale_dropout(const void* x, int dtx, void* y, int dty, long n, float scale, float p,
                                 uint64_t seed, uint64_t off, void* stream);

CFM_EXPORT int cfm_layernorm_bwd_drop(const void* dy, int dtdy, const void* x, int dtx, const float* gamma,
                                      const float* mean, const float* rstd, const void* dres, int dtres, void* dx,
                                      int dtdx, float* dgamma, float* dbeta, float* ws, long M, int D, void* g2,
                                      float g2_scale, float g2_p, uint64_t g2_seed, void* stream) {
  CFM_REQUIRE(dy && x && gamma && mean && rstd && dx && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(D > 0 && D <= 64 * MAXJ && M >= 0, CFM_ERR_SHAPE, "D must be in (0, 1024]");
  hipStream_t s = cfm::as_stream(stream);
  const int nb = ln_bwd_blocks(M);
  const LnDrop dr{g2, g2_scale, g2_p, g2_seed, cfm::g_rng_salt};
  bool fast = ln_bwd_fast<2>(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, ws, M, D, nb, s, dr) ||
              ln_bwd_fast<4>(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, ws, M, D, nb, s, dr) ||
              ln_bwd_fast<8>(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, ws, M, D, nb, s, dr) ||
              ln_bwd_fast<16>(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, ws, M, D, nb, s, dr) ||
              ln_bwd_grouped(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, ws, M, D, nb, s, dr);
  bool g2_done = fast && g2 != nullptr;
  if (!fast && g2) {   // no fused path for this shape: the vectorised kernel without g2, then a separate pass
    const LnDrop none{nullptr, 0.f, 0.f, 0, nullptr};
    fast = ln_bwd_fast<2>(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, ws, M, D, nb, s, none) ||
           ln_bwd_fast<4>(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, ws, M, D, nb, s, none) ||
           ln_bwd_fast<8>(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, ws, M, D, nb, s, none) ||
           ln_bwd_fast<16>(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, ws, M, D, nb, s, none) ||
           ln_bwd_grouped(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, ws, M, D, nb, s, none);
  }
  if (!fast)
    hipLaunchKernelGGL(ln_bwd_kernel, dim3(nb), dim3(256), 0, s, dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres,
                       dx, dtdx, ws, M, D);
  if (g2 && !g2_done) {
    const int rc = cfm_scale_dropout(dx, dtdx, g2, CFM_BF16, M * D, g2_scale, g2_p, g2_seed, 0, stream);
    if (rc != CFM_OK) return rc;
  }
  if (dgamma && dbeta && dbeta == dgamma + D) {
    cfm::colreduce(ws, nb, 2L * D, dgamma, 0, s);               // one pass for [dgamma | dbeta]
  } else {
    if (dgamma) cfm::colreduce(ws, nb, D, dgamma, 0, s, 2L * D);
    if (dbeta) cfm::colreduce(ws + D, nb, D, dbeta, 0, s, 2L * D);
  }
  return cfm::check_launch("cfm_layernorm_bwd");
}

CFM_EXPORT int cfm_layernorm_bwd(const void* dy, int dtdy, const void* x, int dtx, const float* gamma,
                                 const float* mean, const float* rstd, const void* dres, int dtres, void* dx,
                                 int dtdx, float* dgamma, float* dbeta, float* ws, long M, int D,
                                 void* stream) {
  return cfm_layernorm_bwd_drop(dy, dtdy, x, dtx, gamma, mean, rstd, dres, dtres, dx, dtdx, dgamma, dbeta, ws, M, D,
                                nullptr, 0.f, 0.f, 0, stream);
}
