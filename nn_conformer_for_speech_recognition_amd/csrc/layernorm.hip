// layernorm.hip — nn.LayerNorm(D) forward/backward over token rows (one wave per row).
//
// Used by every LayerNorm of the torchaudio ConformerLayer (ffn*.sequential.0,
// self_attn_layer_norm, conv_module.layer_norm, final_layer_norm).  The residual stream is
// fp32; the normalised output feeds the next GEMM in the compute dtype (bf16 or fp32).
// Backward fuses the residual-gradient add (dx = LN'(dy) + dres) and produces dgamma/dbeta
// through per-wave partial sums reduced by a second tiny kernel (deterministic, no atomics).
#include "cfm_common.h"

namespace {
constexpr int MAXJ = 16;   // D <= 1024

__global__ __launch_bounds__(256) void ln_fwd_kernel(const void* __restrict__ x, int dtx,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, void* __restrict__ y,
                                                     int dty, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, long M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[MAXJ];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < D ? ld_dyn(x, dtx, row * D + c) : 0.f;
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
  // combine the 4 waves' dgamma/dbeta partials in LDS -> one partial row per workgroup
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
}  // namespace

CFM_EXPORT int cfm_layernorm_fwd(const void* x, int dtx, const float* gamma, const float* beta, void* y,
                                 int dty, float* mean, float* rstd, long M, int D, float eps, void* stream) {
  CFM_REQUIRE(x && gamma && beta && y && mean && rstd, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(D > 0 && D <= 64 * MAXJ && M >= 0, CFM_ERR_SHAPE, "D must be in (0, 1024]");
  if (M == 0) return CFM_OK;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, cfm::as_stream(stream), x,
                     dtx, gamma, beta, y, dty, mean, rstd, M, D, eps);
  return cfm::check_launch("cfm_layernorm_fwd");
}

CFM_EXPORT size_t cfm_layernorm_ws_bytes(long M, int D) {
  return (size_t)ln_bwd_blocks(M) * 2 * D * sizeof(float);
}

CFM_EXPORT int cfm_layernorm_bwd(const void* dy, int dtdy, const void* x, int dtx, const float* gamma,
                                 const float* mean, const float* rstd, const void* dres, int dtres, void* dx,
                                 int dtdx, float* dgamma, float* dbeta, float* ws, long M, int D,
                                 void* stream) {
  CFM_REQUIRE(dy && x && gamma && mean && rstd && dx && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(D > 0 && D <= 64 * MAXJ && M >= 0, CFM_ERR_SHAPE, "D must be in (0, 1024]");
  hipStream_t s = cfm::as_stream(stream);
  const int nb = ln_bwd_blocks(M);
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(nb), dim3(256), 0, s, dy, dtdy, x, dtx, gamma, mean, rstd, dres,
                     dtres, dx, dtdx, ws, M, D);
  if (dgamma) cfm::colreduce(ws, nb, D, dgamma, 0, s, 2L * D);
  if (dbeta) cfm::colreduce(ws + D, nb, D, dbeta, 0, s, 2L * D);
  return cfm::check_launch("cfm_layernorm_bwd");
}
