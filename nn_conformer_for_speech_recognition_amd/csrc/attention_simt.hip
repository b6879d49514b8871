// attention_simt.hip — vector-ALU attention for the fp32 parity mode and for relative positions.
//
// Semantics (one (batch, head) slice, scale = 1/sqrt(dk)):
//   none: s_ij = scale * q_i.k_j
//   rel : s_ij = scale * ((q_i+u).k_j + (q_i+v).p_{T-1-i+j})   (transformers Wav2Vec2Conformer
//         SelfAttention, modeling_wav2vec2_conformer.py:528-565; p = linear_pos(pe), 2T-1 rows)
//   keys j >= len[b] are masked (nn.MultiheadAttention key_padding_mask); every query row is
//   computed (padded queries included, as torchaudio does); probabilities may be dropped
//   (counter-based mask, regenerated in backward); lse_i = log sum_j exp(s_ij) is saved.
// One wavefront per query row (forward, dQ) or per key row (dK/dV) or per relative offset
// (dpos); lanes run over keys for the scores and over the head dimension for the outputs.
// The MFMA kernels (attention.hip) replace this path for bf16 without relative positions.
#include "cfm_common.h"

namespace {

struct AttnP {
  const void* qkv; int dt;   // operand dtype
  int B, T, H, dk, D3;       // D3 = 3*H*dk (row stride of qkv)
  const int32_t* len;
  const void* pos;           // (2T-1, H*dk) or null
  const float* pu; const float* pv;
  float scale;
  float drop_p; uint64_t seed;
  const uint64_t* salt;      // bound dropout step counter or nullptr
};

__device__ __forceinline__ float qkv_at(const AttnP& p, int b, int t, int which, int h, int d) {
  return ld_dyn(p.qkv, p.dt, ((long)b * p.T + t) * p.D3 + which * p.H * p.dk + h * p.dk + d);
}
__device__ __forceinline__ float pos_at(const AttnP& p, int r, int h, int d) {
  return ld_dyn(p.pos, p.dt, (long)r * p.H * p.dk + h * p.dk + d);
}
// attention-dropout element index: rows of an EVEN stride (T rounded up to even), so keys 2m and
// 2m+1 of a row share one 32-bit hash (same convention as attention.hip's didx)
__device__ __forceinline__ uint64_t drop_idx(const AttnP& p, int b, int h, int i, int j) {
  return (((uint64_t)b * p.H + h) * p.T + i) * (uint64_t)(p.T + (p.T & 1)) + j;
}

// score for (i, j): lanes hold their own j; qa/qb are broadcast from LDS
__device__ __forceinline__ float score(const AttnP& p, int b, int h, int i, int j, const float* qa, const float* qb) {
  float s = 0.f;
  const long krow = ((long)b * p.T + j) * p.D3 + p.H * p.dk + h * p.dk;
  for (int d = 0; d < p.dk; ++d) s += qa[d] * ld_dyn(p.qkv, p.dt, krow + d);
  if (p.pos) {
    const long prow = (long)(p.T - 1 - i + j) * p.H * p.dk + h * p.dk;
    for (int d = 0; d < p.dk; ++d) s += qb[d] * ld_dyn(p.pos, p.dt, prow + d);
  }
  return s * p.scale;
}

// grid (ceil(T/4), H, B), 256 threads: one wave per query
__global__ __launch_bounds__(256) void attn_simt_fwd(AttnP p, void* __restrict__ o, float* __restrict__ lse) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  __shared__ float sq[4][2][64];
  __shared__ float sp[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 4 + wv, h = blockIdx.y, b = blockIdx.z;
  if (i >= p.T) return;
  const int len = p.len[b];
  if (lane < p.dk) {
    const float q = qkv_at(p, b, i, 0, h, lane);
    sq[wv][0][lane] = q + (p.pos ? p.pu[h * p.dk + lane] : 0.f);
    sq[wv][1][lane] = q + (p.pos ? p.pv[h * p.dk + lane] : 0.f);
  }
  __builtin_amdgcn_wave_barrier();
  float m = -INFINITY, l = 0.f, acc = 0.f;
  for (int j0 = 0; j0 < len; j0 += 64) {
    const int j = j0 + lane;
    float s = -INFINITY;
    if (j < len) s = score(p, b, h, i, j, sq[wv][0], sq[wv][1]);
    const float mn = fmaxf(m, wave_max(s));
    const float e = (j < len) ? __expf(s - mn) : 0.f;
    const float alpha = __expf(m - mn);
    l = l * alpha + wave_sum(e);
    acc *= alpha;
    m = mn;
    sp[wv][lane] = (j < len) ? e * attn_dropout_scale(p.drop_p, p.seed, drop_idx(p, b, h, i, j)) : 0.f;
    __builtin_amdgcn_wave_barrier();
    if (lane < p.dk) {
      const int jn = min(64, len - j0);
      for (int jj = 0; jj < jn; ++jj) acc += sp[wv][jj] * qkv_at(p, b, j0 + jj, 2, h, lane);
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (lane < p.dk) st_dyn(o, p.dt, ((long)b * p.T + i) * p.H * p.dk + h * p.dk + lane, acc / l);
  if (lane == 0) lse[((long)b * p.H + h) * p.T + i] = m + __logf(l);
}

// dQ (+ dS materialised for dK / dpos, + D_i).  grid (ceil(T/4), H, B)
// ws_ds: (B, H, T, T) fp32 of scale*dS (zero for masked keys);  dD: (B,H,T)
__global__ __launch_bounds__(256) void attn_simt_bwd_dq(AttnP p, const void* __restrict__ o,
                                                        const void* __restrict__ dout, const float* __restrict__ lse,
                                                        void* __restrict__ dqkv, float* __restrict__ ws_ds,
                                                        float* __restrict__ dpu, float* __restrict__ dpv) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  __shared__ float sq[4][2][64];
  __shared__ float sdo[4][64];
  __shared__ float sds[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 4 + wv, h = blockIdx.y, b = blockIdx.z;
  if (i >= p.T) return;
  const int len = p.len[b];
  const int HD = p.H * p.dk;
  float dOo = 0.f;
  if (lane < p.dk) {
    const float q = qkv_at(p, b, i, 0, h, lane);
    sq[wv][0][lane] = q + (p.pos ? p.pu[h * p.dk + lane] : 0.f);
    sq[wv][1][lane] = q + (p.pos ? p.pv[h * p.dk + lane] : 0.f);
    const float g = ld_dyn(dout, p.dt, ((long)b * p.T + i) * HD + h * p.dk + lane);
    sdo[wv][lane] = g;
    dOo = g * ld_dyn(o, p.dt, ((long)b * p.T + i) * HD + h * p.dk + lane);
  }
  const float Di = wave_sum(dOo);
  __builtin_amdgcn_wave_barrier();
  const float L = lse[((long)b * p.H + h) * p.T + i];
  float dqa = 0.f, dqb = 0.f;
  float* dsrow = ws_ds + (((long)b * p.H + h) * p.T + i) * p.T;
  for (int j0 = 0; j0 < p.T; j0 += 64) {
    const int j = j0 + lane;
    float ds = 0.f;
    if (j < len) {
      const float s = score(p, b, h, i, j, sq[wv][0], sq[wv][1]);
      const float pr = __expf(s - L);
      float dp = 0.f;
      const long vrow = ((long)b * p.T + j) * p.D3 + 2 * HD + h * p.dk;
      for (int d = 0; d < p.dk; ++d) dp += sdo[wv][d] * ld_dyn(p.qkv, p.dt, vrow + d);
      dp *= attn_dropout_scale(p.drop_p, p.seed, drop_idx(p, b, h, i, j));
      ds = pr * (dp - Di) * p.scale;
    }
    if (j < p.T) dsrow[j] = ds;
    sds[wv][lane] = ds;
    __builtin_amdgcn_wave_barrier();
    if (lane < p.dk) {
      const int jn = min(64, len - j0);
      for (int jj = 0; jj < jn; ++jj) {
        const float g = sds[wv][jj];
        dqa += g * qkv_at(p, b, j0 + jj, 1, h, lane);
        if (p.pos) dqb += g * pos_at(p, p.T - 1 - i + j0 + jj, h, lane);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (lane < p.dk) {
    st_dyn(dqkv, p.dt, ((long)b * p.T + i) * p.D3 + h * p.dk + lane, dqa + dqb);
    if (p.pos) {
      atomicAdd(dpu + h * p.dk + lane, dqa);
      atomicAdd(dpv + h * p.dk + lane, dqb);
    }
  }
}

// dK, dV.  grid (ceil(T/4), H, B): one wave per key j
__global__ __launch_bounds__(256) void attn_simt_bwd_dkdv(AttnP p, const void* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          void* __restrict__ dqkv, const float* __restrict__ ws_ds) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  __shared__ float sk[4][64];
  __shared__ float sw[4][2][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = blockIdx.x * 4 + wv, h = blockIdx.y, b = blockIdx.z;
  if (j >= p.T) return;
  const int len = p.len[b];
  const int HD = p.H * p.dk;
  float dk_acc = 0.f, dv_acc = 0.f;
  if (j < len) {
    if (lane < p.dk) sk[wv][lane] = qkv_at(p, b, j, 1, h, lane);
    __builtin_amdgcn_wave_barrier();
    for (int i0 = 0; i0 < p.T; i0 += 64) {
      const int i = i0 + lane;
      float pd = 0.f, ds = 0.f;
      if (i < p.T) {
        ds = ws_ds[(((long)b * p.H + h) * p.T + i) * p.T + j];
        // recompute p_ij for dV
        float s = 0.f;
        for (int d = 0; d < p.dk; ++d) {
          const float q = qkv_at(p, b, i, 0, h, d);
          s += (q + (p.pos ? p.pu[h * p.dk + d] : 0.f)) * sk[wv][d];
          if (p.pos) s += (q + p.pv[h * p.dk + d]) * pos_at(p, p.T - 1 - i + j, h, d);
        }
        s *= p.scale;
        pd = __expf(s - lse[((long)b * p.H + h) * p.T + i]) * attn_dropout_scale(p.drop_p, p.seed, drop_idx(p, b, h, i, j));
      }
      sw[wv][0][lane] = pd;
      sw[wv][1][lane] = ds;
      __builtin_amdgcn_wave_barrier();
      if (lane < p.dk) {
        const int in = min(64, p.T - i0);
        for (int ii = 0; ii < in; ++ii) {
          const int iq = i0 + ii;
          dv_acc += sw[wv][0][ii] * ld_dyn(dout, p.dt, ((long)b * p.T + iq) * HD + h * p.dk + lane);
          dk_acc += sw[wv][1][ii] * (qkv_at(p, b, iq, 0, h, lane) + (p.pos ? p.pu[h * p.dk + lane] : 0.f));
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (lane < p.dk) {
    st_dyn(dqkv, p.dt, ((long)b * p.T + j) * p.D3 + HD + h * p.dk + lane, dk_acc);
    st_dyn(dqkv, p.dt, ((long)b * p.T + j) * p.D3 + 2 * HD + h * p.dk + lane, dv_acc);
  }
}

// dpos[r][h][d] = sum_{b,i} dS[b,h,i,j=r-(T-1)+i] * (q_i+v)[d].  grid (ceil((2T-1)/4), H)
__global__ __launch_bounds__(256) void attn_simt_bwd_dpos(AttnP p, const float* __restrict__ ws_ds,
                                                          float* __restrict__ dpos) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + wv, h = blockIdx.y;
  if (r >= 2 * p.T - 1 || lane >= p.dk) return;
  const int shift = r - (p.T - 1);     // j = i + shift
  float acc = 0.f;
  for (int b = 0; b < p.B; ++b) {
    const int i0 = max(0, -shift), i1 = min(p.T, p.T - shift);
    for (int i = i0; i < i1; ++i) {
      const float ds = ws_ds[(((long)b * p.H + h) * p.T + i) * p.T + (i + shift)];
      if (ds != 0.f) acc += ds * (qkv_at(p, b, i, 0, h, lane) + p.pv[h * p.dk + lane]);
    }
  }
  dpos[(long)r * p.H * p.dk + h * p.dk + lane] = acc;
}

}  // namespace

namespace cfm {
int attn_simt_fwd_launch(const void* qkv, void* o, float* lse, const int32_t* len, const void* pos, const float* pu,
                         const float* pv, int B, int T, int H, int dk, int dtype, float drop_p, uint64_t seed,
                         hipStream_t s) {
  AttnP p{qkv, dtype, B, T, H, dk, 3 * H * dk, len, pos, pu, pv, 1.f / sqrtf((float)dk), drop_p, seed, cfm::g_rng_salt};
  hipLaunchKernelGGL(attn_simt_fwd, dim3(cdiv(T, 4), H, B), dim3(256), 0, s, p, o, lse);
  return check_launch("cfm_attn_fwd(simt)");
}

size_t attn_simt_ws_bytes(int B, int T, int H) { return (size_t)B * H * T * T * sizeof(float); }

int attn_simt_bwd_launch(const void* qkv, const void* o, const void* dout, const float* lse, const int32_t* len,
                         const void* pos, const float* pu, const float* pv, void* dqkv, float* dpos, float* dpu,
                         float* dpv, int B, int T, int H, int dk, int dtype, float drop_p, uint64_t seed,
                         float* ws, hipStream_t s) {
  AttnP p{qkv, dtype, B, T, H, dk, 3 * H * dk, len, pos, pu, pv, 1.f / sqrtf((float)dk), drop_p, seed, cfm::g_rng_salt};
  if (pos) {
    (void)hipMemsetAsync(dpu, 0, sizeof(float) * H * dk, s);
    (void)hipMemsetAsync(dpv, 0, sizeof(float) * H * dk, s);
  }
  hipLaunchKernelGGL(attn_simt_bwd_dq, dim3(cdiv(T, 4), H, B), dim3(256), 0, s, p, o, dout, lse, dqkv, ws, dpu, dpv);
  hipLaunchKernelGGL(attn_simt_bwd_dkdv, dim3(cdiv(T, 4), H, B), dim3(256), 0, s, p, dout, lse, dqkv, ws);
  if (pos) hipLaunchKernelGGL(attn_simt_bwd_dpos, dim3(cdiv(2 * T - 1, 4), H), dim3(256), 0, s, p, ws, dpos);
  return check_launch("cfm_attn_bwd(simt)");
}
}  // namespace cfm
