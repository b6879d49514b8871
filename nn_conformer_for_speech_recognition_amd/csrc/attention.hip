// attention.hip — fused flash-style multi-head self-attention on MFMA (bf16), fwd + bwd.
//
// Core of nn.MultiheadAttention(need_weights=False, key_padding_mask) inside torchaudio's
// ConformerLayer: softmax(q k^T / sqrt(dk) + mask) v per (batch, head), never materialising
// the T x T score matrix.  qkv is the packed in_proj output (B*T, 3*H*dk); o is (B*T, H*dk).
//
// Forward: one workgroup = 4 waves = 128 queries of one (b, h); each wave keeps its 32 queries
// in registers (as the B operand) and computes S^T = K Q^T (keys on the accumulator rows,
// queries on the lanes), so the softmax row reductions are lane-local plus one lane^32
// exchange.  The S^T accumulator feeds O^T += V^T P^T directly as an MFMA operand (no LDS
// round trip for P); V^T comes from the V tile through ds_read_b64_tr_b16.  K/V tiles of 64
// keys are staged in LDS (double buffered, register prefetch) and the loop stops at the
// utterance's last valid key (key_padding_mask), so padded keys cost nothing.
// Backward (FA2-style, deterministic, no atomics): dK/dV kernel (keys on the lanes, loops over
// query tiles: S, dP, dV^T += dO^T P, dK^T += Q^T dS) and dQ kernel (queries on the lanes,
// loops over key tiles: S^T, dP^T, dQ^T += K^T dS^T), plus a tiny D = rowsum(dO*O) kernel.
// Head dims below 64 (Conformer-S: 36) are zero-padded to 64 in LDS/registers.
// lse is saved in natural-log units of the scaled scores (same convention as attention_simt).
#include "cfm_common.h"

namespace cfm {
int attn_simt_fwd_launch(const void*, void*, float*, const int32_t*, const void*, const float*, const float*, int,
                         int, int, int, int, float, uint64_t, hipStream_t);
size_t attn_simt_ws_bytes(int B, int T, int H);
size_t attn_rel_ws_bytes(int B, int T, int H, int dk);
extern int g_rel_mode;   // attention_rel.hip: cfm_attn_set_mode's bits for the rel-pos kernels
int attn_rel_fwd_launch(const void* qkv, void* o, float* lse, const int32_t* len, const void* pos, const float* pu,
                        const float* pv, int B, int T, int H, int dk, float drop_p, uint64_t seed, hipStream_t s);
int attn_rel_bwd_launch(const void* qkv, const void* dout, const float* lse, const int32_t* len, const void* pos,
                        const float* pu, const float* pv, void* dqkv, void* dpos, int dpos_dt, float* dpu, float* dpv,
                        int B, int T, int H, int dk, float drop_p, uint64_t seed, float* ws, hipStream_t s);
int attn_simt_bwd_launch(const void*, const void*, const void*, const float*, const int32_t*, const void*,
                         const float*, const float*, void*, float*, float*, float*, int, int, int, int, int, float,
                         uint64_t, float*, hipStream_t);
}  // namespace cfm

#include "attn_common.h"

namespace {

// ------------------------------------------------------------------------------------ forward
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnM p, bf16* __restrict__ o, float* __restrict__ lse) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  const uint32_t dkey = drop_key(p.seed, 0), dthr = drop_thr(p.drop_p);
  const float dkeep = drop_keep_scale(dthr);
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TILE * KS];   // [buf][K,V][64][72]  36 KiB
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5;
  const int h = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * 128 + wv * 32;
  const int len = p.len[b];
  const bf16* qbase = p.qkv + (long)b * p.T * p.D3 + h * p.dk;
  bf16x8 qf[4];
  load_bfrags(p, qbase, p.D3, q0 + (lane & 31), p.T, qf, lane);

  f32x16 o0 = (f32x16){0}, o1 = (f32x16){0};
  float m = -INFINITY, l = 0.f;
  const float c = p.scale * LOG2E;
  const int nkt = (len + TILE - 1) / TILE;
  uint4 rk[2], rv[2];
  const int kcol = p.HD + h * p.dk, vcol = 2 * p.HD + h * p.dk;
  if (nkt > 0) {
    tile_load(p, b, 0, kcol, rk, tid);
    tile_load(p, b, 0, vcol, rv, tid);
    tile_store(smem, rk, tid);
    tile_store(smem + TILE * KS, rv, tid);
    __syncthreads();
  }
  const int qi = q0 + (lane & 31);
  for (int kt = 0; kt < nkt; ++kt) {
    const bf16* sK = smem + (kt & 1) * 2 * TILE * KS;
    const bf16* sV = sK + TILE * KS;
    if (kt + 1 < nkt) {
      tile_load(p, b, (kt + 1) * TILE, kcol, rk, tid);
      tile_load(p, b, (kt + 1) * TILE, vcol, rv, tid);
    }
    f32x16 s0 = (f32x16){0}, s1 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 0, 16 * s, lane), qf[s], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 32, 16 * s, lane), qf[s], s1, 0, 0, 0);
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k0 = kt * TILE + acc_row(r, hh);
      s0[r] = (k0 < len) ? s0[r] * c : -INFINITY;
      s1[r] = (k0 + 32 < len) ? s1[r] * c : -INFINITY;
      mloc = fmaxf(mloc, fmaxf(s0[r], s1[r]));
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float mn = fmaxf(m, mloc);
    const float alpha = exp2f(m - mn);
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s0[r] = exp2f(s0[r] - mn);
      s1[r] = exp2f(s1[r] - mn);
      ls += s0[r] + s1[r];
    }
    ls += __shfl_xor(ls, 32, 64);
    l = l * alpha + ls;
    m = mn;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      o0[r] *= alpha;
      o1[r] *= alpha;
    }
    if (p.drop_p > 0.f) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k0 = kt * TILE + acc_row(r, hh);
        s0[r] *= dropout_keyed(dthr, dkeep, dkey, didx(p, b, h, qi, k0));
        s1[r] *= dropout_keyed(dthr, dkeep, dkey, didx(p, b, h, qi, k0 + 32));
      }
    }
    // O^T[d][q] += sum_key V[key][d] P^T[key][q]
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc2frag(t == 0 ? s0 : s1, s);
        o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sV, 32 * t + 16 * s, 0, lane), pf, o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sV, 32 * t + 16 * s, 32, lane), pf, o1, 0, 0, 0);
      }
    }
    if (kt + 1 < nkt) {
      bf16* nK = smem + ((kt + 1) & 1) * 2 * TILE * KS;
      tile_store(nK, rk, tid);
      tile_store(nK + TILE * KS, rv, tid);
    }
    __syncthreads();
  }
  // epilogue: O = O^T / l (transposed through LDS), lse in natural-log units
  float* stage = reinterpret_cast<float*>(smem) + wv * 32 * 65;
  const float inv = 1.f / l;   // l is per query column (lane & 31); both lane halves agree
  store_transposed(stage, o0, o1, inv, o + (long)b * p.T * p.HD + h * p.dk, p.HD, q0, min(32, p.T - q0), p.dk,
                   lane);
  if (hh == 0 && qi < p.T) lse[((long)b * p.H + h) * p.T + qi] = (m + __log2f(l)) * LN2;
}

// ------------------------------------------------------------------------------------ whole-head kernels
// T <= HEAD_TMAX: ONE workgroup per (b, h) stages the head's whole K and V in LDS once (16-byte
// loads, eight in flight per thread), then every wave runs its 32-query block over the staged keys
// with no further barriers.  B*H workgroups (256 at Conformer-L B=32: one per CU) instead of
// ceil(T/128)*B*H workgroups that each re-stream K/V tile by tile behind a barrier per tile.
constexpr int HEAD_TMAX = 384;      // 12 waves of 32 queries; K+V images 2 * 384 * 144 B = 108 KiB

// the whole-head kernels' work split: when B*H workgroups would leave CUs idle (Conformer-S / M: 4 heads, B*H = 128
// on 256 CUs) each (b, h) runs as p.qs workgroups, each staging the whole head and sweeping its own contiguous range
// of 32-row blocks (queries: fwd / dQ; keys: dK/dV).  -> (b, h, first block of this workgroup)
struct HeadPart { int b, h, blk0; };
__device__ __forceinline__ HeadPart head_part(const AttnM& p) {
  const int qs = p.qs > 1 ? p.qs : 1;
  const int bh = blockIdx.x / qs, part = blockIdx.x - bh * qs;
  return {bh / p.H, bh % p.H, part * (int)(blockDim.x >> 6)};
}


// stage rows [0, nrows) of two head slices (dk <= 64 columns at base0 / base1, row stride ld) into
// LDS images [nrows][KS]; rows >= T read as zero
__device__ __forceinline__ void head_stage(const AttnM& p, const bf16* base0, const bf16* base1, long ld0, long ld1,
                                           int nrows, bf16* img0, bf16* img1, int tid, int nthreads) {
  const int nch = nrows * 8;                      // 16-B chunks per image
  if (p.vec && p.dk == 64) {
    // rows >= T clamp to row T-1 (finite data; those keys are masked by len <= T)
    for (int i0 = 0; i0 < 2 * nch; i0 += 8 * nthreads) {
      uint4 r[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = min(i0 + u * nthreads + tid, 2 * nch - 1);
        const int which = i >= nch, j = i - which * nch;
        const int row = min(j >> 3, p.T - 1);
        r[u] = *reinterpret_cast<const uint4*>((which ? base1 + (long)row * ld1 : base0 + (long)row * ld0) + (j & 7) * 8);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * nthreads + tid;
        if (i < 2 * nch) {
          const int which = i >= nch, j = i - which * nch;
          *reinterpret_cast<uint4*>((which ? img1 : img0) + (j >> 3) * KS + (j & 7) * 8) = r[u];
        }
      }
    }
    return;
  }
  for (int i0 = 0; i0 < 2 * nch; i0 += 8 * nthreads) {
    uint4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * nthreads + tid;
      const int which = i >= nch, j = i - which * nch;
      r[u] = i < 2 * nch ? ld8(which ? base1 : base0, which ? ld1 : ld0, j >> 3, p.T, (j & 7) * 8, p.dk, p.vec,
                               p.vec4)
                         : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * nthreads + tid;
      if (i < 2 * nch) {
        const int which = i >= nch, j = i - which * nch;
        *reinterpret_cast<uint4*>((which ? img1 : img0) + (j >> 3) * KS + (j & 7) * 8) = r[u];
      }
    }
  }
}

// forward: grid (B*H), block 64 * ceil(T/32); dynamic LDS head_lds_bytes(T)
__global__ __launch_bounds__(64 * HEAD_TMAX / 32) void attn_fwd_head_kernel(AttnM p, bf16* __restrict__ o,
                                                                            float* __restrict__ lse) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  const uint32_t dkey = drop_key(p.seed, 0), dthr = drop_thr(p.drop_p);
  const float dkeep = drop_keep_scale(dthr);
  extern __shared__ __attribute__((aligned(16))) bf16 hsm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5;
  const HeadPart hp = head_part(p);
  const int b = hp.b, h = hp.h;
  const int len = p.len[b];
  const int nkt = (len + TILE - 1) / TILE, Tp = nkt * TILE;
  bf16* sKall = hsm;
  bf16* sVall = hsm + (long)Tp * KS;
  const bf16* kvbase = p.qkv + (long)b * p.T * p.D3;
  head_stage(p, kvbase + p.HD + h * p.dk, kvbase + 2 * p.HD + h * p.dk, p.D3, p.D3, Tp, sKall, sVall, tid,
             blockDim.x);
  const int q0 = (hp.blk0 + wv) * 32;
  bf16x8 qf[4];
  load_bfrags(p, kvbase + h * p.dk, p.D3, q0 + (lane & 31), p.T, qf, lane);
  __syncthreads();
  if (p.dbg & 2) {   // timing experiment: staging only
    if (tid == 0 && hsm[5] == (bf16)-12345.f) lse[0] = 1.f;
    return;
  }
  f32x16 o0 = (f32x16){0}, o1 = (f32x16){0};
  float m = -INFINITY, l = 0.f;
  const float c = p.scale * LOG2E;
  const int qi = q0 + (lane & 31);
  // The dropout keep scale is applied once to the output (o * keep / l), not to every P entry.  (Round 4: issuing
  // tile kt+1's S MFMAs before tile kt's softmax VALU, unrolled by two, measured 27.08 vs 26.86 us at L15 --
  // three waves per SIMD already overlap one wave's VALU with another's MFMAs -- and was removed.)
  const bool late = p.drop_p > 0.f;
  auto qk = [&](int kt, f32x16& s0, f32x16& s1) {
    const bf16* sK = sKall + kt * TILE * KS;
    s0 = (f32x16){0};
    s1 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 0, 16 * s, lane), qf[s], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 32, 16 * s, lane), qf[s], s1, 0, 0, 0);
    }
  };
  auto pv = [&](int kt, const f32x16& s0, const f32x16& s1) {
    const bf16* sV = sVall + kt * TILE * KS;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc2frag(t == 0 ? s0 : s1, s);
        o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sV, 32 * t + 16 * s, 0, lane), pf, o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sV, 32 * t + 16 * s, 32, lane), pf, o1, 0, 0, 0);
      }
    }
  };
  f32x16 sa0, sa1;
  for (int kt = 0; kt < nkt; ++kt) {
    qk(kt, sa0, sa1);
    __builtin_amdgcn_sched_barrier(0);
    softmax_tile<true>(p, sa0, sa1, o0, o1, m, l, c, kt * TILE, len, kt == nkt - 1, b, h, qi, hh, dthr, dkeep, dkey);
    pv(kt, sa0, sa1);
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();     // every wave is done with K/V: the images become the epilogue staging
  float* stage = reinterpret_cast<float*>(hsm) + wv * 32 * 65;
  const float inv = (late ? dkeep : 1.f) / l;
  if (p.dbg & 4) {   // timing experiment: no epilogue stores
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) t += o0[r] + o1[r];
    if (t == -1234.5f) lse[0] = t;
    return;
  }
  if (q0 < p.T)
    store_transposed(stage, o0, o1, inv, o + (long)b * p.T * p.HD + h * p.dk, p.HD, q0, min(32, p.T - q0), p.dk,
                     lane);
  if (hh == 0 && qi < p.T) lse[((long)b * p.H + h) * p.T + qi] = (m + __log2f(l)) * LN2;
}

// dQ: grid (B*H), block 64 * ceil(T/32); K and V staged whole
__global__ __launch_bounds__(64 * HEAD_TMAX / 32) void attn_bwd_dq_head_kernel(AttnM p, const bf16* __restrict__ dout,
                                                                               const float* __restrict__ lse,
                                                                               const float* __restrict__ Dg,
                                                                               bf16* __restrict__ dqkv) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  const uint32_t dkey = drop_key(p.seed, 0), dthr = drop_thr(p.drop_p);
  const float dkeep = drop_keep_scale(dthr);
  extern __shared__ __attribute__((aligned(16))) bf16 hsm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5;
  const HeadPart hp = head_part(p);
  const int b = hp.b, h = hp.h;
  const int len = p.len[b];
  const int nkt = (len + TILE - 1) / TILE, Tp = nkt * TILE;
  bf16* sKall = hsm;
  bf16* sVall = hsm + (long)Tp * KS;
  const bf16* kvbase = p.qkv + (long)b * p.T * p.D3;
  head_stage(p, kvbase + p.HD + h * p.dk, kvbase + 2 * p.HD + h * p.dk, p.D3, p.D3, Tp, sKall, sVall, tid,
             blockDim.x);
  const int q0 = (hp.blk0 + wv) * 32;
  const int qi = q0 + (lane & 31);
  bf16x8 qf[4], gf[4];
  load_bfrags(p, kvbase + h * p.dk, p.D3, qi, p.T, qf, lane);
  load_bfrags(p, dout + (long)b * p.T * p.HD + h * p.dk, p.HD, qi, p.T, gf, lane);
  const bool qvalid = qi < p.T;
  const float L2 = qvalid ? lse[((long)b * p.H + h) * p.T + qi] * LOG2E : INFINITY;   // rows past T: P = 0
  const float Dq = qvalid ? Dg[((long)b * p.H + h) * p.T + qi] : 0.f;
  const float c = p.scale * LOG2E;
  __syncthreads();
  f32x16 a0 = (f32x16){0}, a1 = (f32x16){0};
  // 32-key steps (S^T, dP^T: 32 accumulator registers live -> no spill under the 12-wave cap); dropout
  // pairs (keys k, k+1 in registers r, r+1) hash (didx >> 1) mod 2^32 = (bh T + qi) T2 + k/2 in 32 bits
  const int nks = (len + 31) / 32;
  const uint32_t T2 = (uint32_t)(p.T + (p.T & 1)) >> 1;
  const uint32_t hq = ((uint32_t)(b * p.H + h) * (uint32_t)p.T + (uint32_t)qi) * T2 + (uint32_t)(2 * hh);
  const float keep = p.drop_p > 0.f ? dkeep : 1.f;
  auto sd = [&](int ks, f32x16& s0, f32x16& d0) {
    const int k0 = ks * 32;
    s0 = (f32x16){0};
    d0 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sKall, k0, 16 * s, lane), qf[s], s0, 0, 0, 0);
      d0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sVall, k0, 16 * s, lane), gf[s], d0, 0, 0, 0);
    }
  };
  auto ds = [&](int ks, f32x16& s0, f32x16& d0) {   // s0 <- dS^T = P (dP keep - D), then dQ^T += K^T dS^T
    const int k0 = ks * 32;
    if (p.drop_p > 0.f) {
#pragma unroll
      for (int r = 0; r < 16; r += 2) {     // registers r, r+1 = keys k, k+1 with k even: one hash
        const uint32_t hsh = attn_mix(
            hq + dkey + __builtin_amdgcn_readfirstlane((k0 + (r & 3) + 8 * (r >> 2)) >> 1));
        d0[r] = (hsh & 0xFFFFu) >= dthr ? d0[r] : 0.f;
        d0[r + 1] = (hsh >> 16) >= dthr ? d0[r + 1] : 0.f;
      }
    }
    if (k0 + 32 > len) {     // the last (partial) key step only: masked keys
#pragma unroll
      for (int r = 0; r < 16; ++r) s0[r] = k0 + acc_row(r, hh) < len ? s0[r] : -INFINITY;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p0 = fast_exp2(__builtin_fmaf(s0[r], c, -L2));
      s0[r] = p0 * __builtin_fmaf(d0[r], keep, -Dq);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pf = acc2frag(s0, s);
      a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sKall, k0 + 16 * s, 0, lane), pf, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sKall, k0 + 16 * s, 32, lane), pf, a1, 0, 0, 0);
    }
  };
  f32x16 sa, da;
  for (int ks = 0; ks < nks; ++ks) {
    sd(ks, sa, da);
    __builtin_amdgcn_sched_barrier(0);
    ds(ks, sa, da);
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  float* stage = reinterpret_cast<float*>(hsm) + wv * 32 * 65;
  if (q0 < p.T)
    store_transposed(stage, a0, a1, p.scale, dqkv + (long)b * p.T * p.D3 + h * p.dk, p.D3, q0, min(32, p.T - q0),
                     p.dk, lane);
}

// write a wave's 64(d) x 32(key) f32 accumulator pair transposed into bf16 rows, straight from the
// registers: lane (key c, half hh) owns d = 32t + 8g + 4hh .. +3 of register group g -> one 8-byte store
// each (rows row0 + c < row0 + nvalid, d < dk)
__device__ __forceinline__ void store_acc_rows(const f32x16& a0, const f32x16& a1, float mul, bf16* out, long ld,
                                               int row0, int nvalid, int dk, bool v8, int lane) {
  const int hh = lane >> 5, c = lane & 31;
  if (c >= nvalid) return;
  bf16* o = out + (long)(row0 + c) * ld;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const f32x16& a = t ? a1 : a0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * t + 8 * g + 4 * hh;
      if (v8 && d + 4 <= dk) {
        bf16x4 v = {(bf16)(a[4 * g] * mul), (bf16)(a[4 * g + 1] * mul), (bf16)(a[4 * g + 2] * mul),
                    (bf16)(a[4 * g + 3] * mul)};
        *reinterpret_cast<bf16x4*>(o + d) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (d + e < dk) o[d + e] = (bf16)(a[4 * g + e] * mul);
      }
    }
  }
}

// dK, dV, one wave per 32-key block: grid (B*H), block 64 * ceil(T/32) (three waves per SIMD at
// T = 373); the head's whole Q and dO (and lse, D) are staged once and every wave sweeps 32-query
// steps over them with no further barriers.  Two passes keep every wave under the three-wave register
// cap with nothing spilled: pass 1 forms P and accumulates dV^T += dO^T P (8 MFMAs per step), stores dV
// straight from the registers, and leaves the step's dropout keep bits in LDS; pass 2 recomputes S,
// forms dP and dS and accumulates dK^T += Q^T dS (12 MFMAs per step).  Masked keys enter the exponential
// as -inf (branch-free).  Attention dropout: the hash index of element (q, kj) is (didx >> 1) mod 2^32
// = (bh T + q) T2 + kj/2 (T2 = even T / 2; exact: didx < 2^33), so lanes kj and kj^1 share one 32-bit
// hash per query: the even lane hashes the query of accumulator register r, the odd lane that of r + 1,
// and one DPP swap hands each lane its partner's -- one hash per two elements, 32-bit index arithmetic.
// dsT (round 6, may be null): pass 2 also stores dS^T (bf16, unscaled) key-major -- dsT[(b H + h)][key][query],
// Tq x Tq per head (Tq = T rounded up to 32), four 8-B runs of consecutive queries per lane and step -- for
// attn_bwd_dqs_head_kernel.  Key blocks at or past len store nothing (the consumer masks keys >= len).
__global__ __launch_bounds__(64 * HEAD_TMAX / 32) void attn_bwd_dkdv_wave_kernel(AttnM p, const bf16* __restrict__ dout,
                                                                                 const float* __restrict__ lse,
                                                                                 const float* __restrict__ Dg,
                                                                                 bf16* __restrict__ dqkv,
                                                                                 bf16* __restrict__ dsT) {
  const bool drop = p.drop_p > 0.f;
  if (drop) p.seed = salted_seed(p.seed, p.salt);
  const uint32_t dkey = drop_key(p.seed, 0), dthr = drop_thr(p.drop_p);
  const float dkeep = drop_keep_scale(dthr);
  extern __shared__ __attribute__((aligned(16))) bf16 hsm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5;
  const HeadPart hp = head_part(p);
  const int b = hp.b, h = hp.h;
  const int len = p.len[b];
  const int nq = (p.T + 31) / 32, Tq = nq * 32;
  bf16* sQall = hsm;
  bf16* sGall = hsm + (long)Tq * KS;
  float* sL = reinterpret_cast<float*>(sGall + (long)Tq * KS);      // [Tq] lse * log2(e) (+inf past T)
  float* sD = sL + Tq;                                              // [Tq] D
  unsigned short* sM = reinterpret_cast<unsigned short*>(sD + Tq);  // [wave][step][lane] pass-1 keep bits
  const bf16* qbase = p.qkv + (long)b * p.T * p.D3 + h * p.dk;
  head_stage(p, qbase, dout + (long)b * p.T * p.HD + h * p.dk, p.D3, p.HD, Tq, sQall, sGall, tid, blockDim.x);
  for (int i = tid; i < Tq; i += blockDim.x) {
    sL[i] = i < p.T ? lse[((long)b * p.H + h) * p.T + i] * LOG2E : INFINITY;
    sD[i] = i < p.T ? Dg[((long)b * p.H + h) * p.T + i] : 0.f;
  }
  const int k0w = (hp.blk0 + wv) * 32;
  const int kj = k0w + (lane & 31);
  const bool kvalid = kj < len;
  bf16x8 kf[4], vf[4];
  load_bfrags(p, qbase + p.HD, p.D3, kj, p.T, kf, lane);
  load_bfrags(p, qbase + 2 * p.HD, p.D3, kj, p.T, vf, lane);
  __syncthreads();
  const float c = p.scale * LOG2E;
  const int nqs = k0w < len ? nq : 0;      // key blocks past len: zero gradients
  const int odd = lane & 1, sh = 16 * odd;
  const uint32_t T2 = (uint32_t)(p.T + (p.T & 1)) >> 1;
  const uint32_t hbase = ((uint32_t)(b * p.H + h) * (uint32_t)p.T + (uint32_t)(4 * hh + odd)) * T2 + (uint32_t)(kj >> 1);
  unsigned short* myM = sM + (long)wv * nq * 64 + lane;
  bf16* obase = dqkv + (long)b * p.T * p.D3 + h * p.dk;
  const int nvalid = min(32, p.T - k0w);
  const bool v8 = p.vec && ((uintptr_t)dqkv & 7) == 0;

  // ---- pass 1: P, dV^T += dO^T P
  {
    f32x16 dv0 = (f32x16){0}, dv1 = (f32x16){0};
    auto sc = [&](int qt, f32x16& sa) {
      sa = (f32x16){0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sQall, qt * 32, 16 * s4, lane), kf[s4], sa, 0, 0, 0);
    };
    auto pdv = [&](int qt, const f32x16& sa) {
      const int q0 = qt * 32;
      bf16x8 pf[2];
      unsigned bits = 0u;
#pragma unroll
      for (int g = 0; g < 4; ++g) {          // registers 4g .. 4g+3 = queries q0 + 8g + 4hh + 0..3
        const float4 Lg = *reinterpret_cast<const float4*>(sL + q0 + 8 * g + 4 * hh);
        const float Lr[4] = {Lg.x, Lg.y, Lg.z, Lg.w};
        float mk[4] = {1.f, 1.f, 1.f, 1.f};
        if (drop) {
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            // (the wave-uniform offset through readfirstlane: otherwise the per-register bases are
            // hoisted out of the loop as VGPRs)
            const uint32_t hm = attn_mix(hbase + dkey + __builtin_amdgcn_readfirstlane((q0 + 8 * g + e) * (int)T2));
            const uint32_t ho = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hm, 0xB1, 0xF, 0xF, false);  // lane ^ 1
            const uint32_t h0 = odd ? ho : hm, h1 = odd ? hm : ho;
            const bool k0 = ((h0 >> sh) & 0xFFFFu) >= dthr, k1 = ((h1 >> sh) & 0xFFFFu) >= dthr;
            mk[e] = k0 ? dkeep : 0.f;
            mk[e + 1] = k1 ? dkeep : 0.f;
            bits |= (k0 ? 1u : 0u) << (4 * g + e);
            bits |= (k1 ? 2u : 0u) << (4 * g + e);
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          const float pa = fast_exp2(__builtin_fmaf(sa[r], c, -Lr[e]));   // lse = +inf for q >= T
          pf[r >> 3][r & 7] = (bf16)(pa * mk[e]);
        }
      }
      if (drop) myM[qt * 64] = (unsigned short)bits;
      if (!kvalid) pf[0] = pf[1] = (bf16x8){0};     // keys past len: P = 0 (one select per packed register)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sGall, q0 + 16 * s2, 0, lane), pf[s2], dv0, 0, 0, 0);
        dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sGall, q0 + 16 * s2, 32, lane), pf[s2], dv1, 0, 0, 0);
      }
    };
    f32x16 sa;
    for (int qt = 0; qt < nqs; ++qt) {
      sc(qt, sa);
      __builtin_amdgcn_sched_barrier(0);
      pdv(qt, sa);
      __builtin_amdgcn_sched_barrier(0);
    }
    store_acc_rows(dv0, dv1, 1.f, obase + 2 * p.HD, p.D3, k0w, nvalid, p.dk, v8, lane);
  }
  // ---- pass 2: dP, dS, dK^T += Q^T dS
  {
    const float keep = drop ? dkeep : 1.f;
    f32x16 dk0 = (f32x16){0}, dk1 = (f32x16){0};
    auto sg = [&](int qt, f32x16& sa, f32x16& ga) {
      sa = (f32x16){0};
      ga = (f32x16){0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sQall, qt * 32, 16 * s4, lane), kf[s4], sa, 0, 0, 0);
        ga = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sGall, qt * 32, 16 * s4, lane), vf[s4], ga, 0, 0, 0);
      }
    };
    auto dsk = [&](int qt, const f32x16& sa, const f32x16& ga) {
      const int q0 = qt * 32;
      const unsigned bits = drop ? (unsigned)myM[qt * 64] : 0xFFFFu;
      bf16x8 sf[2];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 Lg = *reinterpret_cast<const float4*>(sL + q0 + 8 * g + 4 * hh);
        const float4 Dq = *reinterpret_cast<const float4*>(sD + q0 + 8 * g + 4 * hh);
        const float Lr[4] = {Lg.x, Lg.y, Lg.z, Lg.w}, Dr[4] = {Dq.x, Dq.y, Dq.z, Dq.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          const float pa = fast_exp2(__builtin_fmaf(sa[r], c, -Lr[e]));
          const float gk = (bits >> r) & 1u ? ga[r] : 0.f;
          sf[r >> 3][r & 7] = (bf16)(pa * __builtin_fmaf(gk, keep, -Dr[e]));
        }
      }
      if (!kvalid) sf[0] = sf[1] = (bf16x8){0};
      if (dsT) {   // registers 4g .. 4g+3 = queries q0 + 8g + 4hh + 0..3 of key kj
        bf16* drow = dsT + ((long)(b * p.H + h) * Tq + kj) * Tq + q0 + 4 * hh;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const bf16x8& v = sf[g >> 1];
          const int o = 4 * (g & 1);
          bf16x4 w = {v[o], v[o + 1], v[o + 2], v[o + 3]};
          *reinterpret_cast<uint2*>(drow + 8 * g) = __builtin_bit_cast(uint2, w);
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sQall, q0 + 16 * s2, 0, lane), sf[s2], dk0, 0, 0, 0);
        dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sQall, q0 + 16 * s2, 32, lane), sf[s2], dk1, 0, 0, 0);
      }
    };
    f32x16 sa, ga;
    for (int qt = 0; qt < nqs; ++qt) {
      sg(qt, sa, ga);
      __builtin_amdgcn_sched_barrier(0);
      dsk(qt, sa, ga);
      __builtin_amdgcn_sched_barrier(0);
    }
    store_acc_rows(dk0, dk1, p.scale, obase + p.HD, p.D3, k0w, nvalid, p.dk, v8, lane);
  }
}

// ------------------------------------------------------------------------------------ dQ from the stored dS^T
// (round 6 default on the whole-head path when the caller passes the full workspace; cfm_attn_set_mode bit 10 keeps
// attn_bwd_dq_head_kernel).  dq_i = scale * sum_j dS_ij k_j over the dS^T that attn_bwd_dkdv_wave_kernel stored:
// 8 MFMAs per 64-key tile and wave, no score / softmax / dropout-hash / dO x V recompute.  Whole-head layout like the
// other head kernels: grid (B*H*qs), one wave per 32-query block; the head's K is staged once (192-B rows: the
// transposed fragment reads are conflict free), then each wave streams its [64 keys][32 queries] dS^T slices through
// a private 4 KiB LDS image (64-B rows, conflict free for the same reads; the next slice in registers while the
// current one runs) -- no workgroup barrier inside the loop.  Keys >= len read as zero.  After the loop the LDS holds
// the waves' f32 stages of the dq store.
constexpr int DQH_KS = 96;
size_t dqs_head_lds_bytes(int T, int waves) {
  const size_t tk = (size_t)cdiv(T, TILE) * TILE;   // K rows: whole 64-key tiles (rows >= T zero)
  const size_t loop = tk * DQH_KS * 2 + (size_t)waves * TILE * 32 * 2, stage = (size_t)waves * 32 * 65 * 4;
  return loop > stage ? loop : stage;
}
__global__ __launch_bounds__(64 * HEAD_TMAX / 32) void attn_bwd_dqs_head_kernel(AttnM p, const bf16* __restrict__ dsT,
                                                                                bf16* __restrict__ dqkv) {
  extern __shared__ __attribute__((aligned(16))) bf16 hsm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const HeadPart hp = head_part(p);
  const int b = hp.b, h = hp.h;
  const int len = p.len[b];
  const int nq = (p.T + 31) / 32, Tq = nq * 32;
  const int Tk = (p.T + TILE - 1) / TILE * TILE;   // the last key tile's rows are all staged (zero past T)
  bf16* sK = hsm;
  bf16* simg = hsm + (long)Tk * DQH_KS + wv * TILE * 32;
  // the head's K rows [0, Tk) (rows >= T read as zero)
  const bf16* kbase = p.qkv + (long)b * p.T * p.D3 + p.HD + h * p.dk;
  for (int i = tid; i < Tk * 8; i += blockDim.x) {
    const int row = i >> 3, c = (i & 7) * 8;
    *reinterpret_cast<uint4*>(sK + row * DQH_KS + c) = ld8(kbase, p.D3, row, p.T, c, p.dk, p.vec, p.vec4);
  }
  __syncthreads();
  const int q0 = (hp.blk0 + wv) * 32;
  const int nkt = q0 < p.T ? (len + TILE - 1) / TILE : 0;
  const bf16* dbase = dsT + (long)(b * p.H + h) * Tq * Tq + (q0 < Tq ? q0 : 0);
  uint4 rd[4];
  auto dload = [&](int kt) {   // chunk idx = lane + 64 i -> key row idx >> 2, queries 8 (idx & 3) .. +7
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = lane + 64 * i, key = kt * TILE + (idx >> 2);
      rd[i] = key < len ? *reinterpret_cast<const uint4*>(dbase + (long)key * Tq + 8 * (idx & 3)) : make_uint4(0, 0, 0, 0);
    }
  };
  auto dstore = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = lane + 64 * i;
      *reinterpret_cast<uint4*>(simg + (idx >> 2) * 32 + 8 * (idx & 3)) = rd[i];
    }
  };
  f32x16 a0 = (f32x16){0}, a1 = (f32x16){0};
  if (nkt > 0) {
    dload(0);
    dstore();
  }
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 1 < nkt) dload(kt + 1);
    // (the slice's stores and these reads are one wave's LDS operations: in order)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 bfr = trfrag_perm_s<32>(simg, 32 * t + 16 * s2, 0, lane);   // dS^T: k = keys, columns = queries
        const int kr = kt * TILE + 32 * t + 16 * s2;
        a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm_s<DQH_KS>(sK, kr, 0, lane), bfr, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm_s<DQH_KS>(sK, kr, 32, lane), bfr, a1, 0, 0, 0);
      }
    if (kt + 1 < nkt) {
      __builtin_amdgcn_wave_barrier();
      dstore();
    }
  }
  __syncthreads();   // every wave's reads of K and of its slice are done before the stages reuse the bytes
  float* st = reinterpret_cast<float*>(hsm) + wv * 32 * 65;
  if (q0 < p.T)
    store_transposed(st, a0, a1, p.scale, dqkv + (long)b * p.T * p.D3 + h * p.dk, p.D3, q0, min(32, p.T - q0), p.dk,
                     lane);
}

size_t dkdv_wave_lds_bytes(int T, int waves) {
  const size_t nq = (size_t)cdiv(T, 32), rows = nq * 32;
  return 2 * rows * KS * sizeof(bf16) + 2 * rows * sizeof(float) + (size_t)waves * nq * 64 * sizeof(unsigned short);
}

// ------------------------------------------------------------------------------------ D = rowsum(dO*O)
// one wave per (b, t) token row: lanes sweep the H*dk features (coalesced), per-head sums via LDS
__global__ __launch_bounds__(256) void attn_bwd_dot_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ o,
                                                           float* __restrict__ D, int B, int T, int H, int dk) {
  __shared__ float sacc[4][1024];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long row = (long)blockIdx.x * 4 + wv;          // b*T + t
  const int HD = H * dk;
  if (row < (long)B * T) {
    const bf16* g = dout + row * HD;
    const bf16* x = o + row * HD;
    for (int c = lane; c < HD; c += 64) sacc[wv][c] = (float)g[c] * (float)x[c];
  }
  __syncthreads();
  if (row < (long)B * T) {
    const int b = (int)(row / T), t = (int)(row % T);
    for (int h = lane; h < H; h += 64) {
      float s = 0.f;
      for (int d = 0; d < dk; ++d) s += sacc[wv][h * dk + d];
      D[((long)b * H + h) * T + t] = s;
    }
  }
}

// ------------------------------------------------------------------------------------ dQ
// grid (ceil(T/128), H, B); wave = 32 queries.  dqkv q-part written (bf16), scaled by 1/sqrt(dk).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void attn_bwd_dq_kernel(AttnM p, const bf16* __restrict__ dout,
                                                          const float* __restrict__ lse, const float* __restrict__ Dg,
                                                          bf16* __restrict__ dqkv) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  const uint32_t dkey = drop_key(p.seed, 0), dthr = drop_thr(p.drop_p);
  const float dkeep = drop_keep_scale(dthr);
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TILE * KS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5;
  const int h = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * 128 + wv * 32;
  const int qi = q0 + (lane & 31);
  const int len = p.len[b];
  bf16x8 qf[4], gf[4];
  load_bfrags(p, p.qkv + (long)b * p.T * p.D3 + h * p.dk, p.D3, qi, p.T, qf, lane);
  load_bfrags(p, dout + (long)b * p.T * p.HD + h * p.dk, p.HD, qi, p.T, gf, lane);
  const bool qvalid = qi < p.T;
  const float L2 = qvalid ? lse[((long)b * p.H + h) * p.T + qi] * LOG2E : 0.f;
  const float Dq = qvalid ? Dg[((long)b * p.H + h) * p.T + qi] : 0.f;
  const float c = p.scale * LOG2E;
  f32x16 a0 = (f32x16){0}, a1 = (f32x16){0};
  const int nkt = (len + TILE - 1) / TILE;
  uint4 rk[2], rv[2];
  const int kcol = p.HD + h * p.dk, vcol = 2 * p.HD + h * p.dk;
  if (nkt > 0) {
    tile_load(p, b, 0, kcol, rk, tid);
    tile_load(p, b, 0, vcol, rv, tid);
    tile_store(smem, rk, tid);
    tile_store(smem + TILE * KS, rv, tid);
    __syncthreads();
  }
  for (int kt = 0; kt < nkt; ++kt) {
    const bf16* sK = smem + (kt & 1) * 2 * TILE * KS;
    const bf16* sV = sK + TILE * KS;
    if (kt + 1 < nkt) {
      tile_load(p, b, (kt + 1) * TILE, kcol, rk, tid);
      tile_load(p, b, (kt + 1) * TILE, vcol, rv, tid);
    }
    f32x16 s0 = (f32x16){0}, s1 = (f32x16){0}, d0 = (f32x16){0}, d1 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 0, 16 * s, lane), qf[s], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 32, 16 * s, lane), qf[s], s1, 0, 0, 0);
      d0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sV, 0, 16 * s, lane), gf[s], d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sV, 32, 16 * s, lane), gf[s], d1, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k0 = kt * TILE + acc_row(r, hh);
      float p0 = (k0 < len && qvalid) ? exp2f(s0[r] * c - L2) : 0.f;
      float p1 = (k0 + 32 < len && qvalid) ? exp2f(s1[r] * c - L2) : 0.f;
      float g0 = d0[r], g1 = d1[r];
      if (p.drop_p > 0.f) {
        g0 *= dropout_keyed(dthr, dkeep, dkey, didx(p, b, h, qi, k0));
        g1 *= dropout_keyed(dthr, dkeep, dkey, didx(p, b, h, qi, k0 + 32));
      }
      s0[r] = p0 * (g0 - Dq);
      s1[r] = p1 * (g1 - Dq);
    }
    // dQ^T[d][q] += sum_key K[key][d] dS^T[key][q]
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc2frag(t == 0 ? s0 : s1, s);
        a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sK, 32 * t + 16 * s, 0, lane), pf, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sK, 32 * t + 16 * s, 32, lane), pf, a1, 0, 0, 0);
      }
    }
    if (kt + 1 < nkt) {
      bf16* nK = smem + ((kt + 1) & 1) * 2 * TILE * KS;
      tile_store(nK, rk, tid);
      tile_store(nK + TILE * KS, rv, tid);
    }
    __syncthreads();
  }
  float* stage = reinterpret_cast<float*>(smem) + wv * 32 * 65;
  store_transposed(stage, a0, a1, p.scale, dqkv + (long)b * p.T * p.D3 + h * p.dk, p.D3, q0, min(32, p.T - q0),
                   p.dk, lane);
}

// ------------------------------------------------------------------------------------ dK, dV
// grid (ceil(T/128), H, B); wave = 32 keys on the lanes; loops over query tiles of 64.
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnM p, const bf16* __restrict__ dout,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ Dg, bf16* __restrict__ dqkv) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  const uint32_t dkey = drop_key(p.seed, 0), dthr = drop_thr(p.drop_p);
  const float dkeep = drop_keep_scale(dthr);
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TILE * KS];   // [buf][Q, dO][64][72]
  __shared__ float sLD[2][2][TILE];                                        // [buf][lse2, D][64]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5;
  const int h = blockIdx.y, b = blockIdx.z;
  const int k0w = blockIdx.x * 128 + wv * 32;
  const int kj = k0w + (lane & 31);
  const int len = p.len[b];
  const bool kvalid = kj < len;
  bf16x8 kf[4], vf[4];
  load_bfrags(p, p.qkv + (long)b * p.T * p.D3 + p.HD + h * p.dk, p.D3, kj, p.T, kf, lane);
  load_bfrags(p, p.qkv + (long)b * p.T * p.D3 + 2 * p.HD + h * p.dk, p.D3, kj, p.T, vf, lane);
  const float c = p.scale * LOG2E;
  f32x16 dk0 = (f32x16){0}, dk1 = (f32x16){0}, dv0 = (f32x16){0}, dv1 = (f32x16){0};
  // the whole block may be past len: still write zeros (outputs must be defined)
  const bool block_live = blockIdx.x * 128 < len;
  const int nqt = block_live ? (p.T + TILE - 1) / TILE : 0;
  uint4 rq[2], rg[2];
  float rl = 0.f, rd = 0.f;
  auto gload = [&](int qt) {
    const int r0 = qt * TILE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + 256 * i;
      rq[i] = ld8(p.qkv + (long)b * p.T * p.D3 + h * p.dk, p.D3, r0 + (v >> 3), p.T, (v & 7) * 8, p.dk, p.vec);
      rg[i] = ld8(dout + (long)b * p.T * p.HD + h * p.dk, p.HD, r0 + (v >> 3), p.T, (v & 7) * 8, p.dk, p.vec);
    }
    if (tid < TILE) {
      const int qi = r0 + tid;
      rl = qi < p.T ? lse[((long)b * p.H + h) * p.T + qi] * LOG2E : INFINITY;
      rd = qi < p.T ? Dg[((long)b * p.H + h) * p.T + qi] : 0.f;
    }
  };
  auto sstore = [&](int buf) {
    bf16* t = smem + buf * 2 * TILE * KS;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + 256 * i;
      *reinterpret_cast<uint4*>(t + (v >> 3) * KS + (v & 7) * 8) = rq[i];
      *reinterpret_cast<uint4*>(t + TILE * KS + (v >> 3) * KS + (v & 7) * 8) = rg[i];
    }
    if (tid < TILE) {
      sLD[buf][0][tid] = rl;
      sLD[buf][1][tid] = rd;
    }
  };
  if (nqt > 0) {
    gload(0);
    sstore(0);
    __syncthreads();
  }
  for (int qt = 0; qt < nqt; ++qt) {
    const int cur = qt & 1;
    const bf16* sQ = smem + cur * 2 * TILE * KS;
    const bf16* sG = sQ + TILE * KS;
    if (qt + 1 < nqt) gload(qt + 1);
    // S[q][key] (rows: 2 tiles of 32 queries), dP[q][key]
    f32x16 s0 = (f32x16){0}, s1 = (f32x16){0}, g0 = (f32x16){0}, g1 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sQ, 0, 16 * s, lane), kf[s], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sQ, 32, 16 * s, lane), kf[s], s1, 0, 0, 0);
      g0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sG, 0, 16 * s, lane), vf[s], g0, 0, 0, 0);
      g1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sG, 32, 16 * s, lane), vf[s], g1, 0, 0, 0);
    }
    f32x16 pd0, pd1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qa = acc_row(r, hh), qb = 32 + qa;
      const int qia = qt * TILE + qa, qib = qt * TILE + qb;
      const float pa = kvalid ? exp2f(s0[r] * c - sLD[cur][0][qa]) : 0.f;   // lse = +inf for q >= T
      const float pb = kvalid ? exp2f(s1[r] * c - sLD[cur][0][qb]) : 0.f;
      float ma = 1.f, mb = 1.f;
      if (p.drop_p > 0.f) {
        ma = dropout_keyed(dthr, dkeep, dkey, didx(p, b, h, qia, kj));
        mb = dropout_keyed(dthr, dkeep, dkey, didx(p, b, h, qib, kj));
      }
      pd0[r] = pa * ma;
      pd1[r] = pb * mb;
      s0[r] = pa * (g0[r] * ma - sLD[cur][1][qa]);
      s1[r] = pb * (g1[r] * mb - sLD[cur][1][qb]);
    }
    // dV^T[d][key] += sum_q dO[q][d] Pd[q][key];  dK^T[d][key] += sum_q Q[q][d] dS[q][key]
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc2frag(t == 0 ? pd0 : pd1, s);
        const bf16x8 sf = acc2frag(t == 0 ? s0 : s1, s);
        dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sG, 32 * t + 16 * s, 0, lane), pf, dv0, 0, 0, 0);
        dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sG, 32 * t + 16 * s, 32, lane), pf, dv1, 0, 0, 0);
        dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sQ, 32 * t + 16 * s, 0, lane), sf, dk0, 0, 0, 0);
        dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sQ, 32 * t + 16 * s, 32, lane), sf, dk1, 0, 0, 0);
      }
    }
    if (qt + 1 < nqt) sstore(cur ^ 1);
    __syncthreads();
  }
  float* stage = reinterpret_cast<float*>(smem) + wv * 32 * 65;
  const int nvalid = min(32, p.T - k0w);
  bf16* base = dqkv + (long)b * p.T * p.D3 + h * p.dk;
  store_transposed(stage, dk0, dk1, p.scale, base + p.HD, p.D3, k0w, nvalid, p.dk, lane);
  store_transposed(stage, dv0, dv1, 1.f, base + 2 * p.HD, p.D3, k0w, nvalid, p.dk, lane);
}

// bf16 runs on MFMA (pos != nullptr: attention_rel.hip); fp32 (the parity mode) on the SIMT kernels.
// cfm_attn_set_mode bit 4 sends bf16 rel-pos back to SIMT (A/B, parity cross-check).
int g_attn_mode = 0;
bool use_mfma(int dtype, const void* pos, int dk) {
  return dtype == CFM_BF16 && dk <= DKP && (pos == nullptr || (g_attn_mode & 16) == 0);
}

// whole-head kernels: T <= HEAD_TMAX; cfm_attn_set_mode bit 0 forces the tiled kernels (A/B, parity)
bool use_head(int T) { return T <= HEAD_TMAX && (g_attn_mode & 1) == 0; }
size_t head_lds_bytes(int T, int waves) {
  const size_t rows = (size_t)cdiv(T, TILE) * TILE;
  const size_t img = 2 * rows * KS * sizeof(bf16);
  const size_t stage = (size_t)waves * 32 * 65 * sizeof(float);
  return img > stage ? img : stage;
}

int attn_num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// workgroups per (b, h) of the whole-head kernels: enough to give every CU one (B*H*qs <= CUs), at most 4 and at most
// one 32-row block each (cfm_attn_set_mode bit 6: always one, A/B)
int head_split(int B, int H, int T) {
  if (g_attn_mode & 64) return 1;
  const int nb = cdiv(T, 32), bh = B * H, cus = attn_num_cus();
  int qs = 1;
  while (qs < 4 && qs < nb && (long)bh * (qs + 1) <= cus) ++qs;
  return qs;
}

}  // namespace

CFM_EXPORT int cfm_attn_fwd(const void* qkv, void* o, float* lse, const int32_t* lengths, const void* pos,
                            const float* pos_u, const float* pos_v, int B, int T, int H, int dk, int dtype,
                            float drop_p, uint64_t seed, void* stream) {
  CFM_REQUIRE(qkv && o && lse && lengths, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(B > 0 && T > 0 && H > 0 && dk > 0 && dk <= 1024, CFM_ERR_SHAPE, "bad shape");
  CFM_REQUIRE(!pos || (pos_u && pos_v), CFM_ERR_ARG, "rel-pos needs pos_u and pos_v");
  CFM_REQUIRE(dtype == CFM_BF16 || dtype == CFM_F32, CFM_ERR_DTYPE, "dtype");
  CFM_REQUIRE(pos || dtype == CFM_F32 || dk <= DKP, CFM_ERR_UNSUPPORTED, "bf16 head dim must be <= 64");
  CFM_REQUIRE((double)B * H * T * (T + 1) < 8589934592.0, CFM_ERR_SHAPE, "attention dropout index space (2^33)");
  hipStream_t s = cfm::as_stream(stream);
  if (!use_mfma(dtype, pos, dk))
    return cfm::attn_simt_fwd_launch(qkv, o, lse, lengths, pos, pos_u, pos_v, B, T, H, dk, dtype, drop_p, seed, s);
  if (pos)
    return cfm::attn_rel_fwd_launch(qkv, o, lse, lengths, pos, pos_u, pos_v, B, T, H, dk, drop_p, seed, s);
  AttnM p{(const bf16*)qkv, B, T, H, dk, 3 * H * dk, H * dk, lengths, 1.f / sqrtf((float)dk), drop_p, seed,
          ((uintptr_t)qkv % 16 == 0) && (dk % 8 == 0) && ((3 * H * dk) % 8 == 0), g_attn_mode & 6,
          cfm::g_rng_salt};
  p.vec4 = ((uintptr_t)qkv % 8 == 0) && (dk % 4 == 0) && ((3 * H * dk) % 4 == 0);
  if (use_head(T)) {
    // LDS sized for the full padded length (lengths are device data; len <= T)
    p.qs = head_split(B, H, T);
    const int waves = cdiv(cdiv(T, 32), p.qs);
    hipLaunchKernelGGL(attn_fwd_head_kernel, dim3(B * H * p.qs), dim3(64 * waves), head_lds_bytes(T, waves), s, p,
                       (bf16*)o, lse);
    return cfm::check_launch("cfm_attn_fwd");
  }
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(cdiv(T, 128), H, B), dim3(256), 0, s, p, (bf16*)o, lse);
  return cfm::check_launch("cfm_attn_fwd");
}

// the whole-head backward's dS^T buffer (dQ from dS): after D in the full workspace
static bool dsT_path(int T) { return use_head(T) && !(g_attn_mode & 1024); }
static size_t d_slot_bytes(int B, int T, int H) { return ((size_t)B * H * T * sizeof(float) + 255) & ~(size_t)255; }
static size_t dsT_bytes(int B, int T, int H) { const size_t tq = (size_t)cdiv(T, 32) * 32; return (size_t)B * H * tq * tq * 2; }

CFM_EXPORT size_t cfm_attn_bwd_ws_bytes(int B, int T, int H, int dk, int rel, int dtype) {
  if (!use_mfma(dtype, rel ? (const void*)1 : nullptr, dk)) return cfm::attn_simt_ws_bytes(B, T, H);
  if (rel) return cfm::attn_rel_ws_bytes(B, T, H, dk);
  if (dsT_path(T)) return d_slot_bytes(B, T, H) + dsT_bytes(B, T, H);
  return (size_t)B * H * T * sizeof(float);
}

static int attn_bwd_impl(const void* qkv, const void* o, const void* dout, const float* lse,
                         const int32_t* lengths, const void* pos, const float* pos_u, const float* pos_v,
                         void* dqkv, void* dpos, int dpos_dt, float* dpos_u, float* dpos_v, int B, int T, int H,
                         int dk, int dtype, float drop_p, uint64_t seed, float* ws, void* stream, bool d_ready,
                         bool full_ws) {
  CFM_REQUIRE(qkv && o && dout && lse && lengths && dqkv && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(B > 0 && T > 0 && H > 0 && dk > 0, CFM_ERR_SHAPE, "bad shape");
  CFM_REQUIRE(!pos || (pos_u && pos_v && dpos && dpos_u && dpos_v), CFM_ERR_ARG, "rel-pos grads need buffers");
  hipStream_t s = cfm::as_stream(stream);
  CFM_REQUIRE(!d_ready || use_mfma(dtype, pos, dk), CFM_ERR_UNSUPPORTED, "precomputed D: bf16 MFMA path only");
  CFM_REQUIRE(dpos_dt == CFM_F32 || (dpos_dt == CFM_BF16 && pos && use_mfma(dtype, pos, dk)), CFM_ERR_DTYPE,
              "dpos: fp32, or bf16 on the rel-pos MFMA path");
  if (!use_mfma(dtype, pos, dk))
    return cfm::attn_simt_bwd_launch(qkv, o, dout, lse, lengths, pos, pos_u, pos_v, dqkv, (float*)dpos, dpos_u,
                                     dpos_v, B, T, H, dk, dtype, drop_p, seed, ws, s);
  AttnM p{(const bf16*)qkv, B, T, H, dk, 3 * H * dk, H * dk, lengths, 1.f / sqrtf((float)dk), drop_p, seed,
          ((uintptr_t)qkv % 16 == 0) && ((uintptr_t)dout % 16 == 0) && (dk % 8 == 0) && ((3 * H * dk) % 8 == 0),
          g_attn_mode & 6, cfm::g_rng_salt};
  p.vec4 = ((uintptr_t)qkv % 8 == 0) && ((uintptr_t)dout % 8 == 0) && (dk % 4 == 0) && ((3 * H * dk) % 4 == 0);
  const long nrow = (long)B * H * T;
  (void)nrow;
  CFM_REQUIRE(H * dk <= 1024, CFM_ERR_UNSUPPORTED, "H*dk must be <= 1024");
  if (!d_ready)
    hipLaunchKernelGGL(attn_bwd_dot_kernel, dim3((unsigned)(((long)B * T + 3) / 4)), dim3(256), 0, s,
                       (const bf16*)dout, (const bf16*)o, ws, B, T, H, dk);
  if (pos)
    return cfm::attn_rel_bwd_launch(qkv, dout, lse, lengths, pos, pos_u, pos_v, dqkv, dpos, dpos_dt, dpos_u, dpos_v, B,
                                    T, H, dk, drop_p, seed, ws, s);
  p.qs = use_head(T) ? head_split(B, H, T) : 1;
  const int hwaves = cdiv(cdiv(T, 32), p.qs);
  // dQ from the dS^T the dK/dV kernel stores: only when the caller passed the full workspace (cfm_attn_bwd, or
  // cfm_attn_bwd_ex with d_ready bit 1; cfm_attn_bwd_with_d's ws may be D alone)
  bf16* dsT = full_ws && dsT_path(T) ? reinterpret_cast<bf16*>(reinterpret_cast<char*>(ws) + d_slot_bytes(B, T, H))
                                     : nullptr;
  if (use_head(T))
    hipLaunchKernelGGL(attn_bwd_dkdv_wave_kernel, dim3(B * H * p.qs), dim3(64 * hwaves), dkdv_wave_lds_bytes(T, hwaves),
                       s, p, (const bf16*)dout, lse, ws, (bf16*)dqkv, dsT);
  else
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3(cdiv(T, 128), H, B), dim3(256), 0, s, p, (const bf16*)dout, lse,
                       ws, (bf16*)dqkv);
  if (dsT)
    hipLaunchKernelGGL(attn_bwd_dqs_head_kernel, dim3(B * H * p.qs), dim3(64 * hwaves), dqs_head_lds_bytes(T, hwaves), s,
                       p, (const bf16*)dsT, (bf16*)dqkv);
  else if (use_head(T))
    hipLaunchKernelGGL(attn_bwd_dq_head_kernel, dim3(B * H * p.qs), dim3(64 * hwaves), head_lds_bytes(T, hwaves), s, p,
                       (const bf16*)dout, lse, ws, (bf16*)dqkv);
  else
    hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3(cdiv(T, 128), H, B), dim3(256), 0, s, p, (const bf16*)dout, lse, ws,
                       (bf16*)dqkv);
  return cfm::check_launch("cfm_attn_bwd");
}

CFM_EXPORT int cfm_attn_bwd(const void* qkv, const void* o, const void* dout, const float* lse,
                            const int32_t* lengths, const void* pos, const float* pos_u, const float* pos_v,
                            void* dqkv, float* dpos, float* dpos_u, float* dpos_v, int B, int T, int H, int dk,
                            int dtype, float drop_p, uint64_t seed, float* ws, void* stream) {
  return attn_bwd_impl(qkv, o, dout, lse, lengths, pos, pos_u, pos_v, dqkv, dpos, CFM_F32, dpos_u, dpos_v, B, T, H, dk,
                       dtype, drop_p, seed, ws, stream, false, true);
}

CFM_EXPORT int cfm_attn_bwd_with_d(const void* qkv, const void* o, const void* dout, const float* lse,
                                   const int32_t* lengths, const void* pos, const float* pos_u, const float* pos_v,
                                   void* dqkv, float* dpos, float* dpos_u, float* dpos_v, int B, int T, int H, int dk,
                                   int dtype, float drop_p, uint64_t seed, float* ws, void* stream) {
  return attn_bwd_impl(qkv, o, dout, lse, lengths, pos, pos_u, pos_v, dqkv, dpos, CFM_F32, dpos_u, dpos_v, B, T, H, dk,
                       dtype, drop_p, seed, ws, stream, true, false);
}

CFM_EXPORT int cfm_attn_bwd_ex(const void* qkv, const void* o, const void* dout, const float* lse,
                               const int32_t* lengths, const void* pos, const float* pos_u, const float* pos_v,
                               void* dqkv, void* dpos, int dtype_dpos, float* dpos_u, float* dpos_v, int B, int T,
                               int H, int dk, int dtype, float drop_p, uint64_t seed, int d_ready, float* ws,
                               void* stream) {
  return attn_bwd_impl(qkv, o, dout, lse, lengths, pos, pos_u, pos_v, dqkv, dpos, dtype_dpos, dpos_u, dpos_v, B, T, H,
                       dk, dtype, drop_p, seed, ws, stream, (d_ready & 1) != 0, (d_ready & 2) != 0);
}

CFM_EXPORT int cfm_attn_set_mode(int mode) {
  g_attn_mode = mode;
  cfm::g_rel_mode = mode;
  return CFM_OK;
}
