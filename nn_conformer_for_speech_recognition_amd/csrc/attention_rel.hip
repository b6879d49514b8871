// attention_rel.hip — relative-position multi-head self-attention on MFMA (bf16), fwd + bwd.
//
// Semantics (transformers Wav2Vec2ConformerSelfAttention, position_embeddings_type="relative",
// modeling_wav2vec2_conformer.py:528-565), one (batch b, head h), scale = 1/sqrt(dk):
//   s_ij = scale * ((q_i + u) . k_j + (q_i + v) . p_{T-1-i+j})      p = linear_pos(pe): (2T-1, H*dk)
// keys j >= len[b] masked (key_padding_mask), attention dropout on the probabilities, o = P v.
//
// The rel-shift is never materialised.  For a block of 32 queries (one wave) and 64 keys the
// relative rows r = T-1-i+j span a BAND of 32+64-1 rows of p.  The band is staged in LDS (a ring
// of 64-row chunks: consecutive key tiles share 128 of their 192 rows, so each tile loads only 64
// new rows), and one MFMA product  X[r'][i] = p_{rb+r'} . (q_i+v)  (12 x v_mfma_f32_32x32x16_bf16)
// gives every bd term the block needs.  The skew bd[j][i] = X[j-i+31][i] is a per-lane column shift
// in the accumulator, done through a per-wave LDS stage (column stride 100 floats: b128 writes and
// the skewed b32 reads are both bank-conflict free).  ac and bd add in fp32 before the softmax.
//
// Backward (deterministic, no atomics):
//   dQ kernel  (round 6 default, attn_rel_bwd_dqs_kernel): runs after dK/dV and reads the dS it stored --
//              dq = scale * (sum_j dS k_j + sum_j dS p_{T-1-i+j}), the band sum as below; no recompute.
//   dQ2 kernel (queries on the lanes, streams key tiles; cfm_attn_set_mode bit 9): recomputes S (same band), dP, dS;
//              dq = scale * (sum_j dS k_j  +  sum_j dS p_{T-1-i+j}) -- the second sum is a plain
//              MFMA over the band once dS^T is scattered into the stage in band coordinates;
//              per-wave column sums of both terms -> du, dv partials (one reduction launch).
//   dK/dV kernel (keys on the lanes, streams query tiles): recomputes S with the band in the
//              transposed role, dV += dO^T P~, dK += (q+u)^T dS, and writes dS (bf16,
//              query-major) for the dpos pass.
//   dpos kernel: dpos_r = scale * sum_{b,i} dS[i, i+r-(T-1)] (q_i+v) -- in (i, r) coordinates a plain
//              GEMM over i whose dS operand rows are contiguous runs of the stored dS rows.
#include "attn_common.h"

namespace {

constexpr int SS = 100;     // fwd / dQ stage column stride (floats): 100 = 4 mod 32, 99 odd
constexpr int SS2 = 68;     // dK/dV stage column stride (floats): 68 = 4 mod 32
constexpr int RING = 4;     // p-band ring: chunks of TILE rows

struct RelP {
  const bf16* pos;          // (2T-1, H*dk) projected relative table
  const float* pu;          // (H*dk) pos_bias_u
  const float* pv;          // (H*dk) pos_bias_v
  bool pvec;                // 16-B vector loads of pos legal
};

// 8 head-dim elements c..c+7 of relative row `row` (valid rows [0, 2T-1)), zero outside
__device__ __forceinline__ uint4 ld8p(const AttnM& p, const RelP& rp, int h, int row, int c) {
  if (row < 0 || row >= 2 * p.T - 1) return make_uint4(0, 0, 0, 0);
  return ld8(rp.pos + h * p.dk, p.HD, row, 2 * p.T - 1, c, p.dk, rp.pvec);
}

// (q + u) and (q + v) B-operand fragments of query row `row` (zero past T / past dk)
__device__ __forceinline__ void load_q_uv(const AttnM& p, const RelP& rp, int b, int h, int row, bf16x8 (&qu)[4],
                                          bf16x8 (&qv)[4], int lane) {
  const bf16* qbase = p.qkv + (long)b * p.T * p.D3 + h * p.dk;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int c = 16 * s + 8 * (lane >> 5);
    const bf16x8 q = __builtin_bit_cast(bf16x8, ld8(qbase, p.D3, row, p.T, c, p.dk, p.vec));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int d = c + e;
      const float u = d < p.dk ? rp.pu[h * p.dk + d] : 0.f;
      const float v = d < p.dk ? rp.pv[h * p.dk + d] : 0.f;
      qu[s][e] = (bf16)((float)q[e] + u);
      qv[s][e] = (bf16)((float)q[e] + v);
    }
  }
}


// 16-B chunk `v` (0..511) of a 64-row chunk of the band: row v>>3, columns (v&7)*8.  VEC: relative rows
// outside [0, 2T-1) clamp to the nearest valid row instead of reading zero (branch-free prefetch, ld8c):
// such rows only ever meet (query, key) pairs outside the valid range, whose probabilities are zero
template <bool VEC>
__device__ __forceinline__ uint4 ring_chunk_load(const AttnM& p, const RelP& rp, int h, int row0, int v) {
  if constexpr (VEC) return ld8c(rp.pos + h * p.dk, p.HD, row0 + (v >> 3), 2 * p.T - 1, (v & 7) * 8);
  else return ld8p(p, rp, h, row0 + (v >> 3), (v & 7) * 8);
}
__device__ __forceinline__ void ring_chunk_store(bf16* slot, const uint4 (&reg)[2], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + 256 * i;
    *reinterpret_cast<uint4*>(slot + (v >> 3) * KS + (v & 7) * 8) = reg[i];
  }
}

// accumulator pair (a0 rows 0..31, a1 rows 32..63; lanes = 32 columns) -> per row d = lane: sum over
// the 32 columns, through the wave's LDS stage [c * 65 + d]
__device__ __forceinline__ float wave_rowsum(float* stage, const f32x16& a0, const f32x16& a1, int lane) {
  const int hh = lane >> 5, c = lane & 31;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    stage[c * 65 + acc_row(r, hh)] = a0[r];
    stage[c * 65 + 32 + acc_row(r, hh)] = a1[r];
  }
  __builtin_amdgcn_wave_barrier();
  float s = 0.f;
  for (int cc = 0; cc < 32; ++cc) s += stage[cc * 65 + lane];
  __builtin_amdgcn_wave_barrier();
  return s;
}

// ------------------------------------------------------------------------------------ S^T for a key tile
// queries on the lanes (wave = 32 queries), 64 keys on the accumulator rows (s0: keys 0..31, s1: 32..63):
// S^T = K (q+u)^T + skew(P_band (q+v)^T), unscaled.  band: the ring slot base of each 32-row block.
struct BandRows {
  const bf16* blk[3];       // LDS row 0 of the wave's three 32-row band blocks
};

__device__ __forceinline__ void scores_qlanes(const bf16* sK, const BandRows& br, const bf16x8 (&qu)[4],
                                              const bf16x8 (&qv)[4], float* st, f32x16& s0, f32x16& s1, int lane) {
  const int hh = lane >> 5, ii = lane & 31;
  float* col = st + ii * SS;
  // X[r'][i] -> stage[i][r'] (16-B stores of 4 consecutive accumulator rows), one 32-row band block at a time:
  // only one X accumulator is live (the three at once pushed the dQ kernel past 256 VGPRs into AGPR copies)
  auto put = [&](const f32x16& x, int base) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int r0 = 8 * g + 4 * hh;
      *reinterpret_cast<float4*>(col + base + r0) = make_float4(x[4 * g], x[4 * g + 1], x[4 * g + 2], x[4 * g + 3]);
    }
  };
  s0 = (f32x16){0};
  s1 = (f32x16){0};
  {
    f32x16 x0 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 0, 16 * s, lane), qu[s], s0, 0, 0, 0);
      x0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(br.blk[0], 0, 16 * s, lane), qv[s], x0, 0, 0, 0);
    }
    put(x0, 0);
  }
  {
    f32x16 x1 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 32, 16 * s, lane), qu[s], s1, 0, 0, 0);
      x1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(br.blk[1], 0, 16 * s, lane), qv[s], x1, 0, 0, 0);
    }
    put(x1, 32);
  }
  {
    f32x16 x2 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s)
      x2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(br.blk[2], 0, 16 * s, lane), qv[s], x2, 0, 0, 0);
    put(x2, 64);
  }
  __builtin_amdgcn_wave_barrier();
  // bd[j][i] = X[j - i + 31][i]
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int jj = acc_row(r, hh);
    s0[r] += col[jj - ii + 31];
    s1[r] += col[jj + 32 - ii + 31];
  }
  __builtin_amdgcn_wave_barrier();
}

// the wave's three band blocks for key tile kt: band rows 32(3-w) + 32m of the tile's 192-row window,
// which starts at ring chunk kt
__device__ __forceinline__ BandRows band_rows_q(const bf16* ring, int kt, int wv) {
  BandRows br;
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int off = 32 * (3 - wv) + 32 * m;
    br.blk[m] = ring + ((kt + (off >> 6)) & (RING - 1)) * TILE * KS + (off & 63) * KS;
  }
  return br;
}

// ------------------------------------------------------------------------------------ band bias column
// (q + v) . p_r = (q + u) . p_r + c_r with c_r = (v - u) . p_r: the two-waves kernels form the band product from
// the (q + u) operand they already hold and add c_r (fp32, per relative row) -- no (q + v) operand in registers
// (dQ: 16 registers; the forward has the registers and keeps (q + v), as the c_r path costs ~80 VALU per tile).
// (Round 4: a two-waves dK/dV built the same way -- 81 KiB, Q+u / dO single-buffered, loads between two barriers --
// ran 351 vs 302 us per layer at L60, profiles/r04/rel_l60_kernels_s2.txt, and was removed: the one-wave kernel's
// double-buffered register prefetch hides the tile loads that the single-buffered form exposes twice per tile.)  c of a ring chunk is computed from the chunk's staged rows: the 8 threads that store one row's 8 16-B
// pieces each dot 8 columns with (v - u) and sum over the 8 lanes (three xor shuffles).
__device__ __forceinline__ void load_dvu8(const AttnM& p, const RelP& rp, int h, int tid, float (&dvu)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int d = (tid & 7) * 8 + e;
    dvu[e] = d < p.dk ? rp.pv[h * p.dk + d] - rp.pu[h * p.dk + d] : 0.f;
  }
}
__device__ __forceinline__ void ring_c_store(float* cslot, const uint4 (&reg)[2], const float (&dvu)[8], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const bf16x8 v = __builtin_bit_cast(bf16x8, reg[i]);
    float t = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) t = __builtin_fmaf((float)v[e], dvu[e], t);
    t += __shfl_xor(t, 1, 64);
    t += __shfl_xor(t, 2, 64);
    t += __shfl_xor(t, 4, 64);
    if ((tid & 7) == 0) cslot[(tid + 256 * i) >> 3] = t;
  }
}
// x (band rows 8g + 4hh + e of a 32-row block on the accumulator rows) += c of those rows
__device__ __forceinline__ void add_band_c(f32x16& x, const float* cb, int hh) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 cv = *reinterpret_cast<const float4*>(cb + 8 * g + 4 * hh);
    x[4 * g] += cv.x; x[4 * g + 1] += cv.y; x[4 * g + 2] += cv.z; x[4 * g + 3] += cv.w;
  }
}

// ------------------------------------------------------------------------------------ forward, two waves per SIMD
// grid (ceil(T/128), H, B), 4 waves x 32 queries; K/V tiles of 64 keys, band ring.  <= 80 KiB of LDS and <= 256
// registers, so two workgroups share a
// CU (two waves per SIMD: one wave's softmax VALU issues beside the other's MFMAs, and the VALU issue cost per
// instruction halves -- one wave alone on a SIMD pays 4 cycles per v_fma, two pay 2 each).  LDS: one K/V tile
// (18 KiB, the next tile prefetched into registers and stored between two barriers), a ring of 3 band chunks
// (27 KiB: tile kt reads chunks kt..kt+2, chunk kt+3 replaces kt), and a 64-row skew stage per wave (34 KiB):
// X0 -> rows 0..31 and X1 -> 32..63 for the s0 block (band rows 0..62), then X1 -> 0..31 and X2 -> 32..63 for the
// s1 block (band rows 32..94): both blocks read the same per-lane addresses (one base + immediate offsets).  The
// dropout keep scale is applied once to the output (o * keep / l).
constexpr int SC = 68;      // 64-row skew stage column stride (floats): 68 = 4 mod 32
template <bool VEC>
__global__ __launch_bounds__(256, 2) void attn_rel_fwd2_kernel(AttnM p, RelP rp, bf16* __restrict__ o,
                                                               float* __restrict__ lse) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  const uint32_t dkey = drop_key(p.seed, 0), dthr = drop_thr(p.drop_p);
  const float dkeep = drop_keep_scale(dthr);
  __shared__ __attribute__((aligned(16))) bf16 skv[2 * TILE * KS];        // [K, V][64][72]        18 KiB
  __shared__ __attribute__((aligned(16))) bf16 sring[3 * TILE * KS];      // band ring of 3 chunks 27 KiB
  __shared__ __attribute__((aligned(16))) float sst[4 * 32 * SC];          // circular skew stages  34 KiB
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, ii = lane & 31;
  const int h = blockIdx.y, b = blockIdx.z;
  const int Q0 = blockIdx.x * 128, q0 = Q0 + wv * 32;
  const int qi = q0 + ii;
  const int len = p.len[b];
  const int rbase = p.T - 1 - Q0 - 127;          // relative row of band row 0 at key tile 0
  bf16x8 qu[4], qv[4];
  load_q_uv(p, rp, b, h, qi, qu, qv, lane);
  float* col = sst + wv * 32 * SC + ii * SC;
  f32x16 o0 = (f32x16){0}, o1 = (f32x16){0};
  float m = -INFINITY, l = 0.f;
  const float c = p.scale * LOG2E;
  const int nkt = (len + TILE - 1) / TILE;
  uint4 rk[2], rv[2], rq[2];
  const int kcol = p.HD + h * p.dk, vcol = 2 * p.HD + h * p.dk;
  if (nkt > 0) {
    tile_load<VEC>(p, b, 0, kcol, rk, tid);
    tile_load<VEC>(p, b, 0, vcol, rv, tid);
    tile_store(skv, rk, tid);
    tile_store(skv + TILE * KS, rv, tid);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
#pragma unroll
      for (int i = 0; i < 2; ++i) rq[i] = ring_chunk_load<VEC>(p, rp, h, rbase + ch * TILE, tid + 256 * i);
      ring_chunk_store(sring + ch * TILE * KS, rq, tid);
    }
    __syncthreads();
  }
  wait_prologue_loads();
  // X[r'][i] -> stage rows (base + r') & 63 of column i (16-B stores of 4 consecutive accumulator rows)
  float* colh = col + 4 * hh;                 // the lane's 4-row groups: rows 8g + 4hh .. +3
  const float* sk = col + 31 - ii + 4 * hh;   // bd of accumulator row acc_row(r, hh): sk[(r & 3) + 8 (r >> 2)]
  auto put = [&](const f32x16& x, int base) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<float4*>(colh + base + 8 * g) = make_float4(x[4 * g], x[4 * g + 1], x[4 * g + 2], x[4 * g + 3]);
  };
  for (int kt = 0; kt < nkt; ++kt) {
    const bf16* sK = skv;
    const bf16* sV = skv + TILE * KS;
    if (kt + 1 < nkt) {
      tile_load<VEC>(p, b, (kt + 1) * TILE, kcol, rk, tid);
      tile_load<VEC>(p, b, (kt + 1) * TILE, vcol, rv, tid);
#pragma unroll
      for (int i = 0; i < 2; ++i) rq[i] = ring_chunk_load<VEC>(p, rp, h, rbase + (kt + 3) * TILE, tid + 256 * i);
    }
    const bf16* blk[3];
#pragma unroll
    for (int mm = 0; mm < 3; ++mm) {
      const int off = 32 * (3 - wv) + 32 * mm;
      blk[mm] = sring + ((kt + (off >> 6)) % 3) * TILE * KS + (off & 63) * KS;
    }
    // S^T = K (q+u)^T + skew(P_band (q+v)^T), unscaled (queries on the lanes, keys on the accumulator rows)
    f32x16 s0 = (f32x16){0}, s1 = (f32x16){0};
    {
      f32x16 x0 = (f32x16){0};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 0, 16 * s, lane), qu[s], s0, 0, 0, 0);
        x0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(blk[0], 0, 16 * s, lane), qv[s], x0, 0, 0, 0);
      }
      put(x0, 0);
    }
    f32x16 x1 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 32, 16 * s, lane), qu[s], s1, 0, 0, 0);
      x1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(blk[1], 0, 16 * s, lane), qv[s], x1, 0, 0, 0);
    }
    put(x1, 32);
    f32x16 x2 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s)
      x2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(blk[2], 0, 16 * s, lane), qv[s], x2, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 16; ++r) s0[r] += sk[(r & 3) + 8 * (r >> 2)];              // band rows 0..62
    __builtin_amdgcn_wave_barrier();
    put(x1, 0);                                                                    // band rows 32..94 -> 0..62
    put(x2, 32);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 16; ++r) s1[r] += sk[(r & 3) + 8 * (r >> 2)];
    __builtin_amdgcn_wave_barrier();
    softmax_tile<true>(p, s0, s1, o0, o1, m, l, c, kt * TILE, len, kt == nkt - 1, b, h, qi, hh, dthr, dkeep, dkey);
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
      __syncthreads();           // every wave is done with K/V (kt) and with band chunk kt
      tile_store(skv, rk, tid);
      tile_store(skv + TILE * KS, rv, tid);
      ring_chunk_store(sring + (kt % 3) * TILE * KS, rq, tid);
      __syncthreads();
    }
  }
  __syncthreads();               // the stage region of store_transposed (32 x 65 floats) spans wave boundaries
  float* st = sst + wv * 32 * SC;
  const float inv = (p.drop_p > 0.f ? dkeep : 1.f) / l;
  if (q0 < p.T)
    store_transposed(st, o0, o1, inv, o + (long)b * p.T * p.HD + h * p.dk, p.HD, q0, min(32, p.T - q0), p.dk, lane);
  if (hh == 0 && qi < p.T) lse[((long)b * p.H + h) * p.T + qi] = (m + __log2f(l)) * LN2;
}

// ------------------------------------------------------------------------------------ dQ (+ du, dv partials)
// grid (ceil(T/128), H, B).  part: (B * 4*gridDim.x, 2*H*dk) fp32 -- row (b, 32-query block): per-column sums over
// the block's queries of scale * sum_j dS k_j (u half) and scale * sum_j dS p_r (v half).
// Two waves per SIMD: <= 80 KiB of LDS and <= 256 registers (two workgroups per CU): one K/V tile
// (the next one loaded between two barriers: a register prefetch across the tile spilled, the partner workgroup
// covers the load), a ring of 3 band chunks, and per wave one 64-row f32 skew
// stage (as attn_rel_fwd2_kernel) whose bytes also hold the bf16 band-coordinate image of dS^T
// ([query][96 + 8 pad] bf16, 6.5 KiB of the wave's 8.5): the scatter writes bf16 directly (the MFMA operand type)
// and the band-term MFMA reads 16-B fragments of it.
constexpr int SB = 104;     // band image column stride (bf16 elements): 208 B
template <bool VEC>
__global__ __launch_bounds__(256, 2) void attn_rel_bwd_dq2_kernel(AttnM p, RelP rp, const bf16* __restrict__ dout,
                                                                  const float* __restrict__ lse,
                                                                  const float* __restrict__ Dg,
                                                                  bf16* __restrict__ dqkv, float* __restrict__ part) {
  if (p.drop_p > 0.f) p.seed = salted_seed(p.seed, p.salt);
  const uint32_t dkey = drop_key(p.seed, 0), dthr = drop_thr(p.drop_p);
  const float dkeep = drop_keep_scale(dthr);
  __shared__ __attribute__((aligned(16))) bf16 skv[2 * TILE * KS];
  __shared__ __attribute__((aligned(16))) bf16 sring[3 * TILE * KS];
  __shared__ __attribute__((aligned(16))) float scr[3 * TILE];              // c of the ring's rows
  __shared__ __attribute__((aligned(16))) float sst[4 * 32 * SC];
  static_assert(32 * SB * 2 <= 32 * SC * 4, "band image fits the wave's stage");
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, ii = lane & 31;
  const int h = blockIdx.y, b = blockIdx.z;
  const int Q0 = blockIdx.x * 128, q0 = Q0 + wv * 32;
  const int qi = q0 + ii;
  const int len = p.len[b];
  const int rbase = p.T - 1 - Q0 - 127;
  bf16x8 qu[4], gf[4];
  {
    bf16x8 qv_unused[4];
    load_q_uv(p, rp, b, h, qi, qu, qv_unused, lane);
  }
  float dvu[8];
  load_dvu8(p, rp, h, tid, dvu);
  load_bfrags(p, dout + (long)b * p.T * p.HD + h * p.dk, p.HD, qi, p.T, gf, lane);
  const bool qvalid = qi < p.T;
  const float L2 = qvalid ? lse[((long)b * p.H + h) * p.T + qi] * LOG2E : INFINITY;   // +inf: P = 0 past T
  const float Dq = qvalid ? Dg[((long)b * p.H + h) * p.T + qi] : 0.f;
  const float c = p.scale * LOG2E;
  float* st = sst + wv * 32 * SC;
  float* col = st + ii * SC;
  bf16* bimg = reinterpret_cast<bf16*>(st);            // [query][SB] band image of dS^T
  bf16* bcol = bimg + ii * SB;
  bf16* bsk = bcol + 31 - ii + 4 * hh;         // band row of (key acc_row(r, hh), query ii): bsk[(r & 3) + 8 (r >> 2)]
  f32x16 a0 = (f32x16){0}, a1 = (f32x16){0}, e0 = (f32x16){0}, e1 = (f32x16){0};   // K-term, band term
  const int nkt = (len + TILE - 1) / TILE;
  uint4 rk[2], rv[2], rq[2];
  const int kcol = p.HD + h * p.dk, vcol = 2 * p.HD + h * p.dk;
  if (nkt > 0) {
    tile_load<VEC>(p, b, 0, kcol, rk, tid);
    tile_load<VEC>(p, b, 0, vcol, rv, tid);
    tile_store(skv, rk, tid);
    tile_store(skv + TILE * KS, rv, tid);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
#pragma unroll
      for (int i = 0; i < 2; ++i) rq[i] = ring_chunk_load<VEC>(p, rp, h, rbase + ch * TILE, tid + 256 * i);
      ring_chunk_store(sring + ch * TILE * KS, rq, tid);
      ring_c_store(scr + ch * TILE, rq, dvu, tid);
    }
    __syncthreads();
  }
  wait_prologue_loads();
  float* colh = col + 4 * hh;                 // the lane's 4-row groups: rows 8g + 4hh .. +3
  const float* sk = col + 31 - ii + 4 * hh;   // bd of accumulator row acc_row(r, hh): sk[(r & 3) + 8 (r >> 2)]
  auto put = [&](const f32x16& x, int base) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<float4*>(colh + base + 8 * g) = make_float4(x[4 * g], x[4 * g + 1], x[4 * g + 2], x[4 * g + 3]);
  };
  for (int kt = 0; kt < nkt; ++kt) {
    const bf16* sK = skv;
    const bf16* sV = skv + TILE * KS;
    const bf16* blk[3];
    const float* cbk[3];
#pragma unroll
    for (int mm = 0; mm < 3; ++mm) {
      const int off = 32 * (3 - wv) + 32 * mm;
      blk[mm] = sring + ((kt + (off >> 6)) % 3) * TILE * KS + (off & 63) * KS;
      cbk[mm] = scr + ((kt + (off >> 6)) % 3) * TILE + (off & 63);
    }
    f32x16 s0 = (f32x16){0}, s1 = (f32x16){0};
    {
      f32x16 x0 = (f32x16){0};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 0, 16 * s, lane), qu[s], s0, 0, 0, 0);
        x0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(blk[0], 0, 16 * s, lane), qu[s], x0, 0, 0, 0);
      }
      add_band_c(x0, cbk[0], hh);
      put(x0, 0);
    }
    f32x16 x1 = (f32x16){0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sK, 32, 16 * s, lane), qu[s], s1, 0, 0, 0);
      x1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(blk[1], 0, 16 * s, lane), qu[s], x1, 0, 0, 0);
    }
    add_band_c(x1, cbk[1], hh);
    put(x1, 32);
    {
      f32x16 x2 = (f32x16){0};
#pragma unroll
      for (int s = 0; s < 4; ++s)
        x2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(blk[2], 0, 16 * s, lane), qu[s], x2, 0, 0, 0);
      add_band_c(x2, cbk[2], hh);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = 0; r < 16; ++r) s0[r] += sk[(r & 3) + 8 * (r >> 2)];
      __builtin_amdgcn_wave_barrier();
      put(x1, 0);
      put(x2, 32);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = 0; r < 16; ++r) s1[r] += sk[(r & 3) + 8 * (r >> 2)];
      __builtin_amdgcn_wave_barrier();
    }
    // per 32-key half t: dP^T = V dO^T, dropout, dS^T = P (dP keep - D) in place of the scores, then the K-term
    // dQ^T[d][q] += sum_key K[key][d] dS^T[key][q] (one dP half live at a time)
    const float keep = p.drop_p > 0.f ? dkeep : 1.f;
    const bool tail = kt == nkt - 1 && kt * TILE + TILE > len;
    const uint32_t rowj = (uint32_t)(didx(p, b, h, qi, kt * TILE) >> 1);   // even: 32-bit pair indices
    auto half = [&](f32x16& sx, int t) {
      __builtin_amdgcn_sched_barrier(0);
      f32x16 dd = (f32x16){0};
#pragma unroll
      for (int s = 0; s < 4; ++s)
        dd = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sV, 32 * t, 16 * s, lane), gf[s], dd, 0, 0, 0);
      if (p.drop_p > 0.f) {
        const uint32_t hb = rowj + dkey + 2u * (uint32_t)hh;   // + a compile-time constant per pair (one add)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const uint32_t hs = attn_mix(hb + (uint32_t)(((r & 3) >> 1) + 4 * (r >> 2) + 16 * t));
          dd[r] = (hs & 0xFFFFu) >= dthr ? dd[r] : 0.f;
          dd[r + 1] = (hs >> 16) >= dthr ? dd[r + 1] : 0.f;
        }
      }
      // P = 2^(c s - lse log2 e); key masking only on the utterance's last tile (uniform)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float x = __builtin_fmaf(sx[r], c, -L2);
        if (tail) x = kt * TILE + 32 * t + acc_row(r, hh) < len ? x : -INFINITY;
        sx[r] = fast_exp2(x) * __builtin_fmaf(dd[r], keep, -Dq);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc2frag(sx, s);
        a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sK, 32 * t + 16 * s, 0, lane), pf, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sK, 32 * t + 16 * s, 32, lane), pf, a1, 0, 0, 0);
      }
    };
    half(s0, 0);
    half(s1, 1);
    __builtin_amdgcn_sched_barrier(0);
    // band term: dS^T in band coordinates, bf16 image [i][j - i + 31] (zero elsewhere), then
    // dQ^T[d][q] += sum_r' P_band[r'][d] dS_band^T[r'][q]
#pragma unroll
    for (int g = 0; g < 6; ++g) *reinterpret_cast<uint4*>(bcol + 48 * hh + 8 * g) = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      bsk[(r & 3) + 8 * (r >> 2)] = (bf16)s0[r];
      bsk[(r & 3) + 8 * (r >> 2) + 32] = (bf16)s1[r];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      // (B element j <-> band row 16s + 8(j >> 2) + 4hh + (j & 3): the k order trfrag_perm's A fragment expects)
      const uint2 lo = *reinterpret_cast<const uint2*>(bcol + 16 * s + 4 * hh);
      const uint2 hi = *reinterpret_cast<const uint2*>(bcol + 16 * s + 8 + 4 * hh);
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      const bf16* bk = blk[s >> 1];
      e0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(bk, 16 * (s & 1), 0, lane), bfr, e0, 0, 0, 0);
      e1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(bk, 16 * (s & 1), 32, lane), bfr, e1, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
    if (kt + 1 < nkt) {
      // the next tile's loads are issued before the barrier (this tile's registers are dead): their latency
      // overlaps the wait for the other waves
      tile_load<VEC>(p, b, (kt + 1) * TILE, kcol, rk, tid);
      tile_load<VEC>(p, b, (kt + 1) * TILE, vcol, rv, tid);
#pragma unroll
      for (int i = 0; i < 2; ++i) rq[i] = ring_chunk_load<VEC>(p, rp, h, rbase + (kt + 3) * TILE, tid + 256 * i);
      __syncthreads();
      tile_store(skv, rk, tid);
      tile_store(skv + TILE * KS, rv, tid);
      ring_chunk_store(sring + (kt % 3) * TILE * KS, rq, tid);
      ring_c_store(scr + (kt % 3) * TILE, rq, dvu, tid);
      __syncthreads();
    }
  }
  __builtin_amdgcn_wave_barrier();   // the band-image reads are done before wave_rowsum reuses the stage
  const float su = wave_rowsum(st, a0, a1, lane) * p.scale;
  const float sv = wave_rowsum(st, e0, e1, lane) * p.scale;
  const long prow = (long)b * (4 * gridDim.x) + blockIdx.x * 4 + wv;
  if (lane < p.dk) {
    part[prow * 2 * p.HD + h * p.dk + lane] = su;
    part[prow * 2 * p.HD + p.HD + h * p.dk + lane] = sv;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    a0[r] += e0[r];
    a1[r] += e1[r];
  }
  if (q0 < p.T)
    store_transposed(st, a0, a1, p.scale, dqkv + (long)b * p.T * p.D3 + h * p.dk, p.D3, q0, min(32, p.T - q0),
                     p.dk, lane);
}

// ------------------------------------------------------------------------------------ dQ from the stored dS
// (default since round 6; cfm_attn_set_mode bit 9 keeps the recomputing dQ2 kernel above, A/B).  The dK/dV kernel
// already writes dS (bf16, unscaled, query-major) for the dpos pass; dQ is a plain product of it with K and, in band
// coordinates, with the projected table:  dq_i = scale * (sum_j dS_ij k_j + sum_j dS_ij p_{T-1-i+j}).  No scores,
// softmax, dropout hash or dO x V recompute: per 64-key tile a wave runs 8 + 12 MFMAs (dQ2: 48) and no exp.
// grid (ceil(T/128), H, B), 4 waves x 32 queries; LDS: the K tile, a ring of 3 band chunks (as dQ2), and per wave
// the band-coordinate image of dS^T ([query][SBQ] bf16, as dQ2, zeroed once); the dS fragments come straight from
// the buffer into registers (two 8-B loads per fragment, one tile ahead): the kernel is bound by its LDS instruction
// count, not by bank conflicts (PMC, profiles/r06/misc/rel_dq_from_ds_ab.txt); the band scatter is 32 explicit 2-byte
// stores per tile (merged by the compiler, they were misaligned 8-B stores, slower).  After the loop the K tile + ring
// bytes hold the waves' f32 stages of the du / dv sums and the dq store.
// dS entries of keys >= len are not defined in the buffer (the dK/dV kernel leaves them unmasked or unwritten):
// they are replaced by zeros on the way into LDS.  part: as dQ2.
// K tile and band ring of the dQ-from-dS kernel: read only through the transposed fragments (ds_read_b64_tr_b16:
// 4 rows x 64 B per 32-lane half), so 192-B rows (48 dwords: an odd multiple of 16) put the four rows on disjoint
// bank quarters -- the 144-B rows the score kernels need for their b128 row fragments leave these reads 2-way
// conflicted
constexpr int KSQ = 96;
// (trfrag_perm_s / tile_store_s: attn_common.h)
template <int STR>
__device__ __forceinline__ void ring_chunk_store_s(bf16* slot, const uint4 (&reg)[2], int tid) { tile_store_s<STR>(slot, reg, tid); }
// The band image's row stride is an odd number of 8-B units (25: 100 elements): its 8-B fragment reads of the 32
// query rows hit 32 distinct bank pairs (a 16-B aligned stride -- 208 B -- puts rows i and i + 16 on one pair).
constexpr int SBQ = 100;                      // band image row stride (bf16 elements): 200 B
constexpr int DQS_WAVE = 32 * SBQ * 2;        // per-wave region (bytes)
template <bool VEC>
__global__ __launch_bounds__(256, 2) void attn_rel_bwd_dqs_kernel(AttnM p, RelP rp, const bf16* __restrict__ dsbuf,
                                                                  int ldS, bf16* __restrict__ dqkv,
                                                                  float* __restrict__ part) {
  // sk and sring adjacent: after the loop their 48 KiB hold the four 32 x 65 f32 stages (33 KiB)
  __shared__ __attribute__((aligned(16))) bf16 skr[4 * TILE * KSQ];
  __shared__ __attribute__((aligned(16))) char swv[4 * DQS_WAVE];
  static_assert(4 * TILE * KSQ * 2 >= 4 * 32 * 65 * 4, "final stages fit the K tile + ring");
  bf16* sk = skr;
  bf16* sring = skr + TILE * KSQ;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, ii = lane & 31;
  const int h = blockIdx.y, b = blockIdx.z;
  const int Q0 = blockIdx.x * 128, q0 = Q0 + wv * 32;
  const int len = p.len[b];
  const int rbase = p.T - 1 - Q0 - 127;
  const int nkt = (len + TILE - 1) / TILE;
  const int kcol = p.HD + h * p.dk;
  char* wreg = swv + wv * DQS_WAVE;
  bf16* bimg = reinterpret_cast<bf16*>(wreg);      // [query][SBQ] band image of dS^T
  bf16* bcol = bimg + ii * SBQ;
  // band position of key k (0..63) of query ii: bcol[31 - ii + k]
  // every tile writes the same band positions of a row (k + 31 - ii, k = 0..63): the rest stay zero from here
#pragma unroll
  for (int g = 0; g < 12; ++g) *reinterpret_cast<uint2*>(bcol + 48 * hh + 4 * g) = make_uint2(0, 0);
  const bf16* dsb = dsbuf + ((long)b * p.H + h) * p.T * (long)ldS;
  // the lane's dS^T B fragments of key tile kt straight from the buffer, in the k order of an accumulator used as the
  // B operand: fragment 2 t + s of query q0 + ii holds keys 32 t + 16 s + 4 hh + {0..3, 8..11} -- two 8-B loads
  // (rows past T and runs past the row's ldS read zero; keys >= len are zeroed on the last tile)
  uint4 fA[4], fB[4];
  const int qrow = q0 + ii;
  const bool qok = qrow < p.T;
  const bf16* dsrow = dsb + (long)(qok ? qrow : 0) * ldS + 4 * hh;
  auto dload = [&](uint4 (&f)[4], int kt) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = kt * TILE + 32 * (q >> 1) + 16 * (q & 1);
      const uint2 lo = qok && k + 4 * hh < ldS ? *reinterpret_cast<const uint2*>(dsrow + k) : make_uint2(0, 0);
      const uint2 hi = qok && k + 8 + 4 * hh < ldS ? *reinterpret_cast<const uint2*>(dsrow + k + 8) : make_uint2(0, 0);
      f[q] = make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
  };
  f32x16 a0 = (f32x16){0}, a1 = (f32x16){0}, e0 = (f32x16){0}, e1 = (f32x16){0};   // K-term, band term
  uint4 rk[2], rq[2];
  if (nkt > 0) {
    dload(fA, 0);
    if (nkt > 1) dload(fB, 1);
    tile_load<VEC>(p, b, 0, kcol, rk, tid);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
#pragma unroll
      for (int i = 0; i < 2; ++i) rq[i] = ring_chunk_load<VEC>(p, rp, h, rbase + ch * TILE, tid + 256 * i);
      ring_chunk_store_s<KSQ>(sring + ch * TILE * KSQ, rq, tid);
    }
    tile_store_s<KSQ>(sk, rk, tid);
    __syncthreads();
  }
  // tile kt's fragments: fA when kt is even, fB when odd; refilled with tile kt + 2 after their last use
  auto step = [&](int kt, uint4 (&fc)[4]) {
    if (kt + 1 < nkt) {                           // the next K tile and band chunk in flight under this tile's MFMAs
      tile_load<VEC>(p, b, (kt + 1) * TILE, kcol, rk, tid);
#pragma unroll
      for (int i = 0; i < 2; ++i) rq[i] = ring_chunk_load<VEC>(p, rp, h, rbase + (kt + 3) * TILE, tid + 256 * i);
    }
    const bf16* blk[3];
#pragma unroll
    for (int mm = 0; mm < 3; ++mm) {
      const int off = 32 * (3 - wv) + 32 * mm;
      blk[mm] = sring + ((kt + (off >> 6)) % 3) * TILE * KSQ + (off & 63) * KSQ;
    }
    bf16x8 f[2][2];
    const bool tail = kt * TILE + TILE > len;     // (uniform)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bf16x8 e = __builtin_bit_cast(bf16x8, fc[q]);
      if (tail) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          e[j] = kt * TILE + 32 * (q >> 1) + 16 * (q & 1) + 8 * (j >> 2) + 4 * hh + (j & 3) < len ? e[j] : (bf16)0.f;
      }
      f[q >> 1][q & 1] = e;
    }
    // K-term: dQ^T[d][q] += sum_key K[key][d] dS^T[key][q]
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm_s<KSQ>(sk, 32 * t + 16 * s2, 0, lane), f[t][s2], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm_s<KSQ>(sk, 32 * t + 16 * s2, 32, lane), f[t][s2], a1, 0, 0,
                                                     0);
      }
    // band term: dS^T in band coordinates, bf16 image [i][j - i + 31], then
    // dQ^T[d][q] += sum_r' P_band[r'][d] dS_band^T[r'][q]
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        // explicit 2-byte stores (volatile, from the packed words): the plain element stores were merged by the
        // compiler into ds_write_b64 at 2-byte-aligned addresses, which the LDS runs slower (dQ 140.5 vs 132.9 us
        // at L60, profiles/r06/misc/rel_dqs_b16_ab.txt)
        typedef volatile __attribute__((address_space(3))) unsigned short lds_u16;
        lds_u16* d = reinterpret_cast<lds_u16*>((__attribute__((address_space(3))) char*)swv + wv * DQS_WAVE) +
                     ii * SBQ + 31 - ii;
        const uint4 w = __builtin_bit_cast(uint4, f[t][s2]);
        const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 8; ++j)
          d[32 * t + 16 * s2 + 8 * (j >> 2) + 4 * hh + (j & 3)] =
              (unsigned short)((j & 1) ? (wd[j >> 1] >> 16) : (wd[j >> 1] & 0xFFFFu));
      }
    if (kt + 2 < nkt) dload(fc, kt + 2);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const uint2 lo = *reinterpret_cast<const uint2*>(bcol + 16 * s + 4 * hh);
      const uint2 hi = *reinterpret_cast<const uint2*>(bcol + 16 * s + 8 + 4 * hh);
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      const bf16* bk = blk[s >> 1];
      e0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm_s<KSQ>(bk, 16 * (s & 1), 0, lane), bfr, e0, 0, 0, 0);
      e1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm_s<KSQ>(bk, 16 * (s & 1), 32, lane), bfr, e1, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();   // this tile's band-image reads before the next tile's scatter
    if (kt + 1 < nkt) {
      __syncthreads();
      tile_store_s<KSQ>(sk, rk, tid);
      ring_chunk_store_s<KSQ>(sring + (kt % 3) * TILE * KSQ, rq, tid);
      __syncthreads();
    }
  };
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt & 1) step(kt, fB);
    else step(kt, fA);
  }
  __syncthreads();   // every wave's reads of the K tile / ring are done before the stages reuse their bytes
  float* st = reinterpret_cast<float*>(skr) + wv * 32 * 65;
  const float su = wave_rowsum(st, a0, a1, lane) * p.scale;
  const float sv = wave_rowsum(st, e0, e1, lane) * p.scale;
  const long prow = (long)b * (4 * gridDim.x) + blockIdx.x * 4 + wv;
  if (lane < p.dk) {
    part[prow * 2 * p.HD + h * p.dk + lane] = su;
    part[prow * 2 * p.HD + p.HD + h * p.dk + lane] = sv;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    a0[r] += e0[r];
    a1[r] += e1[r];
  }
  if (q0 < p.T)
    store_transposed(st, a0, a1, p.scale, dqkv + (long)b * p.T * p.D3 + h * p.dk, p.D3, q0, min(32, p.T - q0),
                     p.dk, lane);
}

// ------------------------------------------------------------------------------------ dK, dV (+ dS store)
// grid (ceil(T/128), H, B); wave = 32 keys on the lanes; query tiles of 64 (two 32-query sub-blocks)
// staged in LDS as q+u, q+v, dO (+ lse, D).  The band for (query tile qt, 128 keys) is 192 rows
// starting at relative row T-64-64qt+J0; it moves DOWN one chunk per query tile (ring chunk kc holds
// rows T-64+J0-64(kc-2) ..+63, tile qt uses chunks qt, qt+1, qt+2).
// dsbuf: (B, H, T, ldS) bf16, dS (unscaled: the dpos pass applies the scale), query-major.
template <bool VEC>
__global__ __launch_bounds__(256) void attn_rel_bwd_dkdv_kernel(AttnM p, RelP rp, const bf16* __restrict__ dout,
                                                                const float* __restrict__ lse,
                                                                const float* __restrict__ Dg,
                                                                bf16* __restrict__ dqkv, bf16* __restrict__ dsbuf,
                                                                int ldS) {
  const bool drop = p.drop_p > 0.f;
  if (drop) p.seed = salted_seed(p.seed, p.salt);
  const uint32_t dkey = drop_key(p.seed, 0), dthr = drop_thr(p.drop_p);
  const float dkeep = drop_keep_scale(dthr);
  __shared__ __attribute__((aligned(16))) bf16 sq[2 * 3 * TILE * KS];      // [buf][Qu, Qv, dO][64][72] 54 KiB
  __shared__ __attribute__((aligned(16))) bf16 sring[RING * TILE * KS];    // 36 KiB
  __shared__ __attribute__((aligned(16))) float sst[4 * 32 * SS2];          // 34 KiB
  __shared__ float sLD[2][2][TILE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, jj = lane & 31;
  const int h = blockIdx.y, b = blockIdx.z;
  const int J0 = blockIdx.x * 128;
  const int k0w = J0 + wv * 32;
  const int kj = k0w + jj;
  const int len = p.len[b];
  const bool kvalid = kj < len;
  const int odd = lane & 1, sh = 16 * odd;
  const uint32_t T2 = (uint32_t)(p.T + (p.T & 1)) >> 1;
  const uint32_t hbase = ((uint32_t)(b * p.H + h) * (uint32_t)p.T + (uint32_t)(4 * hh + odd)) * T2 + (uint32_t)(kj >> 1);
  bf16x8 kf[4], vf[4];
  load_bfrags(p, p.qkv + (long)b * p.T * p.D3 + p.HD + h * p.dk, p.D3, kj, p.T, kf, lane);
  load_bfrags(p, p.qkv + (long)b * p.T * p.D3 + 2 * p.HD + h * p.dk, p.D3, kj, p.T, vf, lane);
  const float c = p.scale * LOG2E;
  f32x16 dk0 = (f32x16){0}, dk1 = (f32x16){0}, dv0 = (f32x16){0}, dv1 = (f32x16){0};
  const bool block_live = J0 < len;
  const int nqt = block_live ? (p.T + TILE - 1) / TILE : 0;
  const int cb = p.T - 64 + J0;                  // relative row of band row 0 at query tile 0
  float* st = sst + wv * 32 * SS2;
  uint4 rq[2], rg[2], rr[2];
  float rl = 0.f, rd = 0.f;
  bool rlv = false;
  const bf16* qbase = p.qkv + (long)b * p.T * p.D3 + h * p.dk;
  const bf16* gbase = dout + (long)b * p.T * p.HD + h * p.dk;
  // next query tile into registers; VEC: branch-free (clamped rows, raw lse / D -- validity and the log2 e
  // scaling applied at the LDS store, so no wait lands here)
  auto gload = [&](int qt) {
    const int r0 = qt * TILE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + 256 * i;
      if constexpr (VEC) {
        rq[i] = ld8c(qbase, p.D3, r0 + (v >> 3), p.T, (v & 7) * 8);
        rg[i] = ld8c(gbase, p.HD, r0 + (v >> 3), p.T, (v & 7) * 8);
      } else {
        rq[i] = ld8(qbase, p.D3, r0 + (v >> 3), p.T, (v & 7) * 8, p.dk, p.vec);
        rg[i] = ld8(gbase, p.HD, r0 + (v >> 3), p.T, (v & 7) * 8, p.dk, p.vec);
      }
    }
    if (tid < TILE) {
      const int qi = r0 + tid;
      rlv = qi < p.T;
      const long li = ((long)b * p.H + h) * p.T + min(qi, p.T - 1);
      rl = lse[li];
      rd = Dg[li];
    }
  };
  // pos_bias_u / pos_bias_v of this thread's 8 staging columns ((tid + 256 i) & 7 == tid & 7 for both
  // chunks), loaded once instead of per query tile
  float pu8[8], pv8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int d = (tid & 7) * 8 + e;
    pu8[e] = d < p.dk ? rp.pu[h * p.dk + d] : 0.f;
    pv8[e] = d < p.dk ? rp.pv[h * p.dk + d] : 0.f;
  }
  auto sstore = [&](int buf) {
    bf16* t = sq + buf * 3 * TILE * KS;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + 256 * i;
      const int row = v >> 3, c8 = (v & 7) * 8;
      const bf16x8 q = __builtin_bit_cast(bf16x8, rq[i]);
      bf16x8 qu, qv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        qu[e] = (bf16)((float)q[e] + pu8[e]);
        qv[e] = (bf16)((float)q[e] + pv8[e]);
      }
      *reinterpret_cast<bf16x8*>(t + row * KS + c8) = qu;
      *reinterpret_cast<bf16x8*>(t + TILE * KS + row * KS + c8) = qv;
      *reinterpret_cast<uint4*>(t + 2 * TILE * KS + row * KS + c8) = rg[i];
    }
    if (tid < TILE) {
      sLD[buf][0][tid] = rlv ? rl * LOG2E : INFINITY;   // lse = +inf for q >= T: P = 0
      sLD[buf][1][tid] = rlv ? rd : 0.f;
    }
  };
  if (nqt > 0) {
    gload(0);
    sstore(0);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
#pragma unroll
      for (int i = 0; i < 2; ++i) rr[i] = ring_chunk_load<VEC>(p, rp, h, cb - 64 * (ch - 2), tid + 256 * i);
      ring_chunk_store(sring + ch * TILE * KS, rr, tid);
    }
    __syncthreads();
  }
  wait_prologue_loads();
  bf16* dsb = dsbuf + ((long)b * p.H + h) * p.T * (long)ldS;
  for (int qt = 0; qt < nqt; ++qt) {
    const int cur = qt & 1;
    const bf16* sQu = sq + cur * 3 * TILE * KS;
    const bf16* sQv = sQu + TILE * KS;
    const bf16* sG = sQv + TILE * KS;
    if (qt + 1 < nqt) {
      gload(qt + 1);
#pragma unroll
      for (int i = 0; i < 2; ++i) rr[i] = ring_chunk_load<VEC>(p, rp, h, cb - 64 * (qt + 1), tid + 256 * i);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      // S[q][key], dP[q][key] of queries 32t..32t+31 of the tile (accumulator rows) x the wave's 32 keys
      f32x16 sa = (f32x16){0}, ga = (f32x16){0}, x0 = (f32x16){0}, x1 = (f32x16){0};
      const int o = 32 * (1 + wv - t);           // band offset of the wave's 64 rows in the tile window
      const bf16* blk0 = sring + ((qt + 2 - (o >> 6)) & (RING - 1)) * TILE * KS + (o & 63) * KS;
      const bf16* blk1 = sring + ((qt + 2 - ((o + 32) >> 6)) & (RING - 1)) * TILE * KS + ((o + 32) & 63) * KS;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sQu, 32 * t, 16 * s, lane), kf[s], sa, 0, 0, 0);
        ga = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(sG, 32 * t, 16 * s, lane), vf[s], ga, 0, 0, 0);
        const bf16x8 qvf = rowfrag(sQv, 32 * t, 16 * s, lane);     // queries as the B operand
        x0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(blk0, 0, 16 * s, lane), qvf, x0, 0, 0, 0);
        x1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag(blk1, 0, 16 * s, lane), qvf, x1, 0, 0, 0);
      }
      // X[r'][i] (lanes = queries) -> stage[i][r']; bd[i][j] = X[j - i + 31][i]
      {
        float* colw = st + jj * SS2;       // lane's column = query jj of the sub-block
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int r0 = 8 * g + 4 * hh;
          *reinterpret_cast<float4*>(colw + r0) = make_float4(x0[4 * g], x0[4 * g + 1], x0[4 * g + 2], x0[4 * g + 3]);
          *reinterpret_cast<float4*>(colw + 32 + r0) =
              make_float4(x1[4 * g], x1[4 * g + 1], x1[4 * g + 2], x1[4 * g + 3]);
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qa = acc_row(r, hh);
          sa[r] += st[qa * SS2 + jj - qa + 31];
        }
        __builtin_amdgcn_wave_barrier();
      }
      const float* tL = sLD[cur][0] + 32 * t;
      const float* tD = sLD[cur][1] + 32 * t;
      // the block's lse / D values up front (broadcast LDS reads, one wait), dropout keep-scales per register in
      // one uniform branch, then a branch-free softmax: (written per register with `kvalid ? ... : -inf` inside
      // the mode branches, the compiler emitted an exec-masked branch + LDS read + wait per register)
      float tl[16], td[16], mk[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        tl[r] = tL[acc_row(r, hh)];
        td[r] = tD[acc_row(r, hh)];
      }
      if (drop) {
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          // dropout of (query of register r / r+1, key kj): lanes kj, kj^1 share one 32-bit hash per query
          // (index (didx >> 1) mod 2^32 = (bh T + q) T2 + kj/2); the even lane hashes register r's query,
          // the odd lane register r+1's, and a DPP swap hands each lane its partner's
          const uint32_t hm = attn_mix(
              hbase + dkey + __builtin_amdgcn_readfirstlane((qt * TILE + 32 * t + (r & 3) + 8 * (r >> 2)) * (int)T2));
          const uint32_t ho = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hm, 0xB1, 0xF, 0xF, false);
          const uint32_t h0 = odd ? ho : hm, h1 = odd ? hm : ho;
          mk[r] = ((h0 >> sh) & 0xFFFFu) >= dthr ? dkeep : 0.f;
          mk[r + 1] = ((h1 >> sh) & 0xFFFFu) >= dthr ? dkeep : 0.f;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) mk[r] = 1.f;
      }
      f32x16 pd;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        // (keys >= len are not masked here: their P only reaches this lane's own dK / dV column, zeroed at the
        // store, and dS entries the dpos pass masks out)
        const float pa = fast_exp2(__builtin_fmaf(sa[r], c, -tl[r]));   // lse = +inf for q >= T: 0
        pd[r] = pa * mk[r];
        sa[r] = pa * (ga[r] * mk[r] - td[r]);
      }
      bf16x8 pf[2], sf[2];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        pf[s2] = acc2frag(pd, s2);
        sf[s2] = acc2frag(sa, s2);
      }
      // dS -> dsbuf[i][j] (query-major, unscaled): the 32 x 32 block goes through the wave's stage (free after
      // the skew reads) as bf16 [query][40] and out as 16-B row chunks, 2 stores per lane instead of 16
      // 2-byte ones.  Keys >= T (zero dS) land in the row's padding [T, ldS); chunks past ldS are skipped.
      {
        bf16* sd = reinterpret_cast<bf16*>(st);
#pragma unroll
        for (int r = 0; r < 16; ++r) sd[acc_row(r, hh) * 40 + jj] = sf[r >> 3][r & 7];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int idx = 64 * it + lane, qr = idx >> 2, kc = k0w + 8 * (idx & 3);
          const int qia = qt * TILE + 32 * t + qr;
          const uint4 v = *reinterpret_cast<const uint4*>(sd + qr * 40 + 8 * (idx & 3));
          if (qia < p.T && kc < ldS) *reinterpret_cast<uint4*>(dsb + (long)qia * ldS + kc) = v;
        }
        __builtin_amdgcn_wave_barrier();
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sG, 32 * t + 16 * s2, 0, lane), pf[s2], dv0, 0, 0, 0);
        dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sG, 32 * t + 16 * s2, 32, lane), pf[s2], dv1, 0, 0, 0);
        dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sQu, 32 * t + 16 * s2, 0, lane), sf[s2], dk0, 0, 0, 0);
        dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sQu, 32 * t + 16 * s2, 32, lane), sf[s2], dk1, 0, 0, 0);
      }
    }
    if (qt + 1 < nqt) {
      sstore(cur ^ 1);
      ring_chunk_store(sring + ((qt + 3) & (RING - 1)) * TILE * KS, rr, tid);
    }
    lds_barrier();     // (not __syncthreads: its fence would wait for this tile's dS stores every tile)
  }
  float* stage = sst + wv * 32 * SS2;    // 32 x 68 >= 32 x 65 floats
  const int nvalid = min(32, p.T - k0w);
  if (nvalid > 0) {
    bf16* base = dqkv + (long)b * p.T * p.D3 + h * p.dk;
#pragma unroll
    for (int r = 0; r < 16; ++r) {      // keys >= len: zero gradients (a select: their unmasked P may overflow)
      dk0[r] = kvalid ? dk0[r] : 0.f;
      dk1[r] = kvalid ? dk1[r] : 0.f;
      dv0[r] = kvalid ? dv0[r] : 0.f;
      dv1[r] = kvalid ? dv1[r] : 0.f;
    }
    store_transposed(stage, dk0, dk1, p.scale, base + p.HD, p.D3, k0w, nvalid, p.dk, lane);
    store_transposed(stage, dv0, dv1, 1.f, base + 2 * p.HD, p.D3, k0w, nvalid, p.dk, lane);
  }
}

// ------------------------------------------------------------------------------------ dpos
// grid (ceil((2T-1)/64), H, B): 64 relative rows R0.. of head h for utterance b -> part[b] (the per-utterance
// partials are summed by one deterministic column reduction); 4 waves = (d half, r half).
// part[b][r][h*dk+d] = scale * sum_i dsbuf[b,h,i, i+r-(T-1)] * (q_i + v)[d]   (keys j < len[b] only)
// The next 64-query tile is loaded into registers while the current one runs through the MFMAs.
template <bool VEC>
__global__ __launch_bounds__(256) void attn_rel_bwd_dpos_kernel(AttnM p, RelP rp, const bf16* __restrict__ dsbuf,
                                                                int ldS, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) bf16 sA[2][TILE * KS];    // (q+v)[ii][d]
  __shared__ __attribute__((aligned(16))) bf16 sB[2][TILE * KS];    // dS_diag[ii][rr]
  float* const sO = reinterpret_cast<float*>(&sA[0][0]);   // [TILE][65] after the loop (fits sA: 18 KiB)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int R0 = blockIdx.x * TILE, h = blockIdx.y, b = blockIdx.z;
  const int dh = wv & 1, rh = wv >> 1;
  const int T = p.T, nrel = 2 * T - 1;
  const int len = min(p.len[b], T);
  // i range with a key j = i + r - (T-1) in [0, len) for some r of the tile
  const int ilo = max(0, T - 1 - (R0 + TILE - 1));
  const int ihi = min(T - 1, len - 1 + T - 1 - R0);
  const bf16* dsb = dsbuf + ((long)b * p.H + h) * T * (long)ldS;
  const bf16* qbase = p.qkv + (long)b * T * p.D3 + h * p.dk;
  // this thread's two 8-column chunks: rows (tid + 256k) >> 3, columns c8 (the same for both)
  const int c8 = (tid & 7) * 8;
  float pv8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) pv8[e] = c8 + e < p.dk ? rp.pv[h * p.dk + c8 + e] : 0.f;
  const int nch = ldS >> 3;        // 16-B chunks per dS row
  auto load = [&](int I0, uint4 (&ra)[2], uint4 (&rb)[2]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int row = (tid + 256 * k) >> 3, i = I0 + row;
      const int j0 = i + R0 + c8 - (T - 1);
      if constexpr (VEC) {
        // q + v: one clamped 16-B load (rows >= T zeroed below)
        const bf16x8 q = __builtin_bit_cast(bf16x8, ld8c(qbase, p.D3, i, T, c8));
        bf16x8 qv;
#pragma unroll
        for (int e = 0; e < 8; ++e) qv[e] = (bf16)(i < T ? (float)q[e] + pv8[e] : 0.f);
        ra[k] = __builtin_bit_cast(uint4, qv);
        // dS[i][j0 .. j0+7] (j0 unaligned): the two aligned 16-B chunks around it (chunk indices clamped to the
        // row: a clamped chunk only ever supplies columns outside [0, len), which are zeroed), then a per-lane
        // funnel shift by j0 & 7 elements and the validity mask -- branch-free, no per-element 2-B loads
        const bf16* srow = dsb + (long)min(i, T - 1) * ldS;
        const int cA = j0 >> 3;      // floor (j0 may be negative)
        const uint4 A = *reinterpret_cast<const uint4*>(srow + 8 * min(max(cA, 0), nch - 1));
        const uint4 Bc = *reinterpret_cast<const uint4*>(srow + 8 * min(max(cA + 1, 0), nch - 1));
        const uint32_t w[8] = {A.x, A.y, A.z, A.w, Bc.x, Bc.y, Bc.z, Bc.w};
        const int o = j0 & 7, oh = o >> 1;
        uint32_t out[4];
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          // words oh + q4 and oh + q4 + 1 (oh in 0..3): select by the bits of oh
          const uint32_t a01 = (oh & 1) ? w[q4 + 1] : w[q4], a23 = (oh & 1) ? w[q4 + 3] : w[q4 + 2];
          const uint32_t b01 = (oh & 1) ? w[q4 + 2] : w[q4 + 1], b23 = (oh & 1) ? w[q4 + 4] : w[q4 + 3];
          const uint32_t lo = (oh & 2) ? a23 : a01, hi = (oh & 2) ? b23 : b01;
          const uint32_t v = (o & 1) ? __builtin_amdgcn_alignbit(hi, lo, 16) : lo;
          const int ja = j0 + 2 * q4;
          const bool va = i < T && ja >= 0 && ja < len && R0 + c8 + 2 * q4 < nrel;
          const bool vb = i < T && ja + 1 >= 0 && ja + 1 < len && R0 + c8 + 2 * q4 + 1 < nrel;
          out[q4] = v & ((va ? 0xFFFFu : 0u) | (vb ? 0xFFFF0000u : 0u));
        }
        rb[k] = make_uint4(out[0], out[1], out[2], out[3]);
      } else {
        const bf16x8 q = __builtin_bit_cast(bf16x8, ld8(qbase, p.D3, i, T, c8, p.dk, p.vec));
        bf16x8 qv;
#pragma unroll
        for (int e = 0; e < 8; ++e) qv[e] = (bf16)(i < T && c8 + e < p.dk ? (float)q[e] + pv8[e] : 0.f);
        ra[k] = __builtin_bit_cast(uint4, qv);
        const unsigned short* srow = reinterpret_cast<const unsigned short*>(dsb + (long)min(i, T - 1) * ldS);
        unsigned short t8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int j = j0 + e;
          t8[e] = (i < T && j >= 0 && j < len && R0 + c8 + e < nrel) ? srow[j] : (unsigned short)0;
        }
        rb[k] = make_uint4(t8[0] | (t8[1] << 16), t8[2] | (t8[3] << 16), t8[4] | (t8[5] << 16), t8[6] | (t8[7] << 16));
      }
    }
  };
  auto store = [&](int buf, const uint4 (&ra)[2], const uint4 (&rb)[2]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int row = (tid + 256 * k) >> 3;
      *reinterpret_cast<uint4*>(sA[buf] + row * KS + c8) = ra[k];
      *reinterpret_cast<uint4*>(sB[buf] + row * KS + c8) = rb[k];
    }
  };
  f32x16 acc = (f32x16){0};
  const int it0 = ilo & ~(TILE - 1);
  const int nit = (len > 0 && ihi >= ilo) ? (ihi - it0) / TILE + 1 : 0;
  // two register stages ahead of the LDS double buffer: tile it+2 is loaded while tile it runs through the MFMAs
  // and tile it+1 goes to LDS (four MFMAs per wave per tile cannot cover a load issued one tile ahead)
  uint4 ra0[2], rb0[2], ra1[2], rb1[2];
  if (nit > 0) {
    load(it0, ra0, rb0);
    if (nit > 1) load(it0 + TILE, ra1, rb1);
    store(0, ra0, rb0);
    __syncthreads();
  }
  auto step = [&](int it, uint4 (&af)[2], uint4 (&bfree)[2], const uint4 (&an)[2], const uint4 (&bn)[2]) {
    const int cur = it & 1;
    if (it + 2 < nit) load(it0 + (it + 2) * TILE, af, bfree);
#pragma unroll
    for (int s = 0; s < 4; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag_perm(sA[cur], 16 * s, 32 * dh, lane),
                                                    trfrag_perm(sB[cur], 16 * s, 32 * rh, lane), acc, 0, 0, 0);
    if (it + 1 < nit) store(cur ^ 1, an, bn);
    __syncthreads();
  };
  for (int it = 0; it < nit; it += 2) {
    step(it, ra0, rb0, ra1, rb1);                          // ra0 (tile it, stored) refills with tile it+2
    if (it + 1 < nit) step(it + 1, ra1, rb1, ra0, rb0);    // ra1 (tile it+1, stored) refills with tile it+3
  }
  // acc: rows d (32 dh + acc_row), lanes rr (32 rh + lane&31) -> sO[rr][d] -> this utterance's partial rows
  const int hh = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) sO[(32 * rh + (lane & 31)) * 65 + 32 * dh + acc_row(r, hh)] = acc[r] * p.scale;
  __syncthreads();
  float* dst = part + (long)b * nrel * p.HD;
  for (int idx = tid; idx < TILE * 64; idx += 256) {
    const int rr = idx >> 6, d = idx & 63;
    if (R0 + rr < nrel && d < p.dk) dst[(long)(R0 + rr) * p.HD + h * p.dk + d] = sO[rr * 65 + d];
  }
}

// dpos, round 5 (dk = 64 operands): 128 relative rows x 64 d per workgroup, the (b, h) pairs dealt to XCDs.
// The round-4 kernel above read 802 MB of HBM for 287 MB of dS at L60 (profiles/r05/rel_l60_pmc.txt: L2 hit rate
// 0.19) -- the r-tiles of one (b, h) sat on eight XCDs, so the cache lines two neighbouring r-tiles share (a band row
// segment is not line-aligned) and the (q+v) rows every r-tile of the pair re-reads were fetched once per XCD -- and
// spent ~300 VALU per wave per tile building the skewed dS chunks from two aligned 16-B loads with data-dependent
// selects.  Here:
//  * 1-D grid, workgroup L runs on XCD L % 8 (round-robin placement: a speed hint, never correctness); XCD x takes
//    the pairs x, x + 8, ... one after another, all r-tiles of a pair consecutively, so the pair's dS lines and
//    (q+v) rows are shared through that XCD's L2;
//  * the band skew moves to the LDS store: each row's needed dS run (128 elements from j = i + r0 - (T-1)) is read as
//    17 ALIGNED 16-B chunks (one buffer load each; a (b, h) slab's buffer range turns every out-of-slab read into
//    zeros, so no clamps) and each element is stored with ds_write_b16 at its band column r' = j - i - r0 + (T-1) of
//    a padded [row][8 + 136] image -- the round-4 / first round-5 forms spent ~300 VALU per wave per tile on funnel
//    shifts and clamps in registers; masks only on the edge tiles of the (i, r) parallelogram (a workgroup-uniform
//    test per tile);
//  * 128 r per workgroup halves the (q+v) tile traffic per output; 4 waves = (d half, r half of 64), 8 MFMAs per
//    wave per 64-row i-tile.
constexpr int DP_R = 128;              // relative rows per workgroup
// sB row stride (elements): 320 B = 80 dwords.  With the chunk-to-lane deal below (each 32-lane half of a store:
// rows r, r+2, r+4, r+6 x 8 consecutive chunks) every ds_write_b16 of the band image and every transposed
// fragment read is bank-conflict free (the 400-B stride with the row-major deal: ~740 extra LDS cycles per tile,
// 20.6 M in profiles/r05/rel_l60_pmc_final.txt -- the stores, whose lanes met on banks 4 and more ways)
constexpr int DP_KS = 160;
constexpr int DP_PADL = 8;             // band image column of r' = 0 (r' = -7 .. 135 are written, 0 .. 127 read)
constexpr int DP_CH = DP_R / 8 + 1;    // aligned 8-element dS chunks per row (17)

struct DposRegs {
  uint4 q[2];         // raw q rows (q + v is formed at store time: converting at load time waits for the load)
  uint4 w[5];         // raw dS: five aligned 8-element chunks (the fifth a real one for tid < 64 only)
};

__global__ __launch_bounds__(256) void attn_rel_bwd_dpos3_kernel(AttnM p, RelP rp, const bf16* __restrict__ dsbuf,
                                                                 int ldS, float* __restrict__ part, int nrt) {
  __shared__ __attribute__((aligned(16))) bf16 sA[2][TILE * KS];     // (q+v)[ii][d]
  __shared__ __attribute__((aligned(16))) bf16 sB[2][TILE * DP_KS];  // dS_band[ii][rr]
  float* const sO = reinterpret_cast<float*>(&sB[0][0]);            // [DP_R][65] after the loop (33 KiB <= 40 KiB)
  static_assert(DP_R * 65 * 4 <= 2 * TILE * DP_KS * 2, "the output stage fits in sB");
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nbh = p.B * p.H;
  const int xcd = blockIdx.x & 7, kx = blockIdx.x >> 3;
  const int bh = xcd + 8 * (kx / nrt), rt = kx % nrt;
  if (bh >= nbh) return;   // padding of the XCD deal (uniform over the workgroup)
  const int b = bh / p.H, h = bh % p.H;
  const int R0 = rt * DP_R;
  const int dh = wv & 1, rq = wv >> 1;
  const int T = p.T, nrel = 2 * T - 1;
  const int len = min(p.len[b], T);
  // i range with a key j = i + r - (T-1) in [0, len) for some r of the tile
  const int ilo = max(0, T - 1 - (R0 + DP_R - 1));
  const int ihi = min(T - 1, len - 1 + T - 1 - R0);
  // the pair's dS slab as a buffer resource: reads outside it (j < 0 on row 0, rows >= T) return zeros
  const __amdgpu_buffer_rsrc_t rs = head_rsrc(dsbuf + ((long)b * p.H + h) * T * (long)ldS, (long)T * ldS * 2);
  const bf16* qbase = p.qkv + (long)b * T * p.D3 + h * p.dk;
  const int c8 = (tid & 7) * 8;        // (q+v) chunk column
  float pv8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) pv8[e] = rp.pv[h * p.dk + c8 + e];
  // this thread's band chunks of the tile's 64 x 17: k < 4 -- 32-lane group G = 8k + 2 wv + (lane >> 5) takes rows
  // 8m + par + {0, 2, 4, 6} (G >> 1 = 2m + par) x chunks 8 (G & 1) .. +7 (conflict-free stores, see DP_KS; a wave
  // loads 4 rows x 16 whole chunks); k = 4 -- chunk 16 of row `lane` (wave 0; the other waves re-load their first
  // chunk, not stored).  Per chunk: row, chunk column, the row's skew s = (row + r0 - (T-1)) & 7 (row i's run starts
  // s elements into its first aligned chunk; I0 is a multiple of 64) and its element offset in the slab for tile
  // I0: I0 * (ldS + 1) + base
  int crow[5], ccol[5], csk[5], cbase[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int G = 8 * (k < 4 ? k : 0) + 2 * wv + (lane >> 5), rs = G >> 1;
    crow[k] = 8 * (rs >> 1) + (rs & 1) + 2 * ((lane & 31) >> 3);
    ccol[k] = 8 * (G & 1) + (lane & 7);
    if (k == 4 && wv == 0) {
      crow[k] = lane;
      ccol[k] = 16;
    }
    const int j0 = crow[k] + R0 - (T - 1);
    csk[k] = j0 & 7;
    cbase[k] = crow[k] * ldS + (j0 - csk[k]) + 8 * ccol[k];
  }
  auto interior = [&](int I0) {
    return I0 + TILE - 1 < T && I0 + R0 - (T - 1) >= 0 && I0 + TILE - 1 + R0 + DP_R - 1 - (T - 1) < len &&
           R0 + DP_R - 1 < nrel;
  };
  auto load = [&](int I0, DposRegs& g) {
#pragma unroll
    for (int k = 0; k < 2; ++k) g.q[k] = ld8c(qbase, p.D3, I0 + ((tid + 256 * k) >> 3), T, c8);
    // one aligned 16-B buffer load per chunk, no branch and no clamp (a branch here makes the compiler wait for the
    // loads at its join, and the prefetch ahead becomes a stall); negative offsets wrap past the range: zeros
    const int off0 = I0 * (ldS + 1);
#pragma unroll
    for (int k = 0; k < 5; ++k)
      g.w[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, 2 * (off0 + cbase[k]), 0, 0));
  };
  auto store = [&](int buf, int I0, const DposRegs& g) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = I0 + ((tid + 256 * k) >> 3);
      const bf16x8 q = __builtin_bit_cast(bf16x8, g.q[k]);
      bf16x8 qv;
#pragma unroll
      for (int e = 0; e < 8; ++e) qv[e] = (bf16)(i < T ? (float)q[e] + pv8[e] : 0.f);
      *reinterpret_cast<uint4*>(sA[buf] + ((tid + 256 * k) >> 3) * KS + c8) = __builtin_bit_cast(uint4, qv);
    }
    const bool in = interior(I0);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      if (k == 4 && tid >= TILE * DP_CH - 1024) break;
      uint32_t o[4] = {g.w[k].x, g.w[k].y, g.w[k].z, g.w[k].w};
      const int row = crow[k], i = I0 + row;
      // element e: j = I0 + row + r0 - (T-1) - sk + 8c + e, band column r' = 8c + e - sk
      const int rp0 = 8 * ccol[k] - csk[k];
      if (!in) {   // valid: i < T, 0 <= j < len, r0 + r' < nrel
        const int j0 = i + R0 - (T - 1) + rp0;
        const int lo = max(0, -j0), hi = i < T ? min(8, min(len - j0, nrel - R0 - rp0)) : 0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          o[u] &= ((2 * u >= lo && 2 * u < hi) ? 0xFFFFu : 0u) | ((2 * u + 1 >= lo && 2 * u + 1 < hi) ? 0xFFFF0000u : 0u);
      }
      // (volatile: 2-byte stores at 2-byte-aligned addresses; merged, they became misaligned ds_write_b128)
      typedef volatile __attribute__((address_space(3))) unsigned short lds_u16;
      lds_u16* d = reinterpret_cast<lds_u16*>((__attribute__((address_space(3))) bf16*)sB[buf]) + row * DP_KS + DP_PADL +
                   rp0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        d[2 * u] = (unsigned short)(o[u] & 0xFFFFu);
        d[2 * u + 1] = (unsigned short)(o[u] >> 16);
      }
    }
  };
  f32x16 acc0 = (f32x16){0}, acc1 = (f32x16){0};
  const int it0 = ilo & ~(TILE - 1);
  const int nit = (len > 0 && ihi >= ilo) ? (ihi - it0) / TILE + 1 : 0;
  // four register stages ahead of the LDS double buffer: step it issues tile it+3's loads, computes tile it from
  // LDS and stores tile it+1 (loaded two steps earlier) into the other buffer.  Every load and store is issued
  // unconditionally (tile indices clamped to the last tile), so the compiler's vmcnt waits stay counted -- a
  // conditional load makes the wait at its join a vmcnt(0) that also waits for the prefetch.  The 4-step unroll
  // leaves the loop after the last tile (a workgroup-uniform exit, nothing in flight is needed after it): running the
  // surplus steps of the last group (loads, band stores and a barrier each, ~1.5 of a workgroup's ~13 tiles at L60)
  // cost 8 us of 106 (profiles/r06/misc/dpos_exit_ab.txt)
  auto tile_of = [&](int it) { return it0 + min(it, nit - 1) * TILE; };
  auto step = [&](int it, DposRegs& gl, const DposRegs& gs) {
    load(tile_of(it + 3), gl);
    {
      const int cur = it & 1;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 a = trfrag_perm(sA[cur], 16 * s, 32 * dh, lane);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            a, trfrag_perm_s<DP_KS>(sB[cur], 16 * s, DP_PADL + 64 * rq, lane), acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            a, trfrag_perm_s<DP_KS>(sB[cur], 16 * s, DP_PADL + 64 * rq + 32, lane), acc1, 0, 0, 0);
      }
    }
    store((it + 1) & 1, tile_of(it + 1), gs);
    lds_barrier();
  };
  if (nit > 0) {
    DposRegs g[4];
#pragma unroll
    for (int k = 0; k < 3; ++k) load(tile_of(k), g[k]);
    store(0, tile_of(0), g[0]);
    lds_barrier();
    for (int it = 0; it < nit; it += 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {   // (this form keeps the stages in VGPRs; breaks between four named
        if (k > 0 && it + k >= nit) break;   // stages pushed ~100 registers into AGPRs: one wave per SIMD)
        step(it + k, g[(k + 3) & 3], g[(k + 1) & 3]);
      }
    }
  }
  // acc0/acc1: rows d (32 dh + acc_row), lanes rr (64 rq + 32 j + lane&31) -> sO[rr][d] -> the partial rows
  const int hh = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    sO[(64 * rq + (lane & 31)) * 65 + 32 * dh + acc_row(r, hh)] = acc0[r] * p.scale;
    sO[(64 * rq + 32 + (lane & 31)) * 65 + 32 * dh + acc_row(r, hh)] = acc1[r] * p.scale;
  }
  __syncthreads();
  float* dst = part + (long)b * nrel * p.HD;
  for (int idx = tid; idx < DP_R * 64; idx += 256) {
    const int rr = idx >> 6, d = idx & 63;
    if (R0 + rr < nrel) dst[(long)(R0 + rr) * p.HD + h * p.dk + d] = sO[rr * 65 + d];
  }
}

}  // namespace

namespace cfm {

// workspace of the rel-pos MFMA backward: [D (B*H*T f32)] [du/dv partials] [dS (B*H*T*ldS bf16)]
// [per-utterance dpos partials (B*(2T-1)*H*dk f32)]
static inline int rel_ldS(int T) { return (T + 7) & ~7; }
static inline size_t rel_part_floats(int B, int T, int H, int dk) { return (size_t)B * 4 * cdiv(T, 128) * 2 * H * dk; }

size_t attn_rel_ws_bytes(int B, int T, int H, int dk) {
  const size_t d = (size_t)B * H * T * sizeof(float);
  const size_t part = rel_part_floats(B, T, H, dk) * sizeof(float);
  const size_t ds = (size_t)B * H * T * rel_ldS(T) * sizeof(bf16);
  const size_t dpos_part = (size_t)B * (2 * T - 1) * H * dk * sizeof(float);
  return ((d + 255) & ~(size_t)255) + ((part + 255) & ~(size_t)255) + ((ds + 255) & ~(size_t)255) + dpos_part;
}

static RelP make_relp(const void* pos, const float* pu, const float* pv, int dk) {
  return RelP{(const bf16*)pos, pu, pv, ((uintptr_t)pos % 16 == 0) && (dk % 8 == 0)};
}

// branch-free prefetch kernels (ld8c): dk = 64 with 16-B aligned rows of qkv / dout / pos.  cfm_attn_set_mode
// bit 6 keeps the zero-filling loads (A/B)
int g_rel_mode = 0;
static bool rel_vec(const AttnM& p, const RelP& rp) { return p.vec && rp.pvec && p.dk == 64 && !(g_rel_mode & 64); }

static AttnM make_attnm(const void* qkv, const void* dout, const int32_t* len, int B, int T, int H, int dk,
                        float drop_p, uint64_t seed) {
  AttnM p{(const bf16*)qkv, B, T, H, dk, 3 * H * dk, H * dk, len, 1.f / sqrtf((float)dk), drop_p, seed,
          ((uintptr_t)qkv % 16 == 0) && ((uintptr_t)dout % 16 == 0) && (dk % 8 == 0) && ((3 * H * dk) % 8 == 0), 0,
          g_rng_salt};
  return p;
}

int attn_rel_fwd_launch(const void* qkv, void* o, float* lse, const int32_t* len, const void* pos, const float* pu,
                        const float* pv, int B, int T, int H, int dk, float drop_p, uint64_t seed, hipStream_t s) {
  const AttnM p = make_attnm(qkv, qkv, len, B, T, H, dk, drop_p, seed);
  const RelP rp = make_relp(pos, pu, pv, p.dk);
  const dim3 grid(cdiv(p.T, 128), p.H, p.B);
  if (rel_vec(p, rp)) hipLaunchKernelGGL(attn_rel_fwd2_kernel<true>, grid, dim3(256), 0, s, p, rp, (bf16*)o, lse);
  else hipLaunchKernelGGL(attn_rel_fwd2_kernel<false>, grid, dim3(256), 0, s, p, rp, (bf16*)o, lse);
  return check_launch("cfm_attn_fwd(rel)");
}

// D (rowsum dO*O per head) must already be in ws[0 .. B*H*T)
int attn_rel_bwd_launch(const void* qkv, const void* dout, const float* lse, const int32_t* len, const void* pos,
                        const float* pu, const float* pv, void* dqkv, void* dpos, int dpos_dt, float* dpu, float* dpv,
                        int B, int T, int H, int dk, float drop_p, uint64_t seed, float* ws, hipStream_t s) {
  AttnM p = make_attnm(qkv, dout, len, B, T, H, dk, drop_p, seed);
  const RelP rp = make_relp(pos, pu, pv, p.dk);
  const size_t d_bytes = ((size_t)p.B * p.H * p.T * sizeof(float) + 255) & ~(size_t)255;
  float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + d_bytes);
  const size_t part_bytes = (rel_part_floats(p.B, p.T, p.H, p.dk) * sizeof(float) + 255) & ~(size_t)255;
  bf16* dsbuf = reinterpret_cast<bf16*>(reinterpret_cast<char*>(part) + part_bytes);
  const int ldS = rel_ldS(p.T);
  const dim3 grid(cdiv(p.T, 128), p.H, p.B);
  // dK / dV (+ the dS buffer), then dQ: from the stored dS (default) or recomputed (cfm_attn_set_mode bit 9)
  const bool dq_recompute = (g_rel_mode & 512) != 0;
  if (rel_vec(p, rp)) {
    hipLaunchKernelGGL(attn_rel_bwd_dkdv_kernel<true>, grid, dim3(256), 0, s, p, rp, (const bf16*)dout, lse, ws,
                       (bf16*)dqkv, dsbuf, ldS);
    if (dq_recompute)
      hipLaunchKernelGGL(attn_rel_bwd_dq2_kernel<true>, grid, dim3(256), 0, s, p, rp, (const bf16*)dout, lse, ws,
                         (bf16*)dqkv, part);
    else
      hipLaunchKernelGGL(attn_rel_bwd_dqs_kernel<true>, grid, dim3(256), 0, s, p, rp, (const bf16*)dsbuf, ldS,
                         (bf16*)dqkv, part);
  } else {
    hipLaunchKernelGGL(attn_rel_bwd_dkdv_kernel<false>, grid, dim3(256), 0, s, p, rp, (const bf16*)dout, lse, ws,
                       (bf16*)dqkv, dsbuf, ldS);
    if (dq_recompute)
      hipLaunchKernelGGL(attn_rel_bwd_dq2_kernel<false>, grid, dim3(256), 0, s, p, rp, (const bf16*)dout, lse, ws,
                         (bf16*)dqkv, part);
    else
      hipLaunchKernelGGL(attn_rel_bwd_dqs_kernel<false>, grid, dim3(256), 0, s, p, rp, (const bf16*)dsbuf, ldS,
                         (bf16*)dqkv, part);
  }
  const size_t ds_bytes = ((size_t)p.B * p.H * p.T * ldS * sizeof(bf16) + 255) & ~(size_t)255;
  float* dpos_part = reinterpret_cast<float*>(reinterpret_cast<char*>(dsbuf) + ds_bytes);
  if (rel_vec(p, rp) && !(g_rel_mode & 128)) {
    const int nrt = cdiv(2 * p.T - 1, DP_R);
    hipLaunchKernelGGL(attn_rel_bwd_dpos3_kernel, dim3(8 * cdiv(p.B * p.H, 8) * nrt), dim3(256), 0, s, p, rp,
                       (const bf16*)dsbuf, ldS, dpos_part, nrt);
  } else if (rel_vec(p, rp))
    hipLaunchKernelGGL(attn_rel_bwd_dpos_kernel<true>, dim3(cdiv(2 * p.T - 1, TILE), p.H, p.B), dim3(256), 0, s, p, rp,
                       (const bf16*)dsbuf, ldS, dpos_part);
  else
    hipLaunchKernelGGL(attn_rel_bwd_dpos_kernel<false>, dim3(cdiv(2 * p.T - 1, TILE), p.H, p.B), dim3(256), 0, s, p,
                       rp, (const bf16*)dsbuf, ldS, dpos_part);
  if (dpos_dt == CFM_BF16)   // the compute-dtype copy the dW_pos GEMM reads: no fp32 dpos + cast pass
    colreduce_bf16(dpos_part, p.B, (long)(2 * p.T - 1) * p.HD, (bf16*)dpos, s);
  else
    colreduce(dpos_part, p.B, (long)(2 * p.T - 1) * p.HD, (float*)dpos, 0, s);
  const int nrows = p.B * 4 * cdiv(p.T, 128);
  colreduce_pair(part, part + p.HD, nrows, (long)p.HD, dpu, dpv, s, 2L * p.HD);   // du, dv: one launch
  return check_launch("cfm_attn_bwd(rel)");
}

}  // namespace cfm
