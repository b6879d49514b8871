// attn_common.h — shared pieces of the MFMA attention kernels (attention.hip, attention_rel.hip):
// tile geometry, the per-(b,h) parameter block, attention-dropout indexing, and the fragment
// helpers that move 32x32x16 bf16 MFMA operands between LDS tiles, registers and accumulators.
#pragma once
#include "cfm_common.h"

namespace {

constexpr int DKP = 64;      // padded head dim
constexpr int KS = DKP + 8;  // LDS row stride (elements): 144-B rows, conflict-free ds_read_b128
constexpr int TILE = 64;     // keys (fwd/dQ) or queries (dK/dV) per LDS tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

struct AttnM {
  const bf16* qkv;
  int B, T, H, dk, D3, HD;
  const int32_t* len;
  float scale;
  float drop_p; uint64_t seed;
  bool vec;    // 16-B vector loads legal
  int dbg;     // timing experiments (cfm_attn_set_mode bits 1-2)
  const uint64_t* salt;   // bound dropout step counter or nullptr
  bool vec4;   // 8-B vector loads legal (dk % 4 == 0, 8-B aligned rows: Conformer-S's dk 36)
  int qs;      // whole-head kernels: workgroups per (b, h), each a contiguous range of 32-row blocks (<= 1: one)
};

// attention-dropout element index: rows of an EVEN stride (T rounded up to even), so the keys 2m and
// 2m+1 of one (query, key-pair) share one 32-bit hash (low / high 16 bits): kernels holding both keys of
// a pair in one lane (accumulator registers r, r+1 for even r) hash once per pair (dropout_pair)
__device__ __forceinline__ uint64_t didx(const AttnM& p, int b, int h, int i, int j) {
  return (((uint64_t)b * p.H + h) * p.T + i) * (uint64_t)(p.T + (p.T & 1)) + j;
}
// keep-scales of elements idx (even) and idx + 1: one mix for both (== dropout_keyed of each)
__device__ __forceinline__ void dropout_pair(uint32_t thr, float keep, uint32_t key, uint64_t idx, float& m0,
                                             float& m1) {
  const uint32_t h = attn_mix((uint32_t)(idx >> 1) + key);
  m0 = (h & 0xFFFFu) >= thr ? keep : 0.f;
  m1 = (h >> 16) >= thr ? keep : 0.f;
}

// v_max3_f32 (IEEE maxNum of three, as two fmaxf)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// 2^x for softmax arguments <= 0: the bare v_exp_f32 (results below 2^-126 flush to 0)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// the same with the pair's hash index j = (idx >> 1) mod 2^32 supplied in 32 bits (idx < 2^33)
__device__ __forceinline__ void dropout_pair32(uint32_t thr, float keep, uint32_t key, uint32_t j, float& m0,
                                               float& m1) {
  const uint32_t h = attn_mix(j + key);
  m0 = (h & 0xFFFFu) >= thr ? keep : 0.f;
  m1 = (h >> 16) >= thr ? keep : 0.f;
}

// 8 consecutive head-dim elements c..c+7 of row `row` of matrix base (row stride ld), zero-padded
// (vec: one 16-B load; vec4: two 8-B loads, the upper one zero past dk -- dk 36 rows start 8-B aligned only)
__device__ __forceinline__ uint4 ld8(const bf16* base, long ld, int row, int nrows, int c, int dk, bool vec,
                                     bool vec4 = false) {
  uint4 r = make_uint4(0, 0, 0, 0);
  if (row >= nrows || c >= dk) return r;
  const bf16* p = base + (long)row * ld + c;
  if (vec && c + 8 <= dk) return *reinterpret_cast<const uint4*>(p);
  if (vec4) {
    const uint2 lo = *reinterpret_cast<const uint2*>(p);
    const uint2 hi = c + 8 <= dk ? *reinterpret_cast<const uint2*>(p + 4) : make_uint2(0, 0);
    return make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
  unsigned short t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = (c + e < dk) ? reinterpret_cast<const unsigned short*>(p)[e] : 0;
  r.x = t[0] | (t[1] << 16); r.y = t[2] | (t[3] << 16); r.z = t[4] | (t[5] << 16); r.w = t[6] | (t[7] << 16);
  return r;
}

// A-operand fragment, natural k order, from a [row][KS] tile: lane (r, hh) gets row r0+r, cols k0+8hh..+7
__device__ __forceinline__ bf16x8 rowfrag(const bf16* tile, int r0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(tile + (r0 + (lane & 31)) * KS + k0 + 8 * (lane >> 5));
}

// A-operand fragment of the TRANSPOSED tile, k order permuted to match an accumulator used as the
// B operand (element j of lane half hh <-> tile row r0 + 8(j>>2) + 4hh + (j&3)); column c0 + (lane&31).
__device__ __forceinline__ bf16x8 trfrag_perm(const bf16* tile, int r0, int c0, int lane) {
  const int hh = lane >> 5, g1 = (lane >> 4) & 1, q = (lane & 15) >> 2, p4 = lane & 3;
  const bf16* base = tile + (r0 + 4 * hh + q) * KS + c0 + 16 * g1 + 4 * p4;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + 8 * KS));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// trfrag_perm with an explicit row stride (the dQ-from-dS kernels' conflict-free images, the rel-pos dpos kernel)
template <int STR>
__device__ __forceinline__ bf16x8 trfrag_perm_s(const bf16* tile, int r0, int c0, int lane) {
  const int hh = lane >> 5, g1 = (lane >> 4) & 1, q = (lane & 15) >> 2, p4 = lane & 3;
  const bf16* base = tile + (r0 + 4 * hh + q) * STR + c0 + 16 * g1 + 4 * p4;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + 8 * STR));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// a [64 rows][64 cols] register tile (tile_load) into LDS rows of STR elements
template <int STR>
__device__ __forceinline__ void tile_store_s(bf16* t, const uint4 (&reg)[2], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + 256 * i;
    *reinterpret_cast<uint4*>(t + (v >> 3) * STR + (v & 7) * 8) = reg[i];
  }
}

// accumulator registers 8s..8s+7 -> bf16 B-operand fragment of k-step s
__device__ __forceinline__ bf16x8 acc2frag(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * s + j];
  return r;
}

// accumulator row of register r for lane half hh
__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// 16 B at row clamp(row, 0, nrows - 1), column c: branch-free, for dk = 64 operands with 16-B aligned rows.
// A prefetch through ld8's zero-fill branches makes the compiler wait for the load at the branch join (an
// s_waitcnt vmcnt(0) right behind the prefetch, which also waits for every older store): with one wave per
// SIMD that exposed a full memory round trip per tile.  Clamped rows hold finite data of the same operand,
// and every consumer masks them (keys >= len, queries >= T, relative rows no valid (i, j) pair reaches).
__device__ __forceinline__ uint4 ld8c(const bf16* base, long ld, int row, int nrows, int c) {
  row = min(max(row, 0), nrows - 1);
  return *reinterpret_cast<const uint4*>(base + (long)row * ld + c);
}

// stage a [64 rows][64 cols] bf16 tile (row r0.., column offset col of qkv) into LDS; 2 x 16 B per thread
// (VEC: ld8c, rows past T clamped)
template <bool VEC = false>
__device__ __forceinline__ void tile_load(const AttnM& p, int b, int r0, int col, uint4 (&reg)[2], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + 256 * i;
    if constexpr (VEC) reg[i] = ld8c(p.qkv + (long)b * p.T * p.D3 + col, p.D3, r0 + (v >> 3), p.T, (v & 7) * 8);
    else reg[i] = ld8(p.qkv + (long)b * p.T * p.D3 + col, p.D3, r0 + (v >> 3), p.T, (v & 7) * 8, p.dk, p.vec);
  }
}
__device__ __forceinline__ void tile_store(bf16* t, const uint4 (&reg)[2], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + 256 * i;
    *reinterpret_cast<uint4*>(t + (v >> 3) * KS + (v & 7) * 8) = reg[i];
  }
}

// B-operand fragments (natural k order) of a 32-row block: lane (r, hh) = row[r][16s + 8hh .. +7]
__device__ __forceinline__ void load_bfrags(const AttnM& p, const bf16* base, long ld, int row, int nrows,
                                            bf16x8 (&f)[4], int lane) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    uint4 u = ld8(base, ld, row, nrows, 16 * s + 8 * (lane >> 5), p.dk, p.vec, p.vec4);
    f[s] = __builtin_bit_cast(bf16x8, u);
  }
}

// write a wave's 64(d) x 32(cols) f32 accumulator pair (dt = 0, 1) transposed into a bf16 matrix:
// out[(row0 + c) * ld + d] = acc[d][c] * mul_c  (c < ncols, d < dk), staged through LDS.
__device__ void store_transposed(float* stage, const f32x16& a0, const f32x16& a1, float mulc, bf16* out, long ld,
                                 int row0, int nvalid, int dk, int lane) {
  const int hh = lane >> 5, c = lane & 31;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    stage[c * 65 + acc_row(r, hh)] = a0[r] * mulc;
    stage[c * 65 + 32 + acc_row(r, hh)] = a1[r] * mulc;
  }
  __builtin_amdgcn_wave_barrier();
  if (dk == 64 && ((uintptr_t)out & 15) == 0 && (ld & 7) == 0) {
    // 16-B stores: lane = (row cc = 8 it + lane / 8, 8-column group lane % 8), whole 128-B rows per 8 lanes
    const int g8 = lane & 7;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int cc = 8 * it + (lane >> 3);
      if (cc < nvalid) {
        const float* src = stage + cc * 65 + 8 * g8;
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)src[e];
        *reinterpret_cast<bf16x8*>(out + (long)(row0 + cc) * ld + 8 * g8) = v;
      }
    }
  } else {
    for (int idx = lane; idx < 32 * 64; idx += 64) {
      const int cc = idx >> 6, d = idx & 63;
      if (cc < nvalid && d < dk) out[(long)(row0 + cc) * ld + d] = (bf16)stage[cc * 65 + d];
    }
  }
  __builtin_amdgcn_wave_barrier();
}

// One key tile of the forward's online softmax for a wave (queries on the lanes, keys k0 + acc_row(r, hh)
// [+ 32] in s0 / s1, raw unscaled scores): masking only on the utterance's last tile (`tail`, uniform), the
// running max kept in scaled log2 units (c = scale * log2 e > 0, so max(c s) = c max(s)), p = 2^(c s - m) as
// one FMA + v_exp; rescales o0/o1 and l; attention dropout applied to p (the returned P is dropped/scaled,
// l stays the undropped sum, as nn.MultiheadAttention: dropout after the softmax).
// LATE: the dropout keep scale 1 / (1 - p) is NOT applied to P here (dropped entries are zeroed by one select per
// score); the caller multiplies it into the output once per element instead (o * keep / l).
template <bool LATE = false>
__device__ __forceinline__ void softmax_tile(const AttnM& p, f32x16& s0, f32x16& s1, f32x16& o0, f32x16& o1,
                                             float& m, float& l, float c, int kbase, int len, bool tail, int b,
                                             int h, int qi, int hh, uint32_t dthr, float dkeep, uint32_t dkey) {
  if (tail && kbase + TILE > len) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k0 = kbase + acc_row(r, hh);
      s0[r] = (k0 < len) ? s0[r] : -INFINITY;
      s1[r] = (k0 + 32 < len) ? s1[r] : -INFINITY;
    }
  }
  // the tile maximum as two chains of v_max3_f32 (fmaxf chains compile to v_max_f32 with a canonicalising
  // v_max per MFMA output in IEEE mode: ~57 instructions per tile, here 17; max is exact either way)
  float ma = max3f(s0[0], s0[1], s0[2]), mb = max3f(s1[0], s1[1], s1[2]);
#pragma unroll
  for (int r = 3; r < 15; r += 2) {
    ma = max3f(ma, s0[r], s0[r + 1]);
    mb = max3f(mb, s1[r], s1[r + 1]);
  }
  float mloc = max3f(ma, mb, fmaxf(s0[15], s1[15]));
  mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
  const float mn = fmaxf(m, mloc * c);
  const float alpha = fast_exp2(m - mn);
  // the scale-and-shift and the o rescale on packed FP32 (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth per
  // instruction, the same IEEE operations per element); the sum keeps its order
  typedef float f32x2v __attribute__((ext_vector_type(2)));
  const f32x2v c2 = {c, c}, nm2 = {-mn, -mn}, a2 = {alpha, alpha};
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const f32x2v x0 = __builtin_elementwise_fma((f32x2v){s0[r], s0[r + 1]}, c2, nm2);
    const f32x2v x1 = __builtin_elementwise_fma((f32x2v){s1[r], s1[r + 1]}, c2, nm2);
    s0[r] = x0.x; s0[r + 1] = x0.y;
    s1[r] = x1.x; s1[r + 1] = x1.y;
  }
  float ls = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    s0[r] = fast_exp2(s0[r]);
    s1[r] = fast_exp2(s1[r]);
    ls += s0[r] + s1[r];
  }
  ls += __shfl_xor(ls, 32, 64);
  l = l * alpha + ls;
  m = mn;
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const f32x2v y0 = (f32x2v){o0[r], o0[r + 1]} * a2, y1 = (f32x2v){o1[r], o1[r + 1]} * a2;
    o0[r] = y0.x; o0[r + 1] = y0.y;
    o1[r] = y1.x; o1[r + 1] = y1.y;
  }
  if (p.drop_p > 0.f) {
    const uint32_t rowj = (uint32_t)(didx(p, b, h, qi, kbase) >> 1);   // even: 32-bit pair indices
    // pair index + key = hb + a compile-time constant per register pair (k0 / 2 = ((r & 3) >> 1) + 4 (r >> 2) + 2 hh):
    // one add per hash instead of two (the same 32-bit sums)
    const uint32_t hb = rowj + dkey + 2u * (uint32_t)hh;
#pragma unroll
    for (int r = 0; r < 16; r += 2) {     // registers r, r+1 = keys k, k+1 with k even: one hash
      const int k0 = acc_row(r, hh);
      if constexpr (LATE) {
        const uint32_t cr = (uint32_t)(((r & 3) >> 1) + 4 * (r >> 2));
        const uint32_t h0 = attn_mix(hb + cr), h1 = attn_mix(hb + cr + 16u);
        s0[r] = (h0 & 0xFFFFu) >= dthr ? s0[r] : 0.f;
        s0[r + 1] = (h0 >> 16) >= dthr ? s0[r + 1] : 0.f;
        s1[r] = (h1 & 0xFFFFu) >= dthr ? s1[r] : 0.f;
        s1[r + 1] = (h1 >> 16) >= dthr ? s1[r + 1] : 0.f;
      } else {
        float m0, m1, m2, m3;
        dropout_pair32(dthr, dkeep, dkey, rowj + (k0 >> 1), m0, m1);
        dropout_pair32(dthr, dkeep, dkey, rowj + (k0 >> 1) + 16, m2, m3);
        s0[r] *= m0; s0[r + 1] *= m1;
        s1[r] *= m2; s1[r + 1] *= m3;
      }
    }
  }
}

// ------------------------------------------------------------------------------------ LDS-DMA head images
// A head operand slice (rows of dk = 64 bf16 = 128 B at row stride ld) staged with `buffer_load ... lds`
// into an unpadded [rows][128 B] image whose 16-B chunk c of row r sits in slot c ^ ((r >> 1) & 7): the
// 32 rows x one chunk of an MFMA operand fragment then hit 16 distinct bank groups per 16 lanes
// (conflict-free ds_read_b128).  One wave-instruction moves one 1-KiB piece = 8 rows; no VGPR round trip,
// so a whole head can be in flight while the first tiles are already being consumed (counted vmcnt +
// s_barrier per tile).  Rows past the operand's `nrows` clamp to its last row (finite data; masked).
__device__ __forceinline__ int himg(int r, int c) { return r * 128 + 16 * (c ^ ((r >> 1) & 7)); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t head_rsrc(const bf16* base, long bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}

// piece `pc` (rows 8 pc .. 8 pc + 7) of the image at `img`: lane l's 16 B from row 8 pc + l / 8
// (m0 is declared clobbered -- the asm does overwrite it -- which clang reports as a reserved register; silenced here)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void head_dma_piece(__amdgpu_buffer_rsrc_t r, char* img, int pc, long ld, int nrows,
                                               int lane) {
  const int row = 8 * pc + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
  const unsigned voff = (unsigned)(((long)min(row, nrows - 1) * ld + 8 * c) * 2);
  const unsigned l = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(img + 1024 * pc));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(l), "v"(voff), "s"(r) : "memory", "m0");
}
#pragma clang diagnostic pop

// s_waitcnt vmcnt(0) as a real instruction the compiler's wait insertion accounts for (inline asm is opaque to
// it): issued once after a kernel's prologue loads (q fragments, K/V of the head) so that their first use inside
// the tile loop does not make the compiler wait for everything outstanding -- the prefetch just issued included --
// on every iteration.  gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15.
__device__ __forceinline__ void wait_prologue_loads() { __builtin_amdgcn_s_waitcnt(0x0F70); }


// s_waitcnt vmcnt(n) for a wave-uniform run-time n
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
#define W(k) case k: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(k) : "memory"); break;
    W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14) W(15) W(16)
#undef W
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// fragments from a head image: A-operand rows r0 + (lane & 31), k = k0 + 8 (lane >> 5) .. +7 (natural order)
__device__ __forceinline__ bf16x8 hfrag(const char* img, int r0, int k0, int lane) {
  const int r = r0 + (lane & 31);
  return *reinterpret_cast<const bf16x8*>(img + himg(r, (k0 >> 3) + (lane >> 5)));
}
// trfrag_perm on a head image (transposed, k order matching an accumulator used as the B operand)
__device__ __forceinline__ bf16x8 htrfrag(const char* img, int r0, int c0, int lane) {
  const int hh = lane >> 5, g1 = (lane >> 4) & 1, q = (lane & 15) >> 2, p4 = lane & 3;
  const int row = r0 + 4 * hh + q, col = c0 + 16 * g1 + 4 * p4;
  const char* a0 = img + himg(row, col >> 3) + (col & 7) * 2;
  const char* a1 = img + himg(row + 8, col >> 3) + (col & 7) * 2;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

}  // namespace
