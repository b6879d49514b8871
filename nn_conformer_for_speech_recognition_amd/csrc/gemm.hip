// gemm.hip — MFMA GEMM with fused epilogues for every dense contraction of the encoder, plus the
// implicit-GEMM forms of the second subsampling convolution (no im2col in HBM).
//
// Tile: 128x128 output per 256-thread workgroup (4 waves as 2x2, 64x64 per wave =
// 2x2 MFMA 32x32 tiles).  bf16 operands: v_mfma_f32_32x32x16_bf16, BK = 32.  fp32 operands:
// v_mfma_f32_32x32x2_f32 (exact f32 products, used for the fp32 parity mode), BK = 16.
// Operand layouts (per operand, compile-time): K-major (k contiguous, e.g. X and W in the
// forward pass) is staged row-wise and read with ds_read_b128; MN-major (m/n contiguous, e.g.
// the token dimension in weight-gradient GEMMs) is staged as [k][m] and read with the gfx950
// ds_read_b64_tr_b16 transposed LDS read, so no operand is ever transposed in HBM.
// Operands are "loader" functors: a plain strided matrix, or an on-the-fly im2col gather for
// the 3x3/stride-2 convolution (forward, weight-grad and data-grad).
// Global->LDS staging goes through registers with one-tile-ahead prefetch and a double-buffered
// LDS ring (one barrier per K tile).
#include "cfm_common.h"

#include <algorithm>
#include <type_traits>
#include <vector>

namespace {

constexpr int BM = 128, BN = 128, NT = 256;

struct GemmP {
  int M, N, K;
  void* C; long ldc, sc; int dtc;
  float alpha;
  const float* bias;
  int act, act_grad;
  void* pre; int dtpre;
  float drop_p; uint64_t seed, doff;
  const uint64_t* salt;   // bound dropout step counter (cfm_rng_bind) or nullptr
  float out_scale;
  const void* res; long ldr; int dtr;
  int split_k, k_per_split;
  int vec_c;   // 8-wide epilogue legal: C/pre/residual/bias 16-B aligned rows
  float* slab; // split-K slabs [batch*split][M][N] (nullptr: atomics into C)
  // output row remap for the conv2 data-grad parity classes: row m = (b, i, j) of the class
  // -> dh1 row (b, 2i+pf, 2j+pt)
  int cmap, cm_F1c, cm_T1c, cm_pf, cm_pt, cm_F1, cm_T1;
  int dbg;     // timing experiments only (cfm_gemm_set_mode bit 3: skip the epilogue's stores; bit 13: the main loop)
  unsigned long long* probe;   // optional timing slot (cfm_gemm_desc.probe)
  float* acs_slab;             // A column-sum partials [split][M] (cfm_gemm_desc.a_colsum) or nullptr
  const bf16* rd_with;         // per-64-column-group row dots with C (cfm_gemm_desc.rowdot_*) or nullptr
  float* rd_out;
  int rd_T;
  const float* alpha_a;        // fp8 operands: per-tensor dequantisation scales (device) or nullptr
  const float* alpha_b;
  uint32_t dkey0, dthr;        // dropout constants hoisted out of the epilogue (gemm_drop_prep)
  float dkeep;
  int efast;                   // staged-epilogue fast path (epi_fast_kind; 0: the generic epilogue_store8 rows)
  const uint8_t* mxa;          // MX fp8 operands (cfm_gemm_desc.mx_a / mx_b): e8m0 block scales [rows][mxk]
  const uint8_t* mxb;
  int mxk;                     // blocks of 32 fp8 per row (K / 32)
  uint8_t* mxo8;               // EF_BF16_SILU_MX: the MX e4m3 copy of the bf16 C (cfm_gemm_desc.mx_out)
  uint8_t* mxos;               //   and its e8m0 block scales [M][N/32]
};

// salt the dropout seed and hoist the per-launch constants (hash key of the low 2^33 index range,
// threshold, keep scale -- the latter an IEEE division) out of the per-8-element epilogue
__device__ __forceinline__ void gemm_drop_prep(GemmP& p) {
  if (p.drop_p > 0.f) {
    p.seed = salted_seed(p.seed, p.salt);
    p.dkey0 = drop_key(p.seed, 0);
    p.dthr = drop_thr(p.drop_p);
    p.dkeep = drop_keep_scale(p.dthr);
  }
}

__device__ __forceinline__ long out_row(const GemmP& p, int m) {
  if (!p.cmap) return m;
  const int j = m % p.cm_T1c, r = m / p.cm_T1c, i = r % p.cm_F1c, b = r / p.cm_F1c;
  return ((long)b * p.cm_F1 + 2 * i + p.cm_pf) * p.cm_T1 + 2 * j + p.cm_pt;
}

template <typename T> struct VecOf;
template <> struct VecOf<bf16> { typedef uint4 type; static constexpr int W = 8; };
template <> struct VecOf<float> { typedef float4 type; static constexpr int W = 4; };

// element-wise fallback: W consecutive elements p[0..W), zero past `n_ok`
template <typename T>
__device__ __forceinline__ typename VecOf<T>::type ld_partial(const T* p, int n_ok) {
  typedef typename VecOf<T>::type V;
  constexpr int W = VecOf<T>::W;
  if constexpr (W == 8) {
    unsigned short t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = e < n_ok ? reinterpret_cast<const unsigned short*>(p)[e] : 0;
    V r;
    r.x = t[0] | (t[1] << 16); r.y = t[2] | (t[3] << 16); r.z = t[4] | (t[5] << 16); r.w = t[6] | (t[7] << 16);
    return r;
  } else {
    float t[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) t[e] = e < n_ok ? p[e] : 0.f;
    return make_float4(t[0], t[1], t[2], t[3]);
  }
}
template <typename T> __device__ __forceinline__ typename VecOf<T>::type vzero() {
  typename VecOf<T>::type r;
  if constexpr (VecOf<T>::W == 8) r = make_uint4(0, 0, 0, 0); else r = make_float4(0.f, 0.f, 0.f, 0.f);
  return r;
}

// Plain strided operand: element (outer, inner) at base[outer*ld + inner] (+ batch stride)
template <typename T> struct StridedOp {
  const T* base; long ld; long bstride; bool vec;
  __device__ __forceinline__ void batch(int z) { base += (long)z * bstride; }
  __device__ __forceinline__ typename VecOf<T>::type load(int outer, int inner, int outer_lim, int inner_lim) const {
    constexpr int W = VecOf<T>::W;
    if (outer >= outer_lim || inner >= inner_lim) return vzero<T>();
    const T* p = base + (long)outer * ld + inner;
    if (vec && inner + W <= inner_lim) return *reinterpret_cast<const typename VecOf<T>::type*>(p);
    return ld_partial<T>(p, inner_lim - inner);
  }
};

// conv2 geometry: h1 NHWC (B, F1, T1, C1); output rows m = (b, t2, f2); taps (kh, kw) 3x3 stride 2
struct Conv2Geo { int B, F1, T1, C1, F2, T2, C2; };

// forward A (K-major): A(m, k=(kh,kw,c1)) = h1[b, 2f2+kh, 2t2+kw, c1]
template <typename T> struct Conv2FwdA {
  const T* h1; Conv2Geo g;
  __device__ __forceinline__ void batch(int) {}
  __device__ __forceinline__ typename VecOf<T>::type load(int m, int k, int m_lim, int k_lim) const {
    if (m >= m_lim || k >= k_lim) return vzero<T>();
    const int f2 = m % g.F2, r = m / g.F2, t2 = r % g.T2, b = r / g.T2;
    const int tap = k / g.C1, c1 = k % g.C1, kh = tap / 3, kw = tap % 3;
    const T* p = h1 + (((long)b * g.F1 + 2 * f2 + kh) * g.T1 + 2 * t2 + kw) * g.C1 + c1;
    return *reinterpret_cast<const typename VecOf<T>::type*>(p);
  }
};
// weight-grad B (MN-major): B(n=(kh,kw,c1), k=m) = h1[b(m), 2f2+kh, 2t2+kw, c1]
template <typename T> struct Conv2WgradB {
  const T* h1; Conv2Geo g;
  __device__ __forceinline__ void batch(int) {}
  __device__ __forceinline__ typename VecOf<T>::type load(int m, int n, int m_lim, int n_lim) const {
    if (m >= m_lim || n >= n_lim) return vzero<T>();
    const int f2 = m % g.F2, r = m / g.F2, t2 = r % g.T2, b = r / g.T2;
    const int tap = n / g.C1, c1 = n % g.C1, kh = tap / 3, kw = tap % 3;
    const T* p = h1 + (((long)b * g.F1 + 2 * f2 + kh) * g.T1 + 2 * t2 + kw) * g.C1 + c1;
    return *reinterpret_cast<const typename VecOf<T>::type*>(p);
  }
};
// data-grad, one stride-2 parity class (pf, pt) of input pixels at a time: pixel (f1, t1) with
// f1 = 2i + pf, t1 = 2j + pt only receives the taps kh = pf (+2), kw = pt (+2), i.e. 4 / 2 / 2 / 1
// taps for the four classes instead of 9 zero-padded ones (4x fewer MACs than a plain im2col).
struct Conv2Class {
  int pf, pt, F1c, T1c, ntaps;
  int kh[4], kw[4];
};
// A (K-major): rows (b, i, j) of the class, k = (tap, c2) -> dh2[b, t2 = (t1-kw)/2, f2 = (f1-kh)/2, c2]
template <typename T> struct Conv2DgradA {
  const T* dh2; Conv2Geo g; Conv2Class c;
  __device__ __forceinline__ void batch(int) {}
  __device__ __forceinline__ typename VecOf<T>::type load(int pr, int k, int p_lim, int k_lim) const {
    if (pr >= p_lim || k >= k_lim) return vzero<T>();
    const int j = pr % c.T1c, r = pr / c.T1c, i = r % c.F1c, b = r / c.F1c;
    const int ti = k / g.C2, c2 = k % g.C2;
    const int f2 = (2 * i + c.pf - c.kh[ti]) >> 1, t2 = (2 * j + c.pt - c.kw[ti]) >> 1;
    if (f2 < 0 || t2 < 0 || f2 >= g.F2 || t2 >= g.T2) return vzero<T>();
    const T* p = dh2 + (((long)b * g.T2 + t2) * g.F2 + f2) * g.C2 + c2;
    return *reinterpret_cast<const typename VecOf<T>::type*>(p);
  }
};
// B (MN-major): B(n = c1, k = (tap, c2)) = w2r[c2][kh][kw][c1]
template <typename T> struct Conv2DgradB {
  const T* w2r; Conv2Geo g; Conv2Class c;
  __device__ __forceinline__ void batch(int) {}
  __device__ __forceinline__ typename VecOf<T>::type load(int k, int n, int k_lim, int n_lim) const {
    if (k >= k_lim || n >= n_lim) return vzero<T>();
    const int ti = k / g.C2, c2 = k % g.C2;
    const T* p = w2r + ((long)c2 * 9 + c.kh[ti] * 3 + c.kw[ti]) * g.C1 + n;
    return *reinterpret_cast<const typename VecOf<T>::type*>(p);
  }
};

// bf16 LDS geometry (elements)
constexpr int BK16 = 64;
constexpr int KM_STRIDE = BK16 + 8;        // K-major tile [128][72]: 144-B rows, conflict-free b128
constexpr int MN_STRIDE = 128 + 32;        // MN-major tile [64][160]: 320-B rows, conflict-free tr16
constexpr int TILE16 = (128 * KM_STRIDE > BK16 * MN_STRIDE) ? 128 * KM_STRIDE : BK16 * MN_STRIDE;  // 20 KiB
constexpr int KV16 = BK16 / 8;             // vectors per K-major row (8)

// XCD-aware tile order: blocks b and b+8 share an XCD under round-robin dispatch, so hand each
// XCD a contiguous run of (row-major) tiles: neighbouring tiles then share their A panel in that
// XCD's L2 (bijective for any tile count; speed only, never correctness).
__device__ __forceinline__ void xcd_tile(int& tm, int& tn) {
  const int gx = gridDim.x, nwg = gx * gridDim.y;
  const int L = blockIdx.y * gx + blockIdx.x;
  int id = L;
  if (nwg > 8) {
    const int xcd = L & 7, q = nwg >> 3, r = nwg & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
  }
  tm = id / gx;
  tn = id % gx;
}

// The same over the whole 3-D grid (z = batch x split-K slice, slowest): each XCD gets a contiguous
// run of (slice, tile) pairs, i.e. whole K slices -- the 4-8 tiles that re-read one slice's
// operand panels then do so from that XCD's L2 instead of every XCD fetching every panel.
__device__ __forceinline__ void xcd_tile3(int& tm, int& tn, int& zz) {
  const int gx = gridDim.x, gxy = gx * gridDim.y, nwg = gxy * gridDim.z;
  const int L = (blockIdx.z * gridDim.y + blockIdx.y) * gx + blockIdx.x;
  int id = L;
  if (nwg > 8) {
    const int xcd = L & 7, q = nwg >> 3, r = nwg & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
  }
  zz = id / gxy;
  const int t = id % gxy;
  tm = t / gx;
  tn = t % gx;
}

// fp32 LDS geometry: both operands stored [BK][128+4] (k-rows)
constexpr int BK32 = 16;

// Read one 32x32x16 operand fragment (8 bf16, natural k order) from a staged tile.
// MNS: row stride of the MN-major image (rows + 32 elements: 64 mod 256 bytes -> conflict-free tr16)
template <bool KMAJOR, int MNS = MN_STRIDE>
__device__ __forceinline__ bf16x8 frag16(const bf16* tile, int row0, int kk, int lane) {
  if constexpr (KMAJOR) {
    const bf16* p = tile + (row0 + (lane & 31)) * KM_STRIDE + kk + 8 * (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    const int h = lane >> 5, g1 = (lane >> 4) & 1, q = (lane & 15) >> 2, p4 = lane & 3;
    const bf16* base = tile + (kk + 8 * h + q) * MNS + row0 + 16 * g1 + 4 * p4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + 4 * MNS));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// zs: the launch's batch x split-K slice index (selects the split-K slab)
__device__ __forceinline__ void epilogue_store(const GemmP& p, int z, int zs, int m, int n, float acc) {
  if (m >= p.M || n >= p.N) return;
  const long cidx = (long)z * p.sc + out_row(p, m) * p.ldc + n;
  float v = acc * p.alpha;
  if (p.split_k > 1) {
    if (p.slab) {
      p.slab[(long)zs * p.M * p.N + (long)m * p.N + n] = v;
      return;
    }
    if (p.bias && zs % p.split_k == 0) v += p.bias[n];
    atomicAdd(reinterpret_cast<float*>(p.C) + cidx, v);
    return;
  }
  if (p.bias) v += p.bias[n];
  if (p.act_grad) v *= silu_grad_f(ld_dyn(p.pre, p.dtpre, cidx));
  if (p.act == CFM_ACT_SILU) {
    if (p.pre) st_dyn(p.pre, p.dtpre, cidx, v);
    v = silu_f(v);
  }
  if (p.drop_p > 0.f) v *= dropout_scale(p.drop_p, p.seed, p.doff + (uint64_t)((long)z * p.M * p.N + (long)m * p.N + n));
  v *= p.out_scale;
  if (p.res) v += ld_dyn(p.res, p.dtr, (long)z * p.sc + (long)m * p.ldr + n);
  st_dyn(p.C, p.dtc, cidx, v);
}

// split-K partial of one element: the whole epilogue a split-K launch may carry (cfm_gemm requires a plain fp32
// epilogue for split_k > 1): alpha, the bias on the first slice, atomic accumulation -- a small body, so the
// 64-element loops over an accumulator tile unroll fully (epilogue_store's general body did not)
__device__ __forceinline__ void splitk_atomic_store(const GemmP& p, int z, int zs, int m, int n, float acc) {
  if (m >= p.M || n >= p.N) return;
  float v = acc * p.alpha;
  if (p.bias && zs % p.split_k == 0) v += p.bias[n];
  atomicAdd(reinterpret_cast<float*>(p.C) + (long)z * p.sc + out_row(p, m) * p.ldc + n, v);
}

constexpr int EP_STRIDE = 128 + 4;   // f32 staging row stride: rows r and r+4 land 16 banks apart
static_assert(128 * EP_STRIDE * 4 <= 4 * TILE16 * 2, "epilogue staging fits in the K-loop LDS");

// the epilogue of cfm_gemm_desc on 8 consecutive columns (vectorised when legal)
__device__ __forceinline__ void epilogue_store8(const GemmP& p, int z, int zs, int m, int n, float (&v)[8]) {
  if (m >= p.M || n >= p.N) return;
  if (p.split_k > 1 && p.slab && n + 8 <= p.N && (p.N & 3) == 0) {
    float* dst = p.slab + (long)zs * p.M * p.N + (long)m * p.N + n;
    *reinterpret_cast<float4*>(dst) = make_float4(v[0] * p.alpha, v[1] * p.alpha, v[2] * p.alpha, v[3] * p.alpha);
    *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4] * p.alpha, v[5] * p.alpha, v[6] * p.alpha, v[7] * p.alpha);
    return;
  }
  if (!p.vec_c || n + 8 > p.N || p.split_k > 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (n + e < p.N) epilogue_store(p, z, zs, m, n + e, v[e]);
    return;
  }
  const long cidx = (long)z * p.sc + out_row(p, m) * p.ldc + n;
  if (p.alpha != 1.f) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= p.alpha;
  }
  if (p.bias) {
    const float4 a = *reinterpret_cast<const float4*>(p.bias + n);
    const float4 c = *reinterpret_cast<const float4*>(p.bias + n + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += c.x; v[5] += c.y; v[6] += c.z; v[7] += c.w;
  }
  if (p.act_grad) {
    float pr[8];
    ld8_dyn(p.pre, p.dtpre, cidx, pr);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= silu_grad_f(pr[e]);
  }
  if (p.act == CFM_ACT_SILU) {
    if (p.pre) st8_dyn(p.pre, p.dtpre, cidx, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = silu_f(v[e]);
  }
  if (p.drop_p > 0.f) {
    const uint64_t base = p.doff + (uint64_t)((long)z * p.M * p.N + (long)m * p.N + n);
    float ds[8];
    const uint64_t j0 = base >> 1;
    if ((j0 >> 32) == 0 && (uint32_t)j0 <= 0xFFFFFFFBu && !(p.dbg & 2)) {   // (always, below 2^33 elements)
      uint32_t h[5];
      const int odd = (int)(base & 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) h[q] = attn_mix((uint32_t)j0 + q + p.dkey0);
      h[4] = odd ? attn_mix((uint32_t)j0 + 4 + p.dkey0) : 0u;   // (an even base needs 4 pair hashes)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int q = (odd + e) >> 1;
        const uint32_t b = ((odd + e) & 1) ? (h[q] >> 16) : (h[q] & 0xFFFFu);
        ds[e] = b >= p.dthr ? p.dkeep : 0.f;
      }
    } else {
      dropout_scale8(p.drop_p, p.seed, base, ds);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= ds[e];
  }
  if (p.out_scale != 1.f) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= p.out_scale;
  }
  if (p.res) {
    float r[8];
    ld8_dyn(p.res, p.dtr, (long)z * p.sc + (long)m * p.ldr + n, r);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += r[e];
  }
  st8_dyn(p.C, p.dtc, cidx, v);
}

// ---------------------------------------------------------------- bf16 kernel
// BMt x 128 output tile, BMt*2 threads (BMt/64 x 2 waves of 64x64): BMt = 128 (80 KiB LDS, 2
// workgroups/CU) for narrow or split-K shapes, BMt = 256 (112 KiB, 1 workgroup/CU of 8 waves: 1.5x
// the FLOP per staged byte) for the wide token-major GEMMs.
template <int BMt>
struct Geo16 {
  static constexpr int NTt = BMt * 2;
  static constexpr int NVA = BMt * BK16 / 8 / NTt;      // A vectors per thread (4)
  static constexpr int NVB = BN * BK16 / 8 / NTt;       // B vectors per thread (4 or 2)
  static constexpr int MNSA = BMt + 32;                  // MN-major A row stride
  static constexpr int TILEA = (BMt * KM_STRIDE > BK16 * MNSA) ? BMt * KM_STRIDE : BK16 * MNSA;
  static constexpr int TILEB = TILE16;
  static constexpr int LDS = 2 * (TILEA + TILEB);        // elements
};

template <int BMt>
__device__ __forceinline__ void tile_epilogue(const GemmP& p, f32x16 (&acc)[2][2], float* st, int z, int zs, int m0,
                                              int n0, int wm, int wn, int lane, int tid);

template <int BMt, bool AK, bool BKM, class OA, class OB>
__global__ __launch_bounds__(BMt * 2) void gemm_bf16_kernel(GemmP p, OA oa, OB ob) {
  typedef Geo16<BMt> G;
  probe_begin(p.probe);
  gemm_drop_prep(p);
  constexpr int NTt = G::NTt, NVA = G::NVA, NVB = G::NVB, TILEA = G::TILEA;
  __shared__ __attribute__((aligned(16))) bf16 lds[G::LDS];   // [buf][A,B]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int tm, tn;
  xcd_tile(tm, tn);
  const int m0 = tm * BMt, n0 = tn * BN;
  const int z = blockIdx.z / p.split_k, ks = blockIdx.z % p.split_k;
  oa.batch(z);
  ob.batch(z);
  const int kbeg = ks * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + BK16 - 1) / BK16 : 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0};

  constexpr int AV = BMt / 8;     // MN-major A: vectors per k-row
  uint4 ra[NVA], rb[NVB];
  auto gload = [&](int kt) {
    const int k0 = kbeg + kt * BK16;
#pragma unroll
    for (int i = 0; i < NVA; ++i) {
      const int v = tid + NTt * i;
      if constexpr (AK) ra[i] = oa.load(m0 + v / KV16, k0 + (v % KV16) * 8, p.M, kend);
      else ra[i] = oa.load(k0 + v / AV, m0 + (v % AV) * 8, kend, p.M);
    }
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int v = tid + NTt * i;
      if constexpr (BKM) rb[i] = ob.load(n0 + v / KV16, k0 + (v % KV16) * 8, p.N, kend);
      else rb[i] = ob.load(k0 + (v >> 4), n0 + (v & 15) * 8, kend, p.N);
    }
  };
  auto sstore = [&](int buf) {
    bf16* ta = lds + buf * (TILEA + TILE16);
    bf16* tb = ta + TILEA;
#pragma unroll
    for (int i = 0; i < NVA; ++i) {
      const int v = tid + NTt * i;
      bf16* da = AK ? ta + (v / KV16) * KM_STRIDE + (v % KV16) * 8 : ta + (v / AV) * G::MNSA + (v % AV) * 8;
      *reinterpret_cast<uint4*>(da) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int v = tid + NTt * i;
      bf16* db = BKM ? tb + (v / KV16) * KM_STRIDE + (v % KV16) * 8 : tb + (v >> 4) * MN_STRIDE + (v & 15) * 8;
      *reinterpret_cast<uint4*>(db) = rb[i];
    }
  };

  if (nk > 0) {
    gload(0);
    sstore(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const bf16* ta = lds + cur * (TILEA + TILE16);
    const bf16* tb = ta + TILEA;
#pragma unroll
    for (int kk = 0; kk < BK16; kk += 16) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = frag16<AK, G::MNSA>(ta, wm * 64 + i * 32, kk, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = frag16<BKM>(tb, wn * 64 + j * 32, kk, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  tile_epilogue<BMt>(p, acc, reinterpret_cast<float*>(lds), z, blockIdx.z, m0, n0, wm, wn, lane, tid);
  probe_end(p.probe);
}

// Epilogue of one BMt x 128 tile (4-wave rows x 2-wave columns of 64x64 accumulators).  The
// caller guarantees every wave is done reading the staging LDS (`st`, >= 128 x EP_STRIDE floats).
template <int BMt>
__device__ __forceinline__ void tile_epilogue(const GemmP& p, f32x16 (&acc)[2][2], float* st, int z, int zs, int m0,
                                              int n0, int wm, int wn, int lane, int tid) {
  constexpr int NTt = BMt * 2;
  if (p.split_k > 1 && !p.slab) {
    // split-K partials: atomics straight from the accumulators (32 consecutive columns per
    // half-wave = two 128-B segments per instruction, the fast atomic shape)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int n = n0 + wn * 64 + j * 32 + (lane & 31);
          splitk_atomic_store(p, z, zs, m, n, acc[i][j][r]);
        }
    return;
  }
  // stage 128-row halves of the f32 tile in LDS, then every thread finishes 8 consecutive
  // columns of a row -> 16-B / 32-B vector stores.
#pragma unroll
  for (int hf = 0; hf < BMt / 128; ++hf) {
    if ((wm >> 1) == hf) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = (wm & 1) * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const int col = wn * 64 + j * 32 + (lane & 31);
            st[row * EP_STRIDE + col] = acc[i][j][r];
          }
    }
    __syncthreads();
#pragma unroll 2
    for (int it = 0; it < 128 * 16 / NTt; ++it) {
      const int row = it * (NTt / 16) + (tid >> 4), c8 = (tid & 15) * 8;
      const float4 lo = *reinterpret_cast<const float4*>(st + row * EP_STRIDE + c8);
      const float4 hi = *reinterpret_cast<const float4*>(st + row * EP_STRIDE + c8 + 4);
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      epilogue_store8(p, z, zs, m0 + 128 * hf + row, n0 + c8, v);
    }
    if (hf + 1 < BMt / 128) __syncthreads();
  }
}

// Epilogue of one tile held as WM x WN waves of FM x FN 32x32 accumulators (wave band = FM*32
// rows).  Rows are staged through LDS in chunks of CHB bands (<= 128 rows), then every thread
// finishes 8 consecutive columns of a row (16-B / 32-B vector stores).  The caller guarantees every
// wave is done reading the staging LDS (`st`, >= 128 x EP_STRIDE floats).
// (row, col) inside a 32x32 accumulator block of register r: the 32x32x16 MFMA layout, or (M16) four 16x16x32
// blocks packed as r = 4 (2a + b) + q -> block (a, b) of the 32x32, register q
template <bool M16> __device__ __forceinline__ int accr(int r, int lane) {
  return M16 ? 16 * ((r >> 3) & 1) + 4 * (lane >> 4) + (r & 3) : (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}
template <bool M16> __device__ __forceinline__ int accc(int r, int lane) {
  return M16 ? 16 * ((r >> 2) & 1) + (lane & 15) : (lane & 31);
}

// Staged-epilogue fast path (the encoder's launches; host-side selection in epi_fast_kind): split-K 1, vectorised
// C with N % 8 == 0, bf16 pre-activation, f32 residual, the 32-bit dropout hash range, and a feature set fixed
// at compile time per kind (EK, a kernel template parameter: each kernel carries one epilogue body -- the generic
// body's registers spilled in the 128-register two-per-CU kernels, one accumulator inside the MFMA loop):
//   EF_BF16      bf16 C, nothing else (the d-wide data gradients)
//   EF_BF16_BIAS bf16 C; bias (QKV, pointwise-conv-1 forward)
//   EF_BF16_SILU bf16 C; bias, SiLU + bf16 pre-activation store, dropout (FFN-up forward)
//   EF_BF16_ACTG bf16 C; silu'(pre) * dropout (FFN-down data gradient)
//   EF_BF16_RD   bf16 C; rowdot with rd_with (attention out-projection data gradient)
//   EF_F32       f32 C; alpha, bias, SiLU (+ pre), dropout, out_scale as run-time options
//   EF_F32_RES   f32 C; bias, dropout, out_scale, f32 residual (the d-wide residual-stream outputs)
//   EF_BF16_SILU_MX  EF_BF16_SILU + the MX e4m3 copy of the bf16 C (fp8 FFN-up forward: the FFN-down GEMM's
//                operand; the 4 threads of a 32-column block exchange maxima by two xor shuffles)
// Every option a kind does not list is absent by construction (epi_fast_kind checks): a run-time test on a
// uniform kernel argument is flattened by the compiler into per-lane selects with BOTH sides computed (the SiLU
// of the bias-only QKV rows, the alpha and out_scale products), so the encoder's kinds carry no such tests.
// A thread's 8-column chunk is the same on every row it finishes, so its bias is loaded once, and each row's global
// input (the bf16 pre-activation / rd_with, or the f32 residual) is issued ahead of the previous rows' stores:
// vmcnt counts loads and stores in one in-order queue, and the generic rows, which load bias / pre / residual
// between the previous row's stores, waited for every previous row's write acknowledgements (bias-only FFN-up
// epilogue without the main loop: 49 MB in 21.9 us = 2.2 TB/s).  Arithmetic and its order are epilogue_store8's
// (bit-identical outputs).
// residual-stream kinds: EF_F32_RES (fp32 residual in, fp32 out: the parity mode), EF_BF16_RES (bf16 in, bf16 out: the
// bf16 mode's bf16 residual stream), EF_F32R_BF16 (fp32 in, bf16 out: a layer's first residual add, whose input is the
// previous layer's fp32 LayerNorm output); EF_BF16_DELTA: a residual module's output without the residual (bias,
// dropout, out_scale, bf16) -- the add happens in the next LayerNorm (cfm_layernorm_fwd_res)
enum { EF_GENERIC = 0, EF_BF16 = 1, EF_BF16_BIAS = 2, EF_BF16_SILU = 3, EF_BF16_ACTG = 4, EF_BF16_RD = 5, EF_F32 = 6,
       EF_F32_RES = 7, EF_BF16_SILU_MX = 8, EF_BF16_RES = 9, EF_F32R_BF16 = 10, EF_BF16_DELTA = 11 };

// e8m0 block exponent of an MX block (fp8.hip mx_k): the largest k with amax * 2^k <= 448
__device__ __forceinline__ int epi_mx_k(float a) {
  if (!(a > 0.f) || !(a < INFINITY)) return 0;
  int e;
  const float m = 2.f * frexpf(a, &e);
  const int k = (m <= 1.75f ? 8 : 7) - (e - 1);
  return k < 126 ? (k > -126 ? k : -126) : 126;
}

__device__ __forceinline__ void epi_bias8(const GemmP& p, int n, float (&b)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = 0.f;
  if (p.efast && p.bias && n < p.N) {
    const float4 a = *reinterpret_cast<const float4*>(p.bias + n);
    const float4 c = *reinterpret_cast<const float4*>(p.bias + n + 4);
    b[0] = a.x; b[1] = a.y; b[2] = a.z; b[3] = a.w; b[4] = c.x; b[5] = c.y; b[6] = c.z; b[7] = c.w;
  }
}

// dropout of 8 consecutive elements starting at an index of parity ODD whose pair index is j0 (epilogue_store8's
// hash path: element i draws the (i & 1) half of attn_mix(i / 2 + key))
template <bool ODD>
__device__ __forceinline__ void drop8_fast(float (&v)[8], uint32_t j0, const GemmP& p) {
  constexpr int NH = ODD ? 5 : 4;
  uint32_t h[NH];
#pragma unroll
  for (int q = 0; q < NH; ++q) h[q] = attn_mix(j0 + q + p.dkey0);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int q = (ODD + e) >> 1;
    const uint32_t bits = ((ODD + e) & 1) ? (h[q] >> 16) : (h[q] & 0xFFFFu);
    v[e] *= bits >= p.dthr ? p.dkeep : 0.f;
  }
}

// per-row global inputs of a fast epilogue kind: dwords per row, and the holder (IT rows of one thread)
template <int EK> constexpr int epi_nw() {
  return (EK == EF_F32_RES || EK == EF_F32R_BF16) ? 8 : (EK == EF_BF16_ACTG || EK == EF_BF16_RD || EK == EF_BF16_RES) ? 4
                                                                                                                     : 0;
}
template <int EK, int IT> struct EpiIn { uint4 v[IT][epi_nw<EK>() == 8 ? 2 : 1]; };

template <int EK, int IT, int NTt, int CPW>
__device__ __forceinline__ void epi_load_row(const GemmP& p, int z, int mbase, int n0, int tid, int it,
                                             EpiIn<EK, IT>& in) {
  const int n = n0 + (tid % CPW) * 8, m = mbase + it * (NTt / CPW) + tid / CPW;
  if (m < p.M && n < p.N) {
    if constexpr (EK == EF_F32_RES || EK == EF_F32R_BF16) {
      const uint4* s = reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(p.res) + (long)z * p.sc +
                                                      (long)m * p.ldr + n);
      in.v[it][0] = s[0];
      in.v[it][1] = s[1];
    } else if constexpr (EK == EF_BF16_RES) {
      in.v[it][0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p.res) + (long)z * p.sc +
                                                    (long)m * p.ldr + n);
    } else if constexpr (EK == EF_BF16_ACTG) {
      in.v[it][0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p.pre) + (long)z * p.sc +
                                                    (long)m * p.ldc + n);
    } else if constexpr (EK == EF_BF16_RD) {
      in.v[it][0] = *reinterpret_cast<const uint4*>(p.rd_with + (long)m * p.ldc + n);
    }
  }
}

// every row's input, issued up front (the warp-specialised kernel: before its main loop, which hides the latency)
template <int EK, int IT, int NTt, int CPW>
__device__ __forceinline__ void epi_load_all(const GemmP& p, int z, int mbase, int n0, int tid, EpiIn<EK, IT>& in) {
  if constexpr (epi_nw<EK>() > 0) {
#pragma unroll
    for (int it = 0; it < IT; ++it) epi_load_row<EK, IT, NTt, CPW>(p, z, mbase, n0, tid, it, in);
  }
}

// PRE: `in` already holds every row's input (epi_load_all); otherwise row it's input is issued PD rows ahead,
// before the stores of row it - PD (two rows ahead: the 128-register two-per-CU kernels)
template <int EK, int IT, int NTt, int CPW, int EPS, bool PRE = false>
__device__ __forceinline__ void epi_rows_fast(const GemmP& p, const float* st, int z, int mbase, int n0, int tid,
                                              const float (&b)[8], EpiIn<EK, IT>& in) {
  static_assert(EK > EF_GENERIC && EK <= EF_BF16_DELTA, "fast epilogue kind");
  constexpr bool CF32 = EK == EF_F32 || EK == EF_F32_RES, ACTG = EK == EF_BF16_ACTG, RD = EK == EF_BF16_RD;
  constexpr bool RESB = EK == EF_BF16_RES;                      // bf16 residual operand
  constexpr bool RES = EK == EF_F32_RES || RESB || EK == EF_F32R_BF16, GEN = EK == EF_F32;   // GEN: EF_F32's options
  constexpr bool MXO = EK == EF_BF16_SILU_MX, DLT = EK == EF_BF16_DELTA;
  constexpr bool SILU = EK == EF_BF16_SILU || MXO, BIAS = EK == EF_BF16_BIAS || SILU || RES || DLT;
  constexpr bool DROP = SILU || ACTG || RES || GEN || DLT;
  constexpr int NW = epi_nw<EK>();
  constexpr int RPI = NTt / CPW;                       // rows per pass
  const int c8 = (tid % CPW) * 8, n = n0 + c8, r0 = tid / CPW;
  const bool nok = n < p.N;
  constexpr int PD = PRE ? IT : (IT < 2 ? IT : 2);
  if constexpr (NW > 0 && !PRE) {
#pragma unroll
    for (int it = 0; it < PD; ++it) epi_load_row<EK, IT, NTt, CPW>(p, z, mbase, n0, tid, it, in);
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    if constexpr (NW > 0 && !PRE) {
      if (it + PD < IT) epi_load_row<EK, IT, NTt, CPW>(p, z, mbase, n0, tid, it + PD, in);
    }
    const int row = it * RPI + r0, m = mbase + row;
    const float4 lo = *reinterpret_cast<const float4*>(st + row * EPS + c8);
    const float4 hi = *reinterpret_cast<const float4*>(st + row * EPS + c8 + 4);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const bool ok = m < p.M && nok;
    if (ok) {
      const long cidx = (long)z * p.sc + (long)m * p.ldc + n;   // (no row remap: epi_fast_kind)
      if constexpr (GEN) {
        if (p.alpha != 1.f) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= p.alpha;
        }
        if (p.bias) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += b[e];
        }
      }
      if constexpr (BIAS) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += b[e];
      }
      if constexpr (ACTG) {
        const bf16x8 pr = __builtin_bit_cast(bf16x8, in.v[it][0]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= silu_grad_f((float)pr[e]);
      }
      if constexpr (SILU || GEN) {
        if (SILU || p.act == CFM_ACT_SILU) {
          if (SILU || p.pre) {
            bf16x8 q;
#pragma unroll
            for (int e = 0; e < 8; ++e) q[e] = (bf16)v[e];
            *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.pre) + cidx) = __builtin_bit_cast(uint4, q);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = silu_f(v[e]);
        }
      }
      if constexpr (DROP) {
        if (p.drop_p > 0.f) {
          // n and N are multiples of 8: the element index's parity is the offset's (uniform), so the hash-half
          // selection is static in each branch (a per-lane parity cost ~48 selects per row)
          const uint32_t j0 = (uint32_t)((p.doff + (uint64_t)(((long)z * p.M + m) * p.N + n)) >> 1);
          if (p.doff & 1) drop8_fast<true>(v, j0, p);
          else drop8_fast<false>(v, j0, p);
        }
      }
      if constexpr (RES || DLT) {   // (unconditional: x * 1.0f == x, and no per-lane select for the 1.0 launches)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= p.out_scale;
      } else if constexpr (GEN) {
        if (p.out_scale != 1.f) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= p.out_scale;
        }
      }
      if constexpr (RESB) {
        const bf16x8 r = __builtin_bit_cast(bf16x8, in.v[it][0]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)r[e];
      } else if constexpr (RES) {
        const float4 ra = __builtin_bit_cast(float4, in.v[it][0]), rb = __builtin_bit_cast(float4, in.v[it][1]);
        v[0] += ra.x; v[1] += ra.y; v[2] += ra.z; v[3] += ra.w; v[4] += rb.x; v[5] += rb.y; v[6] += rb.z; v[7] += rb.w;
      }
      if constexpr (CF32) {
        float* d = reinterpret_cast<float*>(p.C) + cidx;
        *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        bf16x8 q;
#pragma unroll
        for (int e = 0; e < 8; ++e) q[e] = (bf16)v[e];
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.C) + cidx) = __builtin_bit_cast(uint4, q);
        if constexpr (MXO) {   // (N % 32 == 0: a block's 4 threads share the row, so all four are here)
          float mx = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) mx = fmaxf(mx, fabsf((float)q[e]));
          mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
          mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
          const int k = epi_mx_k(mx);
          const float sc = ldexpf(1.f, k);
          int lo = 0, hi = 0;
          lo = __builtin_amdgcn_cvt_pk_fp8_f32((float)q[0] * sc, (float)q[1] * sc, lo, false);
          lo = __builtin_amdgcn_cvt_pk_fp8_f32((float)q[2] * sc, (float)q[3] * sc, lo, true);
          hi = __builtin_amdgcn_cvt_pk_fp8_f32((float)q[4] * sc, (float)q[5] * sc, hi, false);
          hi = __builtin_amdgcn_cvt_pk_fp8_f32((float)q[6] * sc, (float)q[7] * sc, hi, true);
          *reinterpret_cast<uint2*>(p.mxo8 + (long)m * p.N + n) = make_uint2((unsigned)lo, (unsigned)hi);
          if ((tid & 3) == 0) p.mxos[(long)m * (p.N / 32) + n / 32] = (uint8_t)(127 - k);
        }
      }
    }
    if constexpr (RD) {   // 8-lane group = 64 columns (as tile_epilogue_g's generic rows)
      float t = 0.f;
      if (ok) {
        const bf16x8 w = __builtin_bit_cast(bf16x8, in.v[it][0]);
#pragma unroll
        for (int e = 0; e < 8; ++e) t += (float)(bf16)v[e] * (float)w[e];
      }
      t += __shfl_xor(t, 1, 64);
      t += __shfl_xor(t, 2, 64);
      t += __shfl_xor(t, 4, 64);
      if ((tid & 7) == 0 && ok) {
        const int bb = m / p.rd_T, tt = m - bb * p.rd_T, g = n >> 6;
        p.rd_out[((long)bb * (p.N >> 6) + g) * p.rd_T + tt] = t;
      }
    }
  }
}

template <int FM, int FN, int WM, int WN, int NTt, int BNt = BN, bool M16 = false, int ROWS = 128, int EK = EF_GENERIC>
__device__ __forceinline__ void tile_epilogue_g(const GemmP& p, f32x16 (&acc)[FM][FN], float* st, int z, int zs,
                                                int m0, int n0, int wm, int wn, int lane, int tid) {
  // ROWS: the staging rows `st` holds (ROWS x (BNt + 4) floats)
  constexpr int BAND = FM * 32, CHB = (ROWS / BAND) >= 1 && WM % (ROWS / BAND) == 0 ? ROWS / BAND : 1;
  static_assert(BAND <= ROWS, "one wave band fits the staging");
  constexpr int RC = CHB * BAND;
  constexpr int EPS = BNt + 4;         // staging row stride (floats): = 4 mod 32 for both widths
  constexpr int CPW = BNt / 8;         // 8-column chunks per row
  static_assert(WN * FN * 32 == BNt, "tile width");
  if (EK == EF_GENERIC && p.split_k > 1 && !p.slab) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * BAND + i * 32 + accr<M16>(r, lane);
          const int n = n0 + wn * FN * 32 + j * 32 + accc<M16>(r, lane);
          splitk_atomic_store(p, z, zs, m, n, acc[i][j][r]);
        }
    return;
  }
  float bias8[8];
  if constexpr (EK != EF_GENERIC) epi_bias8(p, n0 + (tid % CPW) * 8, bias8);
  // (one pass per band chunk; not unrolled -- the epilogue body is large and nothing in it is indexed by hf)
#pragma nounroll
  for (int hf = 0; hf < WM / CHB; ++hf) {
    // fast kinds with a per-row global input (pre-activation, residual, rowdot operand): every row of this pass is
    // issued here, before the accumulators are staged -- the loads' latency hides under the staging and its barrier
    // (issued two rows ahead of the stores instead, the FFN-down data gradient's pre-activation reads exposed ~4
    // round trips per pass)
    EpiIn<EK == EF_GENERIC ? EF_BF16 : EK, RC * CPW / NTt> ein;
    if constexpr (EK != EF_GENERIC) epi_load_all<EK, RC * CPW / NTt, NTt, CPW>(p, z, m0 + RC * hf, n0, tid, ein);
    if (wm / CHB == hf) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = (wm % CHB) * BAND + i * 32 + accr<M16>(r, lane);
            const int col = wn * FN * 32 + j * 32 + accc<M16>(r, lane);
            st[row * EPS + col] = acc[i][j][r];
          }
    }
    __syncthreads();
    static_assert((RC * CPW) % NTt == 0 && NTt % CPW == 0, "whole rows per pass");
    if constexpr (EK != EF_GENERIC) {
      epi_rows_fast<EK, RC * CPW / NTt, NTt, CPW, EPS, true>(p, st, z, m0 + RC * hf, n0, tid, bias8, ein);
      if (hf + 1 < WM / CHB) __syncthreads();
      continue;
    }
#pragma unroll 2
    for (int it = 0; it < RC * CPW / NTt; ++it) {
      const int row = it * (NTt / CPW) + tid / CPW, c8 = (tid % CPW) * 8;
      const float4 lo = *reinterpret_cast<const float4*>(st + row * EPS + c8);
      const float4 hi = *reinterpret_cast<const float4*>(st + row * EPS + c8 + 4);
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      const int m = m0 + RC * hf + row;
      epilogue_store8(p, z, zs, m, n0 + c8, v);
      if (p.rd_out) {   // (vectorised bf16 epilogue: v now holds the stored values) 8-lane group = 64 columns
        float t = 0.f;
        if (m < p.M && n0 + c8 < p.N) {
          const uint4 u = *reinterpret_cast<const uint4*>(p.rd_with + (long)m * p.ldc + n0 + c8);
          const bf16x8 w = __builtin_bit_cast(bf16x8, u);
#pragma unroll
          for (int e = 0; e < 8; ++e) t += (float)(bf16)v[e] * (float)w[e];
        }
        t += __shfl_xor(t, 1, 64);
        t += __shfl_xor(t, 2, 64);
        t += __shfl_xor(t, 4, 64);
        if ((tid & 7) == 0 && m < p.M && n0 + c8 < p.N) {
          const int b = m / p.rd_T, tt = m - b * p.rd_T, g = (n0 + c8) >> 6;
          p.rd_out[((long)b * (p.N >> 6) + g) * p.rd_T + tt] = t;
        }
      }
    }
    if (hf + 1 < WM / CHB) __syncthreads();
  }
}

// ---------------------------------------------------------------- bf16 pipelined kernel
// The fast path for plain strided bf16 operands.  Staging is LDS-DMA (buffer_load_dwordx4 ... lds:
// no VGPR round trip, no per-element predicates) into a PS-deep ring of LDS stages: two K tiles
// are in flight while the waves compute on a third, with one raw s_barrier and a counted
// vmcnt per K tile (a __syncthreads would drain the DMA queue every step).
//
// LDS-DMA writes a wave's 64 x 16 B contiguously, so bank-conflict-free images come from
// permuting the *source* chunks:
//   K-major [R][64] image (128-B rows, read by ds_read_b128 along k):
//       chunk c of row r lives at slot c ^ ((r >> 1) & 7)
//   MN-major [64][R] image (R*2-B k-rows, read by ds_read_b64_tr_b16):
//       chunk c of k-row k lives at slot c ^ (4 * (k & 3))
// Rows past M/N are clamped to the last valid row (their outputs are never stored); k-rows past K
// of an MN-major operand read as zero through the buffer resource's range check.
struct PipeOp {
  const bf16* base;
  long ld, bstride;
  int lim;          // valid rows (K-major) / columns (MN-major) of the M or N dimension
  unsigned bytes;   // extent of one batch for the range check
};

// Gathered K-major A operand (implicit-GEMM convolutions): GEMM row m decomposes as
// j = m % Jn, i = (m / Jn) % In, b = m / (Jn * In); its source row (of Cr channels) for tap ti is
// b * sB + i * sI + j * sJ + dR[ti], valid iff 0 <= i - di[ti] < Ilim and 0 <= j - dj[ti] < Jlim
// (invalid rows read zero through an out-of-range buffer offset).  k = (ti, c) with Ck channels per
// tap, so each BKt-deep K tile lies inside one tap (Ck % BKt == 0).
//   conv2 forward:        rows (b, t2, f2) of h1 taps: i = t2, j = f2, row = (b F1 + 2 f2 + kh) T1 + 2 t2 + kw
//   conv2 data-gradient:  rows (b, i, j) of a parity class, source dh2 (b, t2 = j - dj, f2 = i - di)
struct GatherA {
  int Jn, In;
  long sB;
  int sI, sJ, Cr, Ck, Ilim, Jlim;
  int di[9], dj[9], dR[9];
  const void* group_tab;   // grouped launch (GROUP kernels): device WgTask table, one task per GEMM
  int group_n;
  const unsigned* group_sched;   // planned grouped launch: one word per workgroup (cfm_wgrad_group_plan) or nullptr
};

// BMt x 128 tile, BKt-deep K steps, NST-stage ring, NWV waves; the f32 epilogue staging aliases the ring
template <int BMt, int BKt, int NST, int NWV, int BNt = BN>
struct PipeGeo {
  static constexpr int NTt = NWV * 64, NW = NWV;
  static constexpr int ABYTES = BMt * BKt * 2, BBYTES = BNt * BKt * 2;
  static constexpr int STAGE = ABYTES + BBYTES;
  static constexpr int RING = NST * STAGE, EPI = (BMt < 128 ? BMt : 128) * (BNt + 4) * 4;
  static constexpr int LDS = RING > EPI ? RING : EPI;
  // 1-KiB DMA pieces per stage, spread over the waves: wave w issues pieces w, w + NW, ... (AI / BI rounds;
  // when a count is not a multiple of NW the first waves issue one more piece, and their counted waits say so)
  static constexpr int AP = ABYTES / 1024, BP = BBYTES / 1024;
  static constexpr int AI = (AP + NW - 1) / NW, BI = (BP + NW - 1) / NW;
  static_assert(AP * 1024 == ABYTES && BP * 1024 == BBYTES, "whole wave-instructions per stage");
  static constexpr bool EVEN = AI * NW == AP && BI * NW == BP;
};

// s_waitcnt vmcnt(n) for a wave-uniform run-time n (switch over the immediates a ring can need)
__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {
#define W(k) case k: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(k) : "memory"); break;
    W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14) W(15) W(16)
    W(17) W(18) W(19) W(20) W(21) W(22) W(23) W(24)
#undef W
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// the descriptor is wave-uniform by construction; readfirstlane makes that visible to the compiler even
// when the operand comes from memory (grouped launches), so no waterfall loop wraps the buffer loads
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pipe_rsrc(const PipeOp& o, int z) {
  const uint64_t a = (uint64_t)(uintptr_t)(o.base + (long)z * o.bstride);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane((int)o.bytes), 0x00020000);
}

// buffer resource over `bytes` bytes at p (MX block-scale rows; reads past the range return zero)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mx_rsrc(const uint8_t* p, long bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane((int)(bytes > 0 ? bytes : 0)), 0x00020000);
}

// one wave-instruction of LDS-DMA: lane l's 16 B from rsrc + voff land at lds_base + 16 l.
// Issued through inline asm: the compiler then does not know that it writes LDS, and does not put a
// conservative `s_waitcnt vmcnt(0)` in front of the next LDS read it cannot prove disjoint (it did so in the
// grouped weight-gradient loop, where every K step then waited for the DMA it had just issued).  Every
// consumer waits with its own counted vmcnt + barrier, so no compiler-inserted wait is needed.
// (m0 is declared clobbered -- the asm does overwrite it -- which clang reports as a reserved register once per
// instantiation; the warning is silenced here only)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_base, unsigned voff) {
  const unsigned l = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds_base);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(l), "v"(voff), "s"(r) : "memory", "m0");
}
#pragma clang diagnostic pop

// K-major [R][BKt] image: BKt*2-B rows, RPB rows per 256-B bank row, CPR 16-B chunks per row;
// chunk c of row r sits in slot c ^ ((r / RPB) % CPR): 16 consecutive rows read at one k hit 16
// distinct 16-B bank groups (conflict-free ds_read_b128)
template <int BKt>
struct KmSw {
  static constexpr int RB = BKt * 2, CPR = BKt / 8, RPB = 256 / RB;
  __device__ static __forceinline__ int slot(int r, int c) { return c ^ ((r / RPB) & (CPR - 1)); }
};

// byte offset (in the operand) of the 16-B chunk that lands in LDS slot `lc` of an R-row image
template <bool KM, int R, int BKt>
__device__ __forceinline__ unsigned pipe_src(const PipeOp& o, int lc, int row0, int k0) {
  if constexpr (KM) {
    typedef KmSw<BKt> S;
    const int r = lc / S::CPR, c = S::slot(r, lc % S::CPR);
    const int row = row0 + r < o.lim ? row0 + r : o.lim - 1;
    return (unsigned)(((long)row * o.ld + k0 + 8 * c) * 2);
  } else {
    constexpr int CPR = R / 8;
    const int k = lc / CPR, c = (lc % CPR) ^ (4 * (k & 3));
    const int col = row0 + 8 * c < o.lim - 8 ? row0 + 8 * c : o.lim - 8;
    return (unsigned)(((long)(k0 + k) * o.ld + col) * 2);
  }
}

// k offset (elements, within the BKt-deep tile) of the 16-B chunk that lands in K-major LDS slot `lc`
template <int BKt>
__device__ __forceinline__ int pipe_kchunk(int lc) {
  typedef KmSw<BKt> S;
  const int r = lc / S::CPR;
  return 8 * S::slot(r, lc % S::CPR);
}

// one 32x32x16 operand fragment from a swizzled stage image
template <bool KM, int R, int BKt>
__device__ __forceinline__ bf16x8 pipe_frag(const char* img, int row0, int kk, int lane) {
  if constexpr (KM) {
    typedef KmSw<BKt> S;
    const int r = row0 + (lane & 31), c = (kk >> 3) + (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(img + r * S::RB + 16 * S::slot(r, c));
  } else {
    const int h = lane >> 5, g1 = (lane >> 4) & 1, q = (lane & 15) >> 2, p4 = lane & 3;
    const int col = row0 + 16 * g1 + 4 * p4, k = kk + 8 * h + q;   // k & 3 == q for both halves
    const int off = 16 * ((col >> 3) ^ (4 * q)) + (col & 7) * 2;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + k * (R * 2) + off));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + (k + 4) * (R * 2) + off));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// one 16x16x32 operand fragment (rows row0 .. row0+15, k = kk + 8 (lane >> 4) .. +7) from a K-major swizzled
// stage image: conflict-free ds_read_b128 on the 64-deep images (kk a multiple of 16)
template <int BKt>
__device__ __forceinline__ bf16x8 pipe_frag16k(const char* img, int row0, int kk, int lane) {
  typedef KmSw<BKt> S;
  const int r = row0 + (lane & 15), c = (kk >> 3) + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(img + r * S::RB + 16 * S::slot(r, c));
}

// wait until at most `younger` stages (of PER DMA instructions each) are still in flight
template <int PER>
__device__ __forceinline__ void wait_stages(int younger) {
  if (younger >= 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PER) : "memory");
  else if (younger == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER) : "memory");
  else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
  else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// NWV waves as WM x WN, each owning FM x FN 32x32 accumulators: (BMt, NWV, WN) = (256, 8, 2) ->
// 64x64 per wave; (192, 8, 4) -> 96x32 per wave (192-row tiles: 63 x N/128 tiles of the encoder's
// M = 11,936 fill the 256 CUs in whole rounds); (128, 4, 2) -> 64x64.
struct WgTask;   // grouped weight-gradient task (below)
__device__ __forceinline__ bool group_task(const GatherA& ga, GemmP& p, PipeOp& oa, PipeOp& ob, int& tm, int& tn,
                                           int& zz);

// F8: A and B are fp8 e4m3 (OCP), K-major, viewed as bf16 PAIRS by everything up to the LDS image (K, ld and
// the tile geometry in 2-byte units, so DMA, swizzle and ring are byte-identical to the bf16 kernel); each
// 64-fp8 k-step (4 16-B chunks of a row) feeds one v_mfma_scale_f32_32x32x64_f8f6f4: lane (r, h) holds chunks h
// and h + 2 (the instruction's k order, see frag8).  Per-tensor fp8: unit block scales, the dequantisation
// (alpha_a * alpha_b) applied in the epilogue; MX: the e8m0 block scales below.
// M16: the main loop on v_mfma_f32_16x16x32_bf16 (each 32x32 block of a wave's tile as four 16x16 blocks; same
// LDS images, fragments per k and accumulator registers) -- K-major plain operands only.  On random data the
// chip holds a higher clock under the 16x16 shape than under 32x32x16 (MI355X_MICROARCH.md, DVFS item 7).
// MXK > 0 (F8 only): MX operands -- the tile's e8m0 block-scale rows (A rows m0.., B rows n0..: contiguous runs of
// mxk bytes each, mxk <= MXK) are DMA'd into LDS once, before the ring's first stage (so every stage wait covers
// them), and each fragment row's scales of a stage are read as one dword (BKt 64: 4 blocks) / short (BKt 32: 2);
// lane (r, h) of a 64-fp8 k-step q covers block 2q + h of the stage, shifted into the scale register's low byte.
template <int BMt, int BKt, int NST, int OCC, bool AK, bool BKM, int NWV = BMt / 32, int WN = 2, bool GA = false,
          bool GROUP = false, bool F8 = false, int BNt = BN, bool M16 = false, int EK = EF_GENERIC, int MXK = 0>
__global__ __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(OCC * NWV / 4)))
void gemm_pipe_kernel(GemmP p, PipeOp oa, PipeOp ob, GatherA ga) {
  static_assert(!F8 || (AK && BKM && !GA && !GROUP && BKt % 32 == 0), "fp8: K-major plain operands");
  static_assert(MXK == 0 || (F8 && (BKt == 64 || BKt == 32) && ((BMt + BNt) * MXK) % 1024 == 0), "MX: fp8 only");
  static_assert(!M16 || (AK && BKM && !GA && !GROUP && !F8 && BKt % 32 == 0), "16x16x32: K-major plain bf16");
  typedef PipeGeo<BMt, BKt, NST, NWV, BNt> G;
  constexpr int WM = NWV / WN, FM = BMt / WM / 32, FN = BNt / WN / 32;
  static_assert(WM * FM * 32 == BMt && WN * FN * 32 == BNt, "wave tiling");
  static_assert(G::EVEN || (!GA && !GROUP), "uneven DMA split: plain operands only");
  probe_begin(p.probe);
  // (the dropout constants are prepared right before the epilogue: gemm_drop_prep loads the bound step counter,
  // and waiting for that load at the top held back the first DMA stage by one memory round trip)
  static_assert(NST >= 3 && NST <= 6, "ring depth");
  __shared__ __attribute__((aligned(1024))) char lds[G::LDS + (BMt + BNt) * MXK];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  int tm, tn, zz;
  if constexpr (GROUP) {
    unsigned long long* const probe = p.probe;   // the launch's timing slot survives the task's parameters
    // this workgroup's GEMM, tile and K slice of a grouped launch (a planned launch's padding workgroups exit)
    if (!group_task(ga, p, oa, ob, tm, tn, zz)) return;
    p.probe = probe;
    gemm_drop_prep(p);
  } else {
    xcd_tile3(tm, tn, zz);
  }
  const int m0 = tm * BMt, n0 = tn * BNt;
  const int z = zz / p.split_k, ks = zz % p.split_k;
  const __amdgpu_buffer_rsrc_t ra = pipe_rsrc(oa, z), rb = pipe_rsrc(ob, z);
  const int kbeg = __builtin_amdgcn_readfirstlane(ks * p.k_per_split);
  const int kend = __builtin_amdgcn_readfirstlane(min(p.K, kbeg + p.k_per_split));
  const int nk = kend > kbeg && !(p.dbg & 4) ? (kend - kbeg + BKt - 1) / BKt : 0;   // (dbg 4: epilogue only)

  // per-lane source offsets of stage 0; later stages add k0 * (row stride) (MN-major) or k0 * 2
  unsigned offa[G::AI], offb[G::BI];
  int gi[GA ? G::AI : 1], gj[GA ? G::AI : 1];   // gathered rows: class coordinates (i, j); gi < 0: past M
  if constexpr (GA) {
    static_assert(AK, "gathered A is K-major");
    typedef KmSw<BKt> S;
#pragma unroll
    for (int i = 0; i < G::AI; ++i) {
      const int lc = (i * G::NW + wid) * 64 + lane;
      const int r = lc / S::CPR, c = S::slot(r, lc % S::CPR), m = m0 + r;
      if (m < p.M) {
        const int j = m % ga.Jn, q = m / ga.Jn, ii = q % ga.In, b = q / ga.In;
        gi[i] = ii; gj[i] = j;
        offa[i] = (unsigned)((((long)b * ga.sB + (long)ii * ga.sI + (long)j * ga.sJ) * ga.Cr + 8 * c) * 2);
      } else {
        gi[i] = -1000; gj[i] = -1000; offa[i] = 0;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < G::AI; ++i)
      offa[i] = pipe_src<AK, BMt, BKt>(oa, ((i * G::NW + wid) % G::AP) * 64 + lane, m0, kbeg);
  }
#pragma unroll
  for (int i = 0; i < G::BI; ++i)
    offb[i] = pipe_src<BKM, BNt, BKt>(ob, ((i * G::NW + wid) % G::BP) * 64 + lane, n0, kbeg);
  // K tail (K-major operands, K % BKt != 0, K % 8 == 0): the last stage's chunks at k >= kend read zero through an
  // out-of-range offset (a K-major row's tail would otherwise read the next row's head); MN-major operands already
  // read zero past K (their extent ends at row K - 1).  kca / kcb: the k offset of each piece's chunk in its tile
  const bool ktail = ((kend - kbeg) % BKt) != 0;
  int kca[G::AI], kcb[G::BI];
#pragma unroll
  for (int i = 0; i < G::AI; ++i) kca[i] = AK ? pipe_kchunk<BKt>(((i * G::NW + wid) % G::AP) * 64 + lane) : 0;
#pragma unroll
  for (int i = 0; i < G::BI; ++i) kcb[i] = BKM ? pipe_kchunk<BKt>(((i * G::NW + wid) % G::BP) * 64 + lane) : 0;
  // this wave's DMA pieces per stage (all waves alike unless the piece counts do not divide evenly)
  const int per_w = G::EVEN ? G::AI + G::BI
                            : (G::AP / G::NW + (wid < G::AP % G::NW)) + (G::BP / G::NW + (wid < G::BP % G::NW));
  const unsigned stepa = AK ? BKt * 2 : (unsigned)(BKt * oa.ld * 2);
  const unsigned stepb = BKM ? BKt * 2 : (unsigned)(BKt * ob.ld * 2);
  char* const sca = lds + G::LDS;        // MX: the tile's A / B block-scale rows
  char* const scb = sca + BMt * MXK;
  if constexpr (MXK > 0) {
    const int mk = p.mxk;
    const __amdgpu_buffer_rsrc_t rsa = mx_rsrc(p.mxa + (long)m0 * mk, (long)(p.M - m0) * mk);
    const __amdgpu_buffer_rsrc_t rsb = mx_rsrc(p.mxb + (long)n0 * mk, (long)(p.N - n0) * mk);
    const int pa = (BMt * mk + 1023) / 1024, pb = (BNt * mk + 1023) / 1024;
    for (int q = wid; q < pa + pb; q += NWV) {   // (rows past M / N read zero through the range check)
      if (q < pa) dma16(rsa, sca + 1024 * q, (unsigned)(1024 * q + 16 * lane));
      else dma16(rsb, scb + 1024 * (q - pa), (unsigned)(1024 * (q - pa) + 16 * lane));
    }
  }

  auto issue = [&](int kt) {
    char* sa = lds + (kt % NST) * G::STAGE;
    char* sb = sa + G::ABYTES;
    if constexpr (GA) {
      const int k0 = kbeg + kt * BKt, ti = k0 / ga.Ck, c0 = k0 - ti * ga.Ck;
      const int di = ga.di[ti], dj = ga.dj[ti];
      const unsigned shift = (unsigned)((ga.dR[ti] * ga.Cr + c0) * 2);   // mod 2^32: negative row shifts wrap
#pragma unroll
      for (int i = 0; i < G::AI; ++i) {
        const int ii = gi[i] - di, jj = gj[i] - dj;
        const bool ok = ii >= 0 && jj >= 0 && ii < ga.Ilim && jj < ga.Jlim;
        dma16(ra, sa + (i * G::NW + wid) * 1024, ok ? offa[i] + shift : 0xFFFFFF00u);
      }
    } else if (ktail && kt == nk - 1) {   // wave-uniform: the last, partial K tile
      const int lim = kend - kbeg - kt * BKt;
#pragma unroll
      for (int i = 0; i < G::AI; ++i)
        if (G::EVEN || i * G::NW + wid < G::AP)
          dma16(ra, sa + (i * G::NW + wid) * 1024, !AK || kca[i] < lim ? offa[i] + kt * stepa : 0xFFFFFF00u);
#pragma unroll
      for (int i = 0; i < G::BI; ++i)
        if (G::EVEN || i * G::NW + wid < G::BP)
          dma16(rb, sb + (i * G::NW + wid) * 1024, !BKM || kcb[i] < lim ? offb[i] + kt * stepb : 0xFFFFFF00u);
      return;
    } else {
#pragma unroll
      for (int i = 0; i < G::AI; ++i)
        if (G::EVEN || i * G::NW + wid < G::AP) dma16(ra, sa + (i * G::NW + wid) * 1024, offa[i] + kt * stepa);
    }
#pragma unroll
    for (int i = 0; i < G::BI; ++i)
      if (G::EVEN || i * G::NW + wid < G::BP) dma16(rb, sb + (i * G::NW + wid) * 1024, offb[i] + kt * stepb);
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x16){0};
  f32x4 acc4[M16 ? 2 * FM : 1][M16 ? 2 * FN : 1];
#pragma unroll
  for (int i = 0; i < (M16 ? 2 * FM : 1); ++i)
#pragma unroll
    for (int j = 0; j < (M16 ? 2 * FN : 1); ++j) acc4[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // bias gradient of a weight-gradient GEMM: column sums of the staged MN-major A tile ([k][BMt],
  // chunk c of k-row k at slot c ^ 4(k&3)); thread = one 8-column chunk x every RGth k-row
  constexpr int ACH = BMt / 8, RG = G::NTt / ACH;
  const bool acs = !AK && p.acs_slab != nullptr && tn == 0;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int acs_c = tid % ACH, acs_r = tid / ACH;

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s);
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt has landed once only the younger issued stages are outstanding
    const int younger = min(NST - 2, nk - 1 - kt);
    if constexpr (G::EVEN) wait_stages<G::AI + G::BI>(younger);
    else wait_vm_rt(per_w * younger);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NST - 1 < nk) issue(kt + NST - 1);   // refills the stage every wave finished reading at kt-1
    const char* sa = lds + (kt % NST) * G::STAGE;
    const char* sb = sa + G::ABYTES;
    if constexpr (F8) {
      typedef KmSw<BKt> S;
      typedef int i32x8 __attribute__((ext_vector_type(8)));
      constexpr int KS8 = BKt / 32;    // 64-fp8 k-steps per stage
      i32x8 a8[KS8][FM], b8[KS8][FN];
      unsigned sA[FM], sB[FN];           // MX: this stage's block scales of each fragment row
      if constexpr (MXK > 0) {
        const int mk = p.mxk, kb0 = kt * (BKt / 16);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const char* a = sca + (wm * FM * 32 + i * 32 + (lane & 31)) * mk + kb0;
          sA[i] = BKt == 64 ? *reinterpret_cast<const unsigned*>(a) : *reinterpret_cast<const unsigned short*>(a);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const char* b = scb + (wn * FN * 32 + j * 32 + (lane & 31)) * mk + kb0;
          sB[j] = BKt == 64 ? *reinterpret_cast<const unsigned*>(b) : *reinterpret_cast<const unsigned short*>(b);
        }
      }
      // v_mfma_scale_f32_32x32x64_f8f6f4's k order (measured, benchmarks/mx_probe.hip): lane (r, h) bytes 0-15 hold
      // k = 16h .. 16h+15 and bytes 16-31 k = 32+16h .. 32+16h+15 of the 64-step; the scale of lane r covers k 0..31
      // (bytes 0-15 of both halves), that of lane r+32 k 32..63 -- so lane (r, h) loads 16-B chunks h and h + 2 of
      // the step, and MX block 2q + h's scale sits in lane (r, h)
      auto frag8 = [&](const char* img, int row0, int q) {
        const int r = row0 + (lane & 31), c = 4 * q + (lane >> 5);
        const uint4 lo = *reinterpret_cast<const uint4*>(img + r * S::RB + 16 * S::slot(r, c));
        const uint4 hi = *reinterpret_cast<const uint4*>(img + r * S::RB + 16 * S::slot(r, c + 2));
        i32x8 v;
        v[0] = (int)lo.x; v[1] = (int)lo.y; v[2] = (int)lo.z; v[3] = (int)lo.w;
        v[4] = (int)hi.x; v[5] = (int)hi.y; v[6] = (int)hi.z; v[7] = (int)hi.w;
        return v;
      };
#pragma unroll
      for (int q = 0; q < KS8; ++q) {
#pragma unroll
        for (int j = 0; j < FN; ++j) b8[q][j] = frag8(sb, wn * FN * 32 + j * 32, q);
#pragma unroll
        for (int i = 0; i < FM; ++i) a8[q][i] = frag8(sa, wm * FM * 32 + i * 32, q);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < KS8; ++q)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int sh = 8 * (2 * q + (lane >> 5));
            const int sa = MXK > 0 ? (int)(sA[i] >> sh) : 127, sb = MXK > 0 ? (int)(sB[j] >> sh) : 127;
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8[q][i], b8[q][j], acc[i][j], 0, 0, 0,
                                                                        sa, 0, sb);
          }
      continue;
    }
    if constexpr (M16) {
      constexpr int KS32 = BKt / 32;
      bf16x8 a16[KS32][2 * FM], b16[KS32][2 * FN];
#pragma unroll
      for (int q = 0; q < KS32; ++q) {
#pragma unroll
        for (int j = 0; j < 2 * FN; ++j) b16[q][j] = pipe_frag16k<BKt>(sb, wn * FN * 32 + 16 * j, 32 * q, lane);
#pragma unroll
        for (int i = 0; i < 2 * FM; ++i) a16[q][i] = pipe_frag16k<BKt>(sa, wm * FM * 32 + 16 * i, 32 * q, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < KS32; ++q)
#pragma unroll
        for (int i = 0; i < 2 * FM; ++i)
#pragma unroll
          for (int j = 0; j < 2 * FN; ++j)
            acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a16[q][i], b16[q][j], acc4[i][j], 0, 0, 0);
      continue;
    }
    // every fragment of the stage is read up front (the stage is complete after the barrier), so the
    // LDS latency of later k-steps hides under the MFMAs of earlier ones
    constexpr int KST = BKt / 16;
    bf16x8 af[KST][FM], bfr[KST][FN];
#pragma unroll
    for (int q = 0; q < KST; ++q) {
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[q][j] = pipe_frag<BKM, BNt, BKt>(sb, wn * FN * 32 + j * 32, 16 * q, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[q][i] = pipe_frag<AK, BMt, BKt>(sa, wm * FM * 32 + i * 32, 16 * q, lane);
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the MFMAs (the scheduler would sink them)
#pragma unroll
    for (int q = 0; q < KST; ++q)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[q][i], bfr[q][j], acc[i][j], 0, 0, 0);
    if constexpr (!AK) {
      if (acs) {
#pragma unroll
        for (int kq = 0; kq < BKt / RG; ++kq) {
          const int k = acs_r + kq * RG;
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(sa + k * (BMt * 2) + 16 * (acs_c ^ (4 * (k & 3))));
#pragma unroll
          for (int e = 0; e < 8; ++e) csum[e] += (float)v[e];
        }
      }
    }
  }
  if constexpr (!AK) {
    if (acs) {   // combine the RG row groups in LDS (every wave is past its last ring read after this barrier)
      __syncthreads();
      float* red = reinterpret_cast<float*>(lds);
#pragma unroll
      for (int e = 0; e < 8; ++e) red[acs_r * BMt + acs_c * 8 + e] = csum[e];
      __syncthreads();
      if (tid < BMt && m0 + tid < p.M) {
        float t = 0.f;
        for (int g = 0; g < RG; ++g) t += red[g * BMt + tid];
        p.acs_slab[(long)zz * p.M + m0 + tid] = t;
      }
    }
  }
  if constexpr (M16) {   // pack the 16x16 blocks into the 32x32 accumulator registers (accr / accc<true>)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = acc4[2 * i + ((r >> 3) & 1)][2 * j + ((r >> 2) & 1)][r & 3];
  }
  if (p.dbg & 1) {   // timing experiment: keep the accumulators live, store nothing
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) t += acc[i][j][r];
    if (t == -1234.5f) reinterpret_cast<float*>(p.C)[tid] = t;
    return;
  }
  if constexpr (!GROUP) gemm_drop_prep(p);
  __syncthreads();   // every wave done with the ring (no DMA outstanding) -> reuse it for the epilogue
  if constexpr (F8) {   // per-tensor dequantisation of the fp8 operands (device scalars)
    if (p.alpha_a) p.alpha *= p.alpha_a[0];
    if (p.alpha_b) p.alpha *= p.alpha_b[0];
  }
  tile_epilogue_g<FM, FN, WM, WN, G::NTt, BNt, M16, 128, EK>(p, acc, reinterpret_cast<float*>(lds), z, zz, m0, n0, wm, wn, lane,
                                                      tid);
  probe_end(p.probe);
}

// ---------------------------------------------------------------- warp-specialised K-major GEMM
// For the encoder's d-wide outputs (one BMt x 128 tile per CU, K up to 2048): NL loader waves only issue the
// LDS-DMA of the ring's stages, wait for it (their vmcnt counts nothing else) and join the one barrier per K step;
// the WM x WN compute waves never touch vector memory in the main loop, so no stage wait ever stalls an MFMA wave
// and no DMA issue sits between its MFMAs.  The compute waves read the next half-step's fragments (16x16x32 MFMA,
// conflict-free ds_read_b128 from the source-swizzled image) while the current half-step's MFMAs run; the barrier
// sits where the next stage must become visible, and the slot of stage kt - 1 is refilled right after it (NST - 1
// stages issued ahead).  Gemm lab (benchmarks/gemm_lab, M 11,936 N 512 K 2048, naive stores): 33.9 -> 27.0 us.
// Epilogue: the whole f32 tile staged in the ring's LDS, then every wave (loaders included) finishes 8-column
// chunks through epilogue_store8 (+ rowdot), as tile_epilogue_g does.
template <int BMt, int WM, int WN, int NL, int NST, int EK = EF_GENERIC>
__global__ __launch_bounds__((WM * WN + NL) * 64) void gemm_ws_kernel(GemmP p, PipeOp oa, PipeOp ob) {
  constexpr int BKt = 64, BNt = BN, NC = WM * WN, NTt = (NC + NL) * 64;
  constexpr int ABYTES = BMt * BKt * 2, BBYTES = BNt * BKt * 2, STAGE = ABYTES + BBYTES;
  constexpr int AP = ABYTES / 1024, BP = BBYTES / 1024, PW = (AP + BP) / NL;
  static_assert(PW * NL == AP + BP && AP * 1024 == ABYTES && BP * 1024 == BBYTES, "whole DMA pieces per loader");
  constexpr int FM = BMt / WM / 16, FN = BNt / WN / 16;
  static_assert(FM * WM * 16 == BMt && FN * WN * 16 == BNt, "wave tiling");
  constexpr int EPS = BNt + 4, CPW = BNt / 8;
  constexpr int RING = NST * STAGE, EPI = BMt * EPS * 4;
  static_assert(NST >= 3 && NST <= 5, "ring depth");
  __shared__ __attribute__((aligned(1024))) char lds[RING > EPI ? RING : EPI];
  probe_begin(p.probe);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  int tm, tn, zz;
  xcd_tile3(tm, tn, zz);
  const int m0 = tm * BMt, n0 = tn * BNt;
  const int z = zz;                       // split_k == 1: the batch index
  const int nk = (p.dbg & 4) ? 0 : (p.K + BKt - 1) / BKt;   // (dbg 4: epilogue only; a partial last tile: below)
  // the epilogue rows' global inputs (f32 residual / bf16 rd_with / pre-activation), issued before the main loop
  // so their latency hides under it (the loaders' counted stage waits see them as older, completed first)
  constexpr int EIT = BMt * CPW / NTt;
  EpiIn<EK == EF_GENERIC ? EF_BF16 : EK, EIT> ein;
  if constexpr (EK != EF_GENERIC) epi_load_all<EK, EIT, NTt, CPW>(p, z, m0, n0, tid, ein);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (wid >= NC) {
    // ---- loader waves
    const int lw = wid - NC;
    const __amdgpu_buffer_rsrc_t ra = pipe_rsrc(oa, z), rb = pipe_rsrc(ob, z);
    unsigned off[PW];
    int ldo[PW], kc[PW];
    bool isa[PW];
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int q = lw + NL * i;
      isa[i] = q < AP;
      const int qq = isa[i] ? q : q - AP;
      off[i] = isa[i] ? pipe_src<true, BMt, BKt>(oa, qq * 64 + lane, m0, 0)
                      : pipe_src<true, BNt, BKt>(ob, qq * 64 + lane, n0, 0);
      ldo[i] = (isa[i] ? 0 : ABYTES) + qq * 1024;
      kc[i] = pipe_kchunk<BKt>(qq * 64 + lane);
    }
    // K % BKt != 0 (K % 8 == 0): the last tile's chunks at k >= K read zero (out-of-range offset), not the next row
    const int klast = p.K - (nk - 1) * BKt;
    auto issue = [&](int kt) {
      if (kt == nk - 1 && klast < BKt) {   // wave-uniform
#pragma unroll
        for (int i = 0; i < PW; ++i)
          dma16(isa[i] ? ra : rb, lds + (kt % NST) * STAGE + ldo[i], kc[i] < klast ? off[i] + kt * (BKt * 2) : 0xFFFFFF00u);
        return;
      }
#pragma unroll
      for (int i = 0; i < PW; ++i)
        dma16(isa[i] ? ra : rb, lds + (kt % NST) * STAGE + ldo[i], off[i] + kt * (BKt * 2));
    };
    // stage s has landed once only the stages issued after it (up to `last`) are outstanding
    auto wait_stage = [&](int s, int last) {
      const int younger = min(NST - 2, last - s);
      if (younger >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PW) : "memory");
      else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PW) : "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    for (int s = 0; s < NST - 1 && s < nk; ++s) issue(s);
    int last = min(NST - 2, nk - 1);
    wait_stage(0, last);
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt + 1 < nk; ++kt) {
      wait_stage(kt + 1, last);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int kn = kt + NST - 1;          // refills the slot of stage kt - 1 (every wave is past its reads)
      if (kn < nk) {
        issue(kn);
        last = kn;
      }
    }
  } else {
    // ---- compute waves
    const int wm = wid / WN, wn = wid % WN;
    bf16x8 af[2][FM], bfr[2][FN];
    auto read = [&](bf16x8 (&fa)[FM], bf16x8 (&fb)[FN], int kt, int sub) {
      const char* sa = lds + (kt % NST) * STAGE;
      const char* sb = sa + ABYTES;
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = pipe_frag16k<BKt>(sb, wn * FN * 16 + 16 * j, 32 * sub, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = pipe_frag16k<BKt>(sa, wm * FM * 16 + 16 * i, 32 * sub, lane);
    };
    auto mma = [&](const bf16x8 (&fa)[FM], const bf16x8 (&fb)[FN]) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    };
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read(af[0], bfr[0], 0, 0);
    for (int kt = 0; kt < nk; ++kt) {
      read(af[1], bfr[1], kt, 1);
      mma(af[0], bfr[0]);
      if (kt + 1 < nk) {
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        read(af[0], bfr[0], kt + 1, 0);
      }
      mma(af[1], bfr[1]);
    }
  }
  if (p.dbg & 1) {   // timing experiment: keep the accumulators live, store nothing
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) t += acc[i][j][0] + acc[i][j][3];
    if (t == -1234.5f) reinterpret_cast<float*>(p.C)[tid] = t;
    return;
  }
  gemm_drop_prep(p);   // (here, not at the top: its counter load would hold back the loaders' first stage)
  float bias8[8];
  if constexpr (EK != EF_GENERIC) epi_bias8(p, n0 + (tid % CPW) * 8, bias8);
  __syncthreads();   // every DMA landed (the loaders' last wait was vmcnt(0)), every fragment read consumed
  float* st = reinterpret_cast<float*>(lds);
  if (wid < NC) {
    const int wm = wid / WN, wn = wid % WN;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          st[(wm * FM * 16 + 16 * i + 4 * (lane >> 4) + e) * EPS + wn * FN * 16 + 16 * j + (lane & 15)] = acc[i][j][e];
  }
  __syncthreads();
  static_assert((BMt * CPW) % NTt == 0 && NTt % CPW == 0, "whole rows per pass");
  if constexpr (EK != EF_GENERIC) {
    epi_rows_fast<EK, EIT, NTt, CPW, EPS, true>(p, st, z, m0, n0, tid, bias8, ein);
    probe_end(p.probe);
    return;
  }
#pragma unroll 2
  for (int it = 0; it < BMt * CPW / NTt; ++it) {
    const int row = it * (NTt / CPW) + tid / CPW, c8 = (tid % CPW) * 8;
    const float4 lo = *reinterpret_cast<const float4*>(st + row * EPS + c8);
    const float4 hi = *reinterpret_cast<const float4*>(st + row * EPS + c8 + 4);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const int m = m0 + row;
    epilogue_store8(p, z, zz, m, n0 + c8, v);
    if (p.rd_out) {   // (vectorised bf16 epilogue: v now holds the stored values) 8-lane group = 64 columns
      float t = 0.f;
      if (m < p.M && n0 + c8 < p.N) {
        const uint4 u = *reinterpret_cast<const uint4*>(p.rd_with + (long)m * p.ldc + n0 + c8);
        const bf16x8 w = __builtin_bit_cast(bf16x8, u);
#pragma unroll
        for (int e = 0; e < 8; ++e) t += (float)(bf16)v[e] * (float)w[e];
      }
      t += __shfl_xor(t, 1, 64);
      t += __shfl_xor(t, 2, 64);
      t += __shfl_xor(t, 4, 64);
      if ((tid & 7) == 0 && m < p.M && n0 + c8 < p.N) {
        const int b = m / p.rd_T, tt = m - b * p.rd_T, g = (n0 + c8) >> 6;
        p.rd_out[((long)b * (p.N >> 6) + g) * p.rd_T + tt] = t;
      }
    }
  }
  probe_end(p.probe);
}

extern int g_gemm_mode;
// ---------------------------------------------------------------- grouped weight gradients
// All weight-gradient GEMMs dW_i = dY_iᵀ X_i (+ bias gradient sum_rows dY_i) of a backward pass in ONE
// launch: every task reduces over the same token dimension, so each 256x128 output tile is one
// workgroup running the whole K loop (no split-K slabs, no reduce pass), and the ~3000 tiles of the
// encoder's 17 layers fill the chip in whole rounds.  Workgroup -> (task, tile): XCD-contiguous ids
// (xcd_tile order), tasks back to back (tile0 ascending), tiles row-major inside a task.
// Planned form (cfm_wgrad_group_plan, GatherA.group_sched): one schedule word per workgroup -- task, tile, K slice
// -- laid out so that each XCD (workgroups b, b + 8, ... under round-robin placement) runs whole tasks in rounds of
// one tile per CU, i.e. every tile that shares a dY or X column slice with another is co-resident on that XCD and
// streams the slice through its L2 once; the tiles that do not fill whole rounds run split over K slices into fp32
// slabs (the task's p.split_k / k_per_split / slab / acs_slab), summed by wgrad_split_reduce_kernel.
struct WgTask {
  GemmP p;
  PipeOp oa, ob;
  long tile0;
  int tiles_n;
  int red_blocks;      // split task: blocks of wgrad_split_reduce_kernel (0: not split)
  long red0;           // first reduce block of this task
  float* dw;           // split task: the destinations the reduce writes (p.C / p.acs_slab point into the workspace)
  float* db;
};
static_assert(sizeof(WgTask) % 4 == 0, "word-copied task");
constexpr unsigned WG_SCHED_EMPTY = 0xFFFFFFFFu;   // padding workgroup of a planned launch
__host__ __device__ constexpr unsigned wg_sched_word(int task, int ks, int tile) {
  return ((unsigned)task << 20) | ((unsigned)ks << 16) | (unsigned)tile;
}

__device__ __forceinline__ bool group_task(const GatherA& ga, GemmP& p, PipeOp& oa, PipeOp& ob, int& tm, int& tn,
                                           int& zz) {
  const WgTask* tab = reinterpret_cast<const WgTask*>(ga.group_tab);
  int lo, local;
  zz = 0;
  if (ga.group_sched) {
    const unsigned w = __builtin_amdgcn_readfirstlane(ga.group_sched[blockIdx.x]);
    if (w == WG_SCHED_EMPTY) return false;
    lo = (int)(w >> 20);
    zz = (int)((w >> 16) & 15u);
    local = (int)(w & 0xFFFFu);
  } else {
    const int nwg = gridDim.x, L = blockIdx.x;
    int id = L;
    if (nwg > 8) {
      const int xcd = L & 7, q = nwg >> 3, r = nwg & 7;
      id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
    }
    lo = 0;
    int hi = ga.group_n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (__builtin_amdgcn_readfirstlane((int)tab[mid].tile0) <= id) lo = mid; else hi = mid - 1;
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    local = id - (int)__builtin_amdgcn_readfirstlane((int)tab[lo].tile0);
  }
  // copy the task word by word through readfirstlane: the compiler then knows every field (buffer
  // descriptors, loop bounds) is wave-uniform -- SGPRs, no waterfall loops around the buffer loads
  WgTask t;
  const int* src = reinterpret_cast<const int*>(tab + lo);
  int* dst = reinterpret_cast<int*>(&t);
#pragma unroll
  for (int w = 0; w < (int)(sizeof(WgTask) / 4); ++w) dst[w] = __builtin_amdgcn_readfirstlane(src[w]);
  p = t.p;
  oa = t.oa;
  ob = t.ob;
  tm = local / t.tiles_n;
  tn = local % t.tiles_n;
  return true;
}

// sum the K-slice slabs of every split task of a planned grouped launch, in slice order (deterministic):
// dW (N x K, row-major) = sum_s slab[s], db (N) = sum_s acs_slab[s]; block b of task t: 1024 elements of dW and
// (b < N / 256) 256 elements of db; task of a block = the last one whose red0 <= b (unsplit tasks own no blocks)
__global__ __launch_bounds__(256) void wgrad_split_reduce_kernel(const WgTask* __restrict__ tab, int ntasks) {
  const long b = blockIdx.x;
  int lo = 0, hi = ntasks - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].red0 <= b) lo = mid; else hi = mid - 1;
  }
  const WgTask& t = tab[lo];
  const int S = t.p.split_k, N = t.p.M, K = t.p.N;
  const long lb = b - t.red0;
  const long per = (long)N * K;
  const long w = (lb * 256 + threadIdx.x) * 4;
  if (w < per) {
    const float* src = t.p.slab + w;
    float4 s = *reinterpret_cast<const float4*>(src);
    for (int k = 1; k < S; ++k) {
      const float4 a = *reinterpret_cast<const float4*>(src + k * per);
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
    *reinterpret_cast<float4*>(t.dw + w) = s;
  }
  const long n = lb * 256 + threadIdx.x;
  if (t.db && n < N) {
    float s = t.p.acs_slab[n];
    for (int k = 1; k < S; ++k) s += t.p.acs_slab[k * (long)N + n];
    t.db[n] = s;
  }
}

// ---------------------------------------------------------------- fp32 kernel (exact-f32 MFMA)
// exact-f32 MFMA GEMM (v_mfma_f32_32x32x2f32), register-staged K tiles of 16; TBM x TBM output tile, 4 waves
// of (TBM/2)^2: TBM = 128 for the large shapes, 64 (4x the workgroups) when the 128-tile grid would leave the
// chip mostly idle (the folded front-end's small contractions, frontfold.hip)
template <bool AK, bool BKM, class OA, class OB, int TBM = 128>
__global__ __launch_bounds__(NT) void gemm_f32_kernel(GemmP p, OA oa, OB ob) {
  constexpr int FR = TBM / 64, FS = TBM + 4, TT = BK32 * FS, NV = TBM / 64;
  gemm_drop_prep(p);
  __shared__ __attribute__((aligned(16))) float lds[4 * TT];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * TBM, n0 = blockIdx.x * TBM;
  const int z = blockIdx.z / p.split_k, ks = blockIdx.z % p.split_k;
  oa.batch(z);
  ob.batch(z);
  const int kbeg = ks * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + BK32 - 1) / BK32 : 0;

  f32x16 acc[FR][FR];
#pragma unroll
  for (int i = 0; i < FR; ++i)
#pragma unroll
    for (int j = 0; j < FR; ++j) acc[i][j] = (f32x16){0};

  float4 ra[NV], rb[NV];
  // tile = 16 k x TBM rows = 4 * TBM float4
  auto gload = [&](int kt) {
    const int k0 = kbeg + kt * BK32;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + NT * i;
      if constexpr (AK) ra[i] = oa.load(m0 + (v >> 2), k0 + (v & 3) * 4, p.M, kend);
      else ra[i] = oa.load(k0 + v / (TBM / 4), m0 + (v % (TBM / 4)) * 4, kend, p.M);
      if constexpr (BKM) rb[i] = ob.load(n0 + (v >> 2), k0 + (v & 3) * 4, p.N, kend);
      else rb[i] = ob.load(k0 + v / (TBM / 4), n0 + (v % (TBM / 4)) * 4, kend, p.N);
    }
  };
  auto put = [&](float* t, bool kmaj, int v, float4 r) {
    if (kmaj) {
      const int row = v >> 2, kc = (v & 3) * 4;
      t[(kc + 0) * FS + row] = r.x;
      t[(kc + 1) * FS + row] = r.y;
      t[(kc + 2) * FS + row] = r.z;
      t[(kc + 3) * FS + row] = r.w;
    } else {
      *reinterpret_cast<float4*>(t + (v / (TBM / 4)) * FS + (v % (TBM / 4)) * 4) = r;
    }
  };
  auto sstore = [&](int buf) {
    float* ta = lds + buf * 2 * TT;
    float* tb = ta + TT;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + NT * i;
      put(ta, AK, v, ra[i]);
      put(tb, BKM, v, rb[i]);
    }
  };

  if (nk > 0) {
    gload(0);
    sstore(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const float* ta = lds + cur * 2 * TT;
    const float* tb = ta + TT;
#pragma unroll
    for (int kk = 0; kk < BK32; kk += 2) {
      const int kr = kk + (lane >> 5);
      float af[FR], bfr[FR];
#pragma unroll
      for (int i = 0; i < FR; ++i) af[i] = ta[kr * FS + wm * (TBM / 2) + i * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < FR; ++j) bfr[j] = tb[kr * FS + wn * (TBM / 2) + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }
  // (the K loop ends on a barrier: the staging may reuse the operand LDS) one wave band (TBM / 2 rows) of the
  // f32 tile at a time through LDS, then 8-column chunks through epilogue_store8 (was a per-element epilogue the
  // compiler could not unroll, leaving the accumulators run-time indexed)
  static_assert((TBM / 2) * (TBM + 4) <= 4 * TT, "one band of the tile fits the staging");
  tile_epilogue_g<FR, FR, 2, 2, NT, TBM, false, TBM / 2>(p, acc, lds, z, blockIdx.z, m0, n0, wm, wn, lane, tid);
}

GemmP plain_params(int M, int N, int K, void* C, long ldc, int dtc) {
  GemmP p{};
  p.M = M; p.N = N; p.K = K;
  p.C = C; p.ldc = ldc; p.sc = 0; p.dtc = dtc;
  p.alpha = 1.f; p.out_scale = 1.f;
  p.split_k = 1; p.k_per_split = K;
  return p;
}

// C[z][m][n] = sum_s slab[z*split + s][m][n] + bias[n]   (fp32 C, 4 columns per thread)
// grid (ceil(M*N/4 / 256), batch): 32-bit index math (M*N < 2^31), the split slabs summed in order
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, int split, int M, int N,
                                                            float* __restrict__ C, long ldc, long sc,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ acs_slab, float* __restrict__ acs) {
  if (acs_slab && blockIdx.y == 0) {   // A column sums: out[m] = sum_s acs_slab[s][m] (in order)
    const unsigned m = blockIdx.x * 256u + threadIdx.x;
    if (m < (unsigned)M) {
      float t = acs_slab[m];
      for (int k = 1; k < split; ++k) t += acs_slab[(long)k * M + m];
      acs[m] = t;
    }
  }
  const unsigned per = (unsigned)M * (unsigned)N;
  const unsigned q = blockIdx.x * 256u + threadIdx.x;
  if (q * 4u >= per) return;
  const unsigned w = q * 4u;
  const int z = blockIdx.y;
  const unsigned m = w / (unsigned)N, n = w - m * (unsigned)N;
  const float* src = slab + ((long)z * split) * per + w;
  float4 s = *reinterpret_cast<const float4*>(src);
  for (int k = 1; k < split; ++k) {
    const float4 a = *reinterpret_cast<const float4*>(src + (long)k * per);
    s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
  }
  if (bias) {
    s.x += bias[n]; s.y += bias[n + 1]; s.z += bias[n + 2]; s.w += bias[n + 3];
  }
  float* dst = C + (long)z * sc + (long)m * ldc + n;
  if (((uintptr_t)dst & 15) == 0) *reinterpret_cast<float4*>(dst) = s;
  else { dst[0] = s.x; dst[1] = s.y; dst[2] = s.z; dst[3] = s.w; }
}

// kernel-selection switch (cfm_gemm_set_mode) for A/B measurements:
// bit 0 = 256-row register-staged tiles allowed, bit 1 = LDS-DMA pipelined kernel allowed
int g_gemm_mode = 3;

int vec_epilogue_ok(const GemmP& p) {
  auto al = [](const void* q) { return q == nullptr || (uintptr_t)q % 16 == 0; };
  return (p.ldc % 8 == 0) && (p.sc % 8 == 0) && al(p.C) && al(p.pre) && al(p.bias) &&
         (p.res == nullptr || (al(p.res) && p.ldr % 8 == 0));
}

int split_k_for(const GemmP& p, int bk) {
  return ((p.K + p.split_k - 1) / p.split_k + bk - 1) / bk * bk;
}

template <bool AK, bool BKM, class OA, class OB>
int launch_typed(int /*dtype: implied by the loaders' element type*/, GemmP p, OA oa, OB ob, int batch,
                 hipStream_t s) {
  p.vec_c = vec_epilogue_ok(p);
  typedef decltype(oa.load(0, 0, 0, 0)) V;
  if constexpr (std::is_same<V, uint4>::value) {
    // 256-row tiles when the grid still fills the chip (>= ~2 tiles per CU) without split-K
    const bool wide = p.split_k == 1 && (long)cdiv(p.M, 256) * cdiv(p.N, BN) * batch >= 512 && (g_gemm_mode & 1);
    if (wide) {
      dim3 grid(cdiv(p.N, BN), cdiv(p.M, 256), batch * p.split_k);
      if (grid.y > 65535 || grid.z > 65535) return cfm::fail(CFM_ERR_SHAPE, "gemm: grid too large");
      hipLaunchKernelGGL((gemm_bf16_kernel<256, AK, BKM, OA, OB>), grid, dim3(512), 0, s, p, oa, ob);
    } else {
      dim3 grid(cdiv(p.N, BN), cdiv(p.M, BM), batch * p.split_k);
      if (grid.y > 65535 || grid.z > 65535) return cfm::fail(CFM_ERR_SHAPE, "gemm: grid too large");
      hipLaunchKernelGGL((gemm_bf16_kernel<128, AK, BKM, OA, OB>), grid, dim3(256), 0, s, p, oa, ob);
    }
  } else {
    // 64-row tiles when 128-row tiles would give fewer workgroups than CUs (small fp32 contractions)
    if ((long)cdiv(p.N, BN) * cdiv(p.M, BM) * batch * p.split_k < 256) {
      dim3 grid(cdiv(p.N, 64), cdiv(p.M, 64), batch * p.split_k);
      if (grid.y > 65535 || grid.z > 65535) return cfm::fail(CFM_ERR_SHAPE, "gemm: grid too large");
      hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, OA, OB, 64>), grid, dim3(NT), 0, s, p, oa, ob);
    } else {
      dim3 grid(cdiv(p.N, BN), cdiv(p.M, BM), batch * p.split_k);
      if (grid.y > 65535 || grid.z > 65535) return cfm::fail(CFM_ERR_SHAPE, "gemm: grid too large");
      hipLaunchKernelGGL((gemm_f32_kernel<AK, BKM, OA, OB>), grid, dim3(NT), 0, s, p, oa, ob);
    }
  }
  return CFM_OK;
}

// elements one batch of a strided operand spans: (rows - 1) * ld + row length.  Rows may overlap (ld < row
// length: the folded front-end's windowed view of the packed mels, frontfold.hip); reads past the extent
// return zero through the buffer range check
long pipe_extent(int kmajor, long mn, long K, long ld) {
  return kmajor ? (mn - 1) * ld + K : (K - 1) * ld + mn;
}

// The LDS-DMA kernel takes plain strided bf16 operands whose 16-B chunks never straddle the
// reduction edge: K-major operands need K % 64 == 0, MN-major ones M (N) % 8 == 0, and every
// batch must fit the 32-bit range of a buffer resource.
bool pipe_ok(const cfm_gemm_desc& d, const GemmP& p, bool va, bool vb) {
  if (!va || !vb || p.cmap) return false;
  if (p.k_per_split % BK16) return false;
  auto fits = [](long bytes) { return bytes > 0 && bytes < (1L << 31); };
  const long ea = pipe_extent(d.a_kmajor, d.M, d.K, d.lda), eb = pipe_extent(d.b_kmajor, d.N, d.K, d.ldb);
  if (!fits(ea * 2) || !fits(eb * 2)) return false;
  // K-major: whole 16-B chunks along K; a partial last K tile reads zero past K (the kernels' tail stage), so K need
  // not be a multiple of the tile depth -- Conformer-S's K = 144 / 432 / 288 (d 144) take the pipeline too
  const int kq = p.split_k == 1 ? 8 : BK16;
  if (d.a_kmajor ? d.K % kq != 0 : d.M % 8 != 0) return false;
  if (d.b_kmajor ? d.K % kq != 0 : d.N % 8 != 0) return false;
  return true;
}

// pipelined-kernel variants (cfm_gemm_set_mode bits 4-6 force one for A/B measurements):
//   V256: 256x128 tile, BK 64, 3-stage ring (144 KiB: one workgroup of 8 waves per CU)
//   V256S: 256x128 tile, BK 32, 3-stage ring (72 KiB: two workgroups per CU, one's epilogue
//          overlapping the other's main loop)
//   V192: 192x128 tile for d-wide outputs (warp-specialised for K-major x K-major operands)
//   V192S8: 192x128 tile, 8 waves, BK 32, two workgroups per CU
// (measured slower and removed in round 4, A/B records in DESIGN.md §8: 128-row tiles, 96-row tiles, a persistent
//  register-deferred epilogue, an interleaved-epilogue persistent kernel, a tail-balanced row split, 32x32x16
//  main loops for K-major operands, a 3-deep 192-row ring)
int num_cus();

// f(std::integral_constant<int, EK>) for the launch's epilogue kind (K-major x K-major launches only: the other
// operand layouts keep the generic epilogue, so their kernels are instantiated once)
template <bool KK, class F>
void ek_dispatch(int ek, F&& f) {
  if constexpr (KK) {
    switch (ek) {
      case EF_BF16: f(std::integral_constant<int, EF_BF16>{}); return;
      case EF_BF16_BIAS: f(std::integral_constant<int, EF_BF16_BIAS>{}); return;
      case EF_BF16_SILU: f(std::integral_constant<int, EF_BF16_SILU>{}); return;
      case EF_BF16_ACTG: f(std::integral_constant<int, EF_BF16_ACTG>{}); return;
      case EF_BF16_RD: f(std::integral_constant<int, EF_BF16_RD>{}); return;
      case EF_F32: f(std::integral_constant<int, EF_F32>{}); return;
      case EF_F32_RES: f(std::integral_constant<int, EF_F32_RES>{}); return;
      case EF_BF16_RES: f(std::integral_constant<int, EF_BF16_RES>{}); return;
      case EF_F32R_BF16: f(std::integral_constant<int, EF_F32R_BF16>{}); return;
      case EF_BF16_DELTA: f(std::integral_constant<int, EF_BF16_DELTA>{}); return;
      case EF_BF16_SILU_MX: f(std::integral_constant<int, EF_BF16_SILU_MX>{}); return;
      default: break;
    }
  }
  f(std::integral_constant<int, EF_GENERIC>{});
}

template <bool AK, bool BKM, bool M16 = false>
void launch_pipe_t(const GemmP& p, const PipeOp& oa, const PipeOp& ob, int batch, hipStream_t s) {
  // 0 auto, 1 V256, 2 V256S, 5 V192, 7 V192S8
  const int sel = (g_gemm_mode >> 4) & 7;
  const dim3 g256(cdiv(p.N, BN), cdiv(p.M, 256), batch * p.split_k);
  int v = sel;
  if constexpr (AK && BKM) {
    // auto: 129..160-column outputs (Conformer-S's d = 144) on 64 x 160 tiles, five waves of 64 x 32, BK 64 in a
    // 4-deep ring (84 KiB in flight: one workgroup per CU, 187 of them, each bound by its DMA latency): ONE column tile (the 128-wide tiles took two, the second 16 columns wide -- 126 workgroups for
    // 256 CUs with 44 % of the MFMA work padding); these K <= 576 GEMMs are bandwidth-bound, so the tile's 187 row
    // blocks each stream their A rows once.  cfm_gemm_set_mode bit 22 keeps the 128-wide tiles (A/B)
    if (v == 0 && p.N > 128 && p.N <= 160 && p.split_k == 1 && !(g_gemm_mode & 4194304)) {
      const dim3 g64(1, cdiv(p.M, 64), batch);
      ek_dispatch<true>(p.efast, [&](auto ek) {
        hipLaunchKernelGGL((gemm_pipe_kernel<64, 64, 4, 1, true, true, 5, 5, false, false, false, 160, M16,
                                             decltype(ek)::value>),
                           g64, dim3(320), 0, s, p, oa, ob, GatherA{});
      });
      return;
    }
  }
  if constexpr (AK) {
    // auto: outputs <= 512 columns (the encoder's d-wide outputs) take the 192-row tiles: 63 x 4 = 252
    // tiles fill 256 CUs in one round where 256-row tiles leave 68 CUs idle (A/B: 9-18 % faster)
    if (v == 5 || (v == 0 && p.N <= 512 && p.split_k == 1 && (long)p.M * batch >= 4096)) {
      const dim3 g192(cdiv(p.N, BN), cdiv(p.M, 192), batch * p.split_k);
      if constexpr (BKM) {
        // warp-specialised loading (cfm_gemm_set_mode bit 19 keeps the shared-DMA kernel below for A/B): d-wide
        // layer family 266.6 -> 240.2 us same box (gpurun_out r04b dgemm; 4 compute waves of 96 x 64: 244.4 us)
        if (!(g_gemm_mode & 524288) && p.split_k == 1) {
          // outputs narrow enough that 192-row tiles leave most CUs idle (Conformer-M's d = 256: 63 x 2 = 126 tiles
          // for 256 CUs) take 96-row tiles -- 125 x 2 = 250, one round (cfm_gemm_set_mode bit 23 keeps 192, A/B)
          if ((long)g192.x * g192.y * g192.z * 5 <= (long)num_cus() * 3 && !(g_gemm_mode & 8388608)) {
            const dim3 g96(cdiv(p.N, BN), cdiv(p.M, 96), batch * p.split_k);
            ek_dispatch<true>(p.efast, [&](auto ek) {
              hipLaunchKernelGGL((gemm_ws_kernel<96, 2, 4, 4, 4, decltype(ek)::value>), g96, dim3(768), 0, s, p, oa, ob);
            });
            return;
          }
          ek_dispatch<true>(p.efast, [&](auto ek) {
            hipLaunchKernelGGL((gemm_ws_kernel<192, 2, 4, 4, 4, decltype(ek)::value>), g192, dim3(768), 0, s, p, oa, ob);
          });
          return;
        }
      }
      // 4-deep ring (4 x 40 KiB = the whole 160 KiB LDS): FFN-up data gradient 34.2 -> 32.5 us same-box
      hipLaunchKernelGGL((gemm_pipe_kernel<192, 64, 4, 1, AK, BKM, 8, 4, false, false, false, BN, M16>), g192,
                         dim3(512), 0, s, p, oa, ob, GatherA{});
      return;
    }
    // auto: 1024- / 1536-wide outputs of short reductions (QKV, pointwise-conv-1 forward) take 192-row tiles
    // two per CU: 504 / 756 tiles fill the 512 slots in whole rounds where 256-row tiles leave a sliver
    // (A/B, profiles/r02/gemm_v192s8_ab.txt: QKV 41.1 -> 36.1 us, pw1 27.7 -> 24.8 us)
    // (cfm_gemm_set_mode bit 12 turns this rule off for A/B)
    if (v == 0 && p.N > 512 && p.N <= 1536 && p.k_per_split <= 512 && p.split_k == 1 && p.M >= 4096 &&
        !(g_gemm_mode & 4096))
      v = 7;
    // 1024- / 1536-wide K-major x K-major outputs (QKV, pointwise-conv-1 forward) on the warp-specialised kernel:
    // QKV 32.41 -> 30.97 us, pw1 22.53 -> 21.41 us same box, bit-identical (gpurun_out r04y; the 2048-wide ones
    // stay on the two-per-CU 256-row tiles: 45.5 vs 57.3 us).  cfm_gemm_set_mode bit 21 keeps the 192-row pipeline.
    // (short reductions, K <= 256 -- Conformer-S's FFN up / down-gradient at K 144: three K tiles -- keep the two-per-CU
    // pipeline: S15 step 8.27 -> 8.07 ms same box, gpurun_out r06c)
    if constexpr (BKM) {
      if (v == 7 && sel == 0 && !(g_gemm_mode & 2097152) && p.k_per_split > 256) {
        const dim3 g192(cdiv(p.N, BN), cdiv(p.M, 192), batch * p.split_k);
        ek_dispatch<true>(p.efast, [&](auto ek) {
          hipLaunchKernelGGL((gemm_ws_kernel<192, 2, 4, 4, 4, decltype(ek)::value>), g192, dim3(768), 0, s, p, oa, ob);
        });
        return;
      }
    }
    if (v == 7) {   // 192 x 128 tiles, 8 waves of 96 x 32, BK 32 (uneven A DMA split): two per CU
      const dim3 g192(cdiv(p.N, BN), cdiv(p.M, 192), batch * p.split_k);
      ek_dispatch<AK && BKM>(p.efast, [&](auto ek) {
        hipLaunchKernelGGL((gemm_pipe_kernel<192, 32, 3, 2, AK, BKM, 8, 4, false, false, false, BN, M16,
                                             decltype(ek)::value>),
                           g192, dim3(512), 0, s, p, oa, ob, GatherA{});
      });
      return;
    }
  }
  if (v != 1 && v != 2) v = 0;
  if (!v) {
    // auto: short reductions (K <= 512: the epilogue is a large share of the tile's time) run two
    // 256-row workgroups per CU so one's epilogue hides under the other's MFMAs; long ones keep BK 64
    v = p.k_per_split <= 512 ? 2 : 1;      // (V128S measured no faster for N = 512 outputs)
  }
  if (v == 1)
    hipLaunchKernelGGL((gemm_pipe_kernel<256, 64, 3, 1, AK, BKM, 8, 2, false, false, false, BN, M16>), g256, dim3(512), 0,
                       s, p, oa, ob, GatherA{});
  else
    ek_dispatch<AK && BKM>(p.efast, [&](auto ek) {
      hipLaunchKernelGGL((gemm_pipe_kernel<256, 32, 3, 2, AK, BKM, 8, 2, false, false, false, BN, M16, decltype(ek)::value>),
                         g256, dim3(512), 0, s, p, oa, ob, GatherA{});
    });
}

int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// the staged-epilogue fast path a launch can take (EF_*, epi_rows_fast; EF_GENERIC: the epilogue_store8 rows)
int epi_fast_kind(const GemmP& p, int batch) {
  if (p.split_k != 1 || !p.vec_c || p.N % 8 || p.cmap || (p.dbg & 2) || (g_gemm_mode & 16384)) return EF_GENERIC;
  if (p.drop_p > 0.f && (p.doff + (uint64_t)batch * p.M * p.N) / 2 + 8 > 0xFFFFFFFBull) return EF_GENERIC;
  const bool f32 = p.dtc == CFM_F32, bf = p.dtc == CFM_BF16, silu = p.act == CFM_ACT_SILU;
  const bool a1 = p.alpha == 1.f, s1 = p.out_scale == 1.f;
  if (!f32 && !bf) return EF_GENERIC;
  if (p.res) {
    if (!p.bias || !a1 || silu || p.act_grad || p.rd_out) return EF_GENERIC;
    if (f32) return p.dtr == CFM_F32 ? EF_F32_RES : EF_GENERIC;
    return p.dtr == CFM_BF16 ? EF_BF16_RES : p.dtr == CFM_F32 ? EF_F32R_BF16 : EF_GENERIC;
  }
  if (p.act_grad)
    return bf && p.dtpre == CFM_BF16 && !p.bias && a1 && s1 && !silu && !p.rd_out ? EF_BF16_ACTG : EF_GENERIC;
  if (p.rd_out)
    return bf && !p.bias && a1 && s1 && !silu && p.drop_p <= 0.f ? EF_BF16_RD : EF_GENERIC;
  if (f32) return silu && p.pre && p.dtpre != CFM_BF16 ? EF_GENERIC : EF_F32;
  if (silu) return p.pre && p.dtpre == CFM_BF16 && p.bias && a1 && s1 ? (p.mxo8 ? EF_BF16_SILU_MX : EF_BF16_SILU)
                                                                        : EF_GENERIC;
  if (p.drop_p > 0.f || !s1)
    return bf && p.bias && a1 && p.act == CFM_ACT_NONE && !p.pre ? EF_BF16_DELTA : EF_GENERIC;
  if (!a1) return EF_GENERIC;
  return p.bias ? EF_BF16_BIAS : EF_BF16;
}

int launch_pipe(const cfm_gemm_desc& d, GemmP p, hipStream_t s) {
  p.vec_c = vec_epilogue_ok(p);
  p.dbg = ((g_gemm_mode & 8) ? 1 : 0) | ((g_gemm_mode & 1024) ? 2 : 0)    // bit 10: generic dropout path (A/B)
          | ((g_gemm_mode & 8192) ? 4 : 0);                                     // bit 13: skip the main loop (timing)
  p.efast = d.a_kmajor && d.b_kmajor ? epi_fast_kind(p, d.batch) : EF_GENERIC;                                  // bit 14: generic epilogue rows (A/B)
  if (cdiv(p.M, 128) > 65535 || (long)d.batch * p.split_k > 65535) return cfm::fail(CFM_ERR_SHAPE, "gemm: grid too large");
  const long ea = pipe_extent(d.a_kmajor, d.M, d.K, d.lda), eb = pipe_extent(d.b_kmajor, d.N, d.K, d.ldb);
  const PipeOp oa{(const bf16*)d.A, d.lda, d.stride_a, d.M, (unsigned)(ea * 2)};
  const PipeOp ob{(const bf16*)d.B, d.ldb, d.stride_b, d.N, (unsigned)(eb * 2)};
  const bool ak = d.a_kmajor != 0, bkm = d.b_kmajor != 0;
  // the K-major x K-major GEMMs (forward and data-gradient) run 16x16x32 MFMA main loops (L15 step 25.0 -> 24.7 ms
  // same-box A/B)
  if (ak && bkm) launch_pipe_t<true, true, true>(p, oa, ob, d.batch, s);
  else if (ak) launch_pipe_t<true, false>(p, oa, ob, d.batch, s);
  else if (bkm) launch_pipe_t<false, true>(p, oa, ob, d.batch, s);
  else launch_pipe_t<false, false>(p, oa, ob, d.batch, s);
  return CFM_OK;
}

// fp8 e4m3 x e4m3 (K-major both) on the LDS-DMA pipeline with the block-scaled MFMA (2x the bf16 rate):
// operands viewed as bf16 pairs (K/2 "elements" per row), so DMA / swizzle / epilogue are the bf16 kernel's
int launch_fp8(const cfm_gemm_desc& d, GemmP p, hipStream_t s) {
  p.K = d.K / 2;
  p.split_k = 1;
  p.k_per_split = p.K;
  p.vec_c = vec_epilogue_ok(p);
  p.alpha_a = d.alpha_a_dev;
  p.alpha_b = d.alpha_b_dev;
  const PipeOp oa{(const bf16*)d.A, d.lda / 2, 0, d.M, (unsigned)((long)d.M * d.lda)};
  const PipeOp ob{(const bf16*)d.B, d.ldb / 2, 0, d.N, (unsigned)((long)d.N * d.ldb)};
  if (d.mx_a) {
    // MX operands: block scales applied inside the MFMA, so alpha stays 1 and the fast epilogue kinds apply
    p.mxa = d.mx_a;
    p.mxb = d.mx_b;
    p.mxk = d.K / 32;
    p.mxo8 = (uint8_t*)d.mx_out;
    p.mxos = d.mx_out_scales;
    p.efast = epi_fast_kind(p, 1);
    if (p.mxo8 && p.efast != EF_BF16_SILU_MX)
      return cfm::fail(CFM_ERR_UNSUPPORTED, "cfm_gemm: mx_out needs the FFN-up epilogue (bias + SiLU + bf16 pre, "
                                            "bf16 C, ldc == N, N % 32 == 0)");
    if (p.N <= 512 || d.K > 512) {
      // d-wide outputs, and any K > 512 (the 2048-deep scale rows -- 20 KiB -- do not fit beside a two-per-CU ring)
      const dim3 g(cdiv(p.N, BN), cdiv(p.M, 192), 1);
      ek_dispatch<true>(p.efast, [&](auto ek) {
        hipLaunchKernelGGL((gemm_pipe_kernel<192, 64, 3, 1, true, true, 8, 4, false, false, true, BN, false,
                                             decltype(ek)::value, 64>), g, dim3(512), 0, s, p, oa, ob, GatherA{});
      });
    } else {
      // K <= 512 (FFN up, QKV): the scale rows (6 KiB) fit beside the 72 KiB ring -- two workgroups per CU
      const dim3 g(cdiv(p.N, BN), cdiv(p.M, 256), 1);
      ek_dispatch<true>(p.efast, [&](auto ek) {
        hipLaunchKernelGGL((gemm_pipe_kernel<256, 32, 3, 2, true, true, 8, 2, false, false, true, BN, false,
                                             decltype(ek)::value, 16>), g, dim3(512), 0, s, p, oa, ob, GatherA{});
      });
    }
    return cfm::check_launch("cfm_gemm(fp8 mx)");
  }
  if (p.N <= 512) {
    const dim3 g(cdiv(p.N, BN), cdiv(p.M, 192), 1);
    hipLaunchKernelGGL((gemm_pipe_kernel<192, 64, 3, 1, true, true, 8, 4, false, false, true>), g, dim3(512), 0, s, p,
                       oa, ob, GatherA{});
  } else {
    const dim3 g(cdiv(p.N, BN), cdiv(p.M, 256), 1);
    hipLaunchKernelGGL((gemm_pipe_kernel<256, 32, 3, 2, true, true, 8, 2, false, false, true>), g, dim3(512), 0, s, p,
                       oa, ob, GatherA{});
  }
  return cfm::check_launch("cfm_gemm(fp8)");
}

}  // namespace

CFM_EXPORT int cfm_gemm_set_mode(int mode) {
  g_gemm_mode = mode;
  return CFM_OK;
}

CFM_EXPORT int cfm_gemm(const cfm_gemm_desc* d, void* stream) {
  CFM_REQUIRE(d != nullptr, CFM_ERR_ARG, "null descriptor");
  CFM_REQUIRE(d->M >= 0 && d->N >= 0 && d->K >= 0 && d->batch >= 1, CFM_ERR_SHAPE, "bad M/N/K/batch");
  CFM_REQUIRE(d->dtype_ab == CFM_F32 || d->dtype_ab == CFM_BF16 || d->dtype_ab == CFM_FP8, CFM_ERR_DTYPE, "dtype_ab");
  CFM_REQUIRE(d->A && d->B && d->C, CFM_ERR_ARG, "null operand");
  CFM_REQUIRE(d->act == CFM_ACT_NONE || d->act == CFM_ACT_SILU, CFM_ERR_ARG, "act");
  CFM_REQUIRE(!d->act_grad || d->pre, CFM_ERR_ARG, "act_grad needs pre");
  const int split = d->split_k < 1 ? 1 : d->split_k;
  CFM_REQUIRE(split == 1 || (d->dtype_c == CFM_F32 && d->act == CFM_ACT_NONE && !d->act_grad &&
                             !d->residual && d->drop_p <= 0.f),
              CFM_ERR_ARG, "split_k needs a plain fp32 epilogue");
  // A and B are read-only: rows may overlap (ld below the row length -- the folded front-end's windowed view
  // of the packed mels, frontfold.hip) when the caller says so (allow_overlap); C rows may not
  CFM_REQUIRE(d->lda >= 1 && d->ldb >= 1, CFM_ERR_SHAPE, "lda / ldb");
  CFM_REQUIRE(d->allow_overlap || (d->lda >= (d->a_kmajor ? d->K : d->M) && d->ldb >= (d->b_kmajor ? d->K : d->N)),
              CFM_ERR_SHAPE, "lda / ldb below the row length (overlapping rows need allow_overlap)");
  CFM_REQUIRE(d->ldc >= d->N, CFM_ERR_SHAPE, "ldc");
  if (d->M == 0 || d->N == 0) return CFM_OK;

  GemmP p = plain_params(d->M, d->N, d->K, d->C, d->ldc, d->dtype_c);
  p.sc = d->stride_c;
  p.alpha = d->alpha; p.bias = d->bias; p.act = d->act; p.act_grad = d->act_grad;
  p.pre = d->pre; p.dtpre = d->dtype_pre;
  p.drop_p = d->drop_p; p.seed = d->drop_seed; p.doff = d->drop_offset; p.salt = cfm::g_rng_salt;
  p.out_scale = d->out_scale; p.res = d->residual; p.ldr = d->ldr; p.dtr = d->dtype_r;
  p.split_k = split;
  p.probe = d->probe;
  CFM_REQUIRE(!d->mx_out || d->dtype_ab == CFM_FP8, CFM_ERR_UNSUPPORTED, "mx_out: fp8 MX launches only");
  if (d->dtype_ab == CFM_FP8) {
    CFM_REQUIRE(d->a_kmajor && d->b_kmajor && d->K % 128 == 0 && d->lda % 16 == 0 && d->ldb % 16 == 0 &&
                    (uintptr_t)d->A % 16 == 0 && (uintptr_t)d->B % 16 == 0 && split == 1 && d->batch == 1 &&
                    !d->rowdot_out && !d->a_colsum && (long)d->M * d->lda < (1L << 31) &&
                    (long)d->N * d->ldb < (1L << 31),
                CFM_ERR_UNSUPPORTED, "fp8: K-major A and B, K % 128 == 0, 16-B aligned rows, no split-K / batch");
    CFM_REQUIRE(!d->mx_a == !d->mx_b && (!d->mx_a || (d->K <= 2048 && !d->alpha_a_dev && !d->alpha_b_dev)),
                CFM_ERR_ARG, "fp8 MX: both scale tensors, K <= 2048, no per-tensor alpha");
    CFM_REQUIRE(!d->mx_out || (d->mx_a && d->mx_out_scales && d->dtype_c == CFM_BF16 && d->ldc == d->N &&
                               d->N % 32 == 0 && (uintptr_t)d->mx_out % 8 == 0),
                CFM_ERR_UNSUPPORTED, "mx_out: MX operands, bf16 C with ldc == N, N % 32 == 0");
    return launch_fp8(*d, p, cfm::as_stream(stream));
  }
  const bool bf = d->dtype_ab == CFM_BF16;
  p.k_per_split = split_k_for(p, bf ? BK16 : BK32);
  const int vlen = bf ? 8 : 4;
  const bool va = ((uintptr_t)d->A % 16 == 0) && (d->lda % vlen == 0) && (d->stride_a % vlen == 0);
  const bool vb = ((uintptr_t)d->B % 16 == 0) && (d->ldb % vlen == 0) && (d->stride_b % vlen == 0);
  hipStream_t s = cfm::as_stream(stream);
  const bool ak = d->a_kmajor != 0, bkm = d->b_kmajor != 0;
  int rc;
  auto go = [&](auto tag) {
    typedef decltype(tag) T;
    StridedOp<T> oa{(const T*)d->A, d->lda, d->stride_a, va};
    StridedOp<T> ob{(const T*)d->B, d->ldb, d->stride_b, vb};
    if (ak && bkm) rc = launch_typed<true, true>(d->dtype_ab, p, oa, ob, d->batch, s);
    else if (ak) rc = launch_typed<true, false>(d->dtype_ab, p, oa, ob, d->batch, s);
    else if (bkm) rc = launch_typed<false, true>(d->dtype_ab, p, oa, ob, d->batch, s);
    else rc = launch_typed<false, false>(d->dtype_ab, p, oa, ob, d->batch, s);
  };
  if (split > 1 && d->workspace) {
    CFM_REQUIRE(d->N % 4 == 0 && d->ldc % 4 == 0, CFM_ERR_SHAPE, "slab split-K needs N % 4 == 0");
    p.slab = d->workspace;
  }
  if (d->rowdot_out) {
    CFM_REQUIRE(bf && d->dtype_c == CFM_BF16 && d->rowdot_with && d->N % 64 == 0 && d->rowdot_T > 0 &&
                d->M % d->rowdot_T == 0 && split == 1 && d->batch == 1 && (g_gemm_mode & 2) &&
                pipe_ok(*d, p, va, vb) && ((uintptr_t)d->rowdot_with % 16) == 0,
                CFM_ERR_UNSUPPORTED, "rowdot needs bf16 C on the LDS-DMA path, N % 64 == 0, no split-K, batch 1");
    p.rd_with = (const bf16*)d->rowdot_with;
    p.rd_out = d->rowdot_out;
    p.rd_T = d->rowdot_T;
  }
  if (d->a_colsum) {
    CFM_REQUIRE(bf && !d->a_kmajor && p.slab && d->batch == 1 && (g_gemm_mode & 2) && pipe_ok(*d, p, va, vb),
                CFM_ERR_UNSUPPORTED, "a_colsum needs the bf16 LDS-DMA path, MN-major A, slab split-K, batch 1");
    p.acs_slab = p.slab + (long)split * d->M * d->N;
  }
  if (bf && (g_gemm_mode & 2) && pipe_ok(*d, p, va, vb)) rc = launch_pipe(*d, p, s);
  else if (bf) go(bf16{});
  else go(float{});
  if (rc != CFM_OK) return rc;
  if (p.slab) {
    CFM_REQUIRE((long)d->M * d->N < (1L << 31) && d->batch <= 65535, CFM_ERR_SHAPE, "split-K slab too large");
    const long n4 = (long)d->M * d->N / 4;
    const unsigned gx = (unsigned)((n4 + 255) / 256) > (unsigned)cdiv(d->M, 256) ? (unsigned)((n4 + 255) / 256)
                                                                                : (unsigned)cdiv(d->M, 256);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(gx, d->batch), dim3(256), 0, s, p.slab, split, d->M, d->N,
                       (float*)d->C, d->ldc, d->stride_c, d->bias, p.acs_slab, d->a_colsum);
  }
  return cfm::check_launch("cfm_gemm");
}

CFM_EXPORT size_t cfm_wgrad_group_task_bytes(void) { return sizeof(WgTask); }
// grouped weight-gradient launch: 256 x 256 output tiles, BK 32, 4-deep ring (half the dY panel re-reads of
// 256 x 128; 17 layers 5.46 -> 4.89 ms, L15 step -0.8 ms same-box; 256 x 128 BK 32 two per CU, 256 x 128 BK 64 and
// plain dispatch order measured slower and were removed in round 4; a 256 x 256 BK 64 double-buffered form spilled
// and ran 2.4x slower)
// (round 4: a warp-specialised 256 x 128 form -- 4 loader waves folding the bias sums, 8 compute waves -- ran
// 2.889 vs 2.870 ms for the 17-layer launch, gpurun_out r04b wgrad, and was removed)
constexpr int WG_BN = 256;
CFM_EXPORT long cfm_wgrad_group_tiles(int N, int K) { return (long)cdiv(N, 256) * cdiv(K, WG_BN); }

// fill task i of a HOST table: dW (N x K, fp32) = dYᵀ X over M tokens, dY (M x N) / X (M x K) bf16
// row-major; db (N, fp32, may be NULL) = sum_rows dY; tile0 = first workgroup id of the task
CFM_EXPORT int cfm_wgrad_group_fill(void* host_tab, int i, const void* dy, const void* x, float* dw, float* db, int M,
                                    int N, int K, long tile0) {
  CFM_REQUIRE(host_tab && dy && x && dw && i >= 0, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(M > 0 && N > 0 && K > 0 && N % 8 == 0 && K % 8 == 0, CFM_ERR_SHAPE, "N, K multiples of 8");
  CFM_REQUIRE((long)M * N * 2 < (1L << 31) && (long)M * K * 2 < (1L << 31), CFM_ERR_SHAPE, "operands < 2 GiB");
  CFM_REQUIRE((uintptr_t)dy % 16 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)dw % 16 == 0, CFM_ERR_ALIGN,
              "16-B aligned operands");
  WgTask t{};
  t.p = plain_params(N, K, M, dw, K, CFM_F32);
  t.p.k_per_split = split_k_for(t.p, BK16);
  t.p.vec_c = vec_epilogue_ok(t.p);
  t.p.acs_slab = db;   // single K slice: the column sums go straight to db
  t.oa = PipeOp{(const bf16*)dy, N, 0, N, (unsigned)((long)M * N * 2)};
  t.ob = PipeOp{(const bf16*)x, K, 0, K, (unsigned)((long)M * K * 2)};
  t.tile0 = tile0;
  t.tiles_n = cdiv(K, WG_BN);
  reinterpret_cast<WgTask*>(host_tab)[i] = t;
  return CFM_OK;
}

// the same for a planned launch: task i of the table as cfm_wgrad_group_fill, and when split > 1 (the plan's
// task_split[i]) its K range cut into `split` slices of whole 32-token steps whose fp32 partials go to the workspace
// ws (cfm_wgrad_group_ws_floats(N, K, split) floats: split dW slabs, then split db rows), summed into dw / db by the
// reduce pass; red0 = the task's first reduce block (running sum of cfm_wgrad_group_red_blocks over earlier tasks)
CFM_EXPORT long cfm_wgrad_group_ws_floats(int N, int K, int split) {
  return split > 1 ? (long)split * ((long)N * K + N) : 0;
}
CFM_EXPORT long cfm_wgrad_group_red_blocks(int N, int K, int split) {
  if (split <= 1) return 0;
  const long a = cdiv((long)N * K, 1024), b = cdiv(N, 256);
  return a > b ? a : b;
}
CFM_EXPORT int cfm_wgrad_group_fill_split(void* host_tab, int i, const void* dy, const void* x, float* dw, float* db,
                                          int M, int N, int K, int split, float* ws, long red0) {
  const int rc = cfm_wgrad_group_fill(host_tab, i, dy, x, dw, db, M, N, K, 0);
  if (rc != CFM_OK) return rc;
  CFM_REQUIRE(split >= 1 && split <= 15, CFM_ERR_ARG, "split in 1..15");
  WgTask& t = reinterpret_cast<WgTask*>(host_tab)[i];
  t.red0 = red0;
  t.dw = dw;
  t.db = db;
  if (split > 1) {
    CFM_REQUIRE(ws && (uintptr_t)ws % 16 == 0, CFM_ERR_ALIGN, "16-B aligned workspace");
    CFM_REQUIRE((long)split * N * K < (1L << 31), CFM_ERR_SHAPE, "split slabs too large");
    t.p.split_k = split;
    t.p.k_per_split = ((M + split - 1) / split + 31) / 32 * 32;
    t.p.slab = ws;
    t.p.acs_slab = db ? ws + (long)split * N * K : nullptr;
    t.red_blocks = (int)cfm_wgrad_group_red_blocks(N, K, split);
  }
  return CFM_OK;
}

// Plan a grouped launch of ntasks GEMMs of task_tiles[i] output tiles each (cfm_wgrad_group_tiles) on nxcd XCDs
// of `cus` CUs (one workgroup per CU: the kernel holds a 128-KiB ring):
//  * tasks (cut into pieces of at most `cus` tiles) are packed first-fit-decreasing into bins of `cus` tiles;
//  * each XCD x gets R = (full bins) / nxcd full bins -- workgroup ids x, x + nxcd, ... in bin order, so a bin's
//    tiles start together on one XCD and every dY / X slice a bin reads is streamed into that XCD's L2 once;
//  * the tiles of the remaining bins (the ragged last round) are split over S = min(8, nxcd * cus / tail) K slices
//    (task_split[i] = S for their tasks, 1 otherwise) and dealt to the XCDs slice by slice, so the last round
//    fills the chip instead of running a few tiles alone; with S < 2 (or a task cut across main and tail bins)
//    they run unsplit as extra bins.
// Writes grid words to sched (capacity cap; WG_SCHED_EMPTY pads the shorter XCD lists) and returns the grid size,
// or a negative error code.
CFM_EXPORT long cfm_wgrad_group_plan(const long* task_tiles, int ntasks, int nxcd, int cus, unsigned* sched,
                                     long cap, int* task_split) {
  if (!task_tiles || !sched || !task_split || ntasks <= 0 || ntasks > 4095 || nxcd <= 0 || cus <= 0)
    return cfm::fail(CFM_ERR_ARG, "cfm_wgrad_group_plan: bad arguments");
  struct Piece { int task, off, n; };
  std::vector<Piece> pieces;
  for (int i = 0; i < ntasks; ++i) {
    if (task_tiles[i] <= 0 || task_tiles[i] > 65535)
      return cfm::fail(CFM_ERR_SHAPE, "cfm_wgrad_group_plan: tiles per task in 1..65535");
    for (int o = 0; o < task_tiles[i]; o += cus) pieces.push_back({i, o, (int)std::min<long>(cus, task_tiles[i] - o)});
    task_split[i] = 1;
  }
  std::stable_sort(pieces.begin(), pieces.end(), [](const Piece& a, const Piece& b) { return a.n > b.n; });
  std::vector<std::vector<Piece>> bins;
  std::vector<int> fill;
  for (const Piece& pc : pieces) {
    size_t k = 0;
    while (k < bins.size() && fill[k] + pc.n > cus) ++k;
    if (k == bins.size()) { bins.emplace_back(); fill.push_back(0); }
    bins[k].push_back(pc);
    fill[k] += pc.n;
  }
  std::vector<int> full, rest;
  for (size_t k = 0; k < bins.size(); ++k) (fill[k] == cus ? full : rest).push_back((int)k);
  const int R = (int)full.size() / nxcd;
  for (size_t k = (size_t)R * nxcd; k < full.size(); ++k) rest.push_back(full[k]);
  full.resize((size_t)R * nxcd);
  std::vector<std::vector<unsigned>> lists(nxcd);
  auto emit_bin = [&](std::vector<unsigned>& l, int k, int ks) {
    for (const Piece& pc : bins[k])
      for (int t = 0; t < pc.n; ++t) l.push_back(wg_sched_word(pc.task, ks, pc.off + t));
  };
  for (int x = 0; x < nxcd; ++x)
    for (int r = 0; r < R; ++r) emit_bin(lists[x], full[(size_t)x * R + r], 0);
  long tail = 0;
  std::vector<char> in_main(ntasks, 0), in_tail(ntasks, 0);
  for (int k : full) for (const Piece& pc : bins[k]) in_main[pc.task] = 1;
  for (int k : rest) for (const Piece& pc : bins[k]) { in_tail[pc.task] = 1; tail += pc.n; }
  bool cut = false;
  for (int i = 0; i < ntasks; ++i) cut |= in_main[i] && in_tail[i];
  const int S = tail > 0 && !cut ? (int)std::min<long>(8, (long)nxcd * cus / tail) : 1;
  if (S >= 2) {
    std::vector<unsigned> parts;   // slice-major: XCD x gets a contiguous run (one slice per XCD when S == nxcd)
    for (int ks = 0; ks < S; ++ks)
      for (int k : rest) emit_bin(parts, k, ks);
    const long np = (long)parts.size();
    for (long q = 0; q < np; ++q) lists[(int)(q * nxcd / np)].push_back(parts[q]);
    for (int i = 0; i < ntasks; ++i) if (in_tail[i]) task_split[i] = S;
  } else {
    for (size_t j = 0; j < rest.size(); ++j) emit_bin(lists[j % nxcd], rest[j], 0);
  }
  size_t len = 0;
  for (auto& l : lists) len = std::max(len, l.size());
  const long grid = (long)len * nxcd;
  if (grid > cap) return cfm::fail(CFM_ERR_ARG, "cfm_wgrad_group_plan: schedule capacity too small");
  for (size_t j = 0; j < len; ++j)
    for (int x = 0; x < nxcd; ++x) sched[j * nxcd + x] = j < lists[x].size() ? lists[x][j] : WG_SCHED_EMPTY;
  return grid;
}

// planned launch: dev_sched (grid words from cfm_wgrad_group_plan, on the device) over the table of
// cfm_wgrad_group_fill_split tasks, then the reduce pass over the split tasks' slabs (red_blocks = the sum of the
// tasks' cfm_wgrad_group_red_blocks; 0: no split task)
CFM_EXPORT int cfm_wgrad_group_sched(const void* dev_tab, int ntasks, const unsigned* dev_sched, long grid,
                                     long red_blocks, unsigned long long* probe, void* stream) {
  CFM_REQUIRE(dev_tab && dev_sched && ntasks > 0 && grid > 0 && grid < (1L << 31) && red_blocks >= 0 &&
              red_blocks < (1L << 31), CFM_ERR_ARG, "bad plan");
  GemmP gp{};
  gp.probe = probe;
  GatherA ga{};
  ga.group_tab = dev_tab;
  ga.group_n = ntasks;
  ga.group_sched = dev_sched;
  hipStream_t s = cfm::as_stream(stream);
  hipLaunchKernelGGL((gemm_pipe_kernel<256, 32, 4, 1, false, false, 8, 2, false, true, false, WG_BN>),
                     dim3((unsigned)grid), dim3(512), 0, s, gp, PipeOp{}, PipeOp{}, ga);
  if (red_blocks > 0)
    hipLaunchKernelGGL(wgrad_split_reduce_kernel, dim3((unsigned)red_blocks), dim3(256), 0, s,
                       reinterpret_cast<const WgTask*>(dev_tab), ntasks);
  return cfm::check_launch("cfm_wgrad_group_sched");
}

CFM_EXPORT int cfm_wgrad_group_probed(const void* dev_tab, int ntasks, long total_tiles, unsigned long long* probe,
                                      void* stream) {
  CFM_REQUIRE(dev_tab && ntasks > 0 && total_tiles > 0 && total_tiles < (1L << 31), CFM_ERR_ARG, "bad table");
  GemmP gp{};
  gp.probe = probe;
  GatherA ga{};
  ga.group_tab = dev_tab;
  ga.group_n = ntasks;
  // (round 4: a 5-deep ring -- 5 x 32 KiB, the whole 160 KiB LDS -- ran 3.132 vs 2.896 ms, gpurun_out r04u)
  hipLaunchKernelGGL((gemm_pipe_kernel<256, 32, 4, 1, false, false, 8, 2, false, true, false, WG_BN>),
                     dim3((unsigned)total_tiles), dim3(512), 0, cfm::as_stream(stream), gp, PipeOp{}, PipeOp{}, ga);
  return cfm::check_launch("cfm_wgrad_group");
}

CFM_EXPORT int cfm_wgrad_group(const void* dev_tab, int ntasks, long total_tiles, void* stream) {
  return cfm_wgrad_group_probed(dev_tab, ntasks, total_tiles, nullptr, stream);
}

// ---------------------------------------------------------------------------- conv2 (3x3, s2)
static Conv2Geo conv2_geo(int B, int F1, int T1, int C1, int C2) {
  Conv2Geo g{B, F1, T1, C1, (F1 - 3) / 2 + 1, (T1 - 3) / 2 + 1, C2};
  return g;
}

CFM_EXPORT int cfm_conv2_fwd(const void* h1, const void* w2r, const float* b2, void* h2, int dtype_h2, int dtype,
                             int B, int F1, int T1, int C1, int C2, void* stream) {
  CFM_REQUIRE(h1 && w2r && h2, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(C1 % 8 == 0 && F1 >= 3 && T1 >= 3 && B > 0 && C2 > 0, CFM_ERR_SHAPE, "conv2: C1 % 8, F1/T1 >= 3");
  CFM_REQUIRE((uintptr_t)h1 % 16 == 0 && (uintptr_t)w2r % 16 == 0, CFM_ERR_ALIGN, "16-B aligned operands");
  const Conv2Geo g = conv2_geo(B, F1, T1, C1, C2);
  GemmP p = plain_params(B * g.T2 * g.F2, C2, 9 * C1, h2, C2, dtype_h2);
  p.bias = b2;
  hipStream_t s = cfm::as_stream(stream);
  const long h1_bytes = (long)B * F1 * T1 * C1 * 2;
  if (dtype == CFM_BF16 && (g_gemm_mode & 2) && C1 % 64 == 0 && h1_bytes < (1L << 31) - 4096 &&
      cdiv(p.M, 256) <= 65535) {
    // LDS-DMA pipeline with h1 rows gathered per tap: rows m = (b, t2, f2), tap (kh, kw) reads h1 row
    // (b F1 + 2 f2 + kh) T1 + 2 t2 + kw -- every tap in range (no padding)
    GatherA ga{};
    ga.Jn = g.F2; ga.In = g.T2;
    ga.sB = (long)F1 * T1; ga.sI = 2; ga.sJ = 2 * T1; ga.Cr = C1; ga.Ck = C1;
    ga.Ilim = 0x7FFFFFFF; ga.Jlim = 0x7FFFFFFF;
    for (int kh = 0; kh < 3; ++kh)
      for (int kw = 0; kw < 3; ++kw) ga.dR[kh * 3 + kw] = kh * T1 + kw;
    p.split_k = 1;
    p.k_per_split = 9 * C1;
    p.vec_c = vec_epilogue_ok(p);
    const PipeOp oa{(const bf16*)h1, C1, 0, p.M, (unsigned)h1_bytes};
    const PipeOp ob{(const bf16*)w2r, 9L * C1, 0, C2, (unsigned)((long)C2 * 9 * C1 * 2)};
    hipLaunchKernelGGL((gemm_pipe_kernel<256, 64, 3, 1, true, true, 8, 2, true>), dim3(cdiv(C2, BN), cdiv(p.M, 256), 1),
                       dim3(512), 0, s, p, oa, ob, ga);
    return cfm::check_launch("cfm_conv2_fwd");
  }
  int rc;
  if (dtype == CFM_BF16)
    rc = launch_typed<true, true>(dtype, p, Conv2FwdA<bf16>{(const bf16*)h1, g},
                                  StridedOp<bf16>{(const bf16*)w2r, 9L * C1, 0, true}, 1, s);
  else
    rc = launch_typed<true, true>(dtype, p, Conv2FwdA<float>{(const float*)h1, g},
                                  StridedOp<float>{(const float*)w2r, 9L * C1, 0, true}, 1, s);
  if (rc != CFM_OK) return rc;
  return cfm::check_launch("cfm_conv2_fwd");
}

// conv2 weight gradient dW2r (C2 x 9*C1, fp32) = dh2^T im2col(h1) over M = B*T2*F2 tokens.  Split-K over the
// tokens into DETERMINISTIC slabs (ws: split x C2 x 9*C1 floats, each slab written whole by its K slice) summed in
// slice order by splitk_reduce_kernel -- no atomics and no memset: the round-2 form zeroed dW with
// hipMemsetAsync and accumulated with atomics, and inside a replayed HIP graph that left part of dW unzeroed /
// stale (the round-2 NaN losses: nan_hunt showed this gradient alone going non-finite under poisoned memory).
static int conv2_wgrad_split(int B, int F1, int T1, int C1, int C2) {
  const Conv2Geo g = conv2_geo(B, F1, T1, C1, C2);
  const int Mrows = B * g.T2 * g.F2;
  const int tiles = cdiv(C2, BM) * cdiv(9 * C1, BN);
  // ~1024 workgroups (4 per CU: the register-staged 128 x 128 kernel needs them to hide its loads; 512 measured
  // 609 vs 485 us for the atomics form at L15), each slice >= 512 tokens
  int split = 1024 / (tiles > 0 ? tiles : 1);
  split = split < 1 ? 1 : (split > 32 ? 32 : split);
  if (Mrows / 512 < split) split = Mrows / 512 > 1 ? Mrows / 512 : 1;
  return split;
}

CFM_EXPORT size_t cfm_conv2_bwd_weight_ws_bytes(int B, int F1, int T1, int C1, int C2) {
  const int split = conv2_wgrad_split(B, F1, T1, C1, C2);
  return split > 1 ? (size_t)split * C2 * 9 * C1 * sizeof(float) : 0;
}

CFM_EXPORT int cfm_conv2_bwd_weight_ws(const void* dh2, const void* h1, float* dw2r, int dtype, int B, int F1, int T1,
                                       int C1, int C2, float* ws, void* stream) {
  CFM_REQUIRE(dh2 && h1 && dw2r, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(C1 % 8 == 0 && C2 % 8 == 0, CFM_ERR_SHAPE, "conv2: C1 and C2 must be multiples of 8");
  const Conv2Geo g = conv2_geo(B, F1, T1, C1, C2);
  const int Mrows = B * g.T2 * g.F2;
  GemmP p = plain_params(C2, 9 * C1, Mrows, dw2r, 9L * C1, CFM_F32);
  const int split = ws ? conv2_wgrad_split(B, F1, T1, C1, C2) : 1;
  p.split_k = split;
  p.k_per_split = split_k_for(p, dtype == CFM_BF16 ? BK16 : BK32);
  const int used = cdiv(Mrows, p.k_per_split);       // slices that hold tokens (each writes its whole slab)
  p.split_k = used;
  if (used > 1) {
    CFM_REQUIRE((long)C2 * 9 * C1 < (1L << 31), CFM_ERR_SHAPE, "conv2 wgrad: slab too large");
    p.slab = ws;
  }
  hipStream_t s = cfm::as_stream(stream);
  int rc;
  if (dtype == CFM_BF16)
    rc = launch_typed<false, false>(dtype, p, StridedOp<bf16>{(const bf16*)dh2, C2, 0, C2 % 8 == 0},
                                    Conv2WgradB<bf16>{(const bf16*)h1, g}, 1, s);
  else
    rc = launch_typed<false, false>(dtype, p, StridedOp<float>{(const float*)dh2, C2, 0, C2 % 4 == 0},
                                    Conv2WgradB<float>{(const float*)h1, g}, 1, s);
  if (rc != CFM_OK) return rc;
  if (used > 1) {
    const long n4 = (long)C2 * 9 * C1 / 4;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n4 + 255) / 256), 1), dim3(256), 0, s, p.slab, used, C2,
                       9 * C1, dw2r, 9L * C1, 0L, (const float*)nullptr, (const float*)nullptr, (float*)nullptr);
  }
  return cfm::check_launch("cfm_conv2_bwd_weight");
}

// (workspace-free form: one K slice, no split -- kept for the C ABI; the host path passes a workspace)
CFM_EXPORT int cfm_conv2_bwd_weight(const void* dh2, const void* h1, float* dw2r, int dtype, int B, int F1, int T1,
                                    int C1, int C2, void* stream) {
  return cfm_conv2_bwd_weight_ws(dh2, h1, dw2r, dtype, B, F1, T1, C1, C2, nullptr, stream);
}

namespace {
// Per-class K-major data-gradient weights: wt[koff(class) + c1 * K_class + ti * C2 + c2] =
// w2r[c2][kh_ti][kw_ti][c1] for the class's taps (classes (pf, pt) in order (0,0) (0,1) (1,0) (1,1):
// 4, 2, 2, 1 taps -> 9 * C1 * C2 elements in all)
__global__ __launch_bounds__(256) void conv2_dgrad_pack(const bf16* __restrict__ w2r, bf16* __restrict__ wt, int C1,
                                                        int C2) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long per = (long)C1 * C2;
  if (e >= 9 * per) return;
  // which class / tap of the class does slab e / per belong to
  const int slab = (int)(e / per);        // 0..8: class (0,0) taps 0-3, (0,1) 4-5, (1,0) 6-7, (1,1) 8
  const int cls = slab < 4 ? 0 : (slab < 6 ? 1 : (slab < 8 ? 2 : 3));
  const int first = cls == 0 ? 0 : (cls == 1 ? 4 : (cls == 2 ? 6 : 8));
  const int ntaps = cls == 0 ? 4 : (cls == 3 ? 1 : 2);
  const int pf = cls >> 1, pt = cls & 1;
  const long r = e - (long)first * per;   // offset inside the class block (C1 x ntaps*C2)
  const int K = ntaps * C2;
  const int c1 = (int)(r / K), k = (int)(r % K), ti = k / C2, c2 = k % C2;
  // taps of the class in (kh, kw) order, kh = pf (+2), kw = pt (+2)
  const int nkw = pt == 0 ? 2 : 1;
  const int kh = pf + 2 * (ti / nkw), kw = pt + 2 * (ti % nkw);
  wt[e] = w2r[((long)c2 * 9 + kh * 3 + kw) * C1 + c1];
}
}  // namespace

CFM_EXPORT int cfm_conv2_bwd_data(const void* dh2, const void* w2r, void* dh1, int dtype, int B, int F1, int T1,
                                  int C1, int C2, void* stream);

CFM_EXPORT size_t cfm_conv2_bwd_data_ws_bytes(int C1, int C2) { return (size_t)9 * C1 * C2 * sizeof(bf16); }

// conv2 data-gradient on the LDS-DMA pipeline (bf16): per parity class, A rows gathered straight from
// dh2 by the DMA (GatherA), B = the class's packed K-major weights (from `ws`, written by
// conv2_dgrad_pack on the same stream), output rows scattered to the class's dh1 pixels (cmap).
// Falls back to the register-staged gather kernel when ws is NULL or the shape does not qualify.
CFM_EXPORT int cfm_conv2_bwd_data_ws(const void* dh2, const void* w2r, void* dh1, int dtype, int B, int F1, int T1,
                                     int C1, int C2, void* ws, void* stream) {
  CFM_REQUIRE(dh2 && w2r && dh1, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(C1 % 8 == 0 && C2 % 8 == 0, CFM_ERR_SHAPE, "conv2: C1 and C2 must be multiples of 8");
  const Conv2Geo g = conv2_geo(B, F1, T1, C1, C2);
  const long dh2_bytes = (long)B * g.T2 * g.F2 * C2 * 2;
  const bool fast = ws && dtype == CFM_BF16 && C2 % 32 == 0 && C1 % 8 == 0 && (g_gemm_mode & 2) &&
                    dh2_bytes < (1L << 31) - 4096 && ((uintptr_t)dh2 % 16) == 0 && ((uintptr_t)dh1 % 16) == 0;
  if (!fast) return cfm_conv2_bwd_data(dh2, w2r, dh1, dtype, B, F1, T1, C1, C2, stream);
  hipStream_t s = cfm::as_stream(stream);
  bf16* wt = (bf16*)ws;
  const long per = (long)C1 * C2;
  hipLaunchKernelGGL(conv2_dgrad_pack, dim3((unsigned)cdiv(9 * per, 256)), dim3(256), 0, s, (const bf16*)w2r, wt, C1,
                     C2);
  long koff = 0;
  for (int pf = 0; pf < 2; ++pf)
    for (int pt = 0; pt < 2; ++pt) {
      GatherA ga{};
      const int F1c = (F1 - pf + 1) / 2, T1c = (T1 - pt + 1) / 2;
      // rows (b, i, j) of the class; source dh2 rows (b, t2, f2) = b T2 F2 + t2 F2 + f2 with f2 = i - di, t2 = j - dj
      ga.Jn = T1c; ga.In = F1c;
      ga.sB = (long)g.T2 * g.F2; ga.sI = 1; ga.sJ = g.F2; ga.Cr = C2; ga.Ck = C2; ga.Ilim = g.F2; ga.Jlim = g.T2;
      int nt = 0;
      for (int kh = pf; kh < 3; kh += 2)
        for (int kw = pt; kw < 3; kw += 2) {
          ga.di[nt] = (kh - pf) / 2;
          ga.dj[nt] = (kw - pt) / 2;
          ga.dR[nt] = -(ga.dj[nt] * g.F2 + ga.di[nt]);
          ++nt;
        }
      const int K = nt * C2;
      const bf16* wc = wt + koff;
      koff += (long)nt * per;
      if (F1c <= 0 || T1c <= 0) continue;
      GemmP p = plain_params(B * F1c * T1c, C1, K, dh1, C1, dtype);
      p.cmap = 1; p.cm_F1c = F1c; p.cm_T1c = T1c; p.cm_pf = pf; p.cm_pt = pt; p.cm_F1 = F1; p.cm_T1 = T1;
      p.split_k = 1;
      p.k_per_split = K;
      p.vec_c = vec_epilogue_ok(p);
      const PipeOp oa{(const bf16*)dh2, C2, 0, p.M, (unsigned)dh2_bytes};
      const PipeOp ob{wc, K, 0, C1, (unsigned)(per * nt * 2)};
      const dim3 grid(cdiv(C1, BN), cdiv(p.M, 256), 1);
      CFM_REQUIRE(grid.y <= 65535, CFM_ERR_SHAPE, "conv2 dgrad: grid too large");
      hipLaunchKernelGGL((gemm_pipe_kernel<256, 32, 3, 2, true, true, 8, 2, true>), grid, dim3(512), 0, s, p, oa, ob,
                         ga);
    }
  return cfm::check_launch("cfm_conv2_bwd_data_ws");
}

CFM_EXPORT int cfm_conv2_bwd_data(const void* dh2, const void* w2r, void* dh1, int dtype, int B, int F1, int T1,
                                  int C1, int C2, void* stream) {
  CFM_REQUIRE(dh2 && w2r && dh1, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(C1 % 8 == 0 && C2 % 8 == 0, CFM_ERR_SHAPE, "conv2: C1 and C2 must be multiples of 8");
  const Conv2Geo g = conv2_geo(B, F1, T1, C1, C2);
  hipStream_t s = cfm::as_stream(stream);
  for (int pf = 0; pf < 2; ++pf)
    for (int pt = 0; pt < 2; ++pt) {
      Conv2Class c{};
      c.pf = pf; c.pt = pt;
      c.F1c = (F1 - pf + 1) / 2;
      c.T1c = (T1 - pt + 1) / 2;
      for (int kh = pf; kh < 3; kh += 2)
        for (int kw = pt; kw < 3; kw += 2) {
          c.kh[c.ntaps] = kh;
          c.kw[c.ntaps] = kw;
          ++c.ntaps;
        }
      if (c.F1c <= 0 || c.T1c <= 0) continue;
      GemmP p = plain_params(B * c.F1c * c.T1c, C1, c.ntaps * C2, dh1, C1, dtype);
      p.cmap = 1; p.cm_F1c = c.F1c; p.cm_T1c = c.T1c; p.cm_pf = pf; p.cm_pt = pt; p.cm_F1 = F1; p.cm_T1 = T1;
      int rc;
      if (dtype == CFM_BF16)
        rc = launch_typed<true, false>(dtype, p, Conv2DgradA<bf16>{(const bf16*)dh2, g, c},
                                       Conv2DgradB<bf16>{(const bf16*)w2r, g, c}, 1, s);
      else
        rc = launch_typed<true, false>(dtype, p, Conv2DgradA<float>{(const float*)dh2, g, c},
                                       Conv2DgradB<float>{(const float*)w2r, g, c}, 1, s);
      if (rc != CFM_OK) return rc;
    }
  return cfm::check_launch("cfm_conv2_bwd_data");
}
