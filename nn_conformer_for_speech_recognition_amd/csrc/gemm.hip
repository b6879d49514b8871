// gemm.hip — MFMA GEMM with fused epilogues for every dense contraction of the encoder.
//
// Tile: 128x128 output per 256-thread workgroup (4 waves as 2x2, 64x64 per wave =
// 2x2 MFMA 32x32 tiles).  bf16 operands: v_mfma_f32_32x32x16_bf16, BK = 32.  fp32 operands:
// v_mfma_f32_32x32x2_f32 (exact f32 products, used for the fp32 parity mode), BK = 16.
// Operand layouts (per operand, compile-time): K-major (k contiguous, e.g. X and W in the
// forward pass) is staged row-wise and read with ds_read_b128; MN-major (m/n contiguous, e.g.
// the token dimension in weight-gradient GEMMs) is staged as [k][m] and read with the gfx950
// ds_read_b64_tr_b16 transposed LDS read, so no operand is ever transposed in HBM.
// Global->LDS staging goes through registers with one-tile-ahead prefetch and a double-buffered
// LDS ring (one barrier per K tile).
#include "cfm_common.h"

namespace {

constexpr int BM = 128, BN = 128, NT = 256;

struct GemmP {
  int M, N, K;
  const void* A; long lda, sa;
  const void* B; long ldb, sb;
  void* C; long ldc, sc; int dtc;
  float alpha;
  const float* bias;
  int act, act_grad;
  void* pre; int dtpre;
  float drop_p; uint64_t seed, doff;
  float out_scale;
  const void* res; long ldr; int dtr;
  int split_k, k_per_split;
  int vec_a, vec_b;   // 16-byte vector loads legal (alignment of base + ld)
};

// ---------------------------------------------------------------- bf16 staging helpers
// Load 8 consecutive elements base[outer*ld + inner .. +7] with zero fill past the limits.
__device__ __forceinline__ uint4 ld8_bf16(const bf16* __restrict__ base, long ld, int outer, int inner,
                                          int outer_lim, int inner_lim, bool vec) {
  uint4 r = make_uint4(0, 0, 0, 0);
  if (outer >= outer_lim) return r;
  const bf16* p = base + (long)outer * ld + inner;
  if (vec && inner + 8 <= inner_lim) return *reinterpret_cast<const uint4*>(p);
  unsigned short tmp[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) tmp[e] = (inner + e < inner_lim) ? reinterpret_cast<const unsigned short*>(p)[e] : 0;
  r.x = tmp[0] | (tmp[1] << 16); r.y = tmp[2] | (tmp[3] << 16);
  r.z = tmp[4] | (tmp[5] << 16); r.w = tmp[6] | (tmp[7] << 16);
  return r;
}
__device__ __forceinline__ float4 ld4_f32(const float* __restrict__ base, long ld, int outer, int inner,
                                          int outer_lim, int inner_lim, bool vec) {
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (outer >= outer_lim) return r;
  const float* p = base + (long)outer * ld + inner;
  if (vec && inner + 4 <= inner_lim) return *reinterpret_cast<const float4*>(p);
  float t[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) t[e] = (inner + e < inner_lim) ? p[e] : 0.f;
  return make_float4(t[0], t[1], t[2], t[3]);
}

// bf16 LDS geometry (elements)
constexpr int BK16 = 32;
constexpr int KM_STRIDE = BK16 + 8;        // K-major tile [128][40]: 80-B rows, conflict-free b128
constexpr int MN_STRIDE = 128 + 32;        // MN-major tile [32][160]: 320-B rows, conflict-free tr16
constexpr int TILE16 = 128 * KM_STRIDE;    // 5120 elements = 10 KiB (== 32*160)
static_assert(TILE16 == BK16 * MN_STRIDE, "both layouts use the same LDS footprint");

// fp32 LDS geometry: both operands stored [BK][128+4] (k-rows)
constexpr int BK32 = 16;
constexpr int F_STRIDE = 128 + 4;
constexpr int TILE32 = BK32 * F_STRIDE;

// Read one 32x32x16 operand fragment (8 bf16) from a staged tile.
// row0: first row (m or n) of the 32-row MFMA block inside the tile; kk: k offset (0 / 16).
template <bool KMAJOR>
__device__ __forceinline__ bf16x8 frag16(const bf16* tile, int row0, int kk, int lane) {
  if constexpr (KMAJOR) {
    const bf16* p = tile + (row0 + (lane & 31)) * KM_STRIDE + kk + 8 * (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    const int h = lane >> 5, g1 = (lane >> 4) & 1, q = (lane & 15) >> 2, p4 = lane & 3;
    const bf16* base = tile + (kk + 8 * h + q) * MN_STRIDE + row0 + 16 * g1 + 4 * p4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + 4 * MN_STRIDE));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

__device__ __forceinline__ void epilogue_store(const GemmP& p, int z, int m, int n, float acc) {
  if (m >= p.M || n >= p.N) return;
  const long cidx = (long)z * p.sc + (long)m * p.ldc + n;
  float v = acc * p.alpha;
  if (p.split_k > 1) {
    if (p.bias && blockIdx.z % p.split_k == 0) v += p.bias[n];
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

// ---------------------------------------------------------------- bf16 kernel
template <bool AK, bool BKM>
__global__ __launch_bounds__(NT) void gemm_bf16_kernel(GemmP p) {
  __shared__ __attribute__((aligned(16))) bf16 lds[4 * TILE16];   // [buf][A,B] 40 KiB
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int z = blockIdx.z / p.split_k, ks = blockIdx.z % p.split_k;
  const bf16* A = reinterpret_cast<const bf16*>(p.A) + (long)z * p.sa;
  const bf16* B = reinterpret_cast<const bf16*>(p.B) + (long)z * p.sb;
  const int kbeg = ks * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + BK16 - 1) / BK16 : 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0};

  uint4 ra[2], rb[2];
  auto gload = [&](int kt) {
    const int k0 = kbeg + kt * BK16;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + NT * i;
      if constexpr (AK) ra[i] = ld8_bf16(A, p.lda, m0 + (v >> 2), k0 + (v & 3) * 8, p.M, kend, p.vec_a);
      else ra[i] = ld8_bf16(A, p.lda, k0 + (v >> 4), m0 + (v & 15) * 8, kend, p.M, p.vec_a);
      if constexpr (BKM) rb[i] = ld8_bf16(B, p.ldb, n0 + (v >> 2), k0 + (v & 3) * 8, p.N, kend, p.vec_b);
      else rb[i] = ld8_bf16(B, p.ldb, k0 + (v >> 4), n0 + (v & 15) * 8, kend, p.N, p.vec_b);
    }
  };
  auto sstore = [&](int buf) {
    bf16* ta = lds + buf * 2 * TILE16;
    bf16* tb = ta + TILE16;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + NT * i;
      bf16* da = AK ? ta + (v >> 2) * KM_STRIDE + (v & 3) * 8 : ta + (v >> 4) * MN_STRIDE + (v & 15) * 8;
      bf16* db = BKM ? tb + (v >> 2) * KM_STRIDE + (v & 3) * 8 : tb + (v >> 4) * MN_STRIDE + (v & 15) * 8;
      *reinterpret_cast<uint4*>(da) = ra[i];
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
    const bf16* ta = lds + cur * 2 * TILE16;
    const bf16* tb = ta + TILE16;
#pragma unroll
    for (int kk = 0; kk < BK16; kk += 16) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = frag16<AK>(ta, wm * 64 + i * 32, kk, lane);
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

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int n = n0 + wn * 64 + j * 32 + (lane & 31);
        epilogue_store(p, z, m, n, acc[i][j][r]);
      }
}

// ---------------------------------------------------------------- fp32 kernel (exact-f32 MFMA)
template <bool AK, bool BKM>
__global__ __launch_bounds__(NT) void gemm_f32_kernel(GemmP p) {
  __shared__ __attribute__((aligned(16))) float lds[4 * TILE32];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int z = blockIdx.z / p.split_k, ks = blockIdx.z % p.split_k;
  const float* A = reinterpret_cast<const float*>(p.A) + (long)z * p.sa;
  const float* B = reinterpret_cast<const float*>(p.B) + (long)z * p.sb;
  const int kbeg = ks * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + BK32 - 1) / BK32 : 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0};

  float4 ra[2], rb[2];
  // tile = 16 k x 128 rows = 512 float4
  auto gload = [&](int kt) {
    const int k0 = kbeg + kt * BK32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + NT * i;
      if constexpr (AK) ra[i] = ld4_f32(A, p.lda, m0 + (v >> 2), k0 + (v & 3) * 4, p.M, kend, p.vec_a);
      else ra[i] = ld4_f32(A, p.lda, k0 + (v >> 5), m0 + (v & 31) * 4, kend, p.M, p.vec_a);
      if constexpr (BKM) rb[i] = ld4_f32(B, p.ldb, n0 + (v >> 2), k0 + (v & 3) * 4, p.N, kend, p.vec_b);
      else rb[i] = ld4_f32(B, p.ldb, k0 + (v >> 5), n0 + (v & 31) * 4, kend, p.N, p.vec_b);
    }
  };
  auto put = [&](float* t, bool kmaj, int v, float4 r) {
    if (kmaj) {
      const int row = v >> 2, kc = (v & 3) * 4;
      t[(kc + 0) * F_STRIDE + row] = r.x;
      t[(kc + 1) * F_STRIDE + row] = r.y;
      t[(kc + 2) * F_STRIDE + row] = r.z;
      t[(kc + 3) * F_STRIDE + row] = r.w;
    } else {
      *reinterpret_cast<float4*>(t + (v >> 5) * F_STRIDE + (v & 31) * 4) = r;
    }
  };
  auto sstore = [&](int buf) {
    float* ta = lds + buf * 2 * TILE32;
    float* tb = ta + TILE32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
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
    const float* ta = lds + cur * 2 * TILE32;
    const float* tb = ta + TILE32;
#pragma unroll
    for (int kk = 0; kk < BK32; kk += 2) {
      const int kr = kk + (lane >> 5);
      float af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = ta[kr * F_STRIDE + wm * 64 + i * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = tb[kr * F_STRIDE + wn * 64 + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int n = n0 + wn * 64 + j * 32 + (lane & 31);
        epilogue_store(p, z, m, n, acc[i][j][r]);
      }
}

template <typename F>
void launch4(bool ak, bool bk, F f) {
  if (ak && bk) f(std::integral_constant<int, 3>{});
  else if (ak) f(std::integral_constant<int, 2>{});
  else if (bk) f(std::integral_constant<int, 1>{});
  else f(std::integral_constant<int, 0>{});
}

}  // namespace

CFM_EXPORT int cfm_gemm(const cfm_gemm_desc* d, void* stream) {
  CFM_REQUIRE(d != nullptr, CFM_ERR_ARG, "null descriptor");
  CFM_REQUIRE(d->M >= 0 && d->N >= 0 && d->K >= 0 && d->batch >= 1, CFM_ERR_SHAPE, "bad M/N/K/batch");
  CFM_REQUIRE(d->dtype_ab == CFM_F32 || d->dtype_ab == CFM_BF16, CFM_ERR_DTYPE, "dtype_ab");
  CFM_REQUIRE(d->A && d->B && d->C, CFM_ERR_ARG, "null operand");
  CFM_REQUIRE(d->act == CFM_ACT_NONE || d->act == CFM_ACT_SILU, CFM_ERR_ARG, "act");
  CFM_REQUIRE(!d->act_grad || d->pre, CFM_ERR_ARG, "act_grad needs pre");
  const int split = d->split_k < 1 ? 1 : d->split_k;
  CFM_REQUIRE(split == 1 || (d->dtype_c == CFM_F32 && d->act == CFM_ACT_NONE && !d->act_grad &&
                             !d->residual && d->drop_p <= 0.f),
              CFM_ERR_ARG, "split_k needs a plain fp32 epilogue");
  CFM_REQUIRE(d->a_kmajor ? d->lda >= d->K : d->lda >= d->M, CFM_ERR_SHAPE, "lda");
  CFM_REQUIRE(d->b_kmajor ? d->ldb >= d->K : d->ldb >= d->N, CFM_ERR_SHAPE, "ldb");
  CFM_REQUIRE(d->ldc >= d->N, CFM_ERR_SHAPE, "ldc");
  if (d->M == 0 || d->N == 0) return CFM_OK;

  GemmP p;
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.A = d->A; p.lda = d->lda; p.sa = d->stride_a;
  p.B = d->B; p.ldb = d->ldb; p.sb = d->stride_b;
  p.C = d->C; p.ldc = d->ldc; p.sc = d->stride_c; p.dtc = d->dtype_c;
  p.alpha = d->alpha; p.bias = d->bias; p.act = d->act; p.act_grad = d->act_grad;
  p.pre = d->pre; p.dtpre = d->dtype_pre;
  p.drop_p = d->drop_p; p.seed = d->drop_seed; p.doff = d->drop_offset;
  p.out_scale = d->out_scale; p.res = d->residual; p.ldr = d->ldr; p.dtr = d->dtype_r;
  p.split_k = split;
  const int bk = d->dtype_ab == CFM_BF16 ? BK16 : BK32;
  p.k_per_split = ((d->K + split - 1) / split + bk - 1) / bk * bk;
  const int esz = d->dtype_ab == CFM_BF16 ? 2 : 4;
  const int vlen = 16 / esz;
  p.vec_a = ((uintptr_t)d->A % 16 == 0) && (d->lda % vlen == 0) && (d->stride_a % vlen == 0);
  p.vec_b = ((uintptr_t)d->B % 16 == 0) && (d->ldb % vlen == 0) && (d->stride_b % vlen == 0);

  dim3 grid(cdiv(d->N, BN), cdiv(d->M, BM), d->batch * split);
  CFM_REQUIRE(grid.y <= 65535 && grid.z <= 65535, CFM_ERR_SHAPE, "grid too large");
  hipStream_t s = cfm::as_stream(stream);
  const bool ak = d->a_kmajor != 0, bkm = d->b_kmajor != 0;
  if (d->dtype_ab == CFM_BF16) {
    launch4(ak, bkm, [&](auto c) {
      constexpr int v = decltype(c)::value;
      hipLaunchKernelGGL((gemm_bf16_kernel<(v & 2) != 0, (v & 1) != 0>), grid, dim3(NT), 0, s, p);
    });
  } else {
    launch4(ak, bkm, [&](auto c) {
      constexpr int v = decltype(c)::value;
      hipLaunchKernelGGL((gemm_f32_kernel<(v & 2) != 0, (v & 1) != 0>), grid, dim3(NT), 0, s, p);
    });
  }
  return cfm::check_launch("cfm_gemm");
}
