// convsub.hip — first subsampling convolution (lib/convsubsampling.py:21, Conv2d(1 -> C1, 7x7,
// stride 2, no padding)) forward and weight-gradient.
//
// The input has ONE channel, so this is 49 MACs per output: HBM-write-bound (C1 = 512 outputs
// per input pixel pair).  Output is NHWC (B, F1, T1, C1) in the compute dtype so that the
// second convolution (implicit GEMM in gemm.hip) reads 16-byte channel chunks.
// Forward: one workgroup per (b, f1, 32-frame tile); the 7 x 69 input patch sits in LDS (all
// lanes read the same pixel: LDS broadcast), each thread owns up to 2 channels with their 49
// taps in registers; stores are 1 KiB-coalesced channel rows.  (VALU-bound: 49 FMAs per output;
// an MFMA im2col form is the next step.)  The weight-gradient stages the block's [32][C1] dh1 rows
// (one contiguous run in NHWC) in LDS with 16-byte loads and keeps the 7x7 input window in registers.
// Weight-gradient: a persistent grid sweeps (b, f1) rows; each thread accumulates 49 tap sums +
// the bias sum for its channels in registers; per-workgroup partials are reduced by a second
// kernel (deterministic).
#include "cfm_common.h"

namespace {
constexpr int KK = 7, ST = 2, TW = 32;   // kernel, stride, output frames per workgroup
constexpr int PW = (TW - 1) * ST + KK;   // 69 input columns per patch
constexpr int CMAX = 512;                // channels supported (2 per thread)

// the 7x7 input window of output frame tt slides by 2 columns per frame: keep it in registers
// (fully unrolled frame loop -> the shifts are register renames) so each frame costs 14 LDS
// broadcast reads for 98 FMAs instead of 49
template <typename TO>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, TO* __restrict__ h1, int F,
                                                        int T, int C1, int F1, int T1) {
  __shared__ float patch[KK][PW + 1];
  const int tid = threadIdx.x;
  const int t10 = blockIdx.x * TW, f1 = blockIdx.y, b = blockIdx.z;
  const float* xb = x + (long)b * F * T;
  for (int i = tid; i < KK * PW; i += 256) {
    const int r = i / PW, cc = i % PW;
    const int fr = ST * f1 + r, tc = ST * t10 + cc;
    patch[r][cc] = (tc < T) ? xb[(long)fr * T + tc] : 0.f;
  }
  float wr[2][KK * KK], bb[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int c = tid + 256 * q;
#pragma unroll
    for (int k = 0; k < KK * KK; ++k) wr[q][k] = c < C1 ? w[c * KK * KK + k] : 0.f;
    bb[q] = c < C1 ? bias[c] : 0.f;
  }
  __syncthreads();
  const int nt = min(TW, T1 - t10);
  for (int tt = 0; tt < nt; ++tt) {
    float a0 = bb[0], a1 = bb[1];
#pragma unroll
    for (int kh = 0; kh < KK; ++kh)
#pragma unroll
      for (int kw = 0; kw < KK; ++kw) {
        const float v = patch[kh][ST * tt + kw];
        a0 += wr[0][kh * KK + kw] * v;
        a1 += wr[1][kh * KK + kw] * v;
      }
    TO* row = h1 + (((long)b * F1 + f1) * T1 + t10 + tt) * C1;
    if (tid < C1) row[tid] = from_f32<TO>(a0);
    if (tid + 256 < C1) row[tid + 256] = from_f32<TO>(a1);
  }
}

// partial dW: ws[blk][c][50] (49 taps + bias)
template <typename TI>
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(const TI* __restrict__ dh1, const float* __restrict__ x,
                                                          int B, int F, int T, int C1, int F1, int T1,
                                                          float* __restrict__ ws) {
  __shared__ float patch[KK][PW + 1];
  __shared__ __attribute__((aligned(16))) TI stage[TW * CMAX];   // the block's [nt][C1] dh1 rows
  const int tid = threadIdx.x;
  float acc[2][KK * KK + 1];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int k = 0; k <= KK * KK; ++k) acc[q][k] = 0.f;
  const int ntile = (T1 + TW - 1) / TW;
  const long nwork = (long)B * F1 * ntile;
  for (long wi = blockIdx.x; wi < nwork; wi += gridDim.x) {
    const int tile = (int)(wi % ntile);
    const long bf = wi / ntile;
    const int f1 = (int)(bf % F1), b = (int)(bf / F1);
    const int t10 = tile * TW;
    __syncthreads();
    const float* xb = x + (long)b * F * T;
    for (int i = tid; i < KK * PW; i += 256) {
      const int r = i / PW, cc = i % PW;
      const int tc = ST * t10 + cc;
      patch[r][cc] = (tc < T) ? xb[(long)(ST * f1 + r) * T + tc] : 0.f;
    }
    const int nt = min(TW, T1 - t10);
    {
      const TI* src = dh1 + (((long)b * F1 + f1) * T1 + t10) * C1;
      const long n = (long)nt * C1;
      constexpr int V = 16 / sizeof(TI);
      if ((C1 % V) == 0 && ((uintptr_t)src % 16) == 0) {
        for (long i = (long)tid * V; i < n; i += 256 * V)
          *reinterpret_cast<uint4*>(stage + i) = *reinterpret_cast<const uint4*>(src + i);
      } else {
        for (long i = tid; i < n; i += 256) stage[i] = src[i];
      }
    }
    __syncthreads();
    float win[KK][KK];
#pragma unroll
    for (int r = 0; r < KK; ++r)
#pragma unroll
      for (int q = 0; q < KK; ++q) win[r][q] = patch[r][q];
#pragma nounroll
    for (int tt = 0; tt < TW; ++tt) {   // (not unrolled: win[][] is statically indexed inside the body)
      if (tt >= nt) break;
      if (tt > 0) {
#pragma unroll
        for (int r = 0; r < KK; ++r) {
#pragma unroll
          for (int q = 0; q < KK - ST; ++q) win[r][q] = win[r][q + ST];
          win[r][KK - 2] = patch[r][ST * tt + KK - 2];
          win[r][KK - 1] = patch[r][ST * tt + KK - 1];
        }
      }
      const float g0 = 2 * tid < C1 ? to_f32(stage[tt * C1 + 2 * tid]) : 0.f;
      const float g1 = 2 * tid + 1 < C1 ? to_f32(stage[tt * C1 + 2 * tid + 1]) : 0.f;
#pragma unroll
      for (int kh = 0; kh < KK; ++kh)
#pragma unroll
        for (int kw = 0; kw < KK; ++kw) {
          acc[0][kh * KK + kw] += g0 * win[kh][kw];
          acc[1][kh * KK + kw] += g1 * win[kh][kw];
        }
      acc[0][KK * KK] += g0;
      acc[1][KK * KK] += g1;
    }
  }
  float* out = ws + (long)blockIdx.x * C1 * (KK * KK + 1);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int c = 2 * tid + q;
    if (c < C1)
#pragma unroll
      for (int k = 0; k <= KK * KK; ++k) out[(long)c * (KK * KK + 1) + k] = acc[q][k];
  }
}

__global__ void conv1_wgrad_reduce(const float* __restrict__ ws, int nblk, int C1, float* __restrict__ dw,
                                   float* __restrict__ db) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int per = KK * KK + 1;
  if (i >= C1 * per) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += ws[(long)b * C1 * per + i];
  const int c = i / per, k = i % per;
  if (k < KK * KK) dw[c * KK * KK + k] = (float)s;
  else if (db) db[c] = (float)s;
}

// ---------------------------------------------------------------- MFMA forms (bf16 h1, C1 = 512)
// The same two convolutions as GEMMs on the matrix cores: a tile is 32 consecutive output frames
// of one (b, f1) row, i.e. 32 contiguous NHWC rows of 512 channels (32 KiB of bf16).
//   forward:  C[c][t] = sum_k W[c][k] * P[k][t]      (M = channels, N = frames, K = taps)
//   wgrad:    dW[c][k] += sum_t dh1[t][c] * P[k][t]  (M = channels, N = taps, K = frames)
// where P[k][t] = x[b][2 f1 + kh][2 (t0 + t) + kw] for tap k = 7 kh + kw < 49.  x (fp32) enters as
// hi + lo bf16 halves (two MFMA passes over the same weights: x is carried to ~16 mantissa
// bits), so the only rounding beyond the fp32 path is that of W (forward) or of dh1 (wgrad).
// The bias rides along as extra taps: forward W[c][49] = bf16(b), W[c][50] = bf16(b - bf16(b)) against
// P = 1 (hi pass); wgrad P[49][t] = 1 so dW[c][49] = sum_t dh1[t][c] = db.
// Every launch is persistent (grid <= 2 workgroups per CU); each workgroup sweeps tiles
// blockIdx.x, blockIdx.x + gridDim.x, ...
constexpr int MT = 32;                       // frames per tile
constexpr int MPW = (MT - 1) * ST + KK;      // 69 input columns per tile
constexpr int MPS = 72;                      // patch row stride (floats)
constexpr int MC = 512;                      // channels (4 waves x 128)
constexpr int FSTR = MC + 8;                 // forward staging row stride (bf16): 2-way-free b64 writes

__device__ __forceinline__ void load_patch(float (*patch)[MPS], const float* __restrict__ xb, int f1, int t0, int T,
                                           int tid) {
  for (int i = tid; i < KK * MPW; i += 256) {
    const int r = i / MPW, cc = i % MPW;
    const int tc = ST * t0 + cc;
    patch[r][cc] = (tc < T) ? xb[(long)(ST * f1 + r) * T + tc] : 0.f;
  }
}

// hi / lo bf16 halves of one P fragment: 8 taps k0..k0+7 (k0 % 8 == 0) at frame t, or 8 frames
// t0..t0+7 at tap k (wgrad); `one_at` = the tap that reads as constant 1 in the hi half (or -1)
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bf16 h = (bf16)v[e];
    hi[e] = h;
    lo[e] = (bf16)(v[e] - (float)h);
  }
}

__global__ __launch_bounds__(256, 2) void conv1_fwd_mfma_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ bias,
                                                                bf16* __restrict__ h1, int F, int T, int F1, int T1,
                                                                int ntile_t, long ntiles) {
  __shared__ __attribute__((aligned(16))) bf16 stage[MT * FSTR];
  __shared__ float patch[KK][MPS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l31 = lane & 31, hh = lane >> 5;
  // weight fragments (A operand: rows = channels, k = taps), loaded once per workgroup
  bf16x8 wa[4][4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int c = wid * 128 + f * 32 + l31;
    const float b = bias[c];
    const bf16 bh = (bf16)b;
    const bf16 bl = (bf16)(b - (float)bh);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = s4 * 16 + 8 * hh + e;
        wa[f][s4][e] = k < 49 ? (bf16)w[c * 49 + k] : (k == 49 ? bh : (k == 50 ? bl : (bf16)0.f));
      }
  }
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int tt = (int)(tile % ntile_t);
    const long bf = tile / ntile_t;
    const int f1 = (int)(bf % F1), b = (int)(bf / F1);
    const int t0 = tt * MT;
    load_patch(patch, x + (long)b * F * T, f1, t0, T, tid);
    __syncthreads();
    // P fragments (B operand: k = taps, col = frame l31)
    bf16x8 ph[4], pl[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = s4 * 16 + 8 * hh + e;
        const int kh = k / 7, kw = k % 7;
        v[e] = k < 49 ? patch[kh][ST * l31 + kw] : (k < 51 ? 1.f : 0.f);
      }
      split8(v, ph[s4], pl[s4]);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (s4 * 16 + 8 * hh + e >= 49) pl[s4][e] = (bf16)0.f;
    }
    f32x16 acc[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[f] = (f32x16){0};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[f][s4], ph[s4], acc[f], 0, 0, 0);
        acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[f][s4], pl[s4], acc[f], 0, 0, 0);
      }
    // accumulator -> LDS [frame][channel] bf16 (4 consecutive channels per 8-B write)
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = wid * 128 + f * 32 + 8 * g + 4 * hh;
        bf16x4 v4 = {(bf16)acc[f][4 * g], (bf16)acc[f][4 * g + 1], (bf16)acc[f][4 * g + 2], (bf16)acc[f][4 * g + 3]};
        *reinterpret_cast<bf16x4*>(stage + l31 * FSTR + c) = v4;
      }
    __syncthreads();
    // 32 contiguous NHWC rows: 1 KiB per wave-instruction of 16-B stores
    bf16* dst = h1 + (((long)b * F1 + f1) * T1 + t0) * MC;
    const int nt = min(MT, T1 - t0);
#pragma unroll
    for (int it = 0; it < MT * MC / 8 / 256; ++it) {
      const int id = it * 256 + tid, r = id >> 6, cc = id & 63;
      if (r < nt)
        *reinterpret_cast<uint4*>(dst + (long)r * MC + cc * 8) = *reinterpret_cast<const uint4*>(stage + r * FSTR + cc * 8);
    }
    __syncthreads();
  }
}

// dh1 tile image for transposed reads: [frame][512] bf16, 16-B chunk c of frame row t at slot
// c ^ (4 (t & 3)) (conflict-free ds_read_b64_tr_b16, as gemm.hip's MN-major stage images)
__device__ __forceinline__ bf16x8 dh1_frag(const bf16* img, int c0, int k0, int lane) {
  const int h = lane >> 5, g1 = (lane >> 4) & 1, q = (lane & 15) >> 2, p4 = lane & 3;
  const int col = c0 + 16 * g1 + 4 * p4, k = k0 + 8 * h + q;
  const int off = 8 * ((col >> 3) ^ (4 * q)) + (col & 7);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(img + k * MC + off));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(img + (k + 4) * MC + off));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// partial dW / db per workgroup: ws[blk][c][50] (49 taps + bias), the layout conv1_wgrad_reduce sums
__global__ __launch_bounds__(256, 2) void conv1_wgrad_mfma_kernel(const bf16* __restrict__ dh1,
                                                                  const float* __restrict__ x, int F, int T, int F1,
                                                                  int T1, int ntile_t, long ntiles,
                                                                  float* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) bf16 img[MT * MC];
  __shared__ float patch[KK][MPS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l31 = lane & 31, hh = lane >> 5;
  f32x16 acc[4][2];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[f][j] = (f32x16){0};
  constexpr int NV = MT * MC / 8 / 256;   // 16-B chunks per thread per tile (8)
  uint4 pf[NV];
  auto fetch = [&](long tile) {
    const int tt = (int)(tile % ntile_t);
    const long bf = tile / ntile_t;
    const int f1 = (int)(bf % F1), b = (int)(bf / F1), t0 = tt * MT;
    const int nt = min(MT, T1 - t0);
    const bf16* src = dh1 + (((long)b * F1 + f1) * T1 + t0) * MC;
#pragma unroll
    for (int it = 0; it < NV; ++it) {
      const int id = it * 256 + tid, r = id >> 6, cc = id & 63;
      pf[it] = r < nt ? *reinterpret_cast<const uint4*>(src + (long)r * MC + cc * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  long tile = blockIdx.x;
  if (tile < ntiles) fetch(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    const int tt = (int)(tile % ntile_t);
    const long bf = tile / ntile_t;
    const int f1 = (int)(bf % F1), b = (int)(bf / F1), t0 = tt * MT;
    const int nt = min(MT, T1 - t0);
    __syncthreads();   // previous tile's reads of img / patch are done
#pragma unroll
    for (int it = 0; it < NV; ++it) {
      const int id = it * 256 + tid, r = id >> 6, cc = id & 63;
      *reinterpret_cast<uint4*>(img + r * MC + 8 * (cc ^ (4 * (r & 3)))) = pf[it];
    }
    load_patch(patch, x + (long)b * F * T, f1, t0, T, tid);
    __syncthreads();
    if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);   // in flight under this tile's MFMAs
    // per 16-frame k-step: P fragments (B operand: rows k = frames, cols = taps j*32 + l31), then
    // the 4 channel fragments of this wave (frames >= nt read 0 from dh1)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 ph[2], pl[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = j * 32 + l31, kh = k / 7, kw = k % 7;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int t = ks * 16 + 8 * hh + e;
          v[e] = k < 49 ? patch[kh][ST * t + kw] : (k == 49 ? 1.f : 0.f);
        }
        split8(v, ph[j], pl[j]);
      }
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const bf16x8 a = dh1_frag(img, wid * 128 + f * 32, ks * 16, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[f][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, ph[j], acc[f][j], 0, 0, 0);
          acc[f][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pl[j], acc[f][j], 0, 0, 0);
        }
      }
    }
    (void)nt;
  }
  float* out = ws + (long)blockIdx.x * MC * (KK * KK + 1);
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = j * 32 + l31;
      if (k <= KK * KK)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = wid * 128 + f * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          out[(long)c * (KK * KK + 1) + k] = acc[f][j][r];
        }
    }
}

// deterministic partial sum: 64 outputs per workgroup, 4 fixed block strides summed in order
__global__ __launch_bounds__(256) void conv1_wgrad_reduce2(const float* __restrict__ ws, int nblk, int C1,
                                                           float* __restrict__ dw, float* __restrict__ db) {
  __shared__ double part[4][64];
  const int per = KK * KK + 1, n = C1 * per;
  const int o = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + o;
  double s = 0.0;
  if (i < n)
    for (int b = g; b < nblk; b += 4) s += ws[(long)b * n + i];
  part[g][o] = s;
  __syncthreads();
  if (g == 0 && i < n) {
    const double t = part[0][o] + part[1][o] + part[2][o] + part[3][o];
    const int c = i / per, k = i % per;
    if (k < KK * KK) dw[c * KK * KK + k] = (float)t;
    else if (db) db[c] = (float)t;
  }
}

constexpr int MFMA_BLOCKS = 512;     // persistent grids: 2 workgroups per CU
constexpr int WGRAD_BLOCKS = 512;   // 2 workgroups per CU (174 VGPRs)
}  // namespace

CFM_EXPORT int cfm_conv1_fwd(const float* x, const float* w1, const float* b1, void* h1, int dtype_h, int B, int F,
                             int T, int C1, void* stream) {
  CFM_REQUIRE(x && w1 && b1 && h1, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(C1 > 0 && C1 <= CMAX, CFM_ERR_UNSUPPORTED, "conv1 supports up to 512 channels");
  CFM_REQUIRE(F >= KK && T >= KK && B > 0, CFM_ERR_SHAPE, "input smaller than the 7x7 kernel");
  const int F1 = (F - KK) / ST + 1, T1 = (T - KK) / ST + 1;
  CFM_REQUIRE(F1 <= 65535, CFM_ERR_SHAPE, "too many mel bins");
  dim3 grid(cdiv(T1, TW), F1, B);
  hipStream_t s = cfm::as_stream(stream);
  if (dtype_h == CFM_BF16 && C1 == MC) {
    const int ntt = cdiv(T1, MT);
    const long ntiles = (long)B * F1 * ntt;
    const int nblk = (int)(ntiles < MFMA_BLOCKS ? ntiles : MFMA_BLOCKS);
    hipLaunchKernelGGL(conv1_fwd_mfma_kernel, dim3(nblk), dim3(256), 0, s, x, w1, b1, (bf16*)h1, F, T, F1, T1, ntt,
                       ntiles);
  } else if (dtype_h == CFM_BF16)
    hipLaunchKernelGGL(conv1_fwd_kernel<bf16>, grid, dim3(256), 0, s, x, w1, b1, (bf16*)h1, F, T, C1, F1, T1);
  else
    hipLaunchKernelGGL(conv1_fwd_kernel<float>, grid, dim3(256), 0, s, x, w1, b1, (float*)h1, F, T, C1, F1, T1);
  return cfm::check_launch("cfm_conv1_fwd");
}

CFM_EXPORT size_t cfm_conv1_bwd_ws_bytes(int B, int F, int T, int C1) {
  (void)B; (void)F; (void)T;
  const int nb = WGRAD_BLOCKS > MFMA_BLOCKS ? WGRAD_BLOCKS : MFMA_BLOCKS;
  return (size_t)nb * C1 * (KK * KK + 1) * sizeof(float);
}

CFM_EXPORT int cfm_conv1_bwd_weight(const void* dh1, int dtype_h, const float* x, float* dw1, float* db1, int B, int F,
                                    int T, int C1, float* ws, void* stream) {
  CFM_REQUIRE(dh1 && x && dw1 && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(C1 > 0 && C1 <= CMAX, CFM_ERR_UNSUPPORTED, "conv1 supports up to 512 channels");
  const int F1 = (F - KK) / ST + 1, T1 = (T - KK) / ST + 1;
  const long nwork = (long)B * F1 * cdiv(T1, TW);
  const int nblk = (int)(nwork < WGRAD_BLOCKS ? nwork : WGRAD_BLOCKS);
  hipStream_t s = cfm::as_stream(stream);
  if (dtype_h == CFM_BF16 && C1 == MC) {
    const int ntt = cdiv(T1, MT);
    const long ntiles = (long)B * F1 * ntt;
    const int nb = (int)(ntiles < MFMA_BLOCKS ? ntiles : MFMA_BLOCKS);
    hipLaunchKernelGGL(conv1_wgrad_mfma_kernel, dim3(nb), dim3(256), 0, s, (const bf16*)dh1, x, F, T, F1, T1, ntt,
                       ntiles, ws);
    hipLaunchKernelGGL(conv1_wgrad_reduce2, dim3(cdiv((long)C1 * (KK * KK + 1), 64)), dim3(256), 0, s, ws, nb, C1,
                       dw1, db1);
    return cfm::check_launch("cfm_conv1_bwd_weight");
  }
  if (dtype_h == CFM_BF16)
    hipLaunchKernelGGL(conv1_wgrad_kernel<bf16>, dim3(nblk), dim3(256), 0, s, (const bf16*)dh1, x, B, F, T, C1, F1,
                       T1, ws);
  else
    hipLaunchKernelGGL(conv1_wgrad_kernel<float>, dim3(nblk), dim3(256), 0, s, (const float*)dh1, x, B, F, T, C1, F1,
                       T1, ws);
  hipLaunchKernelGGL(conv1_wgrad_reduce, dim3(cdiv((long)C1 * (KK * KK + 1), 256)), dim3(256), 0, s, ws, nblk, C1,
                     dw1, db1);
  return cfm::check_launch("cfm_conv1_bwd_weight");
}
