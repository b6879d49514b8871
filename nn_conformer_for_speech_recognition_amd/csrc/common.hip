// common.hip — error plumbing, version, dtype casts and small elementwise kernels.
#include "cfm_common.h"

#include <type_traits>

namespace cfm {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CFM_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e));
  return CFM_OK;
}
}  // namespace cfm

namespace cfm {
const uint64_t* g_rng_salt = nullptr;
}

CFM_EXPORT int cfm_version(void) { return 1; }

CFM_EXPORT int cfm_rng_bind(const uint64_t* counter) {
  cfm::g_rng_salt = counter;
  return CFM_OK;
}
CFM_EXPORT const char* cfm_get_last_error(void) { return cfm::g_last_error.c_str(); }

namespace {
template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ x, TO* __restrict__ y, long n) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long stride = (long)gridDim.x * blockDim.x * 4;
  for (; i < n; i += stride) {
    if (i + 4 <= n) {
#pragma unroll
      for (int e = 0; e < 4; ++e) y[i + e] = from_f32<TO>(to_f32(x[i + e]));
    } else {
      for (long e = i; e < n; ++e) y[e] = from_f32<TO>(to_f32(x[e]));
    }
  }
}

__global__ void scale_dropout_kernel(const void* x, int dtx, void* y, int dty, long n, float scale,
                                     float p, uint64_t seed, uint64_t off, const uint64_t* salt) {
  if (p > 0.f) seed = salted_seed(seed, salt);
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    float v = ld_dyn(x, dtx, i) * scale;
    if (p > 0.f) v *= dropout_scale(p, seed, off + (uint64_t)i);
    st_dyn(y, dty, i, v);
  }
}
// 8 elements per thread (n % 8 == 0, 16-B aligned x / y)
__global__ void scale_dropout8_kernel(const void* x, int dtx, void* y, int dty, long n8, float scale,
                                      float p, uint64_t seed, uint64_t off, const uint64_t* salt) {
  if (p > 0.f) seed = salted_seed(seed, salt);
  for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < n8; q += (long)gridDim.x * blockDim.x) {
    float v[8], s[8];
    ld8_dyn(x, dtx, q * 8, v);
    if (p > 0.f) dropout_scale8(p, seed, off + (uint64_t)(q * 8), s);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= p > 0.f ? scale * s[e] : scale;
    st8_dyn(y, dty, q * 8, v);
  }
}
}  // namespace

static int grid_for(long n, int per_thread) {
  long blocks = (n / per_thread + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 8192) blocks = 8192;
  return (int)blocks;
}

CFM_EXPORT int cfm_cast(const void* x, int dtx, void* y, int dty, long n, void* stream) {
  CFM_REQUIRE(x && y && n >= 0, CFM_ERR_ARG, "bad args");
  if (n == 0) return CFM_OK;
  hipStream_t s = cfm::as_stream(stream);
  dim3 g(grid_for(n, 4)), b(256);
  if (dtx == CFM_F32 && dty == CFM_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16>), g, b, 0, s, (const float*)x, (bf16*)y, n);
  else if (dtx == CFM_BF16 && dty == CFM_F32)
    hipLaunchKernelGGL((cast_kernel<bf16, float>), g, b, 0, s, (const bf16*)x, (float*)y, n);
  else if (dtx == CFM_F32 && dty == CFM_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), g, b, 0, s, (const float*)x, (float*)y, n);
  else if (dtx == CFM_BF16 && dty == CFM_BF16)
    hipLaunchKernelGGL((cast_kernel<bf16, bf16>), g, b, 0, s, (const bf16*)x, (bf16*)y, n);
  else
    return cfm::fail(CFM_ERR_DTYPE, "cfm_cast: dtype");
  return cfm::check_launch("cfm_cast");
}

namespace {
constexpr int CAST_BLK = 2048;   // elements per block (256 threads x 8)
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void cast_batch_kernel(const cfm_cast_task* __restrict__ tasks, int ntasks) {
  // the task owning this block: last t with blk0 <= blockIdx.x (binary search, wave-uniform)
  int lo = 0, hi = ntasks - 1;
  const long b = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tasks[mid].blk0 <= b) lo = mid; else hi = mid - 1;
  }
  const cfm_cast_task t = tasks[lo];
  const long e0 = (b - t.blk0) * CAST_BLK + threadIdx.x * 8;
  const TI* x = reinterpret_cast<const TI*>(t.src);
  TO* y = reinterpret_cast<TO*>(t.dst);
  if (e0 + 8 <= t.n && ((uintptr_t)(x + e0) % 16 == 0) && ((uintptr_t)(y + e0) % 16 == 0)) {
    float v[8];
    ld8_dyn(x, std::is_same<TI, bf16>::value ? CFM_BF16 : CFM_F32, e0, v);
    st8_dyn(y, std::is_same<TO, bf16>::value ? CFM_BF16 : CFM_F32, e0, v);
  } else {
    for (long e = e0; e < e0 + 8 && e < t.n; ++e) y[e] = from_f32<TO>(to_f32(x[e]));
  }
}
}  // namespace

CFM_EXPORT int cfm_cast_batch(const cfm_cast_task* tasks, int ntasks, long nblocks, int dtx, int dty,
                              void* stream) {
  CFM_REQUIRE(tasks && ntasks > 0 && nblocks > 0 && nblocks < (1L << 31), CFM_ERR_ARG, "bad task table");
  hipStream_t s = cfm::as_stream(stream);
  if (dtx == CFM_F32 && dty == CFM_BF16)
    hipLaunchKernelGGL((cast_batch_kernel<float, bf16>), dim3((unsigned)nblocks), dim3(256), 0, s, tasks, ntasks);
  else if (dtx == CFM_BF16 && dty == CFM_F32)
    hipLaunchKernelGGL((cast_batch_kernel<bf16, float>), dim3((unsigned)nblocks), dim3(256), 0, s, tasks, ntasks);
  else
    return cfm::fail(CFM_ERR_DTYPE, "cfm_cast_batch: f32 <-> bf16 only");
  return cfm::check_launch("cfm_cast_batch");
}

namespace {
// one 64 x 64 tile of one task per block: float4 row reads (16 lanes per 256-B row) -> optional
// row-major copy (8-B stores) + LDS -> transposed copy (2 x 16-B stores per thread)
template <typename TO>
__global__ __launch_bounds__(256) void cast_t_batch_kernel(const cfm_castT_task* __restrict__ tasks, int ntasks) {
  __shared__ float tile[64][65];
  int lo = 0, hi = ntasks - 1;
  const long b = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tasks[mid].blk0 <= b) lo = mid; else hi = mid - 1;
  }
  const cfm_castT_task t = tasks[lo];
  const int tcols = (t.cols + 63) / 64;
  const int tb = (int)(b - t.blk0), r0 = (tb / tcols) * 64, c0 = (tb % tcols) * 64;
  const float* x = reinterpret_cast<const float*>(t.src);
  TO* yn = reinterpret_cast<TO*>(t.dst_n);
  const int tid = threadIdx.x;
  constexpr int DT = std::is_same<TO, bf16>::value ? CFM_BF16 : CFM_F32;
  {
    const int c4 = (tid & 15) * 4, c = c0 + c4;
    const bool vec = (t.cols % 4) == 0 && c + 4 <= t.cols;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = (tid >> 4) + 16 * i, r = r0 + rr;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (r < t.rows) {
        if (vec) {
          const float4 q = *reinterpret_cast<const float4*>(x + (long)r * t.cols + c);
          v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = c + e < t.cols ? x[(long)r * t.cols + c + e] : 0.f;
        }
        if (yn) {
          TO* d = yn + (long)r * t.cols + c;
          if (vec && DT == CFM_BF16) {
            bf16x4 w4 = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
            *reinterpret_cast<bf16x4*>(d) = w4;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (c + e < t.cols) d[e] = from_f32<TO>(v[e]);
          }
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) tile[rr][c4 + e] = v[e];
    }
  }
  __syncthreads();
  // output row = source column c0 + rr, output columns = source rows r0 + cq .. + 16
  const int rr = tid >> 2, cq = (tid & 3) * 16;
  const int orow = c0 + rr;
  if (orow >= t.cols || r0 + cq >= t.rows) return;
  TO* dst = reinterpret_cast<TO*>(t.dst) + (long)orow * t.rows + r0 + cq;
  float v0[8], v1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { v0[e] = tile[cq + e][rr]; v1[e] = tile[cq + 8 + e][rr]; }
  if (r0 + cq + 16 <= t.rows && ((uintptr_t)dst % 16) == 0) {
    st8_dyn(dst, DT, 0, v0);
    st8_dyn(dst + 8, DT, 0, v1);
  } else {
    for (int e = 0; e < 16 && r0 + cq + e < t.rows; ++e) dst[e] = from_f32<TO>(e < 8 ? v0[e] : v1[e - 8]);
  }
}
}  // namespace

CFM_EXPORT int cfm_cast_transpose_batch(const cfm_castT_task* tasks, int ntasks, long nblocks, int dtx, int dty,
                                        void* stream) {
  CFM_REQUIRE(tasks && ntasks > 0 && nblocks > 0 && nblocks < (1L << 31), CFM_ERR_ARG, "bad task table");
  hipStream_t s = cfm::as_stream(stream);
  if (dtx == CFM_F32 && dty == CFM_BF16)
    hipLaunchKernelGGL((cast_t_batch_kernel<bf16>), dim3((unsigned)nblocks), dim3(256), 0, s, tasks, ntasks);
  else if (dtx == CFM_F32 && dty == CFM_F32)
    hipLaunchKernelGGL((cast_t_batch_kernel<float>), dim3((unsigned)nblocks), dim3(256), 0, s, tasks, ntasks);
  else
    return cfm::fail(CFM_ERR_DTYPE, "cfm_cast_transpose_batch: f32 -> bf16 / f32 only");
  return cfm::check_launch("cfm_cast_transpose_batch");
}

CFM_EXPORT int cfm_scale_dropout(const void* x, int dtx, void* y, int dty, long n, float scale,
                                 float p, uint64_t seed, uint64_t off, void* stream) {
  CFM_REQUIRE(x && y && n >= 0, CFM_ERR_ARG, "bad args");
  if (n == 0) return CFM_OK;
  if (n % 8 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0)
    hipLaunchKernelGGL(scale_dropout8_kernel, dim3(grid_for(n / 8, 1)), dim3(256), 0, cfm::as_stream(stream), x,
                       dtx, y, dty, n / 8, scale, p, seed, off, cfm::g_rng_salt);
  else
    hipLaunchKernelGGL(scale_dropout_kernel, dim3(grid_for(n, 1)), dim3(256), 0, cfm::as_stream(stream), x,
                       dtx, y, dty, n, scale, p, seed, off, cfm::g_rng_salt);
  return cfm::check_launch("cfm_scale_dropout");
}

namespace {
__global__ void silu_bwd_kernel(const void* dy, int dtdy, const void* pre, int dtpre, void* dx, int dtdx, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    st_dyn(dx, dtdx, i, ld_dyn(dy, dtdy, i) * silu_grad_f(ld_dyn(pre, dtpre, i)));
}
}  // namespace

CFM_EXPORT int cfm_silu_bwd(const void* dy, int dtdy, const void* pre, int dtpre, void* dx, int dtdx, long n,
                            void* stream) {
  CFM_REQUIRE(dy && pre && dx && n >= 0, CFM_ERR_ARG, "bad args");
  if (n == 0) return CFM_OK;
  hipLaunchKernelGGL(silu_bwd_kernel, dim3(grid_for(n, 1)), dim3(256), 0, cfm::as_stream(stream), dy, dtdy, pre,
                     dtpre, dx, dtdx, n);
  return cfm::check_launch("cfm_silu_bwd");
}

// --------------------------------------------------------------------------- column reductions
// Deterministic two-level column sums.  Level 1 (colsum_partial): grid (ceil(N/64), NCHUNK), each
// block = 4 waves over a contiguous row chunk, lane = column, waves interleave rows, LDS combine ->
// one partial row per block.  Level 2 (colreduce_kernel): block = 16 waves over 64 columns, each
// wave sums every 16th partial row, LDS combine.  Also used by LayerNorm / BatchNorm / depthwise
// weight-gradient partial sums.
namespace {
constexpr int COLSUM_CHUNKS = 256;

__global__ __launch_bounds__(256) void colsum_partial(const void* __restrict__ x, int dtx, long M, int N, long ld,
                                                      long rows_per, float* __restrict__ ws) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + lane;
  const long r0 = (long)blockIdx.y * rows_per;
  const long r1 = min(M, r0 + rows_per);
  float s = 0.f;
  if (n < N) {
    if (dtx == CFM_BF16) {
      const bf16* p = reinterpret_cast<const bf16*>(x) + n;
#pragma unroll 4
      for (long r = r0 + wv; r < r1; r += 4) s += (float)p[r * ld];
    } else {
      const float* p = reinterpret_cast<const float*>(x) + n;
#pragma unroll 4
      for (long r = r0 + wv; r < r1; r += 4) s += p[r * ld];
    }
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && n < N) ws[(long)blockIdx.y * N + n] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

__global__ __launch_bounds__(1024) void colreduce_kernel(const float* __restrict__ part, int nparts, long N,
                                                         long ldp, float* __restrict__ out, int acc) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long n = (long)blockIdx.x * 64 + lane;
  float s = 0.f;
  if (n < N) {
#pragma unroll 4
    for (int p = wv; p < nparts; p += 16) s += part[(long)p * ldp + n];
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][lane];
    out[n] = acc ? out[n] + t : t;
  }
}
// two independent column reductions in one launch (blockIdx.y selects): BatchNorm's (sum, sumsq) /
// (dbeta, dgamma) partial pairs
__global__ __launch_bounds__(1024) void colreduce2_kernel(const float* __restrict__ partA, const float* __restrict__ partB,
                                                          int nparts, long N, long ldp, float* __restrict__ outA,
                                                          float* __restrict__ outB) {
  __shared__ float red[16][64];
  const float* part = blockIdx.y ? partB : partA;
  float* out = blockIdx.y ? outB : outA;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long n = (long)blockIdx.x * 64 + lane;
  float s = 0.f;
  if (n < N) {
    // 16 of the wave's parts loaded before any is added (the round-4 `unroll 4` paid 3 memory round trips for the
    // 12 parts a wave holds at 192 partial rows); same order of additions: bit-identical
    for (int p0 = wv; p0 < nparts; p0 += 16 * 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p0 + 16 * u < nparts ? part[(long)(p0 + 16 * u) * ldp + n] : 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][lane];
    out[n] = t;
  }
}
// few partial rows over many columns (the rel-pos dpos per-utterance partials: 8 rows x 1.5 M columns): the
// 16-wave-per-64-columns kernel above left half its waves idle and launched 24 K blocks; here each thread sums
// float4 columns over the parts in the same order (0 + p0 + p1 + ...: bit-identical to colreduce_kernel for
// nparts <= 16, whose waves hold at most one part each)
__global__ __launch_bounds__(256) void colreduce_few_kernel(const float* __restrict__ part, int nparts, long N,
                                                            long ldp, float* __restrict__ out, int acc) {
  const long n4 = N / 4;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < nparts; ++p) {
      const float4 v = *reinterpret_cast<const float4*>(part + (long)p * ldp + 4 * i);
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    float4* o = reinterpret_cast<float4*>(out + 4 * i);
    if (acc) {
      const float4 u = *o;
      t = make_float4(u.x + t.x, u.y + t.y, u.z + t.z, u.w + t.w);
    }
    *o = t;
  }
}
// the same writing bf16 (each column's fp32 sum rounded as cfm_cast rounds it; out 8-B aligned)
__global__ __launch_bounds__(256) void colreduce_few_bf16_kernel(const float* __restrict__ part, int nparts, long N,
                                                                 long ldp, bf16* __restrict__ out) {
  const long n4 = N / 4;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < nparts; ++p) {
      const float4 v = *reinterpret_cast<const float4*>(part + (long)p * ldp + 4 * i);
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    bf16x4 o = {from_f32<bf16>(t.x), from_f32<bf16>(t.y), from_f32<bf16>(t.z), from_f32<bf16>(t.w)};
    *reinterpret_cast<bf16x4*>(out + 4 * i) = o;
  }
}
}  // namespace

namespace cfm {
// out (bf16) = sum_p part[p * ldp + n]: the few-rows kernel when it applies, else the fp32 reduction into part's
// row 0 (in place: every column's parts are read before its sum is written) and a cast
void colreduce_bf16(float* part, int nparts, long N, bf16* out, hipStream_t s, long ldp) {
  const long lp = ldp > 0 ? ldp : N;
  if (nparts <= 16 && N % 4 == 0 && lp % 4 == 0 && (uintptr_t)part % 16 == 0 && (uintptr_t)out % 8 == 0 &&
      N >= 65536) {
    const long blocks = (N / 4 + 255) / 256;
    hipLaunchKernelGGL(colreduce_few_bf16_kernel, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(256), 0, s,
                       part, nparts, N, lp, out);
    return;
  }
  colreduce(part, nparts, N, part, 0, s, lp);
  cfm_cast(part, CFM_F32, out, CFM_BF16, N, s);
}
void colreduce_pair(const float* partA, const float* partB, int nparts, long N, float* outA, float* outB,
                    hipStream_t s, long ldp) {
  hipLaunchKernelGGL(colreduce2_kernel, dim3((unsigned)((N + 63) / 64), 2), dim3(1024), 0, s, partA, partB, nparts, N,
                     ldp > 0 ? ldp : N, outA, outB);
}
void colreduce(const float* part, int nparts, long N, float* out, int accumulate, hipStream_t s, long ldp) {
  const long lp = ldp > 0 ? ldp : N;
  if (nparts <= 16 && N % 4 == 0 && lp % 4 == 0 && (uintptr_t)part % 16 == 0 && (uintptr_t)out % 16 == 0 &&
      N >= 65536) {
    const long blocks = (N / 4 + 255) / 256;
    hipLaunchKernelGGL(colreduce_few_kernel, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(256), 0, s, part,
                       nparts, N, lp, out, accumulate);
    return;
  }
  hipLaunchKernelGGL(colreduce_kernel, dim3((unsigned)((N + 63) / 64)), dim3(1024), 0, s, part, nparts, N,
                     ldp > 0 ? ldp : N, out, accumulate);
}
}  // namespace cfm

CFM_EXPORT int cfm_colreduce(const float* part, int nparts, long N, long ldp, float* out, int accumulate,
                             void* stream) {
  CFM_REQUIRE(part && out && nparts > 0 && N > 0 && ldp >= N, CFM_ERR_ARG, "bad args");
  cfm::colreduce(part, nparts, N, out, accumulate, cfm::as_stream(stream), ldp);
  return cfm::check_launch("cfm_colreduce");
}

CFM_EXPORT int cfm_colsum(const void* x, int dtx, long M, int N, long ld, float* out, int accumulate,
                          float* ws, void* stream) {
  CFM_REQUIRE(x && out && ws && N > 0 && M >= 0 && ld >= N, CFM_ERR_ARG, "bad args");
  int nblk = (int)((M + 63) / 64);
  if (nblk > COLSUM_CHUNKS) nblk = COLSUM_CHUNKS;
  if (nblk < 1) nblk = 1;
  const long rows_per = (M + nblk - 1) / nblk;
  hipStream_t s = cfm::as_stream(stream);
  hipLaunchKernelGGL(colsum_partial, dim3(cdiv(N, 64), nblk), dim3(256), 0, s, x, dtx, M, N, ld,
                     rows_per > 0 ? rows_per : 1, ws);
  cfm::colreduce(ws, nblk, N, out, accumulate, s);
  return cfm::check_launch("cfm_colsum");
}

// --------------------------------------------------------------------------- probes
// A probed kernel records its own first-workgroup start and last-workgroup end (s_memrealtime) in
// slot[0] / slot[1]; these one-lane kernels reset the slot before it and accumulate the interval
// after it, on the same stream (so they work as nodes of a captured HIP graph too).
namespace {
__global__ void probe_slot_kernel(unsigned long long* s, int mode) {
  if (mode == 0 || mode == 2) {
    s[0] = ~0ull;
    s[1] = 0ull;
    if (mode == 2) s[4] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
  } else {
    if (s[1] > s[0]) s[2] += s[1] - s[0];
    if (mode == 3) s[5] += (unsigned long long)__builtin_amdgcn_s_memrealtime() - s[4];
    s[3] += 1;
  }
}
}  // namespace

CFM_EXPORT int cfm_probe_slot(unsigned long long* slot, int mode, void* stream) {
  CFM_REQUIRE(slot && mode >= 0 && mode <= 3, CFM_ERR_ARG, "bad args");
  hipLaunchKernelGGL(probe_slot_kernel, dim3(1), dim3(1), 0, cfm::as_stream(stream), slot, mode);
  return cfm::check_launch("cfm_probe_slot");
}

CFM_EXPORT int cfm_wallclock_khz(void) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 0;
  return khz;
}

// --------------------------------------------------------------------------- grouped column reductions
// Every small deferred reduction of a backward pass (LayerNorm dgamma|dbeta partial rows, depthwise-conv
// weight/bias partials) in ONE launch at the end: 85 side-stream launches per Conformer-L step were worth
// ~1.9 ms of wall time (same-box A/B).  Task i: out[n] = sum_p part[p*ldp + n], n < N, summed in a fixed
// order (16 waves per 64-column block, wave w takes parts w, w+16, ...; LDS combine) -- deterministic.
// mode 1 (depthwise conv): column n = k*C + c of the [K+1][C] sums goes to dw[c*K + k] (k < K) / db[c].
namespace {
struct RedTask {
  const float* part;
  float* out;
  float* out2;
  long N, ldp;
  long block0;
  int nparts, mode, C, K;
};

__global__ __launch_bounds__(1024) void colreduce_group_kernel(const RedTask* __restrict__ tab, int ntasks) {
  __shared__ float red[16][64];
  const long blk = blockIdx.x;
  int lo = 0, hi = ntasks - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (__builtin_amdgcn_readfirstlane((int)tab[mid].block0) <= blk) lo = mid; else hi = mid - 1;
  }
  const RedTask t = tab[__builtin_amdgcn_readfirstlane(lo)];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long n = (blk - t.block0) * 64 + lane;
  float s = 0.f;
  if (n < t.N) {
#pragma unroll 4
    for (int p = wv; p < t.nparts; p += 16) s += t.part[(long)p * t.ldp + n];
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && n < t.N) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) v += red[w][lane];
    if (t.mode == 0) {
      t.out[n] = v;
    } else {
      const int k = (int)(n / t.C), c = (int)(n % t.C);
      if (k < t.K) t.out[(long)c * t.K + k] = v;
      else if (t.out2) t.out2[c] = v;
    }
  }
}
}  // namespace

CFM_EXPORT size_t cfm_colreduce_group_task_bytes(void) { return sizeof(RedTask); }
CFM_EXPORT long cfm_colreduce_group_blocks(long N) { return (N + 63) / 64; }

// task i of a HOST table; mode 0: out[n] = sum_p part[p*ldp + n]; mode 1: depthwise-conv scatter (C, K)
CFM_EXPORT int cfm_colreduce_group_fill(void* host_tab, int i, const float* part, int nparts, long N, long ldp,
                                        float* out, float* out2, int mode, int C, int K, long block0) {
  CFM_REQUIRE(host_tab && part && out && i >= 0 && nparts > 0 && N > 0 && ldp >= N, CFM_ERR_ARG, "bad task");
  CFM_REQUIRE(mode == 0 || (mode == 1 && C > 0 && K > 0 && N == (long)C * (K + 1)), CFM_ERR_ARG, "bad mode");
  RedTask t{part, out, out2, N, ldp, block0, nparts, mode, C, K};
  reinterpret_cast<RedTask*>(host_tab)[i] = t;
  return CFM_OK;
}

CFM_EXPORT int cfm_colreduce_group(const void* dev_tab, int ntasks, long total_blocks, void* stream) {
  CFM_REQUIRE(dev_tab && ntasks > 0 && total_blocks > 0 && total_blocks < (1L << 31), CFM_ERR_ARG, "bad table");
  hipLaunchKernelGGL(colreduce_group_kernel, dim3((unsigned)total_blocks), dim3(1024), 0, cfm::as_stream(stream),
                     (const RedTask*)dev_tab, ntasks);
  return cfm::check_launch("cfm_colreduce_group");
}
