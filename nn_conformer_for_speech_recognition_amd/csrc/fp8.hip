// fp8.hip — per-tensor e4m3 quantisation for the fp8 GEMM path (BASELINE.json configs[4]: the 60 s long-form
// Conformer-L with fp8 MFMA).  Current scaling: amax over the tensor (256 partial maxima, no atomics) ->
// scale = the power of two just below 448 / amax (448: e4m3fn's largest finite value) -> y = e4m3(x * scale), and the dequantisation factor 1/scale is written to a device scalar
// that the GEMM epilogue multiplies in (cfm_gemm_desc.alpha_a_dev / alpha_b_dev).  Everything stays on the
// device (no host sync), so quantisation sits inside a captured HIP graph.  The scale is the power of two
// just below 448/amax (at most one bit of range unused; exact scaling and dequantisation).
#include "cfm_common.h"

namespace {

constexpr int AMAX_BLOCKS = 256;   // partial maxima: no atomics (one word would serialise every wave)

// |x| max: block b writes its partial maximum to part[b] (grid AMAX_BLOCKS, grid-stride)
__global__ __launch_bounds__(256) void amax_kernel(const void* __restrict__ x, int dt, long n,
                                                   float* __restrict__ part) {
  __shared__ float red[4];
  float m = 0.f;
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8];
    ld8_dyn(x, dt, i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
  }
  for (long i = n8 * 8 + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    m = fmaxf(m, fabsf(ld_dyn(x, dt, i)));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// every block of the cast reduces the AMAX_BLOCKS partials itself (1 KiB, L2-resident): no extra launch
__device__ __forceinline__ float block_amax(const float* part) {
  __shared__ float red[4];
  float m = 0.f;
  for (int i = threadIdx.x; i < AMAX_BLOCKS; i += 256) m = fmaxf(m, part[i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// power-of-two scale 2^k, k the largest integer with amax * 2^k <= 448 (= 1.75 * 2^8): exact in both
// directions (x * 2^k and the dequantisation 2^-k lose nothing), bit-reproducible against any host restatement
__device__ __forceinline__ float fp8_scale(float a) {
  if (!(a > 0.f) || !(a < INFINITY)) return 1.f;
  int e;
  const float m = 2.f * frexpf(a, &e);          // a = m * 2^(e-1), m in [1, 2)
  const int k = (m <= 1.75f ? 8 : 7) - (e - 1);
  return ldexpf(1.f, k < 126 ? (k > -126 ? k : -126) : 126);
}

__global__ __launch_bounds__(256) void quant_fp8_kernel(const void* __restrict__ x, int dt, long n,
                                                        const float* __restrict__ part, uint8_t* __restrict__ y,
                                                        float* __restrict__ inv_scale) {
  const float sc = fp8_scale(block_amax(part));
  if (blockIdx.x == 0 && threadIdx.x == 0) inv_scale[0] = 1.f / sc;
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8];
    ld8_dyn(x, dt, i * 8, v);
    int lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * sc, v[1] * sc, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * sc, v[3] * sc, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * sc, v[5] * sc, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * sc, v[7] * sc, hi, true);
    *reinterpret_cast<uint2*>(y + i * 8) = make_uint2((unsigned)lo, (unsigned)hi);
  }
  for (long i = n8 * 8 + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int w = __builtin_amdgcn_cvt_pk_fp8_f32(ld_dyn(x, dt, i) * sc, 0.f, 0, false);
    y[i] = (uint8_t)(w & 0xFF);
  }
}

// e4m3 -> f32 (for tests / dequantised views): byte i of x times inv_scale
__global__ __launch_bounds__(256) void dequant_fp8_kernel(const uint8_t* __restrict__ x, long n,
                                                          const float* __restrict__ inv_scale, float* __restrict__ y) {
  const float s = inv_scale ? inv_scale[0] : 1.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] = __builtin_amdgcn_cvt_f32_fp8((int)x[i], 0) * s;
}

// ---------------------------------------------------------------- batched (one table, two launches)
// task of a block: the last task whose blk0 <= block (wave-uniform binary search over the small table)
__device__ __forceinline__ int q8_task_of(const cfm_q8_task* t, int n, long blk) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t[mid].blk0 <= blk) lo = mid; else hi = mid - 1;
  }
  return lo;
}
__host__ __device__ inline long q8_blocks(long n) {
  const long b = (n / 8 + 255) / 256;
  return b > 64 ? 64 : (b < 1 ? 1 : b);
}

// pass 1: block j of task i writes the partial |x| max of its grid-stride share to part[blk0_i + j]
__global__ __launch_bounds__(256) void amax_batch_kernel(const cfm_q8_task* __restrict__ t, int nt, int dt,
                                                         float* __restrict__ part) {
  __shared__ float red[4];
  const long blk = blockIdx.x;
  const cfm_q8_task q = t[q8_task_of(t, nt, blk)];
  const long j = blk - q.blk0, nb = q8_blocks(q.n);
  float m = 0.f;
  const long n8 = q.n / 8;
  for (long i = j * 256 + threadIdx.x; i < n8; i += nb * 256) {
    float v[8];
    ld8_dyn(q.x, dt, i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
  }
  for (long i = n8 * 8 + j * 256 + threadIdx.x; i < q.n; i += nb * 256) m = fmaxf(m, fabsf(ld_dyn(q.x, dt, i)));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[blk] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// pass 2: every block of task i reduces the task's partials, then casts its share (quant_fp8_kernel's math)
__global__ __launch_bounds__(256) void quant_batch_kernel(const cfm_q8_task* __restrict__ t, int nt, int dt,
                                                          const float* __restrict__ part) {
  __shared__ float red[4];
  const long blk = blockIdx.x;
  const cfm_q8_task q = t[q8_task_of(t, nt, blk)];
  const long j = blk - q.blk0, nb = q8_blocks(q.n);
  float m = 0.f;
  for (long i = threadIdx.x; i < nb; i += 256) m = fmaxf(m, part[q.blk0 + i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  const float sc = fp8_scale(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  if (j == 0 && threadIdx.x == 0) q.inv_scale[0] = 1.f / sc;
  uint8_t* y = reinterpret_cast<uint8_t*>(q.y);
  const long n8 = q.n / 8;
  for (long i = j * 256 + threadIdx.x; i < n8; i += nb * 256) {
    float v[8];
    ld8_dyn(q.x, dt, i * 8, v);
    int lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * sc, v[1] * sc, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * sc, v[3] * sc, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * sc, v[5] * sc, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * sc, v[7] * sc, hi, true);
    *reinterpret_cast<uint2*>(y + i * 8) = make_uint2((unsigned)lo, (unsigned)hi);
  }
  for (long i = n8 * 8 + j * 256 + threadIdx.x; i < q.n; i += nb * 256) {
    const int w = __builtin_amdgcn_cvt_pk_fp8_f32(ld_dyn(q.x, dt, i) * sc, 0.f, 0, false);
    y[i] = (uint8_t)(w & 0xFF);
  }
}

int grid_for(long n) {
  long b = (n / 8 + 255) / 256;
  return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

// ---------------------------------------------------------------- MX (OCP microscaling) e4m3
// Every 32 consecutive elements of a row share one e8m0 scale byte s = 127 - k, k the largest integer with
// amax(block) * 2^k <= 448 (fp8_scale's rule per block; 0 for an all-zero block), y = e4m3(x * 2^k): the block-scaled
// MFMA (v_mfma_scale_f32_32x32x64_f8f6f4) multiplies each 32-element product run by 2^(s_a - 127) 2^(s_b - 127).
// One pass over x (no tensor-wide amax): a thread converts 8 elements, the 4 lanes of a block exchange their maxima
// by two xor shuffles (lanes 4j .. 4j+3 hold consecutive 8-element chunks of one block).
__device__ __forceinline__ int mx_k(float a) {
  if (!(a > 0.f) || !(a < INFINITY)) return 0;
  int e;
  const float m = 2.f * frexpf(a, &e);          // a = m * 2^(e-1), m in [1, 2)
  const int k = (m <= 1.75f ? 8 : 7) - (e - 1);
  return k < 126 ? (k > -126 ? k : -126) : 126;
}

__device__ __forceinline__ void mx_chunk(const float (&v)[8], uint8_t* y, uint8_t* s, bool lead) {
  float m = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
  m = fmaxf(m, __shfl_xor(m, 1, 64));
  m = fmaxf(m, __shfl_xor(m, 2, 64));
  const int k = mx_k(m);
  const float sc = ldexpf(1.f, k);
  int lo = 0, hi = 0;
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * sc, v[1] * sc, lo, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * sc, v[3] * sc, lo, true);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * sc, v[5] * sc, hi, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * sc, v[7] * sc, hi, true);
  *reinterpret_cast<uint2*>(y) = make_uint2((unsigned)lo, (unsigned)hi);
  if (lead) *s = (uint8_t)(127 - k);
}

// chunks [j * 256 + tid, n8) step nb * 256 of a rows x K tensor (K % 32 == 0: the chunk count is a multiple of 4
// and a block's 4 chunks sit in one aligned lane quad, so every quad runs the loop together)
__device__ __forceinline__ void mx_rows(const void* x, int dt, long rows, int K, long ldx, uint8_t* y, uint8_t* s,
                                        long j, long nb) {
  const int c8n = K / 8;
  const long n8 = rows * c8n;
  for (long i = j * 256 + threadIdx.x; i < n8; i += nb * 256) {
    const long row = i / c8n;
    const int c = (int)(i - row * c8n);
    float v[8];
    ld8_dyn(x, dt, row * ldx + 8L * c, v);
    mx_chunk(v, y + row * K + 8L * c, s + row * (K / 32) + c / 4, (c & 3) == 0);
  }
}

__global__ __launch_bounds__(256) void quant_mx_kernel(const void* __restrict__ x, int dt, long rows, int K, long ldx,
                                                       uint8_t* __restrict__ y, uint8_t* __restrict__ s) {
  mx_rows(x, dt, rows, K, ldx, y, s, blockIdx.x, gridDim.x);
}

__host__ __device__ inline long mx_blocks(long rows, int K) {
  const long b = (rows * (K / 8) + 255) / 256;
  return b > 256 ? 256 : (b < 1 ? 1 : b);
}

__device__ __forceinline__ int mx_task_of(const cfm_mx_task* t, int n, long blk) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t[mid].blk0 <= blk) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(256) void quant_mx_batch_kernel(const cfm_mx_task* __restrict__ t, int nt, int dt) {
  const long blk = blockIdx.x;
  const cfm_mx_task q = t[mx_task_of(t, nt, blk)];
  mx_rows(q.x, dt, q.rows, q.K, q.K, reinterpret_cast<uint8_t*>(q.y), q.s, blk - q.blk0, mx_blocks(q.rows, q.K));
}

// e4m3 x e8m0 block scales -> f32 (tests / dequantised views): y = e4m3(x) * 2^(s - 127)
__global__ __launch_bounds__(256) void dequant_mx_kernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ s,
                                                         long n, float* __restrict__ y) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] = ldexpf(__builtin_amdgcn_cvt_f32_fp8((int)x[i], 0), (int)s[i / 32] - 127);
}

}  // namespace

CFM_EXPORT int cfm_quant_mx(const void* x, int dtx, long rows, int K, long ldx, void* y, uint8_t* s, void* stream) {
  CFM_REQUIRE(x && y && s && rows > 0 && K > 0, CFM_ERR_ARG, "null pointer / empty tensor");
  CFM_REQUIRE(dtx == CFM_F32 || dtx == CFM_BF16, CFM_ERR_DTYPE, "x must be fp32 or bf16");
  CFM_REQUIRE(K % 32 == 0 && ldx >= K && ldx % 8 == 0, CFM_ERR_SHAPE, "K % 32 == 0, ldx >= K, ldx % 8 == 0");
  CFM_REQUIRE((uintptr_t)x % 16 == 0 && (uintptr_t)y % 8 == 0, CFM_ERR_ALIGN, "16-B aligned x, 8-B aligned y");
  hipLaunchKernelGGL(quant_mx_kernel, dim3(grid_for(rows * (long)K)), dim3(256), 0, cfm::as_stream(stream), x, dtx,
                     rows, K, ldx, (uint8_t*)y, s);
  return cfm::check_launch("cfm_quant_mx");
}

CFM_EXPORT long cfm_quant_mx_batch_blocks(long rows, int K) { return mx_blocks(rows, K); }

CFM_EXPORT int cfm_quant_mx_batch(const cfm_mx_task* tasks, int ntasks, long nblocks, int dtx, void* stream) {
  CFM_REQUIRE(tasks && ntasks > 0 && nblocks > 0, CFM_ERR_ARG, "null table / empty batch");
  CFM_REQUIRE(dtx == CFM_F32 || dtx == CFM_BF16, CFM_ERR_DTYPE, "x must be fp32 or bf16");
  hipLaunchKernelGGL(quant_mx_batch_kernel, dim3((unsigned)nblocks), dim3(256), 0, cfm::as_stream(stream), tasks,
                     ntasks, dtx);
  return cfm::check_launch("cfm_quant_mx_batch");
}

CFM_EXPORT int cfm_dequant_mx(const void* x, const uint8_t* s, long n, float* y, void* stream) {
  CFM_REQUIRE(x && s && y && n > 0 && n % 32 == 0, CFM_ERR_ARG, "null pointer / n % 32");
  hipLaunchKernelGGL(dequant_mx_kernel, dim3(grid_for(8 * n)), dim3(256), 0, cfm::as_stream(stream),
                     (const uint8_t*)x, s, n, y);
  return cfm::check_launch("cfm_dequant_mx");
}

CFM_EXPORT size_t cfm_quant_fp8_ws_bytes(void) { return AMAX_BLOCKS * sizeof(float); }

CFM_EXPORT int cfm_quant_fp8(const void* x, int dtx, long n, void* y, float* inv_scale, unsigned* amax_ws,
                             void* stream) {
  CFM_REQUIRE(x && y && inv_scale && amax_ws && n > 0, CFM_ERR_ARG, "null pointer / empty tensor");
  CFM_REQUIRE(dtx == CFM_F32 || dtx == CFM_BF16, CFM_ERR_DTYPE, "x must be fp32 or bf16");
  CFM_REQUIRE((uintptr_t)x % 16 == 0 && (uintptr_t)y % 8 == 0, CFM_ERR_ALIGN, "16-B aligned x, 8-B aligned y");
  hipStream_t s = cfm::as_stream(stream);
  hipLaunchKernelGGL(amax_kernel, dim3(AMAX_BLOCKS), dim3(256), 0, s, x, dtx, n, (float*)amax_ws);
  hipLaunchKernelGGL(quant_fp8_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, dtx, n, (const float*)amax_ws,
                     (uint8_t*)y, inv_scale);
  return cfm::check_launch("cfm_quant_fp8");
}

CFM_EXPORT long cfm_quant_fp8_batch_blocks(long n) { return q8_blocks(n); }

CFM_EXPORT int cfm_quant_fp8_batch(const cfm_q8_task* tasks, int ntasks, long nblocks, int dtx, float* amax_ws,
                                   void* stream) {
  CFM_REQUIRE(tasks && amax_ws && ntasks > 0 && nblocks > 0, CFM_ERR_ARG, "null table / empty batch");
  CFM_REQUIRE(dtx == CFM_F32 || dtx == CFM_BF16, CFM_ERR_DTYPE, "x must be fp32 or bf16");
  hipStream_t s = cfm::as_stream(stream);
  hipLaunchKernelGGL(amax_batch_kernel, dim3((unsigned)nblocks), dim3(256), 0, s, tasks, ntasks, dtx, amax_ws);
  hipLaunchKernelGGL(quant_batch_kernel, dim3((unsigned)nblocks), dim3(256), 0, s, tasks, ntasks, dtx,
                     (const float*)amax_ws);
  return cfm::check_launch("cfm_quant_fp8_batch");
}

CFM_EXPORT int cfm_dequant_fp8(const void* x, long n, const float* inv_scale, float* y, void* stream) {
  CFM_REQUIRE(x && y && n > 0, CFM_ERR_ARG, "null pointer / empty tensor");
  hipLaunchKernelGGL(dequant_fp8_kernel, dim3(grid_for(8 * n)), dim3(256), 0, cfm::as_stream(stream),
                     (const uint8_t*)x, n, inv_scale, y);
  return cfm::check_launch("cfm_dequant_fp8");
}
