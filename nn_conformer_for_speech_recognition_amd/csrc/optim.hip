// optim.hip — multi-tensor fused Adafactor step (the reference's optimizer, runner.py:36:
// transformers.Adafactor(lr, beta1=0.9, scale_parameter=False, relative_step=False); defaults
// eps=(1e-30, 1e-3), clip_threshold=1, decay_rate=-0.8, weight_decay=0).
//
// Every parameter is viewed as nb x R x C (leading dims folded into nb).  Factored second moment
// for ndim >= 2 (row/col EMAs of g^2+eps1), full EMA otherwise; update u = g * rsqrt(row_r /
// mean(row)) * rsqrt(col_c) (or g * rsqrt(v)), clipped by max(1, RMS(u)/clip), scaled by lr,
// first moment m = b1*m + (1-b1)*u, p -= m.  All parameters are handled by five launches over a
// device-side parameter table (no per-tensor launches): row stats, column stats, row-stat means,
// u^2 sums (one atomic per workgroup per tensor), apply.  Work items are "tasks" whose shape
// adapts to the tensor: a wide row (C >= 64) is one wave, narrow rows (e.g. the 3x3 taps of the
// conv2 weight, nb = 65536) are packed 64 per wave (one per lane).  HBM-bound.
#include "cfm_common.h"

namespace {

constexpr int EB = 256;          // threads per block
constexpr int CHUNK = 4096;      // elements per block in the elementwise passes

struct AdaP {
  float* p; const float* g; float* m; float* row; float* col;   // col == nullptr: unfactored (row = v)
  long numel; int nb, R, C, factored;
  long row_toff, col_off, blk_off, rm_off, rm_toff;              // prefix offsets (tasks / elements)
};

__device__ __forceinline__ long off_of(const AdaP& q, int which) {
  return which == 0 ? q.row_toff : which == 1 ? q.col_off : which == 2 ? q.blk_off : q.rm_toff;
}
__device__ __forceinline__ int find_param(const AdaP* t, int n, long idx, int which) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off_of(t[mid], which) <= idx) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ void row_update(const AdaP& q, long lr, float s, float b2t) {
  q.row[lr] = b2t * q.row[lr] + (1.f - b2t) * (s / q.C);
}

// row tasks: wide rows -> one wave per row; narrow rows -> 64 rows per wave (lane = row)
__global__ void ada_rows(const AdaP* __restrict__ t, int n, long ntasks, float b2t, float eps1) {
  const int lane = threadIdx.x & 63;
  const long task = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= ntasks) return;
  const AdaP& q = t[find_param(t, n, task, 0)];
  const long lt = task - q.row_toff;
  if (q.C >= 64) {
    const float* g = q.g + lt * q.C;
    float s = 0.f;
    for (int c = lane; c < q.C; c += 64) s += g[c] * g[c] + eps1;
    s = wave_sum(s);
    if (lane == 0) row_update(q, lt, s, b2t);
  } else {
    const long lr = lt * 64 + lane;
    if (lr < (long)q.nb * q.R) {
      const float* g = q.g + lr * q.C;
      float s = 0.f;
      for (int c = 0; c < q.C; ++c) s += g[c] * g[c] + eps1;
      row_update(q, lr, s, b2t);
    }
  }
}

// one thread per factored column: col = b2t*col + (1-b2t)*mean_r(g^2 + eps1)
__global__ void ada_cols(const AdaP* __restrict__ t, int n, long ncols, float b2t, float eps1) {
  const long cidx = (long)blockIdx.x * EB + threadIdx.x;
  if (cidx >= ncols) return;
  const AdaP& q = t[find_param(t, n, cidx, 1)];
  const long lc = cidx - q.col_off;     // = b*C + j
  const int b = (int)(lc / q.C), j = (int)(lc % q.C);
  const float* g = q.g + (long)b * q.R * q.C + j;
  float s = 0.f;
  for (int r = 0; r < q.R; ++r) {
    const float v = g[(long)r * q.C];
    s += v * v + eps1;
  }
  q.col[lc] = b2t * q.col[lc] + (1.f - b2t) * (s / q.R);
}

// mean over R of the row state per (param, b): wide R -> one wave per b; narrow -> 64 b per wave
__global__ void ada_rowmean(const AdaP* __restrict__ t, int n, long ntasks, float* __restrict__ rowmean) {
  const int lane = threadIdx.x & 63;
  const long task = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= ntasks) return;
  const AdaP& q = t[find_param(t, n, task, 3)];
  if (!q.factored) return;
  const long lt = task - q.rm_toff;
  if (q.R >= 64) {
    float s = 0.f;
    for (int r = lane; r < q.R; r += 64) s += q.row[lt * q.R + r];
    s = wave_sum(s);
    if (lane == 0) rowmean[q.rm_off + lt] = s / q.R;
  } else {
    const long b = lt * 64 + lane;
    if (b < q.nb) {
      float s = 0.f;
      for (int r = 0; r < q.R; ++r) s += q.row[b * q.R + r];
      rowmean[q.rm_off + b] = s / q.R;
    }
  }
}

__device__ __forceinline__ float ada_u(const AdaP& q, const float* rowmean, long i, float b2t, float eps1,
                                       bool update_v) {
  const float g = q.g[i];
  if (!q.factored) {
    float v = q.row[i];
    if (update_v) {
      v = b2t * v + (1.f - b2t) * (g * g + eps1);
      q.row[i] = v;
    }
    return g * rsqrtf(v);
  }
  const long rc = (long)q.R * q.C;
  const int b = (int)(i / rc);
  const long w = i % rc;
  const int r = (int)(w / q.C), c = (int)(w % q.C);
  const float rf = rsqrtf(q.row[(long)b * q.R + r] / rowmean[q.rm_off + b]);
  const float cf = rsqrtf(q.col[(long)b * q.C + c]);
  return g * rf * cf;
}

// per-block sum of u^2 -> one atomic per block into sumsq[param]
__global__ void ada_sumsq(const AdaP* __restrict__ t, int n, const float* __restrict__ rowmean, float b2t,
                          float eps1, float* __restrict__ sumsq) {
  __shared__ float red[EB / 64];
  const int pi = find_param(t, n, blockIdx.x, 2);
  const AdaP& q = t[pi];
  const long start = (long)(blockIdx.x - q.blk_off) * CHUNK;
  const long end = min(q.numel, start + CHUNK);
  float s = 0.f;
  for (long i = start + threadIdx.x; i < end; i += EB) {
    const float u = ada_u(q, rowmean, i, b2t, eps1, true);
    s += u * u;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(sumsq + pi, red[0] + red[1] + red[2] + red[3]);
}

__global__ void ada_apply(const AdaP* __restrict__ t, int n, const float* __restrict__ rowmean, float b2t, float eps1,
                          const float* __restrict__ sumsq, float lr, float beta1, float clip) {
  const int pi = find_param(t, n, blockIdx.x, 2);
  const AdaP& q = t[pi];
  const long start = (long)(blockIdx.x - q.blk_off) * CHUNK;
  const long end = min(q.numel, start + CHUNK);
  const float rms = sqrtf(sumsq[pi] / (float)q.numel);
  const float scale = lr / fmaxf(rms / clip, 1.f);
  for (long i = start + threadIdx.x; i < end; i += EB) {
    const float u = ada_u(q, rowmean, i, b2t, eps1, false) * scale;
    float upd = u;
    if (q.m) {
      upd = beta1 * q.m[i] + (1.f - beta1) * u;
      q.m[i] = upd;
    }
    q.p[i] -= upd;
  }
}

}  // namespace

CFM_EXPORT size_t cfm_adafactor_table_bytes(int n_params) { return (size_t)n_params * sizeof(AdaP); }

CFM_EXPORT int cfm_adafactor_fill_table(void* host_table, int i, float* p, const float* g, float* m, float* row,
                                        float* col, long numel, int nb, int R, int C, long row_toff, long col_off,
                                        long blk_off, long rm_off, long rm_toff) {
  CFM_REQUIRE(host_table && p && g && row, CFM_ERR_ARG, "null pointer");
  AdaP* t = reinterpret_cast<AdaP*>(host_table) + i;
  t->p = p; t->g = g; t->m = m; t->row = row; t->col = col;
  t->numel = numel; t->nb = nb; t->R = R; t->C = C; t->factored = col != nullptr;
  t->row_toff = row_toff; t->col_off = col_off; t->blk_off = blk_off; t->rm_off = rm_off; t->rm_toff = rm_toff;
  return CFM_OK;
}

CFM_EXPORT int cfm_adafactor_blocks(long numel) { return (int)((numel + CHUNK - 1) / CHUNK); }

// number of row tasks / row-mean tasks a factored tensor contributes (see ada_rows / ada_rowmean)
CFM_EXPORT long cfm_adafactor_row_tasks(int nb, int R, int C) { return C >= 64 ? (long)nb * R : ((long)nb * R + 63) / 64; }
CFM_EXPORT long cfm_adafactor_rowmean_tasks(int nb, int R) { return R >= 64 ? (long)nb : ((long)nb + 63) / 64; }

CFM_EXPORT int cfm_adafactor_step(const void* dev_table, int n, long nrow_tasks, long ncols, long nblocks,
                                  long nrm_tasks, float* rowmean, float* sumsq, float lr, float beta1, float beta2t,
                                  float eps1, float clip, void* stream) {
  CFM_REQUIRE(dev_table && rowmean && sumsq && n > 0, CFM_ERR_ARG, "bad args");
  const AdaP* t = reinterpret_cast<const AdaP*>(dev_table);
  hipStream_t s = cfm::as_stream(stream);
  (void)hipMemsetAsync(sumsq, 0, sizeof(float) * n, s);
  if (nrow_tasks > 0)
    hipLaunchKernelGGL(ada_rows, dim3((unsigned)((nrow_tasks + 3) / 4)), dim3(256), 0, s, t, n, nrow_tasks, beta2t,
                       eps1);
  if (ncols > 0)
    hipLaunchKernelGGL(ada_cols, dim3((unsigned)((ncols + EB - 1) / EB)), dim3(EB), 0, s, t, n, ncols, beta2t, eps1);
  if (nrm_tasks > 0)
    hipLaunchKernelGGL(ada_rowmean, dim3((unsigned)((nrm_tasks + 3) / 4)), dim3(256), 0, s, t, n, nrm_tasks, rowmean);
  hipLaunchKernelGGL(ada_sumsq, dim3((unsigned)nblocks), dim3(EB), 0, s, t, n, rowmean, beta2t, eps1, sumsq);
  hipLaunchKernelGGL(ada_apply, dim3((unsigned)nblocks), dim3(EB), 0, s, t, n, rowmean, beta2t, eps1, sumsq, lr,
                     beta1, clip);
  return cfm::check_launch("cfm_adafactor_step");
}
