// optim.hip — multi-tensor fused Adafactor step (the reference's optimizer, runner.py:36:
// transformers.Adafactor(lr, beta1=0.9, scale_parameter=False, relative_step=False); defaults
// eps=(1e-30, 1e-3), clip_threshold=1, decay_rate=-0.8, weight_decay=0).
//
// Every parameter is viewed as nb x R x C (leading dims folded into nb).  Factored second moment
// for ndim >= 2 (row/col EMAs of g^2+eps1), full EMA otherwise; update u = g * rsqrt(row_r /
// mean(row)) * rsqrt(col_c) (or g * rsqrt(v)), clipped by max(1, RMS(u)/clip), scaled by lr,
// first moment m = b1*m + (1-b1)*u, p -= m.  All parameters are handled by five launches over a
// device-side parameter table (no per-tensor launches): one pass over g for the row statistics
// and column partial sums of wide matrices (64 <= C <= 2560), row stats of narrow ones, column
// finish (partials in fixed order), row-stat means, u^2 block partials, apply (each block sums its
// tensor's partials in block order: deterministic, no atomics).  float4 paths where aligned.  Work items are "tasks" whose shape
// adapts to the tensor: a wide row (C >= 64) is one wave, narrow rows (e.g. the 3x3 taps of the
// conv2 weight, nb = 65536) are packed 64 per wave (one per lane).  HBM-bound.
#include "cfm_common.h"

namespace {

constexpr int EB = 256;          // threads per block
constexpr int CHUNK = 4096;      // elements per block in the elementwise passes
constexpr int RB = 32;           // rows per column-partial task (wide factored tensors)
constexpr int KMAX = 40;         // 64-column groups a lane keeps in registers: wide means 64 <= C <= 2560

// unsigned 32-bit division by an invariant divisor d >= 1 (Granlund-Montgomery): with l = ceil(log2 d) and
// m = floor(2^32 (2^l - d) / d) + 1, n / d = (t + ((n - t) >> 1)) >> (l - 1) for t = mulhi(m, n) (d >= 2);
// d == 1: m = 0, sh = 0 and the formula is replaced by n.  Exact for every 32-bit n.
struct UDiv { uint32_t m, sh, one; };
static inline UDiv udiv_make(uint32_t d) {
  if (d <= 1) return UDiv{0u, 0u, 1u};
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return UDiv{(uint32_t)m, l - 1, 0u};
}
__device__ __forceinline__ uint32_t udiv(uint32_t n, const UDiv& v) {
  if (v.one) return n;
  const uint32_t t = __umulhi(v.m, n);
  return (t + ((n - t) >> 1)) >> v.sh;
}

struct AdaP {
  float* p; const float* g; float* m; float* row; float* col;   // col == nullptr: unfactored (row = v)
  long numel; int nb, R, C, factored;
  long row_toff, col_off, blk_off, rm_off, rm_toff;              // prefix offsets (tasks / elements)
  long cp_toff, part_off;                                        // column-partial tasks / partial floats
  UDiv div_rc, div_c;                                            // element index -> (matrix, row, column)
};

__host__ __device__ __forceinline__ bool is_wide(int C) { return C >= 64 && C <= 64 * KMAX; }

__device__ __forceinline__ long off_of(const AdaP& q, int which) {
  return which == 0 ? q.row_toff : which == 1 ? q.col_off : which == 2 ? q.blk_off : which == 3 ? q.rm_toff
                                                                                                  : q.cp_toff;
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

// Wide factored tensors (64 <= C <= 2560), one pass over g: task (b, rb) covers rows
// rb*RB .. rb*RB+RB-1 of matrix b.  Row statistics are finished here (wave reduction per row);
// column sums of the block go to part[b][rb][c] (finished by ada_cols, fixed order).
__global__ __launch_bounds__(EB) void ada_colpart(const AdaP* __restrict__ t, int n, long ntasks, float b2t,
                                                  float eps1, float* __restrict__ part) {
  __shared__ float red[4][64 * KMAX];
  const long task = blockIdx.x;
  if (task >= ntasks) return;
  const AdaP& q = t[find_param(t, n, task, 4)];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nrb = (q.R + RB - 1) / RB;
  const long lt = task - q.cp_toff;
  const int b = (int)(lt / nrb), rb = (int)(lt % nrb);
  const int r0 = rb * RB, r1 = min(q.R, r0 + RB);
  const int nk = (q.C + 63) / 64;
  float cacc[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) cacc[k] = 0.f;
  // the wave's RB/4 rows: their sums stay in registers (lane j keeps row j's) and the row EMAs are updated
  // once after the loop -- a read-modify-write per row inside it serialised every row on a memory round trip
  float rsum = 0.f;
  if (q.C % 4 == 0 && ((uintptr_t)q.g & 15) == 0) {
    // float4 columns: lane owns columns 4 lane + 256 k4 .. +3 (k4 < nk4); cacc[4 k4 + e] = column 4 lane + 256 k4 + e
    const int nk4 = (q.C + 255) / 256;
    // the wave's next row is loaded while this one is summed (one row per round trip otherwise)
    float4 cur[KMAX / 4], nxt[KMAX / 4];
    auto load_row = [&](int r, float4 (&dst)[KMAX / 4]) {
      const float* g = q.g + ((long)b * q.R + r) * q.C;
#pragma unroll
      for (int k4 = 0; k4 < KMAX / 4; ++k4) {
        const int c = 4 * lane + 256 * k4;
        if (k4 < nk4 && c < q.C) dst[k4] = *reinterpret_cast<const float4*>(g + c);
      }
    };
    if (r0 + wv < r1) load_row(r0 + wv, cur);
    for (int j = 0; j < RB / 4; ++j) {
      const int r = r0 + wv + 4 * j;
      if (r >= r1) break;
      if (j + 1 < RB / 4 && r + 4 < r1) load_row(r + 4, nxt);
      float s = 0.f;
#pragma unroll
      for (int k4 = 0; k4 < KMAX / 4; ++k4) {
        const int c = 4 * lane + 256 * k4;
        if (k4 < nk4 && c < q.C) {
          const float4 v = cur[k4];
          const float e0 = v.x * v.x + eps1, e1 = v.y * v.y + eps1, e2 = v.z * v.z + eps1, e3 = v.w * v.w + eps1;
          s += (e0 + e1) + (e2 + e3);
          cacc[4 * k4] += e0; cacc[4 * k4 + 1] += e1; cacc[4 * k4 + 2] += e2; cacc[4 * k4 + 3] += e3;
        }
      }
      s = wave_sum(s);
      rsum = lane == j ? s : rsum;
#pragma unroll
      for (int k4 = 0; k4 < KMAX / 4; ++k4) cur[k4] = nxt[k4];
    }
#pragma unroll
    for (int k4 = 0; k4 < KMAX / 4; ++k4)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (k4 < nk4 && 4 * lane + 256 * k4 + e < q.C) red[wv][4 * lane + 256 * k4 + e] = cacc[4 * k4 + e];
  } else {
    for (int j = 0; j < RB / 4; ++j) {   // (the early exit keeps this loop rolled)
      const int r = r0 + wv + 4 * j;
      if (r >= r1) break;
      const float* g = q.g + ((long)b * q.R + r) * q.C;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        const int c = lane + 64 * k;
        if (k < nk && c < q.C) {
          const float v = g[c];
          const float e = v * v + eps1;
          s += e;
          cacc[k] += e;
        }
      }
      s = wave_sum(s);
      rsum = lane == j ? s : rsum;
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < nk) red[wv][lane + 64 * k] = cacc[k];
  }
  {
    const int r = r0 + wv + 4 * lane;
    if (lane < RB / 4 && r < r1) row_update(q, (long)b * q.R + r, rsum, b2t);
  }
  __syncthreads();
  float* dst = part + q.part_off + ((long)b * nrb + rb) * q.C;
  for (int c = threadIdx.x; c < q.C; c += EB) dst[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

// row tasks of NARROW factored tensors: 256 rows per wave (lane = 4 rows; a task per 64 rows left each wave's
// parameter search -- ~9 dependent table loads -- in front of one 4-byte row: ~18.6 M such rows at L15, the
// degenerate (O, I, 1) pointwise-conv weights, ran 95 us)
constexpr int ROWS_PER_TASK = 256;
__global__ void ada_rows(const AdaP* __restrict__ t, int n, long ntasks, float b2t, float eps1) {
  const int lane = threadIdx.x & 63;
  // wave-uniform task made provably uniform: the parameter search and the table fields become scalar loads
  const long task = (long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (task >= ntasks) return;
  const AdaP& q = t[find_param(t, n, task, 0)];
  const long lt = task - q.row_toff;
  if (is_wide(q.C)) {      // (wide rows are done by ada_colpart; kept for a wide tensor with no tasks)
    const float* g = q.g + lt * q.C;
    float s = 0.f;
    for (int c = lane; c < q.C; c += 64) s += g[c] * g[c] + eps1;
    s = wave_sum(s);
    if (lane == 0) row_update(q, lt, s, b2t);
    return;
  }
  const long nrows = (long)q.nb * q.R, base = lt * ROWS_PER_TASK;
  if (q.C == 1 && ((uintptr_t)q.g & 15) == 0 && ((uintptr_t)q.row & 15) == 0 && base + ROWS_PER_TASK <= nrows) {
    // one element per row: lane owns rows base + 4 lane .. +3 (16-B loads of g and of the row state)
    const long lr = base + 4 * lane;
    const float4 g = *reinterpret_cast<const float4*>(q.g + lr);
    float4 v = *reinterpret_cast<const float4*>(q.row + lr);
    v.x = b2t * v.x + (1.f - b2t) * ((g.x * g.x + eps1) / q.C);
    v.y = b2t * v.y + (1.f - b2t) * ((g.y * g.y + eps1) / q.C);
    v.z = b2t * v.z + (1.f - b2t) * ((g.z * g.z + eps1) / q.C);
    v.w = b2t * v.w + (1.f - b2t) * ((g.w * g.w + eps1) / q.C);
    *reinterpret_cast<float4*>(q.row + lr) = v;
    return;
  }
#pragma unroll
  for (int k = 0; k < ROWS_PER_TASK / 64; ++k) {
    const long lr = base + lane + 64 * k;
    if (lr < nrows) {
      const float* g = q.g + lr * q.C;
      float s = 0.f;
#pragma unroll 8     // independent loads in flight (a serial chain of load latencies otherwise)
      for (int c = 0; c < q.C; ++c) s += g[c] * g[c] + eps1;
      row_update(q, lr, s, b2t);
    }
  }
}

// one thread per factored column: col = b2t*col + (1-b2t)*mean_r(g^2 + eps1)
// wide: sum of the ada_colpart partials in row-block order; narrow: direct sum over the R rows
__global__ void ada_cols(const AdaP* __restrict__ t, int n, long ncols, float b2t, float eps1,
                         const float* __restrict__ part) {
  const long cidx = (long)blockIdx.x * EB + threadIdx.x;
  if (cidx >= ncols) return;
  // the block's first column's parameter by a uniform (scalar) search, then a short per-lane forward scan
  int pi = find_param(t, n, (long)blockIdx.x * EB, 1);
  while (pi + 1 < n && t[pi + 1].col_off <= cidx) ++pi;
  const AdaP& q = t[pi];
  const long lc = cidx - q.col_off;     // = b*C + j
  const int b = (int)(lc / q.C), j = (int)(lc % q.C);
  float s = 0.f;
  if (is_wide(q.C)) {
    const int nrb = (q.R + RB - 1) / RB;
    const float* pp = part + q.part_off + (long)b * nrb * q.C + j;
#pragma unroll 8     // (fixed order kept: the unrolled adds still run k = 0, 1, 2, ...)
    for (int k = 0; k < nrb; ++k) s += pp[(long)k * q.C];
  } else if (q.C == 1 && q.R % 4 == 0 && ((uintptr_t)q.g & 15) == 0) {
    // C == 1 (the pointwise-conv weights (O, I, 1): R = I rows of one element): the column is contiguous, so
    // 16-B loads, a quarter of the latency rounds; the adds keep the r = 0, 1, 2, ... order (bit-identical)
    const float4* g4 = reinterpret_cast<const float4*>(q.g + (long)b * q.R);
#pragma unroll 8
    for (int r4 = 0; r4 < q.R / 4; ++r4) {
      const float4 v = g4[r4];
      s += v.x * v.x + eps1;
      s += v.y * v.y + eps1;
      s += v.z * v.z + eps1;
      s += v.w * v.w + eps1;
    }
  } else {
    const float* g = q.g + (long)b * q.R * q.C + j;
#pragma unroll 8
    for (int r = 0; r < q.R; ++r) {
      const float v = g[(long)r * q.C];
      s += v * v + eps1;
    }
  }
  q.col[lc] = b2t * q.col[lc] + (1.f - b2t) * (s / q.R);
}

// mean over R of the row state per (param, b): wide R -> one wave per b; narrow -> 64 b per wave
__global__ void ada_rowmean(const AdaP* __restrict__ t, int n, long ntasks, float* __restrict__ rowmean) {
  const int lane = threadIdx.x & 63;
  const long task = (long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (task >= ntasks) return;
  const AdaP& q = t[find_param(t, n, task, 3)];
  if (!q.factored) return;
  const long lt = task - q.rm_toff;
  if (q.R >= 64) {
    float s = 0.f;
#pragma unroll 8
    for (int r = lane; r < q.R; r += 64) s += q.row[lt * q.R + r];
    s = wave_sum(s);
    if (lane == 0) rowmean[q.rm_off + lt] = s / q.R;
  } else {
    const long b = lt * 64 + lane;
    if (b < q.nb) {
      float s = 0.f;
#pragma unroll 8
      for (int r = 0; r < q.R; ++r) s += q.row[b * q.R + r];
      rowmean[q.rm_off + b] = s / q.R;
    }
  }
}

// The update direction of 4 consecutive elements i..i+3 (same row: C % 4 == 0, i % 4 == 0) or of
// one element (n4 == 1).  32-bit index arithmetic (numel < 2^31, checked on the host).
template <int W>
__device__ __forceinline__ void ada_u(const AdaP& q, const float* rowmean, unsigned i, float b2t, float eps1,
                                      bool update_v, float (&u)[W]) {
  float g[W];
  if constexpr (W == 4) {
    const float4 v = *reinterpret_cast<const float4*>(q.g + i);
    g[0] = v.x; g[1] = v.y; g[2] = v.z; g[3] = v.w;
  } else {
    g[0] = q.g[i];
  }
  if (!q.factored) {
#pragma unroll
    for (int e = 0; e < W; ++e) {
      float v = q.row[i + e];
      if (update_v) {
        v = b2t * v + (1.f - b2t) * (g[e] * g[e] + eps1);
        q.row[i + e] = v;
      }
      u[e] = g[e] * rsqrtf(v);
    }
    return;
  }
  // (the two divisions by the tensor's R*C and C as multiply-high sequences: as plain 32-bit divisions they were
  // ~40 VALU per element group in two HBM-bound passes)
  const unsigned rc = (unsigned)q.R * (unsigned)q.C;
  const unsigned b = udiv(i, q.div_rc), w = i - b * rc;
  const unsigned r = udiv(w, q.div_c), c = w - r * (unsigned)q.C;
  const float rf = rsqrtf(q.row[(long)b * q.R + r] / rowmean[q.rm_off + b]);
  const float* cp = q.col + (long)b * q.C + c;
#pragma unroll
  for (int e = 0; e < W; ++e) u[e] = g[e] * rf * rsqrtf(cp[e]);
}

__device__ __forceinline__ bool vec4_ok(const AdaP& q) {
  return (q.numel % 4 == 0) && (!q.factored || q.C % 4 == 0) && ((uintptr_t)q.g % 16 == 0) &&
         ((uintptr_t)q.p % 16 == 0) && (!q.m || (uintptr_t)q.m % 16 == 0) &&
         (q.factored || (uintptr_t)q.row % 16 == 0);
}

// per-block sum of u^2 -> partial[blk] (summed in block order by ada_apply: deterministic)
__global__ __launch_bounds__(EB) void ada_sumsq(const AdaP* __restrict__ t, int n, const float* __restrict__ rowmean,
                                                float b2t, float eps1, float* __restrict__ partial) {
  __shared__ float red[EB / 64];
  const int pi = find_param(t, n, blockIdx.x, 2);
  const AdaP& q = t[pi];
  const long start = (long)(blockIdx.x - q.blk_off) * CHUNK;
  const long end = min(q.numel, start + CHUNK);
  float s = 0.f;
  if (vec4_ok(q)) {
    // CHUNK / (4 EB) = 4 float4 steps per thread, unrolled: their loads are in flight together
#pragma unroll
    for (int j = 0; j < CHUNK / (4 * EB); ++j) {
      const long i = start + 4 * threadIdx.x + (long)j * 4 * EB;
      if (i < end) {
        float u[4];
        ada_u<4>(q, rowmean, (unsigned)i, b2t, eps1, true, u);
        s += u[0] * u[0] + u[1] * u[1] + u[2] * u[2] + u[3] * u[3];
      }
    }
  } else {
    for (long i = start + threadIdx.x; i < end; i += EB) {
      float u[1];
      ada_u<1>(q, rowmean, (unsigned)i, b2t, eps1, true, u);
      s += u[0] * u[0];
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(EB) void ada_apply(const AdaP* __restrict__ t, int n, const float* __restrict__ rowmean,
                                                float b2t, float eps1, const float* __restrict__ partial, float lr,
                                                float beta1, float clip) {
  __shared__ float red[EB / 64];
  const int pi = find_param(t, n, blockIdx.x, 2);
  const AdaP& q = t[pi];
  // RMS(u) of the whole tensor: its blocks' partials in block order
  const int nblk = (int)((q.numel + CHUNK - 1) / CHUNK);
  float ps = 0.f;
  for (int k = threadIdx.x; k < nblk; k += EB) ps += partial[q.blk_off + k];
  ps = wave_sum(ps);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ps;
  __syncthreads();
  const float sumsq = red[0] + red[1] + red[2] + red[3];
  const long start = (long)(blockIdx.x - q.blk_off) * CHUNK;
  const long end = min(q.numel, start + CHUNK);
  const float rms = sqrtf(sumsq / (float)q.numel);
  const float scale = lr / fmaxf(rms / clip, 1.f);
  if (vec4_ok(q)) {
    // the CHUNK / (4 EB) = 4 steps unrolled with every load (g, factors, m, p) issued before the first store: vmcnt
    // counts loads and stores in one in-order queue, so step j + 1's loads behind step j's stores waited for them
    constexpr int NJ = CHUNK / (4 * EB);
    float u[NJ][4];
    float4 mv[NJ], pv[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const long i = start + 4 * threadIdx.x + (long)j * 4 * EB;
      if (i < end) {
        ada_u<4>(q, rowmean, (unsigned)i, b2t, eps1, false, u[j]);
        if (q.m) mv[j] = *reinterpret_cast<const float4*>(q.m + i);
        pv[j] = *reinterpret_cast<const float4*>(q.p + i);
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const long i = start + 4 * threadIdx.x + (long)j * 4 * EB;
      if (i >= end) break;
      float4 upd = make_float4(u[j][0] * scale, u[j][1] * scale, u[j][2] * scale, u[j][3] * scale);
      if (q.m) {
        const float4 m = mv[j];
        upd.x = beta1 * m.x + (1.f - beta1) * upd.x;
        upd.y = beta1 * m.y + (1.f - beta1) * upd.y;
        upd.z = beta1 * m.z + (1.f - beta1) * upd.z;
        upd.w = beta1 * m.w + (1.f - beta1) * upd.w;
        *reinterpret_cast<float4*>(q.m + i) = upd;
      }
      float4 p = pv[j];
      p.x -= upd.x; p.y -= upd.y; p.z -= upd.z; p.w -= upd.w;
      *reinterpret_cast<float4*>(q.p + i) = p;
    }
  } else {
    for (long i = start + threadIdx.x; i < end; i += EB) {
      float u[1];
      ada_u<1>(q, rowmean, (unsigned)i, b2t, eps1, false, u);
      float upd = u[0] * scale;
      if (q.m) {
        upd = beta1 * q.m[i] + (1.f - beta1) * upd;
        q.m[i] = upd;
      }
      q.p[i] -= upd;
    }
  }
}

}  // namespace

CFM_EXPORT size_t cfm_adafactor_table_bytes(int n_params) { return (size_t)n_params * sizeof(AdaP); }

CFM_EXPORT int cfm_adafactor_fill_table(void* host_table, int i, float* p, const float* g, float* m, float* row,
                                        float* col, long numel, int nb, int R, int C, long row_toff, long col_off,
                                        long blk_off, long rm_off, long rm_toff, long cp_toff, long part_off) {
  CFM_REQUIRE(host_table && p && g && row, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(numel < (1L << 31), CFM_ERR_SHAPE, "tensor too large (2^31 elements)");
  AdaP* t = reinterpret_cast<AdaP*>(host_table) + i;
  t->p = p; t->g = g; t->m = m; t->row = row; t->col = col;
  t->numel = numel; t->nb = nb; t->R = R; t->C = C; t->factored = col != nullptr;
  t->div_rc = udiv_make((uint32_t)R * (uint32_t)C);
  t->div_c = udiv_make((uint32_t)C);
  t->row_toff = row_toff; t->col_off = col_off; t->blk_off = blk_off; t->rm_off = rm_off; t->rm_toff = rm_toff;
  t->cp_toff = cp_toff; t->part_off = part_off;
  return CFM_OK;
}

CFM_EXPORT int cfm_adafactor_blocks(long numel) { return (int)((numel + CHUNK - 1) / CHUNK); }

// number of row tasks / row-mean tasks / column-partial tasks / partial floats a factored tensor
// contributes (see ada_rows / ada_rowmean / ada_colpart)
CFM_EXPORT long cfm_adafactor_row_tasks(int nb, int R, int C) {
  return is_wide(C) ? 0 : ((long)nb * R + ROWS_PER_TASK - 1) / ROWS_PER_TASK;
}
CFM_EXPORT long cfm_adafactor_colpart_tasks(int nb, int R, int C) { return is_wide(C) ? (long)nb * ((R + RB - 1) / RB) : 0; }
CFM_EXPORT long cfm_adafactor_part_floats(int nb, int R, int C) {
  return is_wide(C) ? (long)nb * ((R + RB - 1) / RB) * C : 0;
}
CFM_EXPORT long cfm_adafactor_rowmean_tasks(int nb, int R) { return R >= 64 ? (long)nb : ((long)nb + 63) / 64; }

CFM_EXPORT int cfm_adafactor_step(const void* dev_table, int n, long nrow_tasks, long ncols, long nblocks,
                                  long nrm_tasks, long ncp_tasks, float* rowmean, float* part, float* partial,
                                  float lr, float beta1, float beta2t, float eps1, float clip, void* stream) {
  CFM_REQUIRE(dev_table && rowmean && partial && n > 0 && (ncp_tasks == 0 || part), CFM_ERR_ARG, "bad args");
  const AdaP* t = reinterpret_cast<const AdaP*>(dev_table);
  hipStream_t s = cfm::as_stream(stream);
  if (ncp_tasks > 0)
    hipLaunchKernelGGL(ada_colpart, dim3((unsigned)ncp_tasks), dim3(EB), 0, s, t, n, ncp_tasks, beta2t, eps1, part);
  if (nrow_tasks > 0)
    hipLaunchKernelGGL(ada_rows, dim3((unsigned)((nrow_tasks + 3) / 4)), dim3(256), 0, s, t, n, nrow_tasks, beta2t,
                       eps1);
  if (ncols > 0)
    hipLaunchKernelGGL(ada_cols, dim3((unsigned)((ncols + EB - 1) / EB)), dim3(EB), 0, s, t, n, ncols, beta2t, eps1,
                       part);
  if (nrm_tasks > 0)
    hipLaunchKernelGGL(ada_rowmean, dim3((unsigned)((nrm_tasks + 3) / 4)), dim3(256), 0, s, t, n, nrm_tasks, rowmean);
  hipLaunchKernelGGL(ada_sumsq, dim3((unsigned)nblocks), dim3(EB), 0, s, t, n, rowmean, beta2t, eps1, partial);
  hipLaunchKernelGGL(ada_apply, dim3((unsigned)nblocks), dim3(EB), 0, s, t, n, rowmean, beta2t, eps1, partial, lr,
                     beta1, clip);
  return cfm::check_launch("cfm_adafactor_step");
}
