// ctc.hip — CTC head of the training step and the greedy decoder, on the device.
//
//   cfm_ctc_loss_fwd / cfm_ctc_loss_bwd replace torch.nn.CTCLoss(blank, zero_infinity=True)
//   applied to log_softmax(logits) (runner.py:35,142-143; asrnn.py:45,256): log-softmax,
//   alpha/beta recursions and the gradient w.r.t. the LOGITS (softmax - posterior, i.e. the CTC
//   gradient already pushed through log_softmax) with no host synchronisation, so the whole
//   training step can be captured in one HIP graph.
//   cfm_ctc_greedy_decode replaces ASRNN.predict (asrnn.py:48-58: argmax over the vocabulary)
//   plus the id filtering of Vocab.decode (myvocab.py:211-231: drop <pad>/<blank>, no repeat
//   collapse unless asked).
//
// Kernels (B utterances, T frames, V classes, L_b target labels, S_b = 2 L_b + 1 states):
//   ctc_prep     one wave per frame row: lse = logsumexp(logits row); lpe[b,t,s] = logit of the
//                s-th extended label (blank, l1, blank, l2, ...) - lse          HBM: one row read
//   ctc_alphabeta one workgroup per (utterance, direction), one state per thread; the time loop sequential,
//                the 16 waves pipelined a block of 16 frames apart through edge rings in LDS (no workgroup
//                barrier per frame); lpe rows are prefetched 16 frames ahead into registers
//   ctc_grad     one workgroup per frame row: grad[v] = (exp(logit - lse) - sum_{s: l'(s)=v}
//                exp(alpha + beta + nll - lpe)) * scale; duplicate labels are summed in label order
//                (deterministic, no atomics)
#include "cfm_common.h"

#include <math.h>

namespace {

constexpr float NEG_INF = -INFINITY;
constexpr int PF = 16;   // frames of lpe prefetched per chunk

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == NEG_INF) return NEG_INF;
  return m + logf(expf(a - m) + expf(b - m));
}
// the alpha / beta recursion's 3-way log-sum-exp on the hardware exp2 / log2 (v_exp_f32 / v_log_f32: the
// arguments are <= 0 and the sum is in [1, 3], where both are accurate to about an ulp): the libm expf / logf
// range reductions made this the recursion's critical path (one barrier-separated frame per ~0.9 us at L60)
// the recursion's form: the largest of the three contributes exactly 1, so only the other two need an exponential
// (max3 / med3 / min3 are single instructions; the recursion is VALU-issue bound with 16 waves on 4 SIMDs)
__device__ __forceinline__ float lse3r(float a, float b, float c) {
  constexpr float L2E = 1.4426950408889634f, LN2F = 0.6931471805599453f;
  const float m = fmaxf(fmaxf(a, b), c), md = __builtin_amdgcn_fmed3f(a, b, c), lo = fminf(fminf(a, b), c);
  const float s = 1.f + (__builtin_amdgcn_exp2f((md - m) * L2E) + __builtin_amdgcn_exp2f((lo - m) * L2E));
  const float r = m + __builtin_amdgcn_logf(s) * LN2F;
  return m == NEG_INF ? NEG_INF : r;   // a select, not a branch (all -inf: the NaN of -inf - -inf is discarded)
}
__device__ __forceinline__ float lse3(float a, float b, float c) {
  constexpr float L2E = 1.4426950408889634f, LN2F = 0.6931471805599453f;
  const float m = fmaxf(fmaxf(a, b), c);
  if (m == NEG_INF) return NEG_INF;
  const float s = __builtin_amdgcn_exp2f((a - m) * L2E) + __builtin_amdgcn_exp2f((b - m) * L2E) +
                  __builtin_amdgcn_exp2f((c - m) * L2E);
  return m + __builtin_amdgcn_logf(s) * LN2F;
}

// extended label of state s
// (defined after CtcP: ext_label clamps the label ids)

struct CtcP {
  const float* logits; long sb, st;   // row (b, t) at logits + b*sb + t*st (batch- or time-major)
  const int32_t* tgt; int ldt;        // targets: utterance b at tgt + (off ? off[b] : b*ldt)
  const int32_t* off;
  const int32_t* in_len; const int32_t* tgt_len;
  int B, T, V, Smax, S;               // S = 2*Smax + 1 (state stride of the work arrays)
  int blank;
  float* lse;                         // (B, T)
  float* lpe;                         // (B, T, S)
  float* alpha;                       // (B, T, S)
  float* beta;                        // (B, T, S)
  float* nll_raw;                     // (B) -log p, may be +inf
  int32_t* grp;                       // (B, 2, Smax): per label position u: [0] head flag (first occurrence of
                                      // its class), [1] next position of the same class (-1: none)
  int32_t* ab_abort;                  // (2, B): 1 where the alpha (row 0) / beta (row 1) recursion gave up a wait
  int dbg_abort;                      // debug (cfm_ctc_set_debug): bit d forces direction d's abort path
};

__device__ __forceinline__ const int32_t* tgt_of(const CtcP& p, int b) {
  return p.tgt + (p.off ? (long)p.off[b] : (long)b * p.ldt);
}
// lengths are device data: clamp to the buffers' extents (in_len <= T, tgt_len <= Smax) so that a bad
// length can only give a wrong loss, never an access outside lpe / alpha / beta / sh[] (torch raises
// on such inputs; the host wrapper validates host-side lengths the same way)
__device__ __forceinline__ int in_len_of(const CtcP& p, int b) { return min(max(p.in_len[b], 0), p.T); }
__device__ __forceinline__ int tgt_len_of(const CtcP& p, int b) { return min(max(p.tgt_len[b], 0), p.Smax); }
// label u of an utterance, clamped to the class range (an out-of-range id would index x / corr[] out of bounds)
__device__ __forceinline__ int label_of(const CtcP& p, const int32_t* tg, int u) { return min(max(tg[u], 0), p.V - 1); }
__device__ __forceinline__ int ext_label(const CtcP& p, const int32_t* tg, int s) { return (s & 1) ? label_of(p, tg, s >> 1) : p.blank; }

// ---------------------------------------------------------------------------------- prep
__global__ __launch_bounds__(256) void ctc_prep(CtcP p) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)p.B * p.T) return;
  const int b = (int)(row / p.T), t = (int)(row % p.T);
  if (t >= in_len_of(p, b)) return;
  const float* x = p.logits + b * p.sb + t * p.st;
  float m = NEG_INF;
  const bool v4 = (p.V % 4 == 0) && (p.sb % 4 == 0) && (p.st % 4 == 0) && ((uintptr_t)p.logits % 16 == 0);
  if (v4) {
    for (int v = lane * 4; v < p.V; v += 256) {
      const float4 q = *reinterpret_cast<const float4*>(x + v);
      m = fmaxf(m, fmaxf(fmaxf(q.x, q.y), fmaxf(q.z, q.w)));
    }
  } else {
    for (int v = lane; v < p.V; v += 64) m = fmaxf(m, x[v]);
  }
  m = wave_max(m);
  float s = 0.f;
  if (v4) {
    for (int v = lane * 4; v < p.V; v += 256) {
      const float4 q = *reinterpret_cast<const float4*>(x + v);
      s += expf(q.x - m) + expf(q.y - m) + expf(q.z - m) + expf(q.w - m);
    }
  } else {
    for (int v = lane; v < p.V; v += 64) s += expf(x[v] - m);
  }
  s = wave_sum(s);
  const float l = m + logf(s);
  if (lane == 0) p.lse[row] = l;
  const int Sb = 2 * tgt_len_of(p, b) + 1;
  const int32_t* tg = tgt_of(p, b);
  float* dst = p.lpe + row * p.S;
  for (int st = lane; st < Sb; st += 64) dst[st] = x[ext_label(p, tg, st)] - l;
}

// ---------------------------------------------------------------------------------- alpha / beta
// blockIdx.x = utterance, blockIdx.y = 0 (alpha, forward in time) / 1 (beta, backward in time); 1024 threads.
// Wave-pipelined in blocks of PF frames: wave w owns states 64 w + lane and keeps its state's value of the previous
// frame in a register; the in-wave neighbours s - 1, s - 2 (beta: s + 1, s + 2) arrive by DPP wave shifts, and only
// the two states across a wave boundary come through LDS: the edge lanes store the block's PF values into a ring
// (four 16-B stores each), and the wave then publishes the block index.  Its successor waits for that once per
// block, loads the block's PF edge pairs into lanes 0..PF-1 and reads them per frame with v_readlane, so it
// runs one block behind with no synchronisation inside the block (the barrier form paid a workgroup barrier and
// an LDS round trip on every frame: 0.35 us per frame at L60).  A wait gives up after AB_SPIN polls, so no wave
// can spin forever: either direction's abort is recorded in ab_abort, and ctc_finish turns the utterance's loss
// (nll and the nll_raw ctc_grad reads) into NaN and counts it in the bound abort counter (cfm_ctc_bind_abort_counter),
// apart from genuine non-finite losses.  AB_SPIN polls of s_sleep 1 are ~0.1 s: a delayed co-resident wave
// (a side-stream kernel sharing the CU) slows the step, it does not abort it.
constexpr int AB_NT = 1024;
constexpr int AB_RB = 4;                  // ring depth in blocks
constexpr int AB_RF = AB_RB * PF;         // ring depth in frames
constexpr int AB_SPIN = 1 << 22;
typedef float f32x4e __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) volatile int lds_int;
typedef __attribute__((address_space(3))) volatile float lds_float;

template <int DIR>
__device__ __forceinline__ void ctc_alphabeta_dir(const CtcP& p, float* edge_mem, int* tag_mem, int* abort_mem,
                                                  float* fin) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int Tb = in_len_of(p, b), L = tgt_len_of(p, b), Sb = 2 * L + 1;
  const int32_t* tg = tgt_of(p, b);
  float* out = (DIR == 0 ? p.alpha : p.beta) + (long)b * p.T * p.S;
  const float* lp = p.lpe + (long)b * p.T * p.S;
  lds_int* tags = (lds_int*)tag_mem;
  lds_int* abort_flag = (lds_int*)abort_mem;
  lds_float* edge = (lds_float*)edge_mem;   // [2: nearest / second edge state][wave][frame % AB_RF]
  const int nw = (Sb + 63) >> 6;
  const int s = 64 * w + lane, sc = min(s, Sb - 1);
  const bool valid = s < Sb;
  bool skip;   // alpha may skip from s-2 (beta: from s+2) when the labels differ
  if (DIR == 0) skip = valid && s >= 2 && (s & 1) && ext_label(p, tg, s) != ext_label(p, tg, s - 2);
  else skip = s + 2 < Sb && (s & 1) && ext_label(p, tg, s) != ext_label(p, tg, s + 2);
  const bool has_pred = DIR == 0 ? (w > 0) : (w + 1 < nw);     // the wave whose edge states this one reads
  const bool has_succ = DIR == 0 ? (w + 1 < nw) : (w > 0);     // the wave that reads this one's
  const int pw = DIR == 0 ? w - 1 : w + 1, sw = DIR == 0 ? w + 1 : w - 1;
  const int le0 = DIR == 0 ? 63 : 0, le1 = DIR == 0 ? 62 : 1;   // this wave's edge lanes (nearest first)
  auto frame = [&](int i) { return DIR == 0 ? i : Tb - 1 - i; };
  auto wait_tag = [&](int ww, int want) {   // wave-uniform spin until wave ww has published block `want`
    for (int spin = 0;; ++spin) {
      if (__builtin_amdgcn_readfirstlane(tags[ww]) >= want) return;
      if (spin >= AB_SPIN || __builtin_amdgcn_readfirstlane(*abort_flag)) {
        *abort_flag = 1;
        return;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  };
  // lpe of this state, PF frames per block prefetched one block ahead (unconditional clamped loads)
  float cur[PF], nxt[PF];
  auto fetch = [&](float (&r)[PF], int i0) {
#pragma unroll
    for (int q = 0; q < PF; ++q) r[q] = lp[(long)frame(min(i0 + q, Tb - 1)) * p.S + sc];
  };
  const int nsteps = w < nw ? Tb : 0;
  float prev = NEG_INF;
  if (nsteps) fetch(cur, 0);
  for (int i0 = 0; i0 < nsteps; i0 += PF) {
    const int kb = i0 / PF;
    fetch(nxt, min(i0 + PF, Tb - 1));
    // the predecessor's edge pairs of frames i0 - 1 .. i0 + PF - 2, frame i0 - 1 + j in lane j
    float ex = NEG_INF, ey = NEG_INF, ev[PF];
    if (has_pred) {
      wait_tag(pw, kb);
      const int f = (max(i0 - 1 + lane, 0) & (AB_RF - 1)) + pw * AB_RF;
      ex = edge[f];
      ey = edge[AB_NT / 64 * AB_RF + f];
    }
    // ring reuse: this block overwrites block kb - RB, whose last frame the successor loads when it starts block
    // kb - RB + 1 (after which it publishes kb - RB + 1)
    if (has_succ && kb >= AB_RB) wait_tag(sw, kb - AB_RB + 1);
    // branch-free body (the DPP / readlane are convergent: a data-dependent exit keeps the loop from unrolling);
    // steps past the utterance in the last block change nothing
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int i = i0 + q;
      const bool live = i < nsteps;
      // previous frame's neighbours: alpha lane l <- lane l - 1 (wave_shr), beta lane l <- lane l + 1 (wave_shl);
      // the edge lanes get -inf, then the predecessor's pair
      // (the shifts write 0 into the edge lanes, which the predecessor's pair then replaces -- -inf for the first
      // wave, whose ex / ey stay -inf: no old-value moves and no branch on has_pred)
      constexpr int SH = DIR == 0 ? 0x138 : 0x130;
      constexpr int l0 = DIR == 0 ? 0 : 63, l1 = DIR == 0 ? 1 : 62;
      float n1 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(prev), SH, 0xF, 0xF, true));
      float n2 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(n1), SH, 0xF, 0xF, true));
      const float e0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ex), q));
      const float e1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ey), q));
      n1 = lane == l0 ? e0 : n1;
      n2 = lane == l0 ? e1 : (lane == l1 ? e0 : n2);
      // alpha: s - 1 < 0 only for lane 0 of wave 0, whose n1 is the DPP's -inf; beta: s + 1 >= Sb reads an invalid
      // lane (kept at -inf) or the DPP's -inf
      const float a2 = skip ? n2 : NEG_INF;
      float v = lse3r(prev, n1, a2) + cur[q];
      if (q == 0 && i0 == 0) v = DIR == 0 ? (s <= 1 ? cur[q] : NEG_INF) : (s >= Sb - 2 ? cur[q] : NEG_INF);
      if (!valid) v = NEG_INF;
      if (live && valid) out[(long)frame(i) * p.S + s] = v;
      prev = live ? v : prev;
      ev[q] = v;   // the edge lanes' values of the block, stored once per block below
    }
    if (has_succ) {   // lanes le0 / le1: the block's PF values as four 16-B stores each
      if (lane == le0 || lane == le1) {
        lds_float* dst = edge + (lane == le0 ? 0 : AB_NT / 64 * AB_RF) + w * AB_RF + (i0 & (AB_RF - 1));
#pragma unroll
        for (int q = 0; q < PF; q += 4)
          *(__attribute__((address_space(3))) volatile f32x4e*)(dst + q) = (f32x4e){ev[q], ev[q + 1], ev[q + 2], ev[q + 3]};
      }
    }
    // the block's edge stores land before its index (every wave publishes: the index is also the progress its
    // predecessor's ring reuse waits on)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) tags[w] = kb;
#pragma unroll
    for (int q = 0; q < PF; ++q) cur[q] = nxt[q];
  }
  if (DIR == 0) {
    if (s == Sb - 1) fin[0] = prev;
    if (s == Sb - 2) fin[1] = prev;
  }
}

__global__ __launch_bounds__(AB_NT) void ctc_alphabeta(CtcP p) {
  __shared__ __attribute__((aligned(16))) float edge[2 * (AB_NT / 64) * AB_RF];
  __shared__ int tags[AB_NT / 64];
  __shared__ int abort_flag;
  __shared__ float fin[2];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int Tb = in_len_of(p, b), L = tgt_len_of(p, b);
  if (Tb <= 0) {   // uniform over the workgroup
    if (blockIdx.y == 0 && tid == 0) p.nll_raw[b] = L == 0 ? 0.f : INFINITY;
    if (tid == 0) p.ab_abort[blockIdx.y * p.B + b] = 0;
    return;
  }
  if (tid < AB_NT / 64) tags[tid] = -1;
  if (tid == 0) {
    abort_flag = (p.dbg_abort >> blockIdx.y) & 1;
    fin[0] = fin[1] = NEG_INF;
  }
  __syncthreads();
  if (blockIdx.y == 0) ctc_alphabeta_dir<0>(p, edge, tags, &abort_flag, fin);
  else ctc_alphabeta_dir<1>(p, edge, tags, &abort_flag, fin);
  __syncthreads();
  if (tid == 0) {
    if (blockIdx.y == 0) p.nll_raw[b] = abort_flag ? NAN : -lse2(fin[0], fin[1]);
    p.ab_abort[blockIdx.y * p.B + b] = abort_flag;
  }
}

// nll (B): -log p, or 0 where infinite and zero_infinity; NaN (nll and nll_raw, which ctc_grad reads) where either
// recursion aborted, each such utterance counted in *aborts (nullable)
__global__ void ctc_finish(float* nll_raw, const int32_t* ab_abort, int B, int zero_inf, float* nll,
                           int32_t* aborts) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) {
    float v = nll_raw[b];
    if (ab_abort[b] | ab_abort[B + b]) {
      v = NAN;
      nll_raw[b] = v;
      if (aborts) atomicAdd(aborts, 1);
    }
    nll[b] = (zero_inf && isinf(v)) ? 0.f : v;
  }
}

// reduction 'mean' (torch: mean_b(nll_b / max(L_b, 1))) in one workgroup, sums in a fixed order; a non-finite
// result increments *bad (nullable)
__global__ __launch_bounds__(256) void ctc_mean_kernel(const float* __restrict__ nll, const int32_t* __restrict__ tl,
                                                       int B, float* __restrict__ loss, int32_t* __restrict__ bad) {
  __shared__ float red[4];
  float s = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) s += nll[b] / (float)max(tl[b], 1);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = (red[0] + red[1] + red[2] + red[3]) / (float)B;
    *loss = m;
    if (bad && !isfinite(m)) atomicAdd(bad, 1);
  }
}

// ---------------------------------------------------------------------------------- label classes
// once per utterance (one workgroup): for every label position u, whether it is the first occurrence of its
// class and the next position of the same class.  ctc_grad then sums a class's occurrences by walking that
// chain -- O(L) per frame instead of the O(L^2) first-occurrence scans it did per frame (global label loads
// per comparison: 0.8 ms per step at L60's ~500-label utterances)
__global__ __launch_bounds__(256) void ctc_group(CtcP p) {
  const int b = blockIdx.x, L = tgt_len_of(p, b), Lp = (L + 15) & ~15;
  const int32_t* tg = tgt_of(p, b);
  extern __shared__ int4 lab4[];          // [Smax rounded up to 16] clamped labels of the utterance, -1 past L
  int* lab = reinterpret_cast<int*>(lab4);
  for (int u = threadIdx.x; u < Lp; u += 256) lab[u] = u < L ? label_of(p, tg, u) : -1;
  __syncthreads();
  int32_t* head = p.grp + (long)b * 2 * p.Smax;
  int32_t* nxt = head + p.Smax;
  // both scans read 16 labels (four ds_read_b128) per step: the loops are LDS-latency bound, and a rare class
  // walks the whole utterance (one label per read: 65 us at L60's ~500-label utterances)
  for (int u = threadIdx.x; u < L; u += 256) {
    const int c = lab[u];
    bool first = true;
    for (int w0 = 0; w0 < u && first; w0 += 16) {
      int v[16];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int4 q = lab4[w0 / 4 + k];
        v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) first = first && !(w0 + j < u && v[j] == c);
    }
    int n = -1;
    for (int w0 = (u + 1) & ~15; w0 < L && n < 0; w0 += 16) {
      int v[16];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int4 q = lab4[w0 / 4 + k];
        v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
      }
#pragma unroll
      for (int j = 15; j >= 0; --j)           // descending: the smallest match in the chunk wins
        if (w0 + j > u && v[j] == c) n = w0 + j;
    }
    head[u] = first ? 1 : 0;
    nxt[u] = n;
  }
}

// ---------------------------------------------------------------------------------- gradient
// one workgroup (256 threads) per frame row; corr[V] in dynamic LDS
template <typename TG>
__global__ __launch_bounds__(256) void ctc_grad(CtcP p, const float* grad_out, int go_stride, int reduction,
                                                int zero_inf, TG* __restrict__ g, long gsb, long gst) {
  extern __shared__ float corr[];
  const long row = blockIdx.x;
  const int b = (int)(row / p.T), t = (int)(row % p.T);
  TG* dst = g + b * gsb + t * gst;
  const int Tb = in_len_of(p, b), L = tgt_len_of(p, b);
  const float nll = p.nll_raw[b];
  if (t >= Tb || (zero_inf && isinf(nll))) {   // as torch: padded frames and zeroed infinite losses
    for (int v = threadIdx.x; v < p.V; v += 256) dst[v] = from_f32<TG>(0.f);
    return;
  }
  float scale = grad_out[go_stride * b];
  if (reduction == 1) scale /= (float)p.B * (float)(L > 0 ? L : 1);
  for (int v = threadIdx.x; v < p.V; v += 256) corr[v] = 0.f;
  const long base = row * p.S;
  const int32_t* tg = tgt_of(p, b);
  __syncthreads();
  // blank: sum over the even states in state order (one wave, fixed-order tree)
  if (threadIdx.x < 64) {
    float s = 0.f;
    for (int u = threadIdx.x; u <= L; u += 64) {
      const int st = 2 * u;
      s += expf(p.alpha[base + st] + p.beta[base + st] + nll - p.lpe[base + st]);
    }
    s = wave_sum(s);
    if (threadIdx.x == 0) corr[p.blank] = s;
  }
  // labels: the first occurrence of each class sums all its occurrences in label order (the chain of
  // ctc_group: the same positions in the same order as a scan, so the same sums bit for bit)
  const int32_t* head = p.grp + (long)b * 2 * p.Smax;
  const int32_t* nxt = head + p.Smax;
  for (int u = threadIdx.x - 64; u >= 0 && u < L; u += 192) {
    if (!head[u]) continue;
    const int c = label_of(p, tg, u);
    float s = 0.f;
    for (int w = u; w >= 0; w = nxt[w]) {
      const int st = 2 * w + 1;
      s += expf(p.alpha[base + st] + p.beta[base + st] + nll - p.lpe[base + st]);
    }
    corr[c] = s;
  }
  __syncthreads();
  const float* x = p.logits + b * p.sb + t * p.st;
  const float l = p.lse[row];
  for (int v = threadIdx.x; v < p.V; v += 256) dst[v] = from_f32<TG>((expf(x[v] - l) - corr[v]) * scale);
}

// ---------------------------------------------------------------------------------- greedy decode
// one wave per frame row: argmax (first maximum, as torch.argmax) -> ids (B, T) int64
__global__ __launch_bounds__(256) void greedy_argmax(const float* __restrict__ x, long sb, long st, int B, int T,
                                                     int V, int64_t* __restrict__ ids) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)B * T) return;
  const float* r = x + (row / T) * sb + (row % T) * st;
  float m = NEG_INF;
  int mi = 0x7fffffff;
  for (int v = lane; v < V; v += 64) {
    const float q = r[v];
    if (q > m || (q == m && v < mi) || (isnan(q) && !isnan(m))) { m = q; mi = v; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oi = __shfl_xor(mi, o, 64);
    const bool take = (isnan(om) && !isnan(m)) || om > m || (om == m && oi < mi);
    if (take) { m = om; mi = oi; }
  }
  if (lane == 0) ids[row] = mi == 0x7fffffff ? 0 : mi;
}

// one thread per utterance: compact the ids of frames < len dropping `blank` and `pad`
// (pad < 0: none), optionally collapsing repeats first (standard CTC greedy)
__global__ void greedy_compact(const int64_t* __restrict__ ids, const int32_t* __restrict__ lens, int B, int T,
                               int blank, int pad, int collapse, int32_t* __restrict__ out, int32_t* __restrict__ out_len) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int Tb = lens ? min(lens[b], T) : T;
  int n = 0;
  long prev = -1;
  for (int t = 0; t < Tb; ++t) {
    const long c = ids[(long)b * T + t];
    const bool rep = collapse && c == prev;
    prev = c;
    if (rep || c == blank || c == pad) continue;
    out[(long)b * T + n++] = (int32_t)c;
  }
  for (int t = n; t < T; ++t) out[(long)b * T + t] = -1;
  out_len[b] = n;
}

CtcP make_p(const float* logits, long sb, long st, const int32_t* targets, int ldt, const int32_t* off,
            const int32_t* in_len, const int32_t* tgt_len, int B, int T, int V, int Smax, int blank, float* ws) {
  CtcP p;
  p.logits = logits; p.sb = sb; p.st = st; p.tgt = targets; p.ldt = ldt; p.off = off;
  p.in_len = in_len; p.tgt_len = tgt_len;
  p.B = B; p.T = T; p.V = V; p.Smax = Smax; p.S = 2 * Smax + 1; p.blank = blank;
  const long bt = (long)B * T, bts = bt * p.S;
  p.lse = ws;
  p.lpe = ws + bt;
  p.alpha = p.lpe + bts;
  p.beta = p.alpha + bts;
  p.nll_raw = p.beta + bts;
  p.grp = reinterpret_cast<int32_t*>(p.nll_raw + B);
  p.ab_abort = p.grp + 2L * B * Smax;
  p.dbg_abort = 0;
  return p;
}

int g_ctc_dbg_abort = 0;          // cfm_ctc_set_debug
int32_t* g_ctc_aborts = nullptr;  // cfm_ctc_bind_abort_counter

}  // namespace

CFM_EXPORT size_t cfm_ctc_ws_bytes(int B, int T, int Smax) {
  const long bt = (long)B * T;
  return sizeof(float) * (size_t)(bt + 3 * bt * (2L * Smax + 1) + B) + sizeof(int32_t) * 2 * (size_t)B * Smax +
         sizeof(int32_t) * 2 * (size_t)B;
}

CFM_EXPORT int cfm_ctc_set_debug(int force_abort_mask) {
  CFM_REQUIRE(force_abort_mask >= 0 && force_abort_mask <= 3, CFM_ERR_ARG, "mask: bit 0 alpha, bit 1 beta");
  g_ctc_dbg_abort = force_abort_mask;
  return CFM_OK;
}

CFM_EXPORT int cfm_ctc_bind_abort_counter(int32_t* counter) {
  g_ctc_aborts = counter;
  return CFM_OK;
}

CFM_EXPORT int cfm_ctc_loss_fwd(const float* logits, long sb, long st, const int32_t* targets, int ldt,
                                const int32_t* tgt_off, const int32_t* in_len, const int32_t* tgt_len, int B, int T,
                                int V, int Smax, int blank, int zero_infinity, float* nll, float* ws, void* stream) {
  CFM_REQUIRE(logits && targets && in_len && tgt_len && nll && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(B > 0 && T > 0 && V > 0 && Smax >= 0 && (tgt_off || ldt >= Smax), CFM_ERR_SHAPE, "bad shape");
  CFM_REQUIRE(blank >= 0 && blank < V, CFM_ERR_ARG, "blank out of range");
  const int S = 2 * Smax + 1;
  CFM_REQUIRE(S <= AB_NT, CFM_ERR_UNSUPPORTED, "target length must be <= 511");
  hipStream_t s = cfm::as_stream(stream);
  CtcP p = make_p(logits, sb, st, targets, ldt, tgt_off, in_len, tgt_len, B, T, V, Smax, blank, ws);
  p.dbg_abort = g_ctc_dbg_abort;
  hipLaunchKernelGGL(ctc_prep, dim3((unsigned)(((long)B * T + 3) / 4)), dim3(256), 0, s, p);
  hipLaunchKernelGGL(ctc_alphabeta, dim3(B, 2), dim3(AB_NT), 0, s, p);
  hipLaunchKernelGGL(ctc_finish, dim3(cdiv(B, 256)), dim3(256), 0, s, p.nll_raw, p.ab_abort, B, zero_infinity, nll,
                     g_ctc_aborts);
  return cfm::check_launch("cfm_ctc_loss_fwd");
}

CFM_EXPORT int cfm_ctc_loss_bwd(const float* logits, long sb, long st, const int32_t* targets, int ldt,
                                const int32_t* tgt_off, const int32_t* in_len, const int32_t* tgt_len, int B, int T,
                                int V, int Smax, int blank, int zero_infinity, const float* ws, const float* grad_out,
                                int grad_out_stride, int reduction, void* grad_logits, int dtype_grad, long gsb,
                                long gst, void* stream) {
  CFM_REQUIRE(logits && targets && in_len && tgt_len && ws && grad_out && grad_logits, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(B > 0 && T > 0 && V > 0, CFM_ERR_SHAPE, "bad shape");
  CFM_REQUIRE(reduction >= 0 && reduction <= 2, CFM_ERR_ARG, "reduction: 0 none / 1 mean / 2 sum");
  CFM_REQUIRE((size_t)V * sizeof(float) <= 64 * 1024, CFM_ERR_UNSUPPORTED, "V too large for the LDS row");
  hipStream_t s = cfm::as_stream(stream);
  CtcP p = make_p(logits, sb, st, targets, ldt, tgt_off, in_len, tgt_len, B, T, V, Smax, blank, const_cast<float*>(ws));
  const size_t sh = (size_t)V * sizeof(float);
  const dim3 grid((unsigned)((long)B * T));
  if (Smax > 0) hipLaunchKernelGGL(ctc_group, dim3(B), dim3(256), (size_t)((Smax + 15) & ~15) * sizeof(int), s, p);
  if (dtype_grad == CFM_BF16)
    hipLaunchKernelGGL(ctc_grad<bf16>, grid, dim3(256), sh, s, p, grad_out, grad_out_stride, reduction,
                       zero_infinity, (bf16*)grad_logits, gsb, gst);
  else if (dtype_grad == CFM_F32)
    hipLaunchKernelGGL(ctc_grad<float>, grid, dim3(256), sh, s, p, grad_out, grad_out_stride, reduction,
                       zero_infinity, (float*)grad_logits, gsb, gst);
  else
    return cfm::fail(CFM_ERR_DTYPE, "cfm_ctc_loss_bwd: grad dtype");
  return cfm::check_launch("cfm_ctc_loss_bwd");
}

CFM_EXPORT int cfm_ctc_mean(const float* nll, const int32_t* tgt_len, int B, float* loss, int32_t* nonfinite,
                            void* stream) {
  CFM_REQUIRE(nll && tgt_len && loss && B > 0, CFM_ERR_ARG, "bad args");
  hipLaunchKernelGGL(ctc_mean_kernel, dim3(1), dim3(256), 0, cfm::as_stream(stream), nll, tgt_len, B, loss, nonfinite);
  return cfm::check_launch("cfm_ctc_mean");
}

CFM_EXPORT int cfm_ctc_greedy_decode(const float* logits, long sb, long st, const int32_t* lens, int B, int T, int V,
                                     int blank, int pad, int collapse, int64_t* ids, int32_t* out, int32_t* out_len,
                                     void* stream) {
  CFM_REQUIRE(logits && ids && B > 0 && T > 0 && V > 0, CFM_ERR_ARG, "bad args");
  hipStream_t s = cfm::as_stream(stream);
  hipLaunchKernelGGL(greedy_argmax, dim3((unsigned)(((long)B * T + 3) / 4)), dim3(256), 0, s, logits, sb, st, B, T,
                     V, ids);
  if (out && out_len)
    hipLaunchKernelGGL(greedy_compact, dim3(cdiv(B, 64)), dim3(64), 0, s, ids, lens, B, T, blank, pad, collapse, out,
                       out_len);
  return cfm::check_launch("cfm_ctc_greedy_decode");
}
