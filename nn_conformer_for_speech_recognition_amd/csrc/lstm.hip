// BiLSTM decoder recurrence: the reference's nn.LSTM over ONE unbatched sequence
// of L = B*T_enc steps (/root/reference/lib/standard/asrnn.py:38 constructs it, :252 calls it on the
// 2-D encoder output, which torch treats as a single sequence).  PyTorch gate order i, f, g, o:
//   gates_t = x_t W_ih^T + b_ih + b_hh + h_{t-1} W_hh^T        (the x part: one cfm_gemm over all steps)
//   c_t = sigmoid(f) c_{t-1} + sigmoid(i) tanh(g),  h_t = sigmoid(o) tanh(c_t),  h_{-1} = c_{-1} = 0
// The recurrence is latency bound (L serial mat-vecs of 4H x H), so it runs as ONE cooperative launch per
// pass: each workgroup owns 8 hidden units of one direction, keeps its 32 rows of W_hh (forward) or its 8
// columns of W_hh (backward) in registers for the whole sequence, and the workgroups of a direction
// exchange h_t (forward) / dgates_t (backward) through HBM as tagged 64-bit words (value + step tag, polled
// directly: no counters or cache-maintenance fences on the per-step path).  Both
// directions run concurrently in the same grid.  Co-residency is guaranteed by the cooperative launch
// (it fails instead of over-subscribing); every wait is bounded by a wall-clock limit that raises a device
// error flag and releases all other waiters, so a fault can never leave waves spinning.  The outputs y /
// gates / c / dg are plain stores: they are read only by later launches.
#include "cfm_common.h"

namespace {

constexpr int kUnits = 8;          // hidden units per workgroup
constexpr int kThreads = 256;
constexpr int kMaxH = 1024;
constexpr int kMaxK = kMaxH / 8;   // forward: H/8 weights per thread; backward: 4H/32 weights per thread
constexpr long long kSpinTicks = 200000000LL;   // 2 s of the 100 MHz wall clock

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float r = (1.f - e) / (1.f + e);
  return copysignf(r, x);
}

// Exchange words: (tag << 32) | float bits, written with one 64-bit agent-scope store, so a reader
// polls the data itself -- no counters, no L2 write-back / invalidate fences on the per-step path.
__device__ __forceinline__ void put_word(unsigned long long* p, unsigned tag, float v) {
  __hip_atomic_store(p, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// wait until word p carries `tag`; bounded by the wall-clock limit (then raises *err and returns 0)
__device__ __forceinline__ float get_word(const unsigned long long* p, unsigned tag, int* err) {
  unsigned long long w = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((unsigned)(w >> 32) != tag) {
    const long long t0 = wall_clock64();
    for (;;) {
      __builtin_amdgcn_s_sleep(1);
      w = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((unsigned)(w >> 32) == tag) break;
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return 0.f;
      if (wall_clock64() - t0 > kSpinTicks) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0.f;
      }
    }
  }
  return __uint_as_float((unsigned)w);
}

// gx: (L, ndir*4H) input gates incl. both biases; whh: (ndir, 4H, H); y: (L, ndir*H) outputs; gates_out:
// (L, ndir*4H) post-activation i,f,g,o; c_out: (L, ndir*H); xch: (ndir, 2, H) zeroed tagged words (a ring of
// two steps: a workgroup writes step s+2 only after every workgroup has read step s).  Step s carries tag s+1.
__global__ __launch_bounds__(kThreads) void lstm_fwd_rec(const float* __restrict__ gx, const float* __restrict__ whh,
                                                        float* __restrict__ y, float* __restrict__ gates_out,
                                                        float* __restrict__ c_out, unsigned long long* xch, int* err,
                                                        int L, int H, int nwg, int ndir) {
  __shared__ float hl[kMaxH];
  __shared__ float gl[4 * kUnits];
  const int tid = threadIdx.x;
  const int dir = blockIdx.x / nwg;
  const int u0 = (blockIdx.x % nwg) * kUnits;
  const int r = tid >> 3, q = tid & 7;            // row r of the workgroup's 32 (gate r/8, unit r%8)
  const int grow = (r >> 3) * H + u0 + (r & 7);   // row of W_hh / column of the gate vectors
  const int kpt = H >> 3;
  const long ldg = (long)ndir * 4 * H, ldy = (long)ndir * H;
  float w[kMaxK];
  const float* wr = whh + ((long)dir * 4 * H + grow) * H;
#pragma unroll
  for (int j = 0; j < kMaxK; ++j) w[j] = j < kpt ? wr[q + 8 * j] : 0.f;
  float c = 0.f;
  unsigned long long* xd = xch + (long)dir * 2 * H;
  for (int s = 0; s < L; ++s) {
    const int t = dir ? L - 1 - s : s;
    const float gxv = q == 0 ? gx[t * ldg + (long)dir * 4 * H + grow] : 0.f;
    float acc = 0.f;
    if (s > 0) {
      const unsigned long long* src = xd + (long)((s - 1) & 1) * H;
      for (int k = tid; k < H; k += kThreads) hl[k] = get_word(src + k, (unsigned)s, err);
      __syncthreads();
      float a4[4] = {0.f, 0.f, 0.f, 0.f};   // four independent FMA chains
#pragma unroll
      for (int j = 0; j < kMaxK; ++j)
        if (j < kpt) a4[j & 3] = fmaf(w[j], hl[q + 8 * j], a4[j & 3]);
      acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      acc += __shfl_xor(acc, 1);
      acc += __shfl_xor(acc, 2);
      acc += __shfl_xor(acc, 4);
    }
    if (q == 0) gl[r] = acc + gxv;
    __syncthreads();
    if (tid < kUnits) {
      const float ig = sigm(gl[tid]), fg = sigm(gl[kUnits + tid]);
      const float gg = tanh_f(gl[2 * kUnits + tid]), og = sigm(gl[3 * kUnits + tid]);
      c = fg * c + ig * gg;
      const float h = og * tanh_f(c);
      put_word(xd + (long)(s & 1) * H + u0 + tid, (unsigned)(s + 1), h);
      const long gb = t * ldg + (long)dir * 4 * H + u0 + tid;
      gates_out[gb] = ig;
      gates_out[gb + H] = fg;
      gates_out[gb + 2 * H] = gg;
      gates_out[gb + 3 * H] = og;
      c_out[t * ldy + (long)dir * H + u0 + tid] = c;
      y[t * ldy + (long)dir * H + u0 + tid] = h;
    }
  }
}

// Backward through time.  dy: (L, ndir*H) gradient of y; gates/c: the forward's saved values; dg: (L, ndir*4H)
// pre-activation gate gradients; xch: (ndir, 2, 4H) zeroed tagged words; step s (descending) carries tag L-s.
//   dh_t = dy_t + dgates_{t+1} W_hh,  dc_t = dh_t o (1 - tanh^2 c_t) + dc_{t+1} f_{t+1}
//   di = dc g i(1-i), df = dc c_{t-1} f(1-f), dg = dc i (1-g^2), do = dh tanh(c_t) o(1-o)
__global__ __launch_bounds__(kThreads) void lstm_bwd_rec(const float* __restrict__ dy, const float* __restrict__ whh,
                                                        const float* __restrict__ gates, const float* __restrict__ cst,
                                                        float* __restrict__ dg, unsigned long long* xch, int* err,
                                                        int L, int H, int nwg, int ndir) {
  __shared__ float dl[4 * kMaxH];
  const int tid = threadIdx.x;
  const int dir = blockIdx.x / nwg;
  const int u0 = (blockIdx.x % nwg) * kUnits;
  const int u = tid >> 5, p = tid & 31;   // unit u of the workgroup's 8, rows p + 32 j of W_hh
  const int H4 = 4 * H, kpt = H4 >> 5;
  const long ldg = (long)ndir * H4, ldy = (long)ndir * H;
  float w[kMaxK];
  const float* wc = whh + (long)dir * H4 * H + u0 + u;
#pragma unroll
  for (int j = 0; j < kMaxK; ++j) w[j] = j < kpt ? wc[(long)(p + 32 * j) * H] : 0.f;
  float dc_carry = 0.f;
  unsigned long long* xd = xch + (long)dir * 2 * H4;
  const long col = (long)dir * H + u0 + u;
  const long gcol = (long)dir * H4 + u0 + u;
  for (int s = L - 1; s >= 0; --s) {
    const int t = dir ? L - 1 - s : s;
    // this step's forward values (independent of the other workgroups): issue before the wait
    float dyv = 0.f, ig = 0.f, fg = 0.f, gg = 0.f, og = 0.f, ct = 0.f, cp = 0.f;
    if (p == 0) {
      dyv = dy[t * ldy + col];
      ig = gates[t * ldg + gcol];
      fg = gates[t * ldg + gcol + H];
      gg = gates[t * ldg + gcol + 2 * H];
      og = gates[t * ldg + gcol + 3 * H];
      ct = cst[t * ldy + col];
      if (s > 0) cp = cst[(dir ? t + 1 : t - 1) * ldy + col];
    }
    float acc = 0.f;
    if (s < L - 1) {
      const unsigned long long* src = xd + (long)((s + 1) & 1) * H4;
      for (int k = tid; k < H4; k += kThreads) dl[k] = get_word(src + k, (unsigned)(L - s - 1), err);
      __syncthreads();
      float a4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < kMaxK; ++j)
        if (j < kpt) a4[j & 3] = fmaf(w[j], dl[p + 32 * j], a4[j & 3]);
      acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      acc += __shfl_xor(acc, 1);
      acc += __shfl_xor(acc, 2);
      acc += __shfl_xor(acc, 4);
      acc += __shfl_xor(acc, 8);
      acc += __shfl_xor(acc, 16);
    }
    if (p == 0) {
      const float dh = dyv + acc;
      const float tc = tanh_f(ct);
      const float dc = dh * og * (1.f - tc * tc) + dc_carry;
      const float d_o = dh * tc * og * (1.f - og);
      const float d_i = dc * gg * ig * (1.f - ig);
      const float d_f = dc * cp * fg * (1.f - fg);
      const float d_g = dc * ig * (1.f - gg * gg);
      dc_carry = dc * fg;
      const unsigned tag = (unsigned)(L - s);
      unsigned long long* o = xd + (long)(s & 1) * H4 + u0 + u;
      put_word(o, tag, d_i);
      put_word(o + H, tag, d_f);
      put_word(o + 2 * H, tag, d_g);
      put_word(o + 3 * H, tag, d_o);
      float* og_ = dg + t * ldg + gcol;
      og_[0] = d_i;
      og_[H] = d_f;
      og_[2 * H] = d_g;
      og_[3 * H] = d_o;
    }
    // dl is rewritten by the next step's poll only after every thread passed this barrier
    __syncthreads();
  }
}

int launch_coop(const void* fn, int grid, void** args, hipStream_t s, const char* what) {
  hipError_t e = hipLaunchCooperativeKernel(fn, dim3(grid), dim3(kThreads), args, 0, s);
  if (e != hipSuccess) return cfm::fail(CFM_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e));
  return cfm::check_launch(what);
}

}  // namespace

// ws layout: [2 error flags, padded to 16 B][fwd ring (ndir, 2, H) u64][bwd ring (ndir, 2, 4H) u64]
CFM_EXPORT size_t cfm_lstm_ws_bytes(int H, int ndir) { return 16 + (size_t)ndir * 2 * 5 * H * 8; }

// Forward recurrence of one LSTM layer over one unbatched sequence (nn.LSTM on a 2-D input).
CFM_EXPORT int cfm_lstm_fwd(const float* gx, const float* whh, float* y, float* gates, float* c, int L, int H,
                            int ndir, void* ws, void* stream) {
  CFM_REQUIRE(gx && whh && y && gates && c && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(L > 0 && (ndir == 1 || ndir == 2), CFM_ERR_ARG, "L > 0, ndir 1 or 2");
  CFM_REQUIRE(H >= kUnits && H % kUnits == 0 && H <= kMaxH, CFM_ERR_SHAPE, "hidden size: multiple of 8, <= 1024");
  CFM_REQUIRE(((uintptr_t)ws & 15) == 0, CFM_ERR_ALIGN, "ws 16-B aligned");
  hipStream_t s = cfm::as_stream(stream);
  int* err = (int*)ws;
  unsigned long long* xch = (unsigned long long*)((char*)ws + 16);
  if (hipMemsetAsync(err, 0, sizeof(int), s) != hipSuccess ||
      hipMemsetAsync(xch, 0, (size_t)ndir * 2 * H * 8, s) != hipSuccess)
    return cfm::fail(CFM_ERR_LAUNCH, "cfm_lstm_fwd: memset");
  int nwg = H / kUnits;
  void* args[] = {(void*)&gx, (void*)&whh, (void*)&y, (void*)&gates, (void*)&c, (void*)&xch, (void*)&err,
                  (void*)&L, (void*)&H, (void*)&nwg, (void*)&ndir};
  return launch_coop((const void*)lstm_fwd_rec, nwg * ndir, args, s, "cfm_lstm_fwd");
}

// Backward recurrence: dg (L, ndir*4H) <- pre-activation gate gradients.  ws: the forward's workspace layout
// (its backward ring and second flag are used, so one workspace serves a forward and its backward).
CFM_EXPORT int cfm_lstm_bwd(const float* dy, const float* whh, const float* gates, const float* c, float* dg, int L,
                            int H, int ndir, void* ws, void* stream) {
  CFM_REQUIRE(dy && whh && gates && c && dg && ws, CFM_ERR_ARG, "null pointer");
  CFM_REQUIRE(L > 0 && (ndir == 1 || ndir == 2), CFM_ERR_ARG, "L > 0, ndir 1 or 2");
  CFM_REQUIRE(H >= kUnits && H % kUnits == 0 && H <= kMaxH, CFM_ERR_SHAPE, "hidden size: multiple of 8, <= 1024");
  CFM_REQUIRE(((uintptr_t)ws & 15) == 0, CFM_ERR_ALIGN, "ws 16-B aligned");
  hipStream_t s = cfm::as_stream(stream);
  int* err = (int*)ws + 1;
  unsigned long long* xch = (unsigned long long*)((char*)ws + 16) + (long)ndir * 2 * H;
  if (hipMemsetAsync(err, 0, sizeof(int), s) != hipSuccess ||
      hipMemsetAsync(xch, 0, (size_t)ndir * 2 * 4 * H * 8, s) != hipSuccess)
    return cfm::fail(CFM_ERR_LAUNCH, "cfm_lstm_bwd: memset");
  int nwg = H / kUnits;
  void* args[] = {(void*)&dy, (void*)&whh, (void*)&gates, (void*)&c, (void*)&dg, (void*)&xch, (void*)&err,
                  (void*)&L, (void*)&H, (void*)&nwg, (void*)&ndir};
  return launch_coop((const void*)lstm_bwd_rec, nwg * ndir, args, s, "cfm_lstm_bwd");
}
