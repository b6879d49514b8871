// GEMM lab: standalone experiments on the d-wide GEMM family's main loop (K-major A and B, C bf16), outside
// libcfm.  C[m][n] = sum_k A[m][k] * B[n][k], M = 11,936 tokens, N = 512, K = 2048 (the FFN-up data gradient /
// FFN-down forward shape).  Each variant is timed with HIP events (median of 7 x 20 launches) and checked against a
// naive fp32 reference.  MODE bits: 1 = load-only (no LDS reads / MFMA), 2 = compute-only (no DMA), 4 = DMA pieces
// interleaved with the MFMAs (else issued right after the barrier), 8 = skip the C stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
#include <algorithm>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void* base, unsigned bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_base, unsigned voff) {
  const unsigned l = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds_base);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(l), "v"(voff), "s"(r)
               : "memory", "m0");
}
#pragma clang diagnostic pop

template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// K-major [R][64] bf16 image, 128-B rows: chunk c of row r at slot c ^ ((r >> 1) & 7)
__device__ __forceinline__ int slot64(int r, int c) { return c ^ ((r >> 1) & 7); }

struct P {
  const bf16* A; const bf16* B; bf16* C;
  int M, N, K;
  unsigned abytes, bbytes;
};

// XCD-aware linear tile id (blocks b, b + 8 share an XCD): each XCD gets a contiguous run of tiles
__device__ __forceinline__ int xcd_id(int L, int nwg) {
  if (nwg <= 8) return L;
  const int xcd = L & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
}

// BM x BN tile, BK 64 stages, WM x WN waves of (BM/WM) x (BN/WN) (16x16x32 MFMA blocks), NST-stage ring with PREF
// stages in flight
template <int BM, int BN, int WM, int WN, int NST, int PREF, int MODE>
__global__ __launch_bounds__(WM * WN * 64) void kk_kernel(P p) {
  constexpr int BK = 64, NW = WM * WN;
  constexpr int ABY = BM * BK * 2, BBY = BN * BK * 2, STAGE = ABY + BBY;
  constexpr int AP = ABY / 1024, BPc = BBY / 1024, PIECES = AP + BPc;
  static_assert(PIECES % NW == 0, "even DMA split");
  constexpr int PW = PIECES / NW;                    // DMA pieces per wave per stage
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  static_assert(PREF < NST, "ring");
  __shared__ __attribute__((aligned(1024))) char lds[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = p.N / BN;
  const int id = xcd_id(blockIdx.x, gridDim.x);
  const int tm = id / ntn, tn = id % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const __amdgpu_buffer_rsrc_t ra = mk_rsrc(p.A, p.abytes), rb = mk_rsrc(p.B, p.bbytes);
  // this wave's pieces: piece q = wid + NW * i; q < AP -> A rows 8(q) .. ; else B
  unsigned off[PW];
  int ldsoff[PW];
  bool isA[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int q = wid + NW * i;
    const bool a = q < AP;
    const int qq = a ? q : q - AP;
    const int r = qq * 8 + (lane >> 3), c = slot64(r, lane & 7);
    const int lim = a ? p.M : p.N;
    const int row = (a ? m0 : n0) + r < lim ? (a ? m0 : n0) + r : lim - 1;
    off[i] = (unsigned)(((long)row * p.K + 8 * c) * 2);
    ldsoff[i] = (a ? 0 : ABY) + qq * 1024;
    isA[i] = a;
  }
  const int nk = p.K / BK;
  auto issue_piece = [&](int kt, int i) {
    char* st = lds + (kt % NST) * STAGE;
    dma16(isA[i] ? ra : rb, st + ldsoff[i], off[i] + kt * (BK * 2));
  };
  auto issue = [&](int kt) {
#pragma unroll
    for (int i = 0; i < PW; ++i) issue_piece(kt, i);
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if constexpr (!(MODE & 2)) {
#pragma unroll
    for (int s = 0; s < PREF; ++s) issue(s);
  }
  // fragment read: rows row0.., k chunk kc (16x16x32: lane l -> row l & 15, k 8 (l >> 4) .. +7)
  auto frag = [&](const char* img, int row0, int kk) {
    const int r = row0 + (lane & 15), c = (kk >> 3) + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * slot64(r, c));
  };
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (!(MODE & 2)) {
      // stage kt landed once only the younger issued stages are outstanding
      const int younger = min(PREF - 1, nk - 1 - kt);
      if (younger >= 3) vm_wait<3 * PW>();
      else if (younger == 2) vm_wait<2 * PW>();
      else if (younger == 1) vm_wait<PW>();
      else vm_wait<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool pf = !(MODE & 2) && kt + PREF < nk;
    if constexpr (!(MODE & 4)) {
      if (pf) issue(kt + PREF);
    }
    if constexpr (MODE & 1) continue;
    const char* sa = lds + (kt % NST) * STAGE;
    const char* sb = sa + ABY;
    bf16x8 af[2][FM], bfr[2][FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[0][j] = frag(sb, wn * FN * 16 + 16 * j, 0);
#pragma unroll
    for (int i = 0; i < FM; ++i) af[0][i] = frag(sa, wm * FM * 16 + 16 * i, 0);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[1][j] = frag(sb, wn * FN * 16 + 16 * j, 32);
#pragma unroll
    for (int i = 0; i < FM; ++i) af[1][i] = frag(sa, wm * FM * 16 + 16 * i, 32);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s][i], bfr[s][j], acc[i][j], 0, 0, 0);
        if constexpr (MODE & 4) {
          // spread this wave's PW pieces over the 2 * FM MFMA groups of the step
          constexpr int G = 2 * FM;
          const int g = s * FM + i;
#pragma unroll
          for (int q = 0; q < PW; ++q)
            if (g == (q * G) / PW && pf) issue_piece(kt + PREF, q);
        }
      }
    }
  }
  if constexpr (MODE & 8) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) t += acc[i][j][0] + acc[i][j][3];
    if (t == -1234.5f) p.C[tid] = (bf16)t;
    return;
  }
  // plain store: 16x16 block (i, j): lane -> col l & 15, rows 4 (l >> 4) + e
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * FN * 16 + 16 * j + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * FM * 16 + 16 * i + 4 * (lane >> 4) + e;
        if (m < p.M) p.C[(long)m * p.N + n] = (bf16)acc[i][j][e];
      }
    }
}

// Pipelined variant: the fragments of the next half-step (KSPLIT 1) or next K step (KSPLIT 2) are read while the
// current MFMAs run; one barrier per K step, placed where the next stage must become visible; the freed slot (stage
// kt - 1) is refilled right after it (NST - 1 stages issued ahead).
//   KSPLIT 1: WM x WN waves each own (BM/WM) x (BN/WN) and process both 32-deep halves of every stage.
//   KSPLIT 2: the waves form two groups of WM x WN; group g processes half g of every stage (wave tile twice as big
//             for the same wave count: fewer LDS reads per MFMA); the groups' partial sums are added through LDS.
// MODE bits: 1 load-only, 2 compute-only, 8 no stores, 32 s_setprio(1) around the MFMAs, 64 DMA interleaved.
template <int BM, int BN, int WM, int WN, int KSPLIT, int NST, int MODE>
__global__ __launch_bounds__(WM * WN * KSPLIT * 64) void kk2_kernel(P p) {
  constexpr int BK = 64, NW = WM * WN * KSPLIT;
  constexpr int ABY = BM * BK * 2, BBY = BN * BK * 2, STAGE = ABY + BBY;
  constexpr int AP = ABY / 1024, BPc = BBY / 1024, PIECES = AP + BPc;
  static_assert(PIECES % NW == 0, "even DMA split");
  constexpr int PW = PIECES / NW;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  static_assert(NST >= 3, "ring");
  static_assert(KSPLIT == 1 || BM * (BN + 4) * 4 <= NST * STAGE, "reduction staging fits the ring");
  __shared__ __attribute__((aligned(1024))) char lds[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid / (WM * WN), wl = wid % (WM * WN);
  const int wm = wl / WN, wn = wl % WN;
  const int ntn = p.N / BN;
  const int id = xcd_id(blockIdx.x, gridDim.x);
  const int tm = id / ntn, tn = id % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const __amdgpu_buffer_rsrc_t ra = mk_rsrc(p.A, p.abytes), rb = mk_rsrc(p.B, p.bbytes);
  unsigned off[PW];
  int ldsoff[PW];
  bool isA[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int q = wid + NW * i;
    const bool a = q < AP;
    const int qq = a ? q : q - AP;
    const int r = qq * 8 + (lane >> 3), c = slot64(r, lane & 7);
    const int lim = a ? p.M : p.N;
    const int row = (a ? m0 : n0) + r < lim ? (a ? m0 : n0) + r : lim - 1;
    off[i] = (unsigned)(((long)row * p.K + 8 * c) * 2);
    ldsoff[i] = (a ? 0 : ABY) + qq * 1024;
    isA[i] = a;
  }
  const int nk = p.K / BK;
  auto issue_piece = [&](int kt, int i) {
    dma16(isA[i] ? ra : rb, lds + (kt % NST) * STAGE + ldsoff[i], off[i] + kt * (BK * 2));
  };
  auto issue = [&](int kt) {
#pragma unroll
    for (int i = 0; i < PW; ++i) issue_piece(kt, i);
  };
  auto frag = [&](const char* img, int row0, int kk) {
    const int r = row0 + (lane & 15), c = (kk >> 3) + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * slot64(r, c));
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][FM], bfr[2][FN];
  auto read = [&](int buf, int kt, int sub) {
    const char* sa = lds + (kt % NST) * STAGE;
    const char* sb = sa + ABY;
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[buf][j] = frag(sb, wn * FN * 16 + 16 * j, 32 * sub);
#pragma unroll
    for (int i = 0; i < FM; ++i) af[buf][i] = frag(sa, wm * FM * 16 + 16 * i, 32 * sub);
  };
  auto mma = [&](int buf, bool dma, int kt_dma) {
    if constexpr (MODE & 32) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[buf][i], bfr[buf][j], acc[i][j], 0, 0, 0);
      if constexpr (MODE & 64) {
#pragma unroll
        for (int q = 0; q < PW; ++q)
          if (i == (q * FM) / PW && dma) issue_piece(kt_dma, q);
      }
    }
    if constexpr (MODE & 32) __builtin_amdgcn_s_setprio(0);
  };
  // wait until stage s is complete given the stages issued so far (up to `last`)
  auto wait_stage = [&](int s, int last) {
    const int younger = min(NST - 2, last - s);
    if (younger >= 3) vm_wait<3 * PW>();
    else if (younger == 2) vm_wait<2 * PW>();
    else if (younger == 1) vm_wait<PW>();
    else vm_wait<0>();
  };
  constexpr bool LOADS = !(MODE & 2), MATH = !(MODE & 1);
  int last = -1;
  if constexpr (LOADS) {
    for (int s = 0; s < NST - 1 && s < nk; ++s) issue(s);
    last = min(NST - 2, nk - 1);
    wait_stage(0, last);
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if constexpr (MATH) read(0, 0, KSPLIT == 1 ? 0 : grp);
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    const int kn = kt + NST - 1;                 // the stage that refills slot (kt - 1) after this step's barrier
    const bool pf = LOADS && kn < nk;
    if constexpr (KSPLIT == 1) {
      if constexpr (MATH) {
        read(1, kt, 1);
        mma(0, false, 0);
      }
      if (more) {
        if constexpr (LOADS) wait_stage(kt + 1, last);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (!(MODE & 64) || !MATH) {
          if (pf) issue(kn);
        }
        if (pf) last = kn;
        if constexpr (MATH) read(0, kt + 1, 0);
      }
      if constexpr (MATH) mma(1, (MODE & 64) && pf, kn);
    } else {
      // two K steps per iteration so the fragment buffers are compile-time indexed (a run-time index sends them
      // to scratch)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = kt + u;
        if (k < nk) {
          const bool mr = k + 1 < nk;
          const int kn2 = k + NST - 1;
          const bool pf2 = LOADS && kn2 < nk;
          if (mr) {
            if constexpr (LOADS) wait_stage(k + 1, last);
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (!(MODE & 64) || !MATH) {
              if (pf2) issue(kn2);
            }
            if (pf2) last = kn2;
            if constexpr (MATH) read(1 - u, k + 1, grp);
          }
          if constexpr (MATH) mma(u, (MODE & 64) && pf2, kn2);
        }
      }
      ++kt;
    }
  }
  if constexpr (KSPLIT == 2) {
    // group 1 stages its partial sums in LDS (the ring is free once every wave passed this barrier)
    __syncthreads();
    float* st = reinterpret_cast<float*>(lds);
    constexpr int EPS = BN + 4;
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            st[(wm * FM * 16 + 16 * i + 4 * (lane >> 4) + e) * EPS + wn * FN * 16 + 16 * j + (lane & 15)] = acc[i][j][e];
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[i][j][e] += st[(wm * FM * 16 + 16 * i + 4 * (lane >> 4) + e) * EPS + wn * FN * 16 + 16 * j + (lane & 15)];
  }
  if constexpr (MODE & 8) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) t += acc[i][j][0] + acc[i][j][3];
    if (t == -1234.5f) p.C[tid] = (bf16)t;
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * FN * 16 + 16 * j + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * FM * 16 + 16 * i + 4 * (lane >> 4) + e;
        if (m < p.M) p.C[(long)m * p.N + n] = (bf16)acc[i][j][e];
      }
    }
}

// Warp-specialised loading: NC = WM x WN compute waves (the KSPLIT-1 pipelined loop, no VMEM at all) + NL loader waves
// that only issue the LDS-DMA, wait for it and join the one barrier per K step.
template <int BM, int BN, int WM, int WN, int NL, int NST, int MODE>
__global__ __launch_bounds__((WM * WN + NL) * 64) void kk3_kernel(P p) {
  constexpr int BK = 64, NC = WM * WN;
  constexpr int ABY = BM * BK * 2, BBY = BN * BK * 2, STAGE = ABY + BBY;
  constexpr int AP = ABY / 1024, BPc = BBY / 1024, PIECES = AP + BPc;
  static_assert(PIECES % NL == 0, "even DMA split");
  constexpr int PW = PIECES / NL;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  __shared__ __attribute__((aligned(1024))) char lds[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = p.N / BN;
  const int id = xcd_id(blockIdx.x, gridDim.x);
  const int tm = id / ntn, tn = id % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = p.K / BK;
  if (wid >= NC) {
    const int lw = wid - NC;
    const __amdgpu_buffer_rsrc_t ra = mk_rsrc(p.A, p.abytes), rb = mk_rsrc(p.B, p.bbytes);
    unsigned off[PW];
    int ldsoff[PW];
    bool isA[PW];
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int q = lw + NL * i;
      const bool a = q < AP;
      const int qq = a ? q : q - AP;
      const int r = qq * 8 + (lane >> 3), c = slot64(r, lane & 7);
      const int lim = a ? p.M : p.N;
      const int row = (a ? m0 : n0) + r < lim ? (a ? m0 : n0) + r : lim - 1;
      off[i] = (unsigned)(((long)row * p.K + 8 * c) * 2);
      ldsoff[i] = (a ? 0 : ABY) + qq * 1024;
      isA[i] = a;
    }
    auto issue = [&](int kt) {
#pragma unroll
      for (int i = 0; i < PW; ++i)
        dma16(isA[i] ? ra : rb, lds + (kt % NST) * STAGE + ldsoff[i], off[i] + kt * (BK * 2));
    };
    auto wait_stage = [&](int s, int last) {
      const int younger = min(NST - 2, last - s);
      if (younger >= 3) vm_wait<3 * PW>();
      else if (younger == 2) vm_wait<2 * PW>();
      else if (younger == 1) vm_wait<PW>();
      else vm_wait<0>();
    };
    for (int s = 0; s < NST - 1 && s < nk; ++s) issue(s);
    int last = min(NST - 2, nk - 1);
    wait_stage(0, last);
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt + 1 < nk; ++kt) {
      wait_stage(kt + 1, last);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int kn = kt + NST - 1;
      if (kn < nk) {
        issue(kn);
        last = kn;
      }
    }
    return;
  }
  const int wm = wid / WN, wn = wid % WN;
  auto frag = [&](const char* img, int row0, int kk) {
    const int r = row0 + (lane & 15), c = (kk >> 3) + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * slot64(r, c));
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][FM], bfr[2][FN];
  auto read = [&](int buf, int kt, int sub) {
    const char* sa = lds + (kt % NST) * STAGE;
    const char* sb = sa + ABY;
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[buf][j] = frag(sb, wn * FN * 16 + 16 * j, 32 * sub);
#pragma unroll
    for (int i = 0; i < FM; ++i) af[buf][i] = frag(sa, wm * FM * 16 + 16 * i, 32 * sub);
  };
  auto mma = [&](int buf) {
    if constexpr (MODE & 32) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[buf][i], bfr[buf][j], acc[i][j], 0, 0, 0);
    if constexpr (MODE & 32) __builtin_amdgcn_s_setprio(0);
  };
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read(0, 0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    read(1, kt, 1);
    mma(0);
    if (kt + 1 < nk) {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      read(0, kt + 1, 0);
    }
    mma(1);
  }
  if constexpr (MODE & 8) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) t += acc[i][j][0] + acc[i][j][3];
    if (t == -1234.5f) p.C[tid] = (bf16)t;
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * FN * 16 + 16 * j + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * FM * 16 + 16 * i + 4 * (lane >> 4) + e;
        if (m < p.M) p.C[(long)m * p.N + n] = (bf16)acc[i][j][e];
      }
    }
}

__global__ void ref_kernel(const bf16* A, const bf16* B, float* C, int M, int N, int K) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)M * N) return;
  const int m = idx / N, n = idx % N;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(long)m * K + k] * (float)B[(long)n * K + k];
  C[idx] = s;
}

__global__ void fill_kernel(bf16* x, long n, uint32_t seed) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t h = (uint32_t)i * 2654435761u ^ seed;
  h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
  x[i] = (bf16)(((float)(h & 0xFFFF) / 32768.f - 1.f));
}

static std::vector<float> g_ref;
static int M = 32 * 373, N = 512, K = 2048;

template <int BM, int BN, int WM, int WN, int NST, int PREF, int MODE>
void run(const char* name, P p) {
  auto kfn = kk_kernel<BM, BN, WM, WN, NST, PREF, MODE>;
  const int tiles = ((p.M + BM - 1) / BM) * (p.N / BN);
  dim3 g(tiles), b(WM * WN * 64);
  hipLaunchKernelGGL(kfn, g, b, 0, 0, p);
  CK(hipDeviceSynchronize());
  double maxerr = -1;
  if (!(MODE & 11)) {
    std::vector<bf16> c((size_t)p.M * p.N);
    CK(hipMemcpy(c.data(), p.C, c.size() * 2, hipMemcpyDeviceToHost));
    double num = 0, den = 0;
    for (size_t i = 0; i < c.size(); ++i) {
      const double d = (double)(float)c[i] - g_ref[i];
      num += d * d; den += (double)g_ref[i] * g_ref[i];
    }
    maxerr = sqrt(num / den);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < 7; ++r) {
    CK(hipEventRecord(e0));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kfn, g, b, 0, 0, p);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms * 1000.f / 20);
  }
  std::sort(ts.begin(), ts.end());
  const double us = ts[3];
  printf("%-44s tiles %4d  %8.2f us  %6.0f TF/s  %.3f of peak  relL2 %.2e\n", name, tiles, us,
         2.0 * p.M * p.N * p.K / us / 1e6, 2.0 * p.M * p.N * p.K / us / 1e6 / 2500, maxerr);
}

template <int BM, int BN, int WM, int WN, int KS, int NST, int MODE>
void run2(const char* name, P p) {
  auto kfn = kk2_kernel<BM, BN, WM, WN, KS, NST, MODE>;
  const int tiles = ((p.M + BM - 1) / BM) * (p.N / BN);
  dim3 g(tiles), b(WM * WN * KS * 64);
  hipLaunchKernelGGL(kfn, g, b, 0, 0, p);
  CK(hipDeviceSynchronize());
  double maxerr = -1;
  if (!(MODE & 11)) {
    std::vector<bf16> c((size_t)p.M * p.N);
    CK(hipMemcpy(c.data(), p.C, c.size() * 2, hipMemcpyDeviceToHost));
    double num = 0, den = 0;
    for (size_t i = 0; i < c.size(); ++i) {
      const double d = (double)(float)c[i] - g_ref[i];
      num += d * d; den += (double)g_ref[i] * g_ref[i];
    }
    maxerr = sqrt(num / den);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < 7; ++r) {
    CK(hipEventRecord(e0));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kfn, g, b, 0, 0, p);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms * 1000.f / 20);
  }
  std::sort(ts.begin(), ts.end());
  const double us = ts[3];
  printf("%-44s tiles %4d  %8.2f us  %6.0f TF/s  %.3f of peak  relL2 %.2e\n", name, tiles, us,
         2.0 * p.M * p.N * p.K / us / 1e6, 2.0 * p.M * p.N * p.K / us / 1e6 / 2500, maxerr);
}

template <int BM, int BN, int WM, int WN, int NL, int NST, int MODE>
void run3(const char* name, P p) {
  auto kfn = kk3_kernel<BM, BN, WM, WN, NL, NST, MODE>;
  const int tiles = ((p.M + BM - 1) / BM) * (p.N / BN);
  dim3 g(tiles), b((WM * WN + NL) * 64);
  hipLaunchKernelGGL(kfn, g, b, 0, 0, p);
  CK(hipDeviceSynchronize());
  double maxerr = -1;
  if (!(MODE & 11)) {
    std::vector<bf16> c((size_t)p.M * p.N);
    CK(hipMemcpy(c.data(), p.C, c.size() * 2, hipMemcpyDeviceToHost));
    double num = 0, den = 0;
    for (size_t i = 0; i < c.size(); ++i) {
      const double d = (double)(float)c[i] - g_ref[i];
      num += d * d; den += (double)g_ref[i] * g_ref[i];
    }
    maxerr = sqrt(num / den);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < 7; ++r) {
    CK(hipEventRecord(e0));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kfn, g, b, 0, 0, p);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms * 1000.f / 20);
  }
  std::sort(ts.begin(), ts.end());
  const double us = ts[3];
  printf("%-44s tiles %4d  %8.2f us  %6.0f TF/s  %.3f of peak  relL2 %.2e\n", name, tiles, us,
         2.0 * p.M * p.N * p.K / us / 1e6, 2.0 * p.M * p.N * p.K / us / 1e6 / 2500, maxerr);
}

int main(int argc, char** argv) {
  if (argc > 1) K = atoi(argv[1]);
  if (argc > 2) N = atoi(argv[2]);
  bf16 *A, *B, *C;
  float* R;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  CK(hipMalloc(&R, (size_t)M * N * 4));
  hipLaunchKernelGGL(fill_kernel, dim3((M * (long)K + 255) / 256), dim3(256), 0, 0, A, (long)M * K, 1u);
  hipLaunchKernelGGL(fill_kernel, dim3((N * (long)K + 255) / 256), dim3(256), 0, 0, B, (long)N * K, 2u);
  hipLaunchKernelGGL(ref_kernel, dim3((M * (long)N + 255) / 256), dim3(256), 0, 0, A, B, R, M, N, K);
  CK(hipDeviceSynchronize());
  g_ref.resize((size_t)M * N);
  CK(hipMemcpy(g_ref.data(), R, g_ref.size() * 4, hipMemcpyDeviceToHost));
  P p{A, B, C, M, N, K, (unsigned)((size_t)M * K * 2), (unsigned)((size_t)N * K * 2)};
  printf("M %d N %d K %d\n", M, N, K);
  run<192, 128, 2, 4, 4, 3, 0>("old 192x128 8w(96x32) ring4", p);
  run3<192, 128, 2, 4, 4, 4, 0>("ws 8c(96x32)+4L ring4", p);
  run3<192, 128, 2, 4, 4, 4, 8>("  .. no stores", p);
  run3<192, 128, 2, 2, 4, 4, 0>("ws 4c(96x64)+4L ring4", p);
  run3<192, 128, 2, 2, 4, 4, 8>("  .. no stores", p);
  run3<256, 128, 4, 2, 4, 3, 0>("ws 256x128 8c(64x64)+4L ring3", p);
  run3<256, 128, 4, 2, 4, 3, 8>("  .. no stores", p);
  run3<256, 128, 2, 2, 4, 3, 8>("ws 256x128 4c(128x64)+4L ring3 no stores", p);
  run3<128, 128, 2, 2, 4, 4, 0>("ws 128x128 4c(64x64)+4L ring4", p);
  run3<128, 128, 2, 2, 4, 4, 8>("  .. no stores", p);
  return 0;
}
