// xcd_probe.hip -- where do the workgroups of a one-per-CU launch run?  Each workgroup (512 threads, 128 KiB of
// static LDS: one per CU, as the grouped weight-gradient kernel) records its XCC_ID, HW_ID and s_memrealtime start,
// then spins for a per-workgroup duration (uniform or jittered) before it ends.  The host prints how often
// xcc == blockIdx.x % 8, per round of 256 workgroups, and the start order of the later rounds' workgroups.
// Build: hipcc --offload-arch=gfx950 -O2 benchmarks/xcd_probe.hip -o benchmarks/xcd_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(512) void probe(unsigned* out, int spin_ticks, int jitter) {
  __shared__ char lds[128 * 1024];
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (char)threadIdx.x;
  __syncthreads();
  const long ticks = spin_ticks + (jitter ? (long)((blockIdx.x * 2654435761u) >> 20) % jitter : 0);
  while ((long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) {
    out[4 * blockIdx.x + 0] = xcc & 0xF;
    out[4 * blockIdx.x + 1] = hw;
    out[4 * blockIdx.x + 2] = (unsigned)t0;
    out[4 * blockIdx.x + 3] = (unsigned)(t0 >> 32) + lds[5];
  }
}

int main(int argc, char** argv) {
  const int grid = argc > 1 ? atoi(argv[1]) : 1536;
  const int jitter = argc > 2 ? atoi(argv[2]) : 0;
  unsigned* d;
  (void)hipMalloc(&d, 16 * grid);
  std::vector<unsigned> h(4 * grid);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, d, 2000, jitter);   // 100 MHz clock: 2000 = 20 us
    (void)hipMemcpy(h.data(), d, 16 * grid, hipMemcpyDeviceToHost);
  }
  int match = 0;
  std::vector<int> per_round_match((grid + 255) / 256, 0);
  for (int b = 0; b < grid; ++b) {
    const bool m = (int)h[4 * b] == b % 8;
    match += m;
    per_round_match[b / 256] += m;
  }
  printf("grid %d jitter %d: xcc == b %% 8 for %d of %d workgroups\n", grid, jitter, match, grid);
  for (size_t r = 0; r < per_round_match.size(); ++r) printf("  round %zu: %d of 256\n", r, per_round_match[r]);
  printf("first 16 workgroups: xcc");
  for (int b = 0; b < 16 && b < grid; ++b) printf(" %u", h[4 * b]);
  printf("\nworkgroups 256..271: xcc");
  for (int b = 256; b < 272 && b < grid; ++b) printf(" %u", h[4 * b]);
  // per XCD: count of workgroups and the distinct CUs (HW_ID bits: CU_ID 11:8, SH_ID 12, SE_ID 15:13)
  for (int x = 0; x < 8; ++x) {
    int n = 0;
    std::vector<unsigned> cus;
    for (int b = 0; b < grid; ++b)
      if ((int)h[4 * b] == x) {
        ++n;
        cus.push_back(h[4 * b + 1] & 0xFF00u);
      }
    std::sort(cus.begin(), cus.end());
    const int distinct = (int)(std::unique(cus.begin(), cus.end()) - cus.begin());
    printf("\nxcd %d: %d workgroups on %d distinct CU slots", x, n, distinct);
  }
  printf("\n");
  (void)hipFree(d);
  return 0;
}
