// mx_probe.hip -- empirical operand / scale lane maps of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3) on gfx950.
// One wave per probe: A and B are 32 bytes (8 VGPRs) per lane, scale_a / scale_b one e8m0 byte per lane.
//   probe kind 0 (A data):  A = e4m3 1.0 at (lane L, byte J) only, B = all 1.0, scale_a[lane] = 127 + bit_b(lane)
//                           for b = probe's bit (bit 6 = "no scale bit": all 127): D[r][*] = 2^bit_b(scale lane of
//                           (L, J)) in row r = (L, J)'s row, 0 elsewhere.
//   probe kind 1 (B data):  the same with the roles of A and B swapped (D[*][c] in column c).
// Output per probe: the row (col) holding the nonzero and its value.  Build: hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(int kind, float* out) {
  const int pid = blockIdx.x, lane = threadIdx.x;
  const int L = pid / (32 * 7), J = (pid / 7) % 32, bit = pid % 7;
  union { i32x8 v; unsigned char b[32]; } a, b;
  for (int j = 0; j < 32; ++j) {
    const unsigned char one = 0x38;   // e4m3 1.0
    const unsigned char sel = (lane == L && j == J) ? one : 0;
    if (kind == 0) { a.b[j] = sel; b.b[j] = one; } else { a.b[j] = one; b.b[j] = sel; }
  }
  const int sb = bit < 6 ? ((lane >> bit) & 1) : 0;
  const int sa = kind == 0 ? 127 + sb : 127, sbb = kind == 1 ? 127 + sb : 127;
  f32x16 acc = {0};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a.v, b.v, acc, 0, 0, 0, sa, 0, sbb);
  // C/D: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), col = lane & 31;
    out[(long)pid * 1024 + row * 32 + col] = acc[r];
  }
}

int main() {
  const int np = 64 * 32 * 7;
  float* d;
  (void)hipMalloc(&d, sizeof(float) * np * 1024);
  std::vector<float> h((size_t)np * 1024);
  for (int kind = 0; kind < 2; ++kind) {
    hipLaunchKernelGGL(probe, dim3(np), dim3(64), 0, 0, kind, d);
    (void)hipMemcpy(h.data(), d, sizeof(float) * np * 1024, hipMemcpyDeviceToHost);
    printf("kind %d (%s): lane byte -> %s, value, scale lane\n", kind, kind ? "B" : "A", kind ? "col" : "row");
    int bad = 0;
    for (int L = 0; L < 64; ++L)
      for (int J = 0; J < 32; ++J) {
        int where = -1, slane = 0;
        float val = 0.f;
        for (int bit = 0; bit < 7; ++bit) {
          const float* D = &h[((size_t)(L * 32 + J) * 7 + bit) * 1024];
          int cnt = 0;
          float v = 0.f;
          int w = -1;
          for (int i = 0; i < 32; ++i) {
            // kind 0: rows of column 0; kind 1: columns of row 0 (the other operand is all ones)
            const float x = kind == 0 ? D[i * 32 + 0] : D[0 * 32 + i];
            if (x != 0.f) { ++cnt; v = x; w = i; }
          }
          if (cnt != 1) { ++bad; continue; }
          if (bit == 6) { where = w; val = v; }
          else if (v == 2.f) slane |= 1 << bit;
        }
        printf("%s L%02d B%02d -> %2d  v %.1f  slane %2d\n", kind ? "B" : "A", L, J, where, val, slane);
      }
    printf("kind %d: %d probes without a single nonzero\n", kind, bad);
  }
  (void)hipFree(d);
  return 0;
}
