// writeshape_probe.hip — does the decode's write rate depend on which 4 KB pieces a one-wave workgroup writes?
// Store-only passes over 1 GiB (16-B stores per lane, one 64-lane wave per workgroup), shapes:
//   w4:    4 KB per wave, wave j -> piece j (4 KB pieces)
//   w8:    8 KB per wave, wave j -> pieces 2j, 2j + 1 (the decode's shape)
//   w8x:   8 KB per wave, wave j on XCD x = j % 8, l = j / 8 -> pieces 16 l + x and 16 l + 8 + x: every XCD writes the
//          same 4 KB pieces at the same 32 KB stride as under w4
//   w8h:   8 KB per wave, pieces j and j + P/2 (half the array apart)
//   w8nt:  w8 with non-temporal stores
//   w8w2:  8 KB per workgroup of 2 waves, 4 KB per wave (wave w of workgroup j -> piece 2j + w)
//   w16w4: 16 KB per workgroup of 4 waves, 4 KB per wave
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/writeshape_probe tools/writeshape_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int MODE>
__global__ __launch_bounds__(64) void wr(f32x4* __restrict__ out, long P, float v) {
  const int lane = threadIdx.x;
  const long j = blockIdx.x;
  long p0, p1;
  if (MODE == 0) { p0 = j; p1 = -1; }
  else if (MODE == 1 || MODE == 4) { p0 = 2 * j; p1 = 2 * j + 1; }
  else if (MODE == 2) { const long x = j & 7, l = j >> 3; p0 = 16 * l + x; p1 = 16 * l + 8 + x; }
  else { p0 = j; p1 = j + P / 2; }
  const f32x4 val = {v, v + 1.f, v + 2.f, v + 3.f};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4* a = out + p0 * 256 + q * 64 + lane;
    if (MODE == 4) __builtin_nontemporal_store(val, a); else *a = val;
  }
  if (p1 >= 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4* a = out + p1 * 256 + q * 64 + lane;
      if (MODE == 4) __builtin_nontemporal_store(val, a); else *a = val;
    }
  }
}

template <int W>
__global__ __launch_bounds__(64 * W) void wrw(f32x4* __restrict__ out, float v) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long p0 = (long)blockIdx.x * W + w;
  const f32x4 val = {v, v + 1.f, v + 2.f, v + 3.f};
#pragma unroll
  for (int q = 0; q < 4; ++q) out[p0 * 256 + q * 64 + lane] = val;
}

int main() {
  const long bytes = 1l << 30, P = bytes / 4096;  // 4 KB pieces
  f32x4* out;
  CK(hipMalloc(&out, bytes));
  CK(hipMemset(out, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto t = [&](auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipEventRecord(e0));
    for (int it = 0; it < 10; ++it) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 100.0f;
  };
  for (int round = 0; round < 3; ++round) {
    const float a = t([&] { wr<0><<<P, 64>>>(out, P, 1.f); });
    const float b = t([&] { wr<1><<<P / 2, 64>>>(out, P, 1.f); });
    const float c = t([&] { wr<2><<<P / 2, 64>>>(out, P, 1.f); });
    const float d = t([&] { wr<3><<<P / 2, 64>>>(out, P, 1.f); });
    const float e = t([&] { wr<4><<<P / 2, 64>>>(out, P, 1.f); });
    const float f = t([&] { wrw<2><<<P / 2, 128>>>(out, 1.f); });
    const float g = t([&] { wrw<4><<<P / 4, 256>>>(out, 1.f); });
    printf("round %d: 1 GiB of stores: w4 %.1f us | w8 %.1f | w8x %.1f | w8h %.1f | w8nt %.1f | w8w2 %.1f | w16w4 %.1f\n",
           round, a, b, c, d, e, f, g);
  }
  return 0;
}
