// copyprobe.hip — which copy shape makes the stream-copy comparator a real ceiling?  1 GiB fp32
// copied (2 GiB of traffic), each variant timed with events over 10 launches after 3 warm-ups, two rounds:
//   wgT x F: workgroups of T threads, F float4 per lane, one contiguous T*F*16-B chunk per workgroup;
//            NT = non-temporal loads (nt+) and/or stores (+nt).
// Build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/copyprobe tools/copyprobe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int T, int F, bool NTL, bool NTS>
__global__ __launch_bounds__(T) void cp(const f32x4* __restrict__ x, f32x4* __restrict__ y) {
  const long c0 = (long)blockIdx.x * T * F;
  f32x4 v[F];
#pragma unroll
  for (int j = 0; j < F; ++j) {
    const f32x4* p = x + c0 + j * T + threadIdx.x;
    v[j] = NTL ? __builtin_nontemporal_load(p) : *p;
  }
#pragma unroll
  for (int j = 0; j < F; ++j) {
    f32x4* p = y + c0 + j * T + threadIdx.x;
    if (NTS) __builtin_nontemporal_store(v[j], p);
    else *p = v[j];
  }
}

template <int T, int F, bool NTL, bool NTS>
void run(const char* name, const f32x4* x, f32x4* y, long n4, int round) {
  const unsigned g = (unsigned)(n4 / (T * F));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) cp<T, F, NTL, NTS><<<g, T>>>(x, y);
  CK(hipEventRecord(e0));
  for (int it = 0; it < 10; ++it) cp<T, F, NTL, NTS><<<g, T>>>(x, y);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("round %d %-22s %.1f us per 1 GiB copy (%.0f GB/s of 2 GiB)\n", round, name, ms * 100.0f,
         2.0 * (double)n4 * 16 / (ms / 10 * 1e-3) / 1e9);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const long n4 = (1l << 28) / 4;
  f32x4 *x, *y;
  CK(hipMalloc(&x, n4 * 16));
  CK(hipMalloc(&y, n4 * 16));
  CK(hipMemset(x, 0, n4 * 16));
  CK(hipMemset(y, 0, n4 * 16));
  for (int round = 0; round < 2; ++round) {
    run<256, 4, true, false>("wg256x4 nt+ (flc_copy)", x, y, n4, round);
    run<256, 4, false, false>("wg256x4", x, y, n4, round);
    run<256, 4, true, true>("wg256x4 nt+nt", x, y, n4, round);
    run<64, 4, true, false>("wg64x4 nt+", x, y, n4, round);
    run<64, 8, true, false>("wg64x8 nt+", x, y, n4, round);
    run<64, 16, true, false>("wg64x16 nt+", x, y, n4, round);
    run<128, 8, true, false>("wg128x8 nt+", x, y, n4, round);
    run<256, 8, true, false>("wg256x8 nt+", x, y, n4, round);
    run<256, 2, true, false>("wg256x2 nt+", x, y, n4, round);
    run<512, 4, true, false>("wg512x4 nt+", x, y, n4, round);
    run<1024, 4, true, false>("wg1024x4 nt+", x, y, n4, round);
    run<64, 8, false, false>("wg64x8", x, y, n4, round);
  }
  return 0;
}
