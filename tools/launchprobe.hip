// launchprobe.hip — duration of an (almost) empty persistent launch of the encode kernel's shape
// (256 x 1024 threads, one block per CU, LDS 0 / 64 / 150 KB), back to back, events around 100 launches.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/launchprobe tools/launchprobe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int LDS_WORDS>
__global__ __launch_bounds__(1024) void k_lds(unsigned* out) {
  __shared__ unsigned s[LDS_WORDS > 0 ? LDS_WORDS : 1];
  s[threadIdx.x % (LDS_WORDS > 0 ? LDS_WORDS : 1)] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && s[5] == 12345u) out[blockIdx.x] = s[7];
}
__global__ __launch_bounds__(256) void k_small(unsigned* out) {
  if (threadIdx.x == 0 && out[blockIdx.x] == 12345u) out[blockIdx.x] = 1;
}

template <typename F>
float timeit(F f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 10; ++i) f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < 100; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 10.0f;  // us per launch
}

int main() {
  unsigned* o;
  CK(hipMalloc(&o, 4096 * 4));
  CK(hipMemset(o, 0, 4096 * 4));
  int cu = 256;
  CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  for (int r = 0; r < 2; ++r) {
    printf("1024x%d LDS 0      : %.2f us\n", cu, timeit([&] { k_lds<0><<<cu, 1024>>>(o); }));
    printf("1024x%d LDS 64 KB  : %.2f us\n", cu, timeit([&] { k_lds<16384><<<cu, 1024>>>(o); }));
    printf("1024x%d LDS 150 KB : %.2f us\n", cu, timeit([&] { k_lds<38400><<<cu, 1024>>>(o); }));
    printf("256x128 small      : %.2f us\n", timeit([&] { k_small<<<128, 256>>>(o); }));
    printf("alternating 150KB + small: %.2f us per pair\n", timeit([&] { k_small<<<128, 256>>>(o); k_lds<38400><<<cu, 1024>>>(o); }));
  }
  return 0;
}
