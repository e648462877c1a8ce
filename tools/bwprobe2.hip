// bwprobe2.hip — write-pattern calibration for the sparse decode (1 GiB fp32 output).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// B threads per block, each writes one float4; optional dependent loads before the store (like a
// tile index + entry fetch) and an LDS round trip
template <int B, int NLOAD, bool LDS>
__global__ __launch_bounds__(B) void w1(float4* __restrict__ y, long n4, const unsigned* __restrict__ ts) {
  __shared__ f32x4 s[LDS ? B : 1];
  unsigned a = blockIdx.x;
#pragma unroll
  for (int i = 0; i < NLOAD; ++i) a = ts[(a * 2654435761u) & 1048575u];  // dependent scalar-ish loads
  f32x4 z = {0.f, (float)(a & 1), 2.f, 3.f};
  if (LDS) {
    s[threadIdx.x] = z;
    __syncthreads();
    z = s[(threadIdx.x + 1) % B];
  }
  const long j = (long)blockIdx.x * B + threadIdx.x;
  if (j < n4) *(f32x4*)(y + j) = z;
}

// grid-stride over tiles of B float4, G blocks
template <int B>
__global__ __launch_bounds__(B) void wgs(float4* __restrict__ y, long n4) {
  for (long t = blockIdx.x; t * B < n4; t += gridDim.x) {
    const long j = t * B + threadIdx.x;
    f32x4 z = {0.f, 1.f, 2.f, 3.f};
    if (j < n4) *(f32x4*)(y + j) = z;
  }
}

template <typename F> double timeit(F f, int reps) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a)); for (int r = 0; r < reps; ++r) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

int main() {
  const long n = 268435456; const double bytes = n * 4.0; const long n4 = n / 4;
  float* y; unsigned* ts; CK(hipMalloc(&y, n * 4)); CK(hipMalloc(&ts, 4 << 20)); CK(hipMemset(ts, 0, 4 << 20));
  auto rep = [&](const char* name, double ms) { printf("%-44s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9); };
  const int R = 20;
  rep("w1 B256 0load", timeit([&] { w1<256, 0, false><<<n4 / 256, 256>>>((float4*)y, n4, ts); }, R));
  rep("w1 B256 1load", timeit([&] { w1<256, 1, false><<<n4 / 256, 256>>>((float4*)y, n4, ts); }, R));
  rep("w1 B256 2load", timeit([&] { w1<256, 2, false><<<n4 / 256, 256>>>((float4*)y, n4, ts); }, R));
  rep("w1 B256 2load+LDS", timeit([&] { w1<256, 2, true><<<n4 / 256, 256>>>((float4*)y, n4, ts); }, R));
  rep("w1 B512 0load", timeit([&] { w1<512, 0, false><<<n4 / 512, 512>>>((float4*)y, n4, ts); }, R));
  rep("w1 B512 2load+LDS", timeit([&] { w1<512, 2, true><<<n4 / 512, 512>>>((float4*)y, n4, ts); }, R));
  rep("w1 B1024 0load", timeit([&] { w1<1024, 0, false><<<n4 / 1024, 1024>>>((float4*)y, n4, ts); }, R));
  rep("w1 B1024 1load", timeit([&] { w1<1024, 1, false><<<n4 / 1024, 1024>>>((float4*)y, n4, ts); }, R));
  rep("w1 B1024 2load+LDS", timeit([&] { w1<1024, 2, true><<<n4 / 1024, 1024>>>((float4*)y, n4, ts); }, R));
  for (int g : {4096, 16384, 65536, 131072}) {
    char nm[64]; snprintf(nm, sizeof nm, "wgs B256 grid=%d", g);
    rep(nm, timeit([&] { wgs<256><<<g, 256>>>((float4*)y, n4); }, R));
  }
  for (int g : {4096, 16384, 65536}) {
    char nm[64]; snprintf(nm, sizeof nm, "wgs B1024 grid=%d", g);
    rep(nm, timeit([&] { wgs<1024><<<g, 1024>>>((float4*)y, n4); }, R));
  }
  rep("memset", timeit([&] { CK(hipMemsetAsync(y, 0, n * 4)); }, R));
  return 0;
}
