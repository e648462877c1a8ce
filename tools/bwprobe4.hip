// bwprobe4.hip — write-pattern sweep for the dense decode (1 GiB fp32 of mostly zeros).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bwprobe4 tools/bwprobe4.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// one block per tile of TH*4*U floats, store u of thread t at float4 index t + u*TH (coalesced per u)
template <int TH, int U, int NT>
__global__ __launch_bounds__(TH) void w_tile(float* __restrict__ y, long n) {
  const long t0 = (long)blockIdx.x * TH * 4 * U;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    f32x4* p = (f32x4*)(y + t0) + threadIdx.x + u * TH;
    if (NT == 1) __builtin_nontemporal_store(z, p);
    else *p = z;
  }
}

// lane-contiguous: thread t stores U consecutive float4 (64 B at U = 4)
template <int TH, int U>
__global__ __launch_bounds__(TH) void w_lanecontig(float* __restrict__ y, long n) {
  const long t0 = (long)blockIdx.x * TH * 4 * U;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) ((f32x4*)(y + t0))[threadIdx.x * U + u] = z;
}

// XCD-aware tile order: block b -> tile (b % 8) * (T / 8) + b / 8 so each XCD writes a contiguous region
template <int TH, int U>
__global__ __launch_bounds__(TH) void w_tile_xcd(float* __restrict__ y, long n, long ntiles) {
  const long per = ntiles / 8;
  const long t = (long)(blockIdx.x % 8) * per + blockIdx.x / 8;
  const long t0 = t * TH * 4 * U;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) ((f32x4*)(y + t0))[threadIdx.x + u * TH] = z;
}

// wave-granular: each wave writes 4 KB contiguous (64 lanes x 16 B x 4)
template <int TH>
__global__ __launch_bounds__(TH) void w_wave4k(float* __restrict__ y, long n) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long w = (long)blockIdx.x * (TH / 64) + wid;
  f32x4* p = (f32x4*)(y + w * 1024);
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 4; ++u) p[lane + 64 * u] = z;
}

template <typename F>
double timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const long n = 268435456;
  const double bytes = n * 4.0;
  float* y;
  CK(hipMalloc(&y, n * 4));
  const int reps = 20;
  auto rep = [&](const char* name, double ms) { printf("%-48s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9); };
  for (int pass = 0; pass < 2; ++pass) {
  rep("memset", timeit([&] { CK(hipMemsetAsync(y, 0, n * 4)); }, reps));
  rep("tile TH64 U1", timeit([&] { w_tile<64, 1, 0><<<n / 256, 64>>>(y, n); }, reps));
  rep("tile TH64 U4", timeit([&] { w_tile<64, 4, 0><<<n / 1024, 64>>>(y, n); }, reps));
  rep("tile TH128 U2", timeit([&] { w_tile<128, 2, 0><<<n / 1024, 128>>>(y, n); }, reps));
  rep("tile TH256 U1", timeit([&] { w_tile<256, 1, 0><<<n / 1024, 256>>>(y, n); }, reps));
  rep("tile TH256 U2", timeit([&] { w_tile<256, 2, 0><<<n / 2048, 256>>>(y, n); }, reps));
  rep("tile TH256 U4", timeit([&] { w_tile<256, 4, 0><<<n / 4096, 256>>>(y, n); }, reps));
  rep("tile TH256 U4 nt", timeit([&] { w_tile<256, 4, 1><<<n / 4096, 256>>>(y, n); }, reps));
  rep("tile TH512 U2", timeit([&] { w_tile<512, 2, 0><<<n / 4096, 512>>>(y, n); }, reps));
  rep("tile TH1024 U1", timeit([&] { w_tile<1024, 1, 0><<<n / 4096, 1024>>>(y, n); }, reps));
  rep("tile TH1024 U4", timeit([&] { w_tile<1024, 4, 0><<<n / 16384, 1024>>>(y, n); }, reps));
  rep("lanecontig TH256 U2", timeit([&] { w_lanecontig<256, 2><<<n / 2048, 256>>>(y, n); }, reps));
  rep("lanecontig TH256 U4", timeit([&] { w_lanecontig<256, 4><<<n / 4096, 256>>>(y, n); }, reps));
  rep("tile_xcd TH256 U4", timeit([&] { w_tile_xcd<256, 4><<<n / 4096, 256>>>(y, n, n / 4096); }, reps));
  rep("tile_xcd TH256 U1", timeit([&] { w_tile_xcd<256, 1><<<n / 1024, 256>>>(y, n, n / 1024); }, reps));
  rep("wave4k TH256", timeit([&] { w_wave4k<256><<<n / 4096, 256>>>(y, n); }, reps));
  rep("wave4k TH64", timeit([&] { w_wave4k<64><<<n / 1024, 64>>>(y, n); }, reps));
  }
  return 0;
}
