// bwprobe5.hip — write patterns of a persistent one-block-per-CU kernel whose blocks own grid-interleaved
// 64 KB chunks (block b, step s -> chunk s * G + b): the whole grid writes one contiguous 16 MB window
// per step.  Variants: how a block's 16 waves split the chunk, and the store flavour.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bwprobe5 tools/bwprobe5.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// MODE 0: wave w writes the contiguous 4 KB [w*4K, (w+1)*4K) of the chunk (4 stores of 1 KB)
// MODE 1: the block writes the chunk as 4 block-wide 16 KB stores (thread t: float4 t + u*1024)
// MODE 2: like 0 with nontemporal stores
template <int MODE>
__global__ __launch_bounds__(1024) void w_chunks(float* __restrict__ y, long nchunks) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
    f32x4* base = (f32x4*)(y + c * 16384);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4* p = MODE == 1 ? base + threadIdx.x + u * 1024 : base + wid * 256 + u * 64 + lane;
      if (MODE == 2) __builtin_nontemporal_store(z, p);
      else *p = z;
    }
  }
}

// per-block contiguous ranges (reference: the slow pattern)
__global__ __launch_bounds__(1024) void w_ranges(float* __restrict__ y, long nchunks) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long per = nchunks / gridDim.x;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  for (long c = blockIdx.x * per; c < (blockIdx.x + 1) * per; ++c) {
    f32x4* base = (f32x4*)(y + c * 16384);
#pragma unroll
    for (int u = 0; u < 4; ++u) base[wid * 256 + u * 64 + lane] = z;
  }
}


// one-wave workgroups writing NB KB each (lane-strided 1 KB store instructions, in order)
template <int NB>
__global__ __launch_bounds__(64) void w_wave(float* __restrict__ y) {
  const int lane = threadIdx.x;
  f32x4* p = (f32x4*)(y + (long)blockIdx.x * NB * 256);
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < NB; ++u) p[lane + 64 * u] = z;
}


// one-wave workgroups writing two 4 KB pieces half the array apart (tile g and g + ntiles / 2)
__global__ __launch_bounds__(64) void w_wave_split(float* __restrict__ y, long half_tiles) {
  const int lane = threadIdx.x;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    f32x4* p = (f32x4*)(y + ((long)blockIdx.x + h * half_tiles) * 1024);
#pragma unroll
    for (int u = 0; u < 4; ++u) p[lane + 64 * u] = z;
  }
}
// one-wave workgroups writing 8 KB with the two 4 KB halves' stores interleaved
__global__ __launch_bounds__(64) void w_wave_8k_inter(float* __restrict__ y) {
  const int lane = threadIdx.x;
  f32x4* p = (f32x4*)(y + (long)blockIdx.x * 2048);
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    p[lane + 64 * u] = z;
    p[256 + lane + 64 * u] = z;
  }
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
  const long n = 268435456, nch = n / 16384;
  const double bytes = n * 4.0;
  float* y;
  CK(hipMalloc(&y, n * 4));
  int cu = 256;
  CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  auto rep = [&](const char* nm, double ms) { printf("%-52s %8.1f us  %7.0f GB/s\n", nm, ms * 1e3, bytes / (ms * 1e-3) / 1e9); };
  for (int pass = 0; pass < 2; ++pass) {
    rep("chunks 64KB, wave-contiguous 4KB", timeit([&] { w_chunks<0><<<cu, 1024>>>(y, nch); }, 20));
    rep("chunks 64KB, block-wide 16KB stores", timeit([&] { w_chunks<1><<<cu, 1024>>>(y, nch); }, 20));
    rep("chunks 64KB, wave-contiguous nt", timeit([&] { w_chunks<2><<<cu, 1024>>>(y, nch); }, 20));
    rep("per-block ranges (reference)", timeit([&] { w_ranges<<<cu, 1024>>>(y, nch); }, 20));
    rep("memset", timeit([&] { CK(hipMemsetAsync(y, 0, n * 4)); }, 20));
    rep("1-wave WG, 4 KB", timeit([&] { w_wave<4><<<n / 1024, 64>>>(y); }, 20));
    rep("1-wave WG, 8 KB", timeit([&] { w_wave<8><<<n / 2048, 64>>>(y); }, 20));
    rep("1-wave WG, 16 KB", timeit([&] { w_wave<16><<<n / 4096, 64>>>(y); }, 20));
    rep("1-wave WG, 2 x 4 KB half apart", timeit([&] { w_wave_split<<<n / 2048, 64>>>(y, n / 2048); }, 20));
    rep("1-wave WG, 8 KB halves interleaved", timeit([&] { w_wave_8k_inter<<<n / 2048, 64>>>(y); }, 20));
  }
  return 0;
}
