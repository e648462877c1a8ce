// bwprobe6.hip — persistent 1024-thread read kernels (one block per CU, the filter's shape): per-block
// contiguous ranges vs grid-interleaved 64 KB steps (block b, step s -> s * G + b).  Reports kernel time
// and the spread of per-block finish times (s_memrealtime).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bwprobe6 tools/bwprobe6.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int MODE>  // 0: contiguous ranges, 1: interleaved steps
__global__ __launch_bounds__(1024) void rd(const float4* __restrict__ x, long nsteps, float* out,
                                           unsigned long long* t) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long per = nsteps / gridDim.x;
  float acc = 0.f;
  if (threadIdx.x == 0) t[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  for (long s = 0; s < per; ++s) {
    const long g = MODE == 0 ? blockIdx.x * per + s : s * gridDim.x + blockIdx.x;
    const float4* p = x + g * 4096 + wid * 256 + lane;  // 4096 float4 = 64 KB per step
    f32x4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 64 * q));
#pragma unroll
    for (int q = 0; q < 4; ++q) acc += v[q].x + v[q].y + v[q].z + v[q].w;
  }
  if (acc == 1234.5f) out[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
}

int main() {
  const long n = 268435456, nsteps = n / 16384;
  float4* x;
  float* o;
  unsigned long long* t;
  CK(hipMalloc(&x, n * 4));
  CK(hipMemset(x, 0, n * 4));
  CK(hipMalloc(&o, 4096 * 4));
  CK(hipMalloc(&t, 1024 * 16));
  int cu = 256;
  CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<unsigned long long> h(2 * cu);
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < 2; ++mode) {
      auto launch = [&] {
        if (mode == 0) rd<0><<<cu, 1024>>>(x, nsteps, o, t);
        else rd<1><<<cu, 1024>>>(x, nsteps, o, t);
      };
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      for (int r = 0; r < 10; ++r) launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      CK(hipMemcpy(h.data(), t, 16 * cu, hipMemcpyDeviceToHost));
      unsigned long long t0 = ~0ull;
      for (int i = 0; i < cu; ++i) t0 = std::min(t0, h[2 * i]);
      std::vector<double> fin(cu);
      for (int i = 0; i < cu; ++i) fin[i] = (h[2 * i + 1] - t0) * 0.01;
      std::sort(fin.begin(), fin.end());
      printf("%-12s %7.1f us  %6.0f GB/s   finish min %.1f median %.1f p95 %.1f max %.1f us\n",
             mode == 0 ? "contiguous" : "interleaved", ms * 100.0, n * 4.0 / (ms * 1e-4) / 1e9, fin[0],
             fin[cu / 2], fin[cu * 95 / 100], fin[cu - 1]);
    }
  }
  return 0;
}
