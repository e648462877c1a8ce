// bwprobe7.hip — f1: can a persistent read of TWO streams (local and global parameters, the delta-fused encode's
// pass) run at the one-stream rate?  One 1024-thread block per CU, contiguous per-block ranges, 64 KB per step per
// block, non-temporal 16-B loads: (a) one 2 GiB stream; (b) two 1 GiB streams, 2 float4 per lane from each per step
// (the DeltaSrc shape); (c) two streams, 4 float4 from each (twice the bytes in flight); (d) as (b) with the
// second buffer 1 GiB + 8 MiB away instead of 1 GiB.
// Build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/bwprobe7 tools/bwprobe7.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(1024) void one(const float4* __restrict__ x, long steps_per_block, float* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float acc = 0.f;
  for (long s = 0; s < steps_per_block; ++s) {
    const float4* p = x + (blockIdx.x * steps_per_block + s) * 4096 + wid * 256 + lane;
    f32x4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 64 * q));
#pragma unroll
    for (int q = 0; q < 4; ++q) acc += v[q].x + v[q].y + v[q].z + v[q].w;
  }
  if (acc == 1234.5f) out[threadIdx.x] = acc;
}

template <int SF>
__global__ __launch_bounds__(1024) void two(const float4* __restrict__ l, const float4* __restrict__ g,
                                            long steps_per_block, float* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float acc = 0.f;
  constexpr int span = SF * 64 * 16;  // float4 per block step per stream
  for (long s = 0; s < steps_per_block; ++s) {
    const long off = (blockIdx.x * steps_per_block + s) * span + wid * SF * 64 + lane;
    f32x4 a[SF], b[SF];
#pragma unroll
    for (int q = 0; q < SF; ++q) {
      a[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(l + off + 64 * q));
      b[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g + off + 64 * q));
    }
#pragma unroll
    for (int q = 0; q < SF; ++q) acc += (a[q].x - b[q].x) + (a[q].y - b[q].y) + (a[q].z - b[q].z) + (a[q].w - b[q].w);
  }
  if (acc == 1234.5f) out[threadIdx.x] = acc;
}

int main() {
  const long n = 1L << 28;  // floats per GiB
  float4* buf;
  float* o;
  CK(hipMalloc(&buf, (2 * n + (1L << 21)) * 4));
  CK(hipMemset(buf, 0, (2 * n + (1L << 21)) * 4));
  CK(hipMalloc(&o, 4096 * 4));
  int cu = 256;
  CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const float4* l = buf;
  const float4* g = buf + n / 4;                   // 1 GiB after
  const float4* g2 = buf + n / 4 + (1L << 19);     // 1 GiB + 8 MiB after
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < 4; ++mode) {
      auto launch = [&] {
        if (mode == 0) one<<<cu, 1024>>>(buf, 2 * n / 16384 / cu, o);
        else if (mode == 1) two<2><<<cu, 1024>>>(l, g, n / 8192 / cu, o);
        else if (mode == 2) two<4><<<cu, 1024>>>(l, g, n / 16384 / cu, o);
        else two<2><<<cu, 1024>>>(l, g2, n / 8192 / cu, o);
      };
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      for (int r = 0; r < 10; ++r) launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      const char* names[] = {"one stream", "two SF=2", "two SF=4", "two SF=2 +8MiB"};
      printf("%-16s %7.1f us  %6.0f GB/s\n", names[mode], ms * 100.0, 2 * n * 4.0 / (ms * 1e-4) / 1e9);
    }
  }
  return 0;
}
