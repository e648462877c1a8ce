// bwprobe8.hip — the paired pass (topk.hip filter_phase) streams half the blocks' ranges from the top down.  Does the
// direction of a persistent block's 64 KB steps change the streaming rate?  One 1024-thread block per CU over 1 GiB,
// contiguous 4 MB ranges, 64 KB block steps (16 waves x 4 KB), non-temporal 16-B loads, two steps in flight:
//   mode 0: every block ascending;  1: odd blocks descending;  2: every block descending;
//   mode 3: odd blocks take their range in 8-step chunks from the top down, each chunk ascending;
//   mode 4: odd blocks descending, each wave's 4 KB of a step read last-to-first as well.
// Build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/bwprobe8 tools/bwprobe8.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ long step_of(int mode, long s, long S) {
  const bool odd = blockIdx.x & 1;
  if (mode == 2 || ((mode == 1 || mode == 4) && odd)) return S - 1 - s;
  if (mode == 3 && odd) {
    const long c = s / 8, r = s % 8, nc = S / 8;
    return (nc - 1 - c) * 8 + r;
  }
  return s;
}

__global__ __launch_bounds__(1024) void rd(const float4* __restrict__ x, long S, int mode, float* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool rq = mode == 4 && (blockIdx.x & 1);
  float acc = 0.f;
  f32x4 a[4], b[4];
  auto ld = [&](long s, f32x4 (&v)[4]) {
    const float4* p = x + (blockIdx.x * S + step_of(mode, s, S)) * 4096 + wid * 256 + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 64 * (rq ? 3 - q : q)));
  };
  ld(0, a);
  ld(1, b);
  for (long s = 0; s < S; s += 2) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc += a[q].x + a[q].y + a[q].z + a[q].w;
    ld(s + 2 < S ? s + 2 : s, a);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc += b[q].x + b[q].y + b[q].z + b[q].w;
    ld(s + 3 < S ? s + 3 : s + 1, b);
  }
  if (acc == 1234.5f) out[threadIdx.x] = acc;
}

int main() {
  const long n4 = (1l << 28) / 4;  // 1 GiB of floats, as float4
  const int G = 256;
  const long S = n4 / 4096 / G;  // 64 KB steps per block
  float4* x;
  float* out;
  CK(hipMalloc(&x, n4 * 16));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(x, 0, n4 * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < 2; ++round)
    for (int mode = 0; mode < 5; ++mode) {
      for (int w = 0; w < 3; ++w) rd<<<G, 1024>>>(x, S, mode, out);
      CK(hipEventRecord(e0));
      for (int it = 0; it < 10; ++it) rd<<<G, 1024>>>(x, S, mode, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("round %d mode %d: %.1f us per 1 GiB read (%.2f TB/s)\n", round, mode, ms * 100.0f,
             (double)n4 * 16 / (ms / 10 * 1e-3) / 1e12);
    }
  return 0;
}
