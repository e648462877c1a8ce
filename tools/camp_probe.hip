// camp_probe.hip — do the encode's lockstep block ranges camp on HBM channels?  Block b of the persistent pass reads
// b M + s 64 KB at step s: every block sits at the same offset modulo M = 4 MiB at once.  Read-only passes over 1 GiB
// (one 1024-thread block per CU, contiguous 4 MiB ranges, 64 KB steps, non-temporal 16-B loads, two steps in flight):
//   lock:   every block from its range's first step (the encode's order);
//   rot:    block b from step (7 b) mod 64, wrapping round its range (same bytes, the blocks' offsets spread);
// and the delta-fused encoder's two-stream read (local and global, 64 KB + 64 KB per step) with the two operands
//   2^30 B apart (the bench's layout) or 2^30 + 8 MiB apart, lockstep or rotated.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/camp_probe tools/camp_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <bool TWO>
__global__ __launch_bounds__(1024) void rd(const float4* __restrict__ x, const float4* __restrict__ y, long S, int rot,
                                           float* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int Q = TWO ? 2 : 4;  // float4 per lane per operand per step (the delta encoder: 2 + 2)
  const long r0 = rot ? (7L * blockIdx.x) % S : 0;
  float acc = 0.f;
  f32x4 a[2 * Q], b[2 * Q];
  auto ld = [&](long s, f32x4 (&v)[2 * Q]) {
    const long st = (r0 + (s < S ? s : S - 1)) % S;
    const long base = (blockIdx.x * S + st) * (Q * 1024) + wid * (Q * 64) + lane;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      v[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + base + 64 * q));
      if (TWO) v[Q + q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(y + base + 64 * q));
    }
  };
  ld(0, a);
  ld(1, b);
  for (long s = 0; s < S; s += 2) {
#pragma unroll
    for (int q = 0; q < (TWO ? 2 * Q : Q); ++q) acc += a[q].x + a[q].y + a[q].z + a[q].w;
    ld(s + 2, a);
#pragma unroll
    for (int q = 0; q < (TWO ? 2 * Q : Q); ++q) acc += b[q].x + b[q].y + b[q].z + b[q].w;
    ld(s + 3, b);
  }
  if (acc == 1234.5f) out[threadIdx.x] = acc;
}

int main() {
  const long n4 = (1l << 28) / 4;  // 1 GiB of floats as float4
  const int G = 256;
  float4 *big, *x2;
  float* out;
  // one allocation holding x at 0, y at 2^30 and y' at 2^30 + 8 MiB
  CK(hipMalloc(&big, 2 * n4 * 16 + (8l << 20)));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(big, 0, 2 * n4 * 16 + (8l << 20)));
  x2 = big + n4;
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
  const long S1 = n4 / 4096 / G;         // 64 KB steps per block, one operand (64)
  const long S2 = n4 / 2048 / G;         // 32 KB + 32 KB steps, two operands (128)
  for (int round = 0; round < 2; ++round) {
    const float l1 = t([&] { rd<false><<<G, 1024>>>(big, big, S1, 0, out); });
    const float r1 = t([&] { rd<false><<<G, 1024>>>(big, big, S1, 1, out); });
    const float l2 = t([&] { rd<true><<<G, 1024>>>(big, x2, S2, 0, out); });
    const float r2 = t([&] { rd<true><<<G, 1024>>>(big, x2, S2, 1, out); });
    const float l3 = t([&] { rd<true><<<G, 1024>>>(big, x2 + (8l << 20) / 16, S2, 0, out); });
    const float r3 = t([&] { rd<true><<<G, 1024>>>(big, x2 + (8l << 20) / 16, S2, 1, out); });
    printf("round %d: 1 GiB lock %.1f us | rot %.1f us || 2 x 1 GiB (2^30 apart) lock %.1f | rot %.1f || "
           "(2^30 + 8 MiB apart) lock %.1f | rot %.1f\n", round, l1, r1, l2, r2, l3, r3);
  }
  return 0;
}
