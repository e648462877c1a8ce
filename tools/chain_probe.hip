// chain_probe.hip — what a load chain costs a one-wave, 4 KB-per-workgroup writer (the fast store shape of
// tools/writeshape_probe.hip).  1 GiB of output, 262,144 one-wave workgroups, each: zero a 4 KB LDS tile, scatter the
// tile's ~10 entries into it, store it (16-B stores).  The entries come:
//   c0: from nowhere (stores only);
//   c1: from a fixed slot per tile (one load round trip: slots[t * 16 + lane], 16 slots per tile);
//   c2: from a CSR array through the tile's pointer (two dependent round trips: ptr[t], ptr[t + 1] -> idx[...]: the
//       decode's chain).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/chain_probe tools/chain_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int MODE>
__global__ __launch_bounds__(64) void dec(float4* __restrict__ out, const unsigned* __restrict__ ptr,
                                          const unsigned* __restrict__ idx, const unsigned* __restrict__ slots) {
  __shared__ __attribute__((aligned(16))) float s_tile[1024];
  const int lane = threadIdx.x;
  const unsigned t = blockIdx.x;
  unsigned e = 0xffffffffu;
  if (MODE == 1) {
    e = slots[t * 16 + lane % 16];
  } else if (MODE == 2) {
    const unsigned a = ptr[t], b = ptr[t + 1];
    __builtin_amdgcn_sched_barrier(0);
    if (a + lane < b) e = idx[a + lane];
  }
  float4* t4 = reinterpret_cast<float4*>(s_tile);
#pragma unroll
  for (int u = 0; u < 4; ++u) t4[lane + 64 * u] = make_float4(0.f, 0.f, 0.f, 0.f);
  __builtin_amdgcn_wave_barrier();
  if (e != 0xffffffffu && (e >> 10) == t) s_tile[e & 1023u] = 1.0f;
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int u = 0; u < 4; ++u) out[(size_t)t * 256 + lane + 64 * u] = t4[lane + 64 * u];
}

int main() {
  const unsigned T = 1u << 18;  // 4 KB tiles of 1 GiB
  const unsigned per = 10;      // entries per tile (k = 1 %)
  float4* out;
  unsigned *ptr, *idx, *slots;
  CK(hipMalloc(&out, (size_t)T * 4096));
  CK(hipMalloc(&ptr, (size_t)(T + 1) * 4));
  CK(hipMalloc(&idx, (size_t)T * per * 4));
  CK(hipMalloc(&slots, (size_t)T * 16 * 4));
  unsigned* h = (unsigned*)malloc((size_t)T * per * 4);
  unsigned* hp = (unsigned*)malloc((size_t)(T + 1) * 4);
  unsigned* hs = (unsigned*)malloc((size_t)T * 16 * 4);
  unsigned s = 1;
  for (unsigned t = 0; t < T; ++t) {
    hp[t] = t * per;
    for (unsigned j = 0; j < per; ++j) {
      s = s * 1664525u + 1013904223u;
      h[t * per + j] = t * 1024 + (s >> 22);
    }
    for (unsigned j = 0; j < 16; ++j) hs[t * 16 + j] = j < per ? h[t * per + j] : 0xffffffffu;
  }
  hp[T] = T * per;
  CK(hipMemcpy(ptr, hp, (size_t)(T + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(idx, h, (size_t)T * per * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(slots, hs, (size_t)T * 16 * 4, hipMemcpyHostToDevice));
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
    const float a = t([&] { dec<0><<<T, 64>>>(out, ptr, idx, slots); });
    const float b = t([&] { dec<1><<<T, 64>>>(out, ptr, idx, slots); });
    const float c = t([&] { dec<2><<<T, 64>>>(out, ptr, idx, slots); });
    printf("round %d: 1 GiB, one wave per 4 KB tile: stores only %.1f us | fixed slots (1 load) %.1f | CSR (pointer -> "
           "entries) %.1f\n", round, a, b, c);
  }
  return 0;
}
