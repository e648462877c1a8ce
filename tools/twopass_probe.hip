// twopass_probe.hip — VERDICT r04 item 3: the cache-resident two-pass select for configs[2] (25 M fp32, k = 1 %).
// Its first pass histograms EVERY element's key (no sample) on the top 13 bits (1/16 binade: the bin of the k-th largest
// then holds 0.2-0.4 % of a gaussian input, so the second pass's candidates fit the LDS), its second pass re-reads x
// from the memory-side cache.  This probe times the two new phases in the encode's own shape (one 1024-thread block per
// CU, contiguous block ranges, 16 K-element block steps of 4 float4 per lane, two steps in flight, non-temporal loads):
//   read      the pass with no work: the HBM (or cache) streaming floor of the shape;
//   hist-a    + one LDS atomicAdd per element into an 8192-bin block histogram, nonzero bins flushed to global;
//   hist-w    + the same, aggregated per wave when every lane hits one bin (topk.hip hist_add);
//   hist-8    + an 8-bit histogram (sign + 7 exponent bits: 1 binade per bin), one copy per wave (16 x 256 bins);
//   pass2     `read` right after `hist-a` on the same vector (the second pass, from the 256 MiB memory-side cache);
//   cached    hist-a and pass2 with cached loads (non-temporal loads may not allocate in the memory-side cache);
// on 8 distinct 25 M vectors in rotation (800 MB: every first pass reads HBM).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/twopass_probe tools/twopass_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kT = 1024, kBins = 8192;

__device__ __forceinline__ unsigned okey(float v) {
  const unsigned u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <int MODE, bool NT = true>
__global__ __launch_bounds__(kT) void pass(const float* __restrict__ x, long n, long M, unsigned* __restrict__ gh,
                                           float* sink) {
  __shared__ unsigned h[MODE == 3 ? 16 * 256 : kBins];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (MODE) {
    for (int i = tid; i < (MODE == 3 ? 16 * 256 : kBins); i += kT) h[i] = 0u;
    __syncthreads();
  }
  const long b0 = blockIdx.x * M, b1 = b0 + M < n ? b0 + M : n;
  const long steps = (b1 - b0) / 16384;  // (whole steps; the probe's n is a multiple of 16 K per block)
  float acc = 0.f;
  f32x4 a[4], b[4];
  auto ld = [&](long s, f32x4 (&v)[4]) {
    const long e = b0 + (s < steps ? s : steps - 1) * 16384 + wid * 1024 + 4 * lane;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = NT ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + e + 256 * q))
                : *reinterpret_cast<const f32x4*>(x + e + 256 * q);
  };
  auto work = [&](const f32x4 (&v)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float e4[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const unsigned key = okey(e4[c]);
        if (MODE == 0) {
          acc += e4[c];
        } else if (MODE == 1) {
          atomicAdd(&h[key >> 19], 1u);
        } else if (MODE == 2) {
          const unsigned bin = key >> 19;
          const unsigned b0v = (unsigned)__builtin_amdgcn_readfirstlane((int)bin);
          if (__ballot(bin == b0v) == ~0ull) {
            if (lane == 0) atomicAdd(&h[b0v], 64u);
          } else {
            atomicAdd(&h[bin], 1u);
          }
        } else {
          atomicAdd(&h[wid * 256 + (key >> 24)], 1u);
        }
      }
    }
  };
  ld(0, a);
  ld(1, b);
  for (long s = 0; s < steps; s += 2) {
    work(a);
    ld(s + 2, a);
    if (s + 1 < steps) work(b);
    ld(s + 3, b);
  }
  if (MODE) {
    __syncthreads();
    if (MODE == 3) {
      for (int i = tid; i < 256; i += kT) {
        unsigned t = 0;
        for (int w = 0; w < 16; ++w) t += h[w * 256 + i];
        if (t) atomicAdd(&gh[i], t);
      }
    } else {
      for (int i = tid; i < kBins; i += kT)
        if (h[i]) atomicAdd(&gh[i], h[i]);
    }
  }
  if (acc == 1234.5f) sink[tid] = acc;
}

int main() {
  const int G = 256;
  const long M = 98304;  // 6 steps of 16 K per block (25.2 M elements: configs[2]'s 25 M rounded to whole steps)
  const long n = M * G;
  const int NV = 8;
  float* xs[NV];
  unsigned* gh;
  float* sink;
  CK(hipMalloc(&gh, kBins * 4));
  CK(hipMalloc(&sink, 4096));
  float* hx = (float*)malloc(n * 4);
  for (int v = 0; v < NV; ++v) {
    unsigned s = 12345u + 977u * v;
    for (long i = 0; i < n; ++i) {  // a gaussian-like input (sum of 4 uniforms, centred) times 1e-3
      float t = 0.f;
      for (int r = 0; r < 4; ++r) {
        s = s * 1664525u + 1013904223u;
        t += (float)(s >> 8) * (1.0f / 16777216.0f);
      }
      hx[i] = (t - 2.0f) * 1.7320508f * 1e-3f;
    }
    CK(hipMalloc(&xs[v], n * 4));
    CK(hipMemcpy(xs[v], hx, n * 4, hipMemcpyHostToDevice));
  }
  hipEvent_t evs[4];
  for (auto& ev : evs) CK(hipEventCreate(&ev));
  auto t = [&](auto launch) {  // per-call time over 32 calls (inputs rotated)
    for (int w = 0; w < 8; ++w) launch(w % NV);
    CK(hipEventRecord(evs[0]));
    for (int it = 0; it < 32; ++it) launch(it % NV);
    CK(hipEventRecord(evs[1]));
    CK(hipEventSynchronize(evs[1]));
    float ms;
    CK(hipEventElapsedTime(&ms, evs[0], evs[1]));
    return ms * 1000.0f / 32;
  };
  for (int round = 0; round < 2; ++round) {
    const float r0 = t([&](int v) { pass<0><<<G, kT>>>(xs[v], n, M, gh, sink); });
    const float r1 = t([&](int v) { pass<1><<<G, kT>>>(xs[v], n, M, gh, sink); });
    const float r2 = t([&](int v) { pass<2><<<G, kT>>>(xs[v], n, M, gh, sink); });
    const float r3 = t([&](int v) { pass<3><<<G, kT>>>(xs[v], n, M, gh, sink); });
    const float r12 = t([&](int v) {
      pass<1><<<G, kT>>>(xs[v], n, M, gh, sink);
      pass<0><<<G, kT>>>(xs[v], n, M, gh, sink);
    });
    const float r1c = t([&](int v) { pass<1, false><<<G, kT>>>(xs[v], n, M, gh, sink); });
    const float r12c = t([&](int v) {  // pass 1 with cached loads (allocating in the memory-side cache), pass 2 cached
      pass<1, false><<<G, kT>>>(xs[v], n, M, gh, sink);
      pass<0, false><<<G, kT>>>(xs[v], n, M, gh, sink);
    });
    printf("round %d (%.1f MB per pass): read %.1f us (%.2f TB/s) | hist-a %.1f | hist-w %.1f | hist-8 %.1f | "
           "hist-a + pass2 %.1f (pass2 %.1f us, %.2f TB/s) | cached: hist-a %.1f, + pass2 %.1f (pass2 %.1f us, %.2f TB/s)\n",
           round, n * 4e-6, r0, n * 4 / (r0 * 1e-6) / 1e12, r1, r2, r3, r12, r12 - r1,
           n * 4 / ((r12 - r1) * 1e-6) / 1e12, r1c, r12c, r12c - r1c, n * 4 / ((r12c - r1c) * 1e-6) / 1e12);
  }
  return 0;
}
