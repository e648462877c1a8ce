// writeprobe.hip — can the persistent encode shape (one 1024-thread block per CU) write the dense 1 GiB output
// at the decode's rate?  Variants, all writing zeros over 1 GiB:
//   own      block b writes its own contiguous 4 MB range (the encode's block ranges), 64 KB per step
//   window   grid-wide sweeping window: step i, block b writes 64-KB chunk i * G + b
//   window-nt  the same with non-temporal stores
//   skip64   window order, only 64-B lines without a candidate (x >= t) — the lines the encode could zero early
//   cand64   window order, only the lines WITH a candidate (the rest of the output)
//   decode   reference: one-wave blocks, 4 KB each (the decode kernel's store shape)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/writeprobe tools/writeprobe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define CK(e)                                                                       \
  do {                                                                              \
    hipError_t r_ = (e);                                                            \
    if (r_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(r_));     \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kT = 1024;
constexpr int64_t kChunk = 16384;  // elements per block step (64 KB): 16 waves x 4 KB

__device__ __forceinline__ uint32_t hash32(uint32_t a) {
  a ^= a >> 16; a *= 0x7feb352dU; a ^= a >> 15; a *= 0x846ca68bU; a ^= a >> 16;
  return a;
}
__global__ void init_kernel(float* x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint32_t h = hash32((uint32_t)i * 2654435761u + 17u);
    float s = 0.f;
    for (int j = 0; j < 4; ++j) { h = hash32(h + j); s += (h >> 8) * (1.0f / 16777216.0f); }
    x[i] = (s - 2.0f) * 1.7320508f;
  }
}

// line bitmap: bit l = 64-B line l (16 floats) holds an element >= t
__global__ void bitmap_kernel(const float* x, int64_t n, float t, uint32_t* bm) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one word = 32 lines = 512 elements
  if (w * 512 >= n) return;
  uint32_t b = 0;
  for (int l = 0; l < 32; ++l) {
    bool c = false;
    for (int j = 0; j < 16; ++j) c |= x[w * 512 + l * 16 + j] >= t;
    b |= (uint32_t)c << l;
  }
  bm[w] = b;
}

template <int V>  // 0 own, 1 window, 2 window nt, 3 skip64, 4 cand64
__global__ __launch_bounds__(kT) void pw_kernel(float* __restrict__ out, int64_t n, const uint32_t* __restrict__ bm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const f4 zero = {0.f, 0.f, 0.f, 0.f};
  const int64_t nchunks = n / kChunk, G = gridDim.x;
  const int64_t per = nchunks / G;
  for (int64_t i = 0; i < per; ++i) {
    const int64_t c = V == 0 ? (int64_t)blockIdx.x * per + i : i * G + blockIdx.x;
    const int64_t e0 = c * kChunk + (int64_t)w * 1024;  // this wave's 4 KB
    if (V >= 3) {
      // lane covers 16 elements = one line... 4 KB = 64 lines: one line per lane, four 16-B stores
      const int64_t line = e0 / 16 + lane;
      const bool cand = (bm[line >> 5] >> (line & 31)) & 1u;
      if ((V == 3 && !cand) || (V == 4 && cand)) {
        f4* p = reinterpret_cast<f4*>(out + line * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(zero, p + j);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f4* p = reinterpret_cast<f4*>(out + e0 + (j * 64 + lane) * 4);
        if (V == 2) __builtin_nontemporal_store(zero, p);
        else *p = zero;
      }
    }
  }
}

__global__ __launch_bounds__(64) void wave_kernel(float* __restrict__ out) {
  const f4 zero = {0.f, 0.f, 0.f, 0.f};
  const int64_t e0 = (int64_t)blockIdx.x * 1024;
#pragma unroll
  for (int j = 0; j < 4; ++j) *reinterpret_cast<f4*>(out + e0 + (j * 64 + threadIdx.x) * 4) = zero;
}

int main() {
  const int64_t n = 268435456;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int G = std::min(cus, 256);
  float *x, *out;
  uint32_t* bm;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&bm, n / 512 * 4));
  init_kernel<<<4096, 256>>>(x, n);
  const float t = 2.235f;  // ~1.27 % candidates: the encode's floor at k = 1 %
  bitmap_kernel<<<(unsigned)(n / 512 / 256), 256>>>(x, n, t, bm);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](auto launch) {
    std::vector<float> ts;
    for (int r = 0; r < 14; ++r) {
      hipEventRecord(a);
      launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r >= 4) ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
  };
  printf("G=%d\n", G);
  float us;
  us = timeit([&] { pw_kernel<0><<<G, kT>>>(out, n, bm); });
  printf("own         %7.1f us  %5.2f TB/s\n", us, n * 4.0 / us / 1e6);
  us = timeit([&] { pw_kernel<1><<<G, kT>>>(out, n, bm); });
  printf("window      %7.1f us  %5.2f TB/s\n", us, n * 4.0 / us / 1e6);
  us = timeit([&] { pw_kernel<2><<<G, kT>>>(out, n, bm); });
  printf("window-nt   %7.1f us  %5.2f TB/s\n", us, n * 4.0 / us / 1e6);
  us = timeit([&] { pw_kernel<3><<<G, kT>>>(out, n, bm); });
  const float us3 = us;
  printf("skip64      %7.1f us\n", us);
  us = timeit([&] { pw_kernel<4><<<G, kT>>>(out, n, bm); });
  printf("cand64      %7.1f us  (skip64 + cand64 %7.1f)\n", us, us + us3);
  us = timeit([&] { wave_kernel<<<(unsigned)(n / 1024), 64>>>(out); });
  printf("decode-shape %6.1f us  %5.2f TB/s\n", us, n * 4.0 / us / 1e6);
  std::vector<uint32_t> hb(n / 512);
  CK(hipMemcpy(hb.data(), bm, hb.size() * 4, hipMemcpyDeviceToHost));
  long c = 0;
  for (uint32_t v : hb) c += __builtin_popcount(v);
  printf("candidate lines %.4f of all\n", c / (double)(n / 16));
  return 0;
}
