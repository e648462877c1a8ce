// fuseprobe.hip — can the stacked codec's dense output be written during the encode's HBM read pass?
// Persistent shape of the encode (one 1024-thread block per CU, contiguous 4 MB ranges, 64 KB steps,
// two-deep pipeline), 1 GiB of N(0,1) x; variants:
//   0 read only                                   (the encode's pass today)
//   1 read + write every line (copy)              (full read+write)
//   2 read + write zeros for 64-B lines without a candidate (x >= t), plain stores
//   3 same, non-temporal stores
//   4 read + write zeros for 128-B lines without a candidate, non-temporal
//   5 write-only, every line, persistent shape, non-temporal
// and "defer": one wave per 8 KB output tile writing only the candidate lines of the tile (the lines
// variants 2-4 skipped), zeros + values, as the post-select write would.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/fuseprobe tools/fuseprobe.hip
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
constexpr int kT = 1024, kStep = 16384;

__device__ __forceinline__ uint32_t hash32(uint32_t a) {
  a ^= a >> 16; a *= 0x7feb352dU; a ^= a >> 15; a *= 0x846ca68bU; a ^= a >> 16;
  return a;
}
__global__ void init_kernel(float* x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    // approx N(0,1) from the sum of 4 uniforms (Irwin-Hall, scaled)
    uint32_t h = hash32((uint32_t)i * 2654435761u + 17u);
    float s = 0.f;
    for (int j = 0; j < 4; ++j) { h = hash32(h + j); s += (h >> 8) * (1.0f / 16777216.0f); }
    x[i] = (s - 2.0f) * 1.7320508f;
  }
}

template <int V>
__global__ __launch_bounds__(kT) void pass_kernel(const float* __restrict__ x, float* __restrict__ out, int64_t M,
                                                  float t, float* sink) {
  const int64_t base = (int64_t)blockIdx.x * M;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const f4 zero = {0.f, 0.f, 0.f, 0.f};
  float acc = 0.f;
  f4 cur[4], nxt[4];
  auto addr = [&](int64_t s, int j) { return base + s * kStep + w * 1024 + (j * 64 + lane) * 4; };
  const int64_t steps = M / kStep;
  if (V != 5)
#pragma unroll
    for (int j = 0; j < 4; ++j) cur[j] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x + addr(0, j)));
  for (int64_t s = 0; s < steps; ++s) {
    if (V != 5) {
      const int64_t sn = s + 1 < steps ? s + 1 : s;
#pragma unroll
      for (int j = 0; j < 4; ++j) nxt[j] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x + addr(sn, j)));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f4 v = cur[j];
      const int64_t e = addr(s, j);
      if (V == 0) acc += v.x + v.y + v.z + v.w;
      if (V == 1) *reinterpret_cast<f4*>(out + e) = v;
      if (V == 5) __builtin_nontemporal_store(zero, reinterpret_cast<f4*>(out + e));
      if (V >= 2 && V <= 4) {
        int c = (v.x >= t) | (v.y >= t) | (v.z >= t) | (v.w >= t);
        c |= __builtin_amdgcn_mov_dpp(c, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
        c |= __builtin_amdgcn_mov_dpp(c, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
        if (V == 4) c |= __shfl_xor(c, 4);
        if (!c) {
          if (V == 2) *reinterpret_cast<f4*>(out + e) = zero;
          else __builtin_nontemporal_store(zero, reinterpret_cast<f4*>(out + e));
        }
      }
    }
    if (V != 5)
#pragma unroll
      for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
  }
  if (V == 0 && acc == 12345.678f) sink[0] = acc;
}

// deferred lines: one wave per 8 KB tile (2048 elements = 32 lines of 64 B), writes only lines with a candidate
__global__ __launch_bounds__(256) void defer_kernel(const float* __restrict__ x, float* __restrict__ out, int64_t n,
                                                    float t, int line_bytes) {
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t tile0 = wave * 2048;
  if (tile0 >= n) return;
  // lane handles elements tile0 + k*256 + lane*4 .. +3, k = 0..7 (x is L2-cold: this re-read stands in for the
  // LDS-held candidates the encode would have)
  const int lanes_per_line = line_bytes / 16;
  for (int k = 0; k < 8; ++k) {
    const int64_t e = tile0 + k * 256 + lane * 4;
    const f4 v = *reinterpret_cast<const f4*>(x + e);
    int c = (v.x >= t) | (v.y >= t) | (v.z >= t) | (v.w >= t);
    c |= __builtin_amdgcn_mov_dpp(c, 0xB1, 0xf, 0xf, false);
    c |= __builtin_amdgcn_mov_dpp(c, 0x4E, 0xf, 0xf, false);
    if (lanes_per_line == 8) c |= __shfl_xor(c, 4);
    if (c) {
      f4 o = {v.x >= t ? v.x : 0.f, v.y >= t ? v.y : 0.f, v.z >= t ? v.z : 0.f, v.w >= t ? v.w : 0.f};
      *reinterpret_cast<f4*>(out + e) = o;
    }
  }
}

int main() {
  const int64_t n = 268435456;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int G = std::min(cus, 256);
  const int64_t M = n / G;
  float *x, *out, *sink;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&sink, 64));
  init_kernel<<<4096, 256>>>(x, n);
  CK(hipDeviceSynchronize());
  const float t = 2.235f;  // P(N(0,1) >= t) ~ 1.27 %: the encode's candidate floor at k = 1 %
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](auto launch) {
    std::vector<float> ts;
    for (int r = 0; r < 12; ++r) {
      hipEventRecord(a);
      launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r >= 2) ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
  };
  printf("G=%d M=%lld\n", G, (long long)M);
  float us;
  us = timeit([&] { pass_kernel<0><<<G, kT>>>(x, out, M, t, sink); });
  printf("v0 read only            %7.1f us  %6.2f TB/s\n", us, n * 4.0 / us / 1e6);
  us = timeit([&] { pass_kernel<1><<<G, kT>>>(x, out, M, t, sink); });
  printf("v1 read + write all     %7.1f us  %6.2f TB/s (R+W)\n", us, n * 8.0 / us / 1e6);
  us = timeit([&] { pass_kernel<2><<<G, kT>>>(x, out, M, t, sink); });
  printf("v2 read + zero64 plain  %7.1f us\n", us);
  us = timeit([&] { pass_kernel<3><<<G, kT>>>(x, out, M, t, sink); });
  printf("v3 read + zero64 nt     %7.1f us\n", us);
  us = timeit([&] { pass_kernel<4><<<G, kT>>>(x, out, M, t, sink); });
  printf("v4 read + zero128 nt    %7.1f us\n", us);
  us = timeit([&] { pass_kernel<5><<<G, kT>>>(x, out, M, t, sink); });
  printf("v5 write only nt        %7.1f us  %6.2f TB/s\n", us, n * 4.0 / us / 1e6);
  const unsigned dg = (unsigned)(n / 2048 / 4);
  us = timeit([&] { defer_kernel<<<dg, 256>>>(x, out, n, t, 64); });
  printf("defer64 (re-reads x)    %7.1f us\n", us);
  us = timeit([&] { defer_kernel<<<dg, 256>>>(x, out, n, t, 128); });
  printf("defer128 (re-reads x)   %7.1f us\n", us);
  // candidate-line census
  std::vector<float> hx(1 << 22);
  CK(hipMemcpy(hx.data(), x, hx.size() * 4, hipMemcpyDeviceToHost));
  long c = 0, l64 = 0, l128 = 0;
  for (size_t i = 0; i < hx.size(); ++i) c += hx[i] >= t;
  for (size_t i = 0; i < hx.size(); i += 16) { int h = 0; for (int j = 0; j < 16; ++j) h |= hx[i + j] >= t; l64 += h; }
  for (size_t i = 0; i < hx.size(); i += 32) { int h = 0; for (int j = 0; j < 32; ++j) h |= hx[i + j] >= t; l128 += h; }
  printf("candidates %.4f  lines64 with one %.4f  lines128 %.4f\n", c / (double)hx.size(), l64 * 16.0 / hx.size(),
         l128 * 32.0 / hx.size());
  return 0;
}
