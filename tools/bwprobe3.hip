// bwprobe3.hip — HBM read/write rates of the persistent one-block-per-CU layouts considered for the
// fused encode (each block owns a contiguous range, its waves interleave in per-wave steps of
// STEP float4 per lane, software-pipelined two deep) and for the decode.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/bwprobe3 tools/bwprobe3.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int STEP, bool SYNC>
__global__ void read_persist(const float* __restrict__ x, long n, long per_block, float* sink) {
  __shared__ unsigned s_c[2][32];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const long b0 = (long)blockIdx.x * per_block;
  const long b1 = b0 + per_block < n ? b0 + per_block : n;
  const long wstep = (long)STEP * 256;         // elements per wave step
  const long bstep = wstep * nw;                 // elements per block step
  float acc = 0.f;
  unsigned run = 0;
  f32x4 va[STEP], vb[STEP];
  long s = b0 + wid * wstep;
  int it = 0;
#pragma unroll
  for (int q = 0; q < STEP; ++q) va[q] = __builtin_nontemporal_load((const f32x4*)(x + s + 256 * q + 4 * lane));
  for (; s < b1; s += bstep) {
    const long s2 = s + bstep;
    if (s2 < b1) {
#pragma unroll
      for (int q = 0; q < STEP; ++q) vb[q] = __builtin_nontemporal_load((const f32x4*)(x + s2 + 256 * q + 4 * lane));
    }
    unsigned c = 0;
#pragma unroll
    for (int q = 0; q < STEP; ++q) {
      c += __popcll(__ballot(!(va[q].x < 0.0023f))) + __popcll(__ballot(!(va[q].y < 0.0023f)));
      c += __popcll(__ballot(!(va[q].z < 0.0023f))) + __popcll(__ballot(!(va[q].w < 0.0023f)));
    }
    if (SYNC) {
      if (lane == 0) s_c[it & 1][wid] = c;
      __syncthreads();
      unsigned t = 0;
      for (int w = 0; w < nw; ++w) t += s_c[it & 1][w];
      run += t;
    } else {
      run += c;
    }
    ++it;
#pragma unroll
    for (int q = 0; q < STEP; ++q) va[q] = vb[q];
  }
  acc = (float)run;
  if (acc == 12345.f) *sink = acc;
}

template <int V>
__global__ void write_persist(float* __restrict__ y, long n, long per_block) {
  const long b0 = (long)blockIdx.x * per_block;
  const long b1 = b0 + per_block < n ? b0 + per_block : n;
  const long span = (long)blockDim.x * 4 * V;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  for (long s = b0; s < b1; s += span) {
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const long e = s + 4 * ((long)threadIdx.x + (long)u * blockDim.x);
      if (e < b1) *(f32x4*)(y + e) = z;
    }
  }
}

template <int V>
__global__ void write_tiles(float* __restrict__ y, long n) {  // one block per tile of 1024*V floats
  const long t0 = (long)blockIdx.x * 256 * 4 * V;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const long e = t0 + 4 * ((long)threadIdx.x + u * 256);
    if (e < n) *(f32x4*)(y + e) = z;
  }
}

template <typename F>
double timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
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
  float *x, *y, *sink;
  CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4)); CK(hipMalloc(&sink, 4));
  CK(hipMemset(x, 0, n * 4));
  int cu = 256;
  CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  const int reps = 20;
  auto rep = [&](const char* name, double ms) { printf("%-48s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9); };
  char nm[96];
  for (int bpc : {1, 2}) for (int th : {512, 1024}) {
    if (bpc * th > 1024 * 2) continue;
    const int G = cu * bpc;
    const long per = ((n + G - 1) / G + 32767) / 32768 * 32768;
    snprintf(nm, sizeof nm, "read persist STEP8 sync bpc=%d thr=%d", bpc, th);
    rep(nm, timeit([&] { read_persist<8, true><<<G, th>>>(x, n, per, sink); }, reps));
    snprintf(nm, sizeof nm, "read persist STEP8 nosync bpc=%d thr=%d", bpc, th);
    rep(nm, timeit([&] { read_persist<8, false><<<G, th>>>(x, n, per, sink); }, reps));
    snprintf(nm, sizeof nm, "read persist STEP4 sync bpc=%d thr=%d", bpc, th);
    rep(nm, timeit([&] { read_persist<4, true><<<G, th>>>(x, n, per, sink); }, reps));
    snprintf(nm, sizeof nm, "read persist STEP16 sync bpc=%d thr=%d", bpc, th);
    rep(nm, timeit([&] { read_persist<16, true><<<G, th>>>(x, n, per, sink); }, reps));
  }
  for (int bpc : {1, 2, 4, 8}) for (int th : {256, 1024}) {
    const int G = cu * bpc;
    const long per = ((n + G - 1) / G + 4095) / 4096 * 4096;
    snprintf(nm, sizeof nm, "write persist V4 bpc=%d thr=%d", bpc, th);
    rep(nm, timeit([&] { write_persist<4><<<G, th>>>(y, n, per); }, reps));
  }
  rep("write tiles V4 (one block per 4096)", timeit([&] { write_tiles<4><<<n / 4096, 256>>>(y, n); }, reps));
  rep("write tiles V8", timeit([&] { write_tiles<8><<<n / 8192, 256>>>(y, n); }, reps));
  rep("write tiles V16", timeit([&] { write_tiles<16><<<n / 16384, 256>>>(y, n); }, reps));
  rep("hipMemsetAsync 1 GiB", timeit([&] { CK(hipMemsetAsync(y, 0, n * 4)); }, reps));
  return 0;
}
