// bwprobe.hip — HBM bandwidth calibration on MI355X for the two streaming patterns of the codec:
// read-only (the top-k filter) and write-only (the sparse decode), plus a copy for reference.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bwprobe tools/bwprobe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// grid-stride float4 read, sum into a sink
template <bool NT, int U>
__global__ __launch_bounds__(256) void read_gs(const float4* __restrict__ x, long n4, float* sink) {
  float acc = 0.f;
  const long stride = (long)gridDim.x * 256 * U;
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * 256;
      if (j < n4) v[u] = NT ? __builtin_nontemporal_load((const f32x4*)(x + j)) : *(const f32x4*)(x + j);
      else v[u] = (f32x4){0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 12345.f) *sink = acc;
}

// per-wave contiguous chunks (the filter's layout): each wave reads [w*chunk, (w+1)*chunk) in 4 KB steps
template <bool NT>
__global__ __launch_bounds__(256) void read_wave(const float* __restrict__ x, long n, long chunk, float* sink) {
  const int lane = threadIdx.x & 63;
  const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long b = w * chunk, e = b + chunk < n ? b + chunk : n;
  float acc = 0.f;
  for (long base = b; base < e; base += 1024) {
    f32x4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long i = base + 256 * q + 4 * lane;
      v[q] = NT ? __builtin_nontemporal_load((const f32x4*)(x + i)) : *(const f32x4*)(x + i);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) acc += v[q].x + v[q].y + v[q].z + v[q].w;
  }
  if (acc == 12345.f) *sink = acc;
}

template <bool NT, int U>
__global__ __launch_bounds__(256) void write_gs(float4* __restrict__ y, long n4) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * 256;
      f32x4 z = {0.f, 1.f, 2.f, (float)j};
      if (j < n4) {
        if (NT) __builtin_nontemporal_store(z, (f32x4*)(y + j));
        else *(f32x4*)(y + j) = z;
      }
    }
  }
}

// tile write through LDS like the sparse decode (8192 floats per block)
template <bool NT>
__global__ __launch_bounds__(256) void write_tile(float* __restrict__ y, long n) {
  __shared__ __attribute__((aligned(16))) float t[8192];
  const long t0 = (long)blockIdx.x * 8192;
  f32x4* t4 = (f32x4*)t;
  for (int i = threadIdx.x; i < 2048; i += 256) t4[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  if (threadIdx.x < 82) t[(threadIdx.x * 97) & 8191] = 1.0f;
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += 256) {
    f32x4 v = t4[i];
    if (NT) __builtin_nontemporal_store(v, (f32x4*)(y + t0) + i);
    else *((f32x4*)(y + t0) + i) = v;
  }
}

// one store per thread, no loop
template <int U, int CP>
__global__ __launch_bounds__(256) void write_once(float4* __restrict__ y, long n4) {
  const long i0 = ((long)blockIdx.x * 256 * U) + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long j = i0 + u * 256;
    f32x4 z = {0.f, 1.f, 2.f, 3.f};
    if (j < n4) {
      if (CP == 0) *(f32x4*)(y + j) = z;
      else if (CP == 1) __builtin_nontemporal_store(z, (f32x4*)(y + j));
      else if (CP == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(y + j), "v"(z) : "memory");
      else asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(y + j), "v"(z) : "memory");
    }
  }
}

// each lane writes 64 contiguous bytes (4 x float4)
__global__ __launch_bounds__(256) void write_lane64(float4* __restrict__ y, long n4) {
  const long i0 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  f32x4 z = {0.f, 1.f, 2.f, 3.f};
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (i0 + u < n4) *(f32x4*)(y + i0 + u) = z;
}

__global__ __launch_bounds__(256) void copy_gs(const float4* __restrict__ x, float4* __restrict__ y, long n4) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) y[i] = x[i];
}

template <typename F>
double timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  f();
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
  const long n = 268435456;  // 1 GiB of fp32
  const double bytes = n * 4.0;
  float *x, *y, *sink;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(x, 0, n * 4));
  const long n4 = n / 4;
  const int reps = 20;
  auto rep = [&](const char* name, double ms, double b) { printf("%-40s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, b / (ms * 1e-3) / 1e9); };
  for (int g : {1024, 2048, 4096, 8192, 16384}) {
    char nm[64];
    snprintf(nm, sizeof nm, "read grid-stride U1 grid=%d", g);
    rep(nm, timeit([&] { read_gs<false, 1><<<g, 256>>>((const float4*)x, n4, sink); }, reps), bytes);
    snprintf(nm, sizeof nm, "read grid-stride U4 grid=%d", g);
    rep(nm, timeit([&] { read_gs<false, 4><<<g, 256>>>((const float4*)x, n4, sink); }, reps), bytes);
    snprintf(nm, sizeof nm, "read grid-stride U4 nt grid=%d", g);
    rep(nm, timeit([&] { read_gs<true, 4><<<g, 256>>>((const float4*)x, n4, sink); }, reps), bytes);
  }
  for (int blocks : {1024, 2048, 4096}) {
    const long chunk = n / (blocks * 4);
    char nm[64];
    snprintf(nm, sizeof nm, "read per-wave chunks blocks=%d", blocks);
    rep(nm, timeit([&] { read_wave<false><<<blocks, 256>>>(x, n, chunk, sink); }, reps), bytes);
    snprintf(nm, sizeof nm, "read per-wave chunks nt blocks=%d", blocks);
    rep(nm, timeit([&] { read_wave<true><<<blocks, 256>>>(x, n, chunk, sink); }, reps), bytes);
  }
  for (int g : {2048, 8192, 32768}) {
    char nm[64];
    snprintf(nm, sizeof nm, "write grid-stride U1 grid=%d", g);
    rep(nm, timeit([&] { write_gs<false, 1><<<g, 256>>>((float4*)y, n4); }, reps), bytes);
    snprintf(nm, sizeof nm, "write grid-stride U4 nt grid=%d", g);
    rep(nm, timeit([&] { write_gs<true, 4><<<g, 256>>>((float4*)y, n4); }, reps), bytes);
    snprintf(nm, sizeof nm, "write grid-stride U4 grid=%d", g);
    rep(nm, timeit([&] { write_gs<false, 4><<<g, 256>>>((float4*)y, n4); }, reps), bytes);
  }
  for (int U : {1, 2, 4}) {
    char nm[64];
    const long g = n4 / (256 * U);
    snprintf(nm, sizeof nm, "write once U%d plain", U);
    if (U == 1) rep(nm, timeit([&] { write_once<1, 0><<<g, 256>>>((float4*)y, n4); }, reps), bytes);
    if (U == 2) rep(nm, timeit([&] { write_once<2, 0><<<g, 256>>>((float4*)y, n4); }, reps), bytes);
    if (U == 4) rep(nm, timeit([&] { write_once<4, 0><<<g, 256>>>((float4*)y, n4); }, reps), bytes);
  }
  rep("write once U4 nt", timeit([&] { write_once<4, 1><<<n4 / 1024, 256>>>((float4*)y, n4); }, reps), bytes);
  rep("write once U4 sc0sc1", timeit([&] { write_once<4, 2><<<n4 / 1024, 256>>>((float4*)y, n4); }, reps), bytes);
  rep("write once U4 sc1", timeit([&] { write_once<4, 3><<<n4 / 1024, 256>>>((float4*)y, n4); }, reps), bytes);
  rep("write once U1 sc0sc1", timeit([&] { write_once<1, 2><<<n4 / 256, 256>>>((float4*)y, n4); }, reps), bytes);
  rep("write lane64", timeit([&] { write_lane64<<<n4 / 1024, 256>>>((float4*)y, n4); }, reps), bytes);
  rep("write LDS tile 8192", timeit([&] { write_tile<false><<<n / 8192, 256>>>(y, n); }, reps), bytes);
  rep("write LDS tile 8192 nt", timeit([&] { write_tile<true><<<n / 8192, 256>>>(y, n); }, reps), bytes);
  rep("copy grid-stride grid=8192", timeit([&] { copy_gs<<<8192, 256>>>((const float4*)x, (float4*)y, n4); }, reps), 2 * bytes);
  rep("hipMemsetAsync 1 GiB", timeit([&] { CK(hipMemsetAsync(y, 0, n * 4)); }, reps), bytes);
  return 0;
}
