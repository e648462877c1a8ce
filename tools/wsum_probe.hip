// wsum_probe.hip — shapes of the weighted fold dst = beta*dst + sum_m w_m * src_m (8 x 25 M fp32), timed with HIP
// events, variants interleaved: the product's grid-stride kernel (one float4 per source per iteration, non-temporal
// loads), non-temporal stores, two float4 per source per iteration, block-contiguous chunks, and grid sizes.
// Build on the box: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/wsum_probe tools/wsum_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kSrc = 8;
struct Pack {
  const float* p[kSrc];
  float w[kSrc];
};

__device__ __forceinline__ f32x4 ldnt(const float* p) { return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p)); }

template <bool NTST>
__device__ __forceinline__ void fold1(const Pack& s, float beta, float* dst, int64_t i) {
  f32x4 a = *reinterpret_cast<const f32x4*>(dst + 4 * i);
  a = a * beta;
  f32x4 v[kSrc];
#pragma unroll
  for (int m = 0; m < kSrc; ++m) v[m] = ldnt(s.p[m] + 4 * i);
#pragma unroll
  for (int m = 0; m < kSrc; ++m) {
    a.x = fmaf(s.w[m], v[m].x, a.x);
    a.y = fmaf(s.w[m], v[m].y, a.y);
    a.z = fmaf(s.w[m], v[m].z, a.z);
    a.w = fmaf(s.w[m], v[m].w, a.w);
  }
  if (NTST) __builtin_nontemporal_store(a, reinterpret_cast<f32x4*>(dst + 4 * i));
  else *reinterpret_cast<f32x4*>(dst + 4 * i) = a;
}

// grid-stride, one float4 per source per iteration
template <bool NTST>
__global__ __launch_bounds__(256) void k_stride(Pack s, int64_t n4, float beta, float* dst) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) fold1<NTST>(s, beta, dst, i);
}

// grid-stride, two float4 per source per iteration (both batches of loads in flight)
template <bool NTST>
__global__ __launch_bounds__(256) void k_stride2(Pack s, int64_t n4, float beta, float* dst) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    f32x4 a0 = *reinterpret_cast<const f32x4*>(dst + 4 * i) * beta;
    f32x4 a1 = *reinterpret_cast<const f32x4*>(dst + 4 * (i + stride)) * beta;
    f32x4 v0[kSrc], v1[kSrc];
#pragma unroll
    for (int m = 0; m < kSrc; ++m) {
      v0[m] = ldnt(s.p[m] + 4 * i);
      v1[m] = ldnt(s.p[m] + 4 * (i + stride));
    }
#pragma unroll
    for (int m = 0; m < kSrc; ++m) {
      a0.x = fmaf(s.w[m], v0[m].x, a0.x); a0.y = fmaf(s.w[m], v0[m].y, a0.y);
      a0.z = fmaf(s.w[m], v0[m].z, a0.z); a0.w = fmaf(s.w[m], v0[m].w, a0.w);
      a1.x = fmaf(s.w[m], v1[m].x, a1.x); a1.y = fmaf(s.w[m], v1[m].y, a1.y);
      a1.z = fmaf(s.w[m], v1[m].z, a1.z); a1.w = fmaf(s.w[m], v1[m].w, a1.w);
    }
    if (NTST) {
      __builtin_nontemporal_store(a0, reinterpret_cast<f32x4*>(dst + 4 * i));
      __builtin_nontemporal_store(a1, reinterpret_cast<f32x4*>(dst + 4 * (i + stride)));
    } else {
      *reinterpret_cast<f32x4*>(dst + 4 * i) = a0;
      *reinterpret_cast<f32x4*>(dst + 4 * (i + stride)) = a1;
    }
  }
  for (; i < n4; i += stride) fold1<NTST>(s, beta, dst, i);
}

// block-contiguous chunks: block b folds float4s [b * per, (b + 1) * per), 256 at a time
template <bool NTST>
__global__ __launch_bounds__(256) void k_chunk(Pack s, int64_t n4, float beta, float* dst, int64_t per) {
  const int64_t a = (int64_t)blockIdx.x * per, b = a + per < n4 ? a + per : n4;
  for (int64_t i = a + threadIdx.x; i < b; i += 256) fold1<NTST>(s, beta, dst, i);
}

int main() {
  const int64_t n = 25'000'000, n4 = n / 4;
  std::vector<float*> src(kSrc);
  for (auto& p : src) {
    CK(hipMalloc(&p, n * 4));
    CK(hipMemset(p, 0, n * 4));
  }
  float* dst;
  CK(hipMalloc(&dst, n * 4));
  CK(hipMemset(dst, 0, n * 4));
  Pack s;
  for (int m = 0; m < kSrc; ++m) {
    s.p[m] = src[m];
    s.w[m] = 0.125f;
  }
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (kSrc + 2) * 4.0 * n;
  struct V {
    const char* name;
    int kind;  // 0 stride, 1 stride2, 2 chunk
    bool nt;
    int grid;
  };
  const int full = (int)((n4 + 255) / 256);
  std::vector<V> vs = {{"stride g=4096 (product)", 0, false, 4096}, {"stride g=8192", 0, false, 8192},
                       {"stride g=16384", 0, false, 16384},         {"stride g=full (1 per thread)", 0, false, full},
                       {"stride g=cus*32", 0, false, cus * 32},     {"stride g=cus*64", 0, false, cus * 64},
                       {"stride2 g=8192", 1, false, 8192},          {"stride2 g=full/2", 1, false, (full + 1) / 2},
                       {"stride g=full nt-store", 0, true, full}};
  auto launch = [&](const V& v) {
    if (v.kind == 0) {
      if (v.nt) hipLaunchKernelGGL(k_stride<true>, dim3(v.grid), dim3(256), 0, 0, s, n4, 0.5f, dst);
      else hipLaunchKernelGGL(k_stride<false>, dim3(v.grid), dim3(256), 0, 0, s, n4, 0.5f, dst);
    } else if (v.kind == 1) {
      if (v.nt) hipLaunchKernelGGL(k_stride2<true>, dim3(v.grid), dim3(256), 0, 0, s, n4, 0.5f, dst);
      else hipLaunchKernelGGL(k_stride2<false>, dim3(v.grid), dim3(256), 0, 0, s, n4, 0.5f, dst);
    } else {
      const int64_t per = (n4 + v.grid - 1) / v.grid;
      hipLaunchKernelGGL(k_chunk<false>, dim3(v.grid), dim3(256), 0, 0, s, n4, 0.5f, dst, per);
    }
  };
  for (int rnd = 0; rnd < 3; ++rnd) {
    for (const V& v : vs) {
      for (int w = 0; w < 3; ++w) launch(v);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      const int reps = 20;
      for (int r = 0; r < reps; ++r) launch(v);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps;
      printf("round %d %-26s %7.1f us  %6.0f GB/s\n", rnd, v.name, us, bytes / us * 1e-3);
      fflush(stdout);
    }
  }
  return 0;
}
