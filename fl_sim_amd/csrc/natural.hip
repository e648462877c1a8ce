// natural.hip — natural compression (Horváth et al.) for gfx950
// (reference: fl_sim/compressors/compressors.py:302-325).
//
// Per nonzero element: f = floor(log2|x|) from the exponent bits, pt = 2 - |x| / 2^f (exact in fp32,
// equal to the reference's (2^ceil - |x|) / 2^floor), round down to 2^f iff u < pt, else up to
// 2^(f+1); a power of two maps to itself either way.  Wire: uint16 per element, 0 = zero,
// 0x7fff = NaN, else sign << 15 | (e + 150).  Each thread owns 8 consecutive elements (two 16-B
// loads, one 16-B code store): encode reads 4 B and writes 2 B per element, decode the reverse.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kThreads = 256;
constexpr int kNW = kThreads / kWave;
constexpr int kGroup = 8;
constexpr int kGroupsPerBlock = 1024;

__device__ __forceinline__ uint32_t natural_code(float xv, double u) {
  if (xv == 0.0f) return 0u;
  const uint32_t bits = __float_as_uint(xv);
  const uint32_t sign = bits >> 31;
  const uint32_t ab = bits & 0x7fffffffu;
  if (ab > 0x7f800000u) return 0x7fffu;                    // NaN (the reference raises)
  if (ab == 0x7f800000u) return (sign << 15) | (128 + 150);  // inf (the reference raises)
  const uint32_t E = ab >> 23;
  int f;
  if (E == 0) f = (31 - __clz((int)ab)) - 149;  // subnormal: highest set mantissa bit
  else f = (int)E - 127;
  const float m = ldexpf(__uint_as_float(ab), -f);  // |x| / 2^f in [1, 2), exact
  const float pt = 2.0f - m;                         // exact
  const int e = (u < (double)pt) ? f : f + 1;
  return (sign << 15) | (uint32_t)(e + 150);
}

__device__ __forceinline__ float natural_value(uint32_t code) {
  if (code == 0u) return 0.0f;
  if (code == 0x7fffu) return __uint_as_float(0x7fc00000u);
  const int e = (int)(code & 0x7fffu) - 150;
  const float v = ldexpf(1.0f, e);
  return (code >> 15) ? -v : v;
}

__device__ __forceinline__ void load8(const float* __restrict__ x, int64_t e0, int valid, float v[kGroup]) {
  if (valid == kGroup) {
    const float4 a = *reinterpret_cast<const float4*>(x + e0);
    const float4 b = *reinterpret_cast<const float4*>(x + e0 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < kGroup; ++j) v[j] = j < valid ? x[e0 + j] : 0.0f;
  }
}

__global__ __launch_bounds__(kThreads) void natural_count_kernel(const float* __restrict__ x, int64_t n,
                                                                 int* __restrict__ counts) {
  __shared__ int s_red[kNW];
  const int64_t g_begin = (int64_t)blockIdx.x * kGroupsPerBlock;
  int cnt = 0;
  for (int it = 0; it < kGroupsPerBlock / kThreads; ++it) {
    const int64_t e0 = (g_begin + it * kThreads + threadIdx.x) * kGroup;
    if (e0 >= n) break;
    const int valid = n - e0 < kGroup ? (int)(n - e0) : kGroup;
    float v[kGroup];
    load8(x, e0, valid, v);
#pragma unroll
    for (int j = 0; j < kGroup; ++j) cnt += (j < valid && v[j] != 0.0f) ? 1 : 0;
  }
  const int tot = block_sum<int, kNW>(cnt, s_red);
  if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void natural_scan_kernel(const int* __restrict__ counts, long long* __restrict__ offsets,
                                                            int64_t nchunks) {
  __shared__ long long s_red[16];
  long long running = 0;
  for (int64_t base = 0; base < nchunks; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const long long v = i < nchunks ? counts[i] : 0;
    long long tot;
    const long long ex = block_excl_scan<long long, 16>(v, s_red, &tot);
    if (i < nchunks) offsets[i] = running + ex;
    running += tot;
  }
}

template <bool COMPAT>
__global__ __launch_bounds__(kThreads) void natural_encode_kernel(const float* __restrict__ x, int64_t n, uint64_t seed,
                                                                  uint64_t counter, const double* __restrict__ compat_u,
                                                                  const long long* __restrict__ offsets,
                                                                  uint16_t* __restrict__ codes,
                                                                  unsigned long long* __restrict__ nnz) {
  __shared__ long long s_scan[kNW];
  __shared__ unsigned long long s_nnz;
  const int64_t g_begin = (int64_t)blockIdx.x * kGroupsPerBlock;
  long long running = COMPAT ? offsets[blockIdx.x] : 0;
  if (threadIdx.x == 0) s_nnz = 0;
  __syncthreads();
  unsigned my_nnz = 0;
  for (int it = 0; it < kGroupsPerBlock / kThreads; ++it) {
    const int64_t e0 = (g_begin + it * kThreads + threadIdx.x) * kGroup;
    const int valid = e0 >= n ? 0 : (n - e0 < kGroup ? (int)(n - e0) : kGroup);
    float v[kGroup];
    if (valid > 0) load8(x, e0, valid, v);
    else
#pragma unroll
      for (int j = 0; j < kGroup; ++j) v[j] = 0.0f;
    double u[kGroup];
    int c[kGroup];
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < kGroup; ++j) {
      c[j] = (j < valid && v[j] != 0.0f) ? 1 : 0;
      cnt += c[j];
    }
    my_nnz += cnt;
    if (COMPAT) {
      long long tot;
      const long long ex = block_excl_scan<long long, kNW>((long long)cnt, s_scan, &tot);
      long long r = running + ex;
#pragma unroll
      for (int j = 0; j < kGroup; ++j) {
        u[j] = c[j] ? compat_u[r] : 0.0;
        r += c[j];
      }
      running += tot;
    } else if (valid > 0) {
      const U4 a = philox_group((uint64_t)e0 >> 2, seed, counter);
      const U4 b = philox_group(((uint64_t)e0 >> 2) + 1, seed, counter);
      u[0] = u01(a.x); u[1] = u01(a.y); u[2] = u01(a.z); u[3] = u01(a.w);
      u[4] = u01(b.x); u[5] = u01(b.y); u[6] = u01(b.z); u[7] = u01(b.w);
    }
    if (valid == 0) continue;
    uint32_t cd[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; ++j) cd[j] = natural_code(v[j], u[j]);
    if (valid == kGroup) {
      uint4 p;
      p.x = cd[0] | (cd[1] << 16);
      p.y = cd[2] | (cd[3] << 16);
      p.z = cd[4] | (cd[5] << 16);
      p.w = cd[6] | (cd[7] << 16);
      *reinterpret_cast<uint4*>(codes + e0) = p;
    } else {
      for (int j = 0; j < valid; ++j) codes[e0 + j] = (uint16_t)cd[j];
    }
  }
  if (nnz) {
    const unsigned w = wave_sum(my_nnz);
    if ((threadIdx.x & 63) == 0 && w) atomicAdd(&s_nnz, (unsigned long long)w);
    __syncthreads();
    if (threadIdx.x == 0 && s_nnz) atomicAdd(nnz, s_nnz);
  }
}

template <bool ACC>
__global__ __launch_bounds__(kThreads) void natural_decode_kernel(const uint16_t* __restrict__ codes, int64_t n, float weight,
                                                                  float* __restrict__ out) {
  const int64_t ngroups = (n + kGroup - 1) / kGroup;
  for (int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x; g < ngroups; g += (int64_t)gridDim.x * kThreads) {
    const int64_t e0 = g * kGroup;
    const int valid = n - e0 < kGroup ? (int)(n - e0) : kGroup;
    uint32_t cd[kGroup];
    if (valid == kGroup) {
      const uint4 p = *reinterpret_cast<const uint4*>(codes + e0);
      cd[0] = p.x & 0xffffu; cd[1] = p.x >> 16; cd[2] = p.y & 0xffffu; cd[3] = p.y >> 16;
      cd[4] = p.z & 0xffffu; cd[5] = p.z >> 16; cd[6] = p.w & 0xffffu; cd[7] = p.w >> 16;
    } else {
#pragma unroll
      for (int j = 0; j < kGroup; ++j) cd[j] = j < valid ? codes[e0 + j] : 0u;
    }
    float o[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; ++j) o[j] = natural_value(cd[j]);
    if (ACC) {
      float prev[kGroup];
      load8(out, e0, valid, prev);
#pragma unroll
      for (int j = 0; j < kGroup; ++j) o[j] = fmaf(weight, o[j], prev[j]);
    } else if (weight != 1.0f) {
#pragma unroll
      for (int j = 0; j < kGroup; ++j) o[j] = weight * o[j];
    }
    if (valid == kGroup) {
      *reinterpret_cast<float4*>(out + e0) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(out + e0 + 4) = make_float4(o[4], o[5], o[6], o[7]);
    } else {
      for (int j = 0; j < valid; ++j) out[e0 + j] = o[j];
    }
  }
}

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

size_t flc_natural_workspace_size(int64_t n) {
  Carver c(nullptr, 0);
  const int64_t nblocks = cdiv(n < 1 ? 1 : n, (int64_t)kGroup * kGroupsPerBlock);
  (void)c.take<int>((size_t)nblocks);
  (void)c.take<long long>((size_t)nblocks);
  return c.off;
}

int flc_natural_encode(const float* x, int64_t n, uint64_t seed, uint64_t counter, const double* compat_u,
                       uint16_t* codes, int64_t* nnz, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !codes || n <= 0) return fail(FLC_EINVAL, "flc_natural_encode: bad arguments");
  if (!aligned16(x) || !aligned16(codes)) return fail(FLC_EINVAL, "flc_natural_encode: 16-B aligned buffers required");
  const int64_t nblocks = cdiv(n, (int64_t)kGroup * kGroupsPerBlock);
  hipStream_t st = as_stream(stream);
  unsigned long long* nz = reinterpret_cast<unsigned long long*>(nnz);
  if (nnz) FLC_CHECK_HIP(hipMemsetAsync(nnz, 0, sizeof(int64_t), st));
  if (compat_u) {
    Carver c(ws, ws_bytes);
    int* counts = c.take<int>((size_t)nblocks);
    long long* offsets = c.take<long long>((size_t)nblocks);
    if (!ws || !c.ok()) return fail(FLC_EWORKSPACE, "flc_natural_encode: workspace %zu < %zu", ws_bytes, c.off);
    FLC_LAUNCH("natural_count", natural_count_kernel, dim3((unsigned)nblocks), dim3(kThreads), 0, st, x, n, counts);
    FLC_LAUNCH("natural_scan", natural_scan_kernel, dim3(1), dim3(1024), 0, st, counts, offsets, nblocks);
    FLC_LAUNCH("natural_encode", natural_encode_kernel<true>, dim3((unsigned)nblocks), dim3(kThreads), 0, st, x, n, seed,
               counter, compat_u, offsets, codes, nz);
  } else {
    FLC_LAUNCH("natural_encode", natural_encode_kernel<false>, dim3((unsigned)nblocks), dim3(kThreads), 0, st, x, n,
               seed, counter, compat_u, (const long long*)nullptr, codes, nz);
  }
  return FLC_OK;
}

int flc_natural_decode(const uint16_t* codes, int64_t n, float weight, int accumulate, float* out, void* stream) {
  if (!codes || !out || n <= 0) return fail(FLC_EINVAL, "flc_natural_decode: bad arguments");
  if (!aligned16(out) || !aligned16(codes)) return fail(FLC_EINVAL, "flc_natural_decode: 16-B aligned buffers required");
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(cdiv(n, kGroup), kThreads), 256 * 32);
  if (accumulate)
    FLC_LAUNCH("natural_decode", natural_decode_kernel<true>, dim3(grid), dim3(kThreads), 0, st, codes, n, weight, out);
  else
    FLC_LAUNCH("natural_decode", natural_decode_kernel<false>, dim3(grid), dim3(kThreads), 0, st, codes, n, weight, out);
  return FLC_OK;
}

}  // extern "C"
