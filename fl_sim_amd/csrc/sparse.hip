// sparse.hip — dense decoders of the sparse wires and the elementwise compressors, for gfx950
// (reference: fl_sim/compressors/compressors.py:273-296).
//
//   sparse_decode   dense output tile by tile (8192 outputs = 32 KiB of LDS per block): a 64-ary wave
//                   search finds the tile's slice of the ascending index stream, the tile is zero-filled
//                   in LDS, the slice scattered into it, and the tile streamed out with 16-B stores.
//                   Algorithmic bytes: 4 per output element + 8 (top-k: idx+val) or 5 (stacked:
//                   idx+code) per kept entry.  Optionally fused with the aggregation: out = fmaf(w, v, out).
//   randk_scatter   out[idx[j]] = fp32(D/K) * x[idx[j]] after a zero fill (compressors.py:289-291).
//   elementwise     identical (+x) and lazy (x / p) (compressors.py:273-283).
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kThreads = 256;
constexpr int kTile = 8192;

// 64-ary lower bound by one wave: first i in [0, n) with a[i] >= key (n if none), a ascending
__device__ long long wave_lower_bound(const int* __restrict__ a, long long n, int key) {
  const int lane = threadIdx.x & (kWave - 1);
  long long lo = 0, hi = n;  // a[i] < key for i < lo; a[hi] >= key or hi == n
  while (hi - lo > kWave) {
    const long long stride = (hi - lo + kWave - 1) / kWave;
    const long long p = lo + (long long)lane * stride;
    const bool lt = p < hi && a[p] < key;
    const int cnt = __popcll(__ballot(lt));  // probes below key form a prefix of the lanes
    const long long nlo = cnt > 0 ? lo + (long long)(cnt - 1) * stride + 1 : lo;
    const long long nhi = lo + (long long)cnt * stride < hi ? lo + (long long)cnt * stride : hi;
    lo = nlo;
    hi = nhi;
  }
  const long long p = lo + lane;
  const bool lt = p < hi && a[p] < key;
  return lo + __popcll(__ballot(lt));
}

// ------------------------------------------------------------------------------------------------
// K5: sparse -> dense decode (tile = 8192 outputs, LDS scatter, 16-B stores)
//   MODE 0: v = scale * val[j];  MODE 1: v = dithering decode of codes[j] (s = levels, norm)
// ------------------------------------------------------------------------------------------------
template <int MODE, bool ACC>
__global__ __launch_bounds__(kThreads) void sparse_decode_kernel(const int* __restrict__ idx, const float* __restrict__ val,
                                                                 const uint8_t* __restrict__ codes, long long k, float scale,
                                                                 int levels, double step, const float* __restrict__ norm_ptr,
                                                                 int64_t n, float weight, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float s_tile[kTile];
  __shared__ long long s_lo, s_hi;
  const int64_t t0 = (int64_t)blockIdx.x * kTile;
  const int64_t t1 = t0 + kTile < n ? t0 + kTile : n;
  const int wid = threadIdx.x >> 6;
  if (wid == 0) {
    const long long lo = wave_lower_bound(idx, k, (int)t0);
    if (threadIdx.x == 0) s_lo = lo;
  } else if (wid == 1) {
    const long long hi = t1 >= n ? k : wave_lower_bound(idx, k, (int)t1);
    if (threadIdx.x == kWave) s_hi = hi;
  }
  float4* tile4 = reinterpret_cast<float4*>(s_tile);
  for (int i = threadIdx.x; i < kTile / 4; i += kThreads) tile4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  const long long lo = s_lo, hi = s_hi;
  float nrm = 0.f;
  if (MODE == 1) nrm = *norm_ptr;
  for (long long j = lo + threadIdx.x; j < hi; j += kThreads) {
    float v;
    if (MODE == 0) {
      v = scale * val[j];
    } else {
      const uint32_t code = codes[j];
      if (!(nrm > 0.0f && nrm <= 3.402823466e38f)) {
        v = code == 0u ? 0.0f : __uint_as_float(0x7fc00000u);
      } else {
        const float lv = (float)level_value<0>((int)(code & 127u), levels, step);
        v = ((code >> 7) ? -lv : lv) * nrm;
      }
    }
    const unsigned long long off = (unsigned long long)((long long)idx[j] - (long long)t0);
    if (off < (unsigned long long)kTile) s_tile[off] = v;
  }
  __syncthreads();
  const int64_t len = t1 - t0;
  if (len == kTile && ((reinterpret_cast<uintptr_t>(out) & 15u) == 0)) {
    float4* o4 = reinterpret_cast<float4*>(out + t0);
    for (int i = threadIdx.x; i < kTile / 4; i += kThreads) {
      float4 v = tile4[i];
      if (ACC) {
        const float4 p = o4[i];
        v = make_float4(fmaf(weight, v.x, p.x), fmaf(weight, v.y, p.y), fmaf(weight, v.z, p.z), fmaf(weight, v.w, p.w));
      } else if (weight != 1.0f) {
        v = make_float4(weight * v.x, weight * v.y, weight * v.z, weight * v.w);
      }
      st_stream(out + t0 + 4 * (int64_t)i, v);
    }
  } else {
    for (int64_t i = threadIdx.x; i < len; i += kThreads) {
      float v = s_tile[i];
      if (ACC) v = fmaf(weight, v, out[t0 + i]);
      else if (weight != 1.0f) v = weight * v;
      out[t0 + i] = v;
    }
  }
}

// rand-k scatter: out[idx[j]] = scale * x[idx[j]] (out pre-zeroed)
__global__ __launch_bounds__(kThreads) void randk_scatter_kernel(const float* __restrict__ x, const int* __restrict__ idx,
                                                                 long long k, float scale, float* __restrict__ out) {
  for (long long j = (long long)blockIdx.x * kThreads + threadIdx.x; j < k; j += (long long)gridDim.x * kThreads) {
    const int i = idx[j];
    out[i] = scale * x[i];
  }
}

// out = x / p (lazy) or out = x (identical, p == 1 handled as a copy)
template <bool DIV>
__global__ __launch_bounds__(kThreads) void elementwise_kernel(const float* __restrict__ x, int64_t n, float p,
                                                               float* __restrict__ out) {
  const int64_t n4 = n >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  float4* o4 = reinterpret_cast<float4*>(out);
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
    float4 v = x4[i];
    if (DIV) v = make_float4(v.x / p, v.y / p, v.z / p, v.w / p);
    o4[i] = v;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads)
    out[i] = DIV ? x[i] / p : x[i];
}

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

int flc_sparse_decode(const int32_t* idx, const float* val, int64_t k, float scale, int64_t n, float weight,
                      int accumulate, float* out, void* stream) {
  if (!out || n <= 0 || k < 0 || (k > 0 && (!idx || !val))) return fail(FLC_EINVAL, "flc_sparse_decode: bad arguments");
  if (n >= (1ll << 31)) return fail(FLC_EINVAL, "flc_sparse_decode: n must be < 2^31");
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)cdiv(n, kTile);
  if (accumulate)
    FLC_LAUNCH("sparse_decode", (sparse_decode_kernel<0, true>), dim3(grid), dim3(kThreads), 0, st, idx, val,
               (const uint8_t*)nullptr, (long long)k, scale, 0, 0.0, (const float*)nullptr, n, weight, out);
  else
    FLC_LAUNCH("sparse_decode", (sparse_decode_kernel<0, false>), dim3(grid), dim3(kThreads), 0, st, idx, val,
               (const uint8_t*)nullptr, (long long)k, scale, 0, 0.0, (const float*)nullptr, n, weight, out);
  return FLC_OK;
}

int flc_stacked_decode(const int32_t* idx, const uint8_t* codes, int64_t k, int levels, const float* norm, int64_t n,
                       float weight, int accumulate, float* out, void* stream) {
  if (!out || !norm || n <= 0 || k < 0 || (k > 0 && (!idx || !codes)))
    return fail(FLC_EINVAL, "flc_stacked_decode: bad arguments");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_stacked_decode: levels must be in [1, 127]");
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)cdiv(n, kTile);
  const double step = 1.0 / (double)levels;
  if (accumulate)
    FLC_LAUNCH("stacked_decode", (sparse_decode_kernel<1, true>), dim3(grid), dim3(kThreads), 0, st, idx,
               (const float*)nullptr, codes, (long long)k, 1.0f, levels, step, norm, n, weight, out);
  else
    FLC_LAUNCH("stacked_decode", (sparse_decode_kernel<1, false>), dim3(grid), dim3(kThreads), 0, st, idx,
               (const float*)nullptr, codes, (long long)k, 1.0f, levels, step, norm, n, weight, out);
  return FLC_OK;
}

int flc_copy(const float* x, int64_t n, float* out, void* stream) {
  if (!x || !out || n < 0) return fail(FLC_EINVAL, "flc_copy: bad arguments");
  if (n == 0) return FLC_OK;
  if (!aligned16(x) || !aligned16(out)) return fail(FLC_EINVAL, "flc_copy: 16-B aligned buffers required");
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(cdiv(n, 4), kThreads), 256 * 16);
  FLC_LAUNCH("copy", elementwise_kernel<false>, dim3(grid), dim3(kThreads), 0, st, x, n, 1.0f, out);
  return FLC_OK;
}

int flc_scale_div(const float* x, int64_t n, float p, float* out, void* stream) {
  if (!x || !out || n < 0) return fail(FLC_EINVAL, "flc_scale_div: bad arguments");
  if (n == 0) return FLC_OK;
  if (!aligned16(x) || !aligned16(out)) return fail(FLC_EINVAL, "flc_scale_div: 16-B aligned buffers required");
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(cdiv(n, 4), kThreads), 256 * 16);
  FLC_LAUNCH("scale_div", elementwise_kernel<true>, dim3(grid), dim3(kThreads), 0, st, x, n, p, out);
  return FLC_OK;
}

int flc_randk_apply(const float* x, int64_t n, const int32_t* idx, int64_t k, float scale, float* out, void* stream) {
  if (!x || !out || n <= 0 || k < 0 || (k > 0 && !idx)) return fail(FLC_EINVAL, "flc_randk_apply: bad arguments");
  hipStream_t st = as_stream(stream);
  FLC_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)n * sizeof(float), st));
  if (k == 0) return FLC_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(k, kThreads), 256 * 16);
  FLC_LAUNCH("randk_scatter", randk_scatter_kernel, dim3(grid), dim3(kThreads), 0, st, x, idx, (long long)k, scale, out);
  return FLC_OK;
}

}  // extern "C"

