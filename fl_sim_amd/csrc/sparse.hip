// sparse.hip — dense decoders of the sparse wires and the elementwise compressors, for gfx950
// (reference: fl_sim/compressors/compressors.py:273-296).
//
//   tile_index      tile_start[t] = first kept entry of output tile t (one thread per kept entry).
//   sparse_decode   dense output, one 64-lane wave per two adjacent 1024-output tiles (8 KB): the tiles' kept-entry
//                   ranges from the tile pointers, both tiles' entries in flight together, a scatter into the wave's
//                   LDS tiles, 16-B coalesced stores (the shape whose stores reach the write rate the decode needs,
//                   tools/bwprobe4-5.hip; the other shapes measured are in DESIGN §8).  Accumulating
//                   (out = fmaf(w, v, out), the aggregation fused) takes one wave per tile, its slice of `out` read
//                   first.  Algorithmic bytes: 4 per output element + 8 (top-k: idx+val) or 5 (stacked: idx+code)
//                   per kept entry.
//   randk_scatter   out[idx[j]] = fp32(D/K) * x[idx[j]] after a zero fill (compressors.py:289-291).
//   elementwise     identical (+x) and lazy (x / p) (compressors.py:273-283).
#include <hip/hip_runtime.h>
#include <math.h>

#include <stdlib.h>

#include <algorithm>
#include <atomic>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

#ifndef FLC_DECODE_WT
#define FLC_DECODE_WT 1  // the dense decode's output stores written through (st_wt; 0: plain stores, the A/B switch)
#endif

namespace flc {
namespace {

constexpr int kThreads = 256;

// tile_start[t] = first j with idx[j] >= t * TILE (t = 0 .. ntiles); idx ascending.  One thread per
// kept entry: entry j fills the tiles between its predecessor's tile and its own.
template <int TILE_LOG>
__global__ __launch_bounds__(kThreads) void tile_index_kernel(const int* __restrict__ idx, long long k, long long ntiles,
                                                              unsigned* __restrict__ tile_start) {
  for (long long j = (long long)blockIdx.x * kThreads + threadIdx.x; j <= k; j += (long long)gridDim.x * kThreads) {
    long long tj = j < k ? ((long long)(unsigned)idx[j] >> TILE_LOG) : ntiles;
    tj = tj < ntiles ? tj : ntiles;
    const long long tp = j > 0 ? ((long long)(unsigned)idx[j - 1] >> TILE_LOG) : -1;
    for (long long t = tp + 1; t <= tj; ++t) tile_start[t] = (unsigned)j;
  }
}

// raw wire word of kept entry j (MODE 0: fp32 bits of val; MODE 1: the code byte) and its decoded value
template <int MODE>
__device__ __forceinline__ uint32_t entry_raw(const float* __restrict__ val, const uint8_t* __restrict__ codes,
                                              unsigned j) {
  return MODE == 0 ? __float_as_uint(val[j]) : (uint32_t)codes[j];
}
template <int MODE>
__device__ __forceinline__ float entry_value(uint32_t raw, float scale, int levels, double step, float nrm) {
  if (MODE == 0) return scale * __uint_as_float(raw);
  return stacked_dequant(raw, levels, step, nrm);  // compressors.py:357
}

// One-wave decode: one 64-lane workgroup per 1024-output tile (4 KB of output).  Measured on MI355X
// (tools/bwprobe4.hip), 1 GiB of 16-B stores reaches 6.8-6.9 TB/s when every workgroup writes one
// contiguous 4 KB piece, but only 5.6-6.1 TB/s with 8-16 KB per workgroup; a single wave also needs no
// s_barrier between its LDS scatter and its LDS read.  Per tile: the kept-entry range from tile_start
// (scalar loads), the tile's entries (one per lane, more in a loop), a scatter into the wave's 4 KB LDS
// tile, four 1-KB coalesced stores.
template <int MODE, bool ACC>
__global__ __launch_bounds__(kWave) void sparse_decode_wave_kernel(const int* __restrict__ idx,
                                                                   const float* __restrict__ val,
                                                                   const uint8_t* __restrict__ codes, float scale,
                                                                   int levels, double step,
                                                                   const float* __restrict__ norm_ptr, int64_t n,
                                                                   float weight, float* __restrict__ out,
                                                                   const unsigned* __restrict__ tile_start,
                                                                   unsigned k) {
  constexpr int TILE = 1024;
  __shared__ __attribute__((aligned(16))) float s_tile[TILE];
  const int lane = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * TILE;
  float4 acc[4];
  if (ACC) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = t0 + 4 * (int64_t)(lane + u * kWave);
      acc[u] = e + 4 <= n ? *reinterpret_cast<const float4*>(out + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // (entries clamped to [0, k): a malformed tile pointer never reads past the wire.  Both loads are issued before the
  // clamps — a scalar load's value is waited for with lgkmcnt(0), and a clamp scheduled between the loads made them
  // two round trips)
  unsigned lo = tile_start[blockIdx.x], hi = tile_start[blockIdx.x + 1];
  float4* tile4 = reinterpret_cast<float4*>(s_tile);
#pragma unroll
  for (int u = 0; u < 4; ++u) tile4[lane + u * kWave] = make_float4(0.f, 0.f, 0.f, 0.f);
  __builtin_amdgcn_sched_barrier(0);
  lo = min(lo, k);
  hi = min(hi, k);
  const float nrm = MODE == 1 ? *norm_ptr : 0.0f;
  for (unsigned j = lo + lane; j < hi; j += kWave) {
    const int64_t off = (int64_t)(unsigned)idx[j] - t0;
    if (off >= 0 && off < TILE) s_tile[off] = entry_value<MODE>(entry_raw<MODE>(val, codes, j), scale, levels, step, nrm);
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = lane + u * kWave;
    const int64_t e = t0 + 4 * (int64_t)q;
    float4 v = tile4[q];
    if (e + 4 <= n) {
      if (ACC) {
        v = make_float4(fmaf(weight, v.x, acc[u].x), fmaf(weight, v.y, acc[u].y), fmaf(weight, v.z, acc[u].z),
                        fmaf(weight, v.w, acc[u].w));
      } else if (weight != 1.0f) {
        v = make_float4(weight * v.x, weight * v.y, weight * v.z, weight * v.w);
      }
      *reinterpret_cast<float4*>(out + e) = v;
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int c = 0; c < 4 && e + c < n; ++c) {
        float o = vv[c];
        if (ACC) o = fmaf(weight, o, out[e + c]);
        else if (weight != 1.0f) o = weight * o;
        out[e + c] = o;
      }
    }
  }
}

// One-wave decode, NT tiles of 1024 outputs per wave (adjacent: one NT x 4 KB piece), every load chain
// of the NT tiles in flight together.
template <int MODE, int NT>
__global__ __launch_bounds__(kWave) void sparse_decode_wave2_kernel(const int* __restrict__ idx,
                                                                    const float* __restrict__ val,
                                                                    const uint8_t* __restrict__ codes, float scale,
                                                                    int levels, double step,
                                                                    const float* __restrict__ norm_ptr, int64_t n,
                                                                    float weight, float* __restrict__ out,
                                                                    const unsigned* __restrict__ tile_start,
                                                                    int64_t ntiles, unsigned k, int rev) {
  constexpr int TILE = 1024;
  __shared__ __attribute__((aligned(16))) float s_tile[NT * TILE];
  const int lane = threadIdx.x;
  // plain order (XCD-chunked orders measured no faster); `rev`: from the last pair down
  const int64_t g = rev ? (int64_t)gridDim.x - 1 - blockIdx.x : (int64_t)blockIdx.x;
  const int64_t tb = g * NT;
  const int64_t t0 = tb * TILE;
  unsigned ts[NT + 1];
#pragma unroll
  for (int i = 0; i <= NT; ++i) ts[i] = tile_start[tb + i < ntiles ? tb + i : ntiles];
  float4* tile4 = reinterpret_cast<float4*>(s_tile);
#pragma unroll
  for (int u = 0; u < 4 * NT; ++u) tile4[lane + u * kWave] = make_float4(0.f, 0.f, 0.f, 0.f);
  __builtin_amdgcn_sched_barrier(0);  // (every load and the zeroing issued before the clamps: see above)
#pragma unroll
  for (int i = 0; i <= NT; ++i) ts[i] = min(ts[i], k);
  const float nrm = MODE == 1 ? *norm_ptr : 0.0f;
  // first entry per lane of every tile in flight together, the (rare) rest afterwards
  unsigned e_idx[NT];
  uint32_t e_raw[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const unsigned j = ts[i] + lane;
    e_idx[i] = 0xffffffffu;
    e_raw[i] = 0u;
    if (j < ts[i + 1]) {
      e_idx[i] = (unsigned)idx[j];
      e_raw[i] = entry_raw<MODE>(val, codes, j);
    }
  }
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (e_idx[i] != 0xffffffffu) {
      const int64_t off = (int64_t)e_idx[i] - t0;
      if (off >= 0 && off < NT * TILE) s_tile[off] = entry_value<MODE>(e_raw[i], scale, levels, step, nrm);
    }
    for (unsigned j = ts[i] + kWave + lane; j < ts[i + 1]; j += kWave) {
      const int64_t off = (int64_t)(unsigned)idx[j] - t0;
      if (off >= 0 && off < NT * TILE)
        s_tile[off] = entry_value<MODE>(entry_raw<MODE>(val, codes, j), scale, levels, step, nrm);
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int u = 0; u < 4 * NT; ++u) {
    const int q = lane + u * kWave;
    const int64_t e = t0 + 4 * (int64_t)q;
    float4 v = tile4[q];
    if (e + 4 <= n) {
      if (weight != 1.0f) v = make_float4(weight * v.x, weight * v.y, weight * v.z, weight * v.w);
#if FLC_DECODE_WT
      st_wt(out + e, v);
#else
      *reinterpret_cast<float4*>(out + e) = v;
#endif
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int c = 0; c < 4 && e + c < n; ++c) out[e + c] = weight != 1.0f ? weight * vv[c] : vv[c];
    }
  }
}

// rand-k scatter: out[idx[j]] = scale * x[idx[j]] (out pre-zeroed)
// Rand-K in philox mode: a uniformly random K-subset of [0, n) is the K largest of n i.i.d. random keys.  Key of
// element e: the Philox word the codec's stream gives e (word e & 3 of group e >> 2), shifted right by 2 and read as
// an fp32 bit pattern (a positive finite float: order = the word's order), so the top-k encoder selects the subset
// (ties of the 30-bit keys broken toward higher indices, the encoder's rule).
__global__ __launch_bounds__(kThreads) void randk_keys_kernel(int64_t n, uint64_t seed, uint64_t counter,
                                                              float* __restrict__ keys) {
  const int64_t ng = (n + 3) >> 2;
  for (int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x; g < ng; g += (int64_t)gridDim.x * kThreads) {
    const U4 w = philox_group((uint64_t)g, seed, counter);
    const float4 v = make_float4(__uint_as_float(w.x >> 2), __uint_as_float(w.y >> 2), __uint_as_float(w.z >> 2),
                                 __uint_as_float(w.w >> 2));
    const int64_t e = g << 2;
    if (e + 4 <= n) {
      *reinterpret_cast<float4*>(keys + e) = v;
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int c = 0; c < 4 && e + c < n; ++c) keys[e + c] = vv[c];
    }
  }
}

__global__ __launch_bounds__(kThreads) void randk_scatter_kernel(const float* __restrict__ x, const int* __restrict__ idx,
                                                                 long long k, float scale, float* __restrict__ out) {
  for (long long j = (long long)blockIdx.x * kThreads + threadIdx.x; j < k; j += (long long)gridDim.x * kThreads) {
    const int i = idx[j];
    out[i] = scale * x[i];
  }
}

// out = x / p (lazy) or out = x (identical, p == 1 handled as a copy): one short workgroup per 16 KB chunk (4 float4
// per lane in flight, every load issued before the first store), the tail elements by the last workgroup.  (A
// grid-stride form moving one float4 per lane per iteration copied 1 GiB at 5.2 TB/s.)
constexpr int kCopyF4 = 4;
constexpr int64_t kCopyChunk = (int64_t)kThreads * kCopyF4 * 4;  // elements per workgroup
template <bool DIV>
__global__ __launch_bounds__(kThreads) void stream_kernel(const float* __restrict__ x, int64_t n, float p,
                                                          float* __restrict__ out) {
  const int64_t c0 = (int64_t)blockIdx.x * kCopyChunk;
  const int t = threadIdx.x;
  if (c0 + kCopyChunk <= n) {
    float4 v[kCopyF4];
#pragma unroll
    for (int j = 0; j < kCopyF4; ++j) v[j] = ld_stream(x + c0 + 4 * (j * kThreads + t));
#pragma unroll
    for (int j = 0; j < kCopyF4; ++j) {
      float4 a = v[j];
      if (DIV) a = make_float4(a.x / p, a.y / p, a.z / p, a.w / p);
      st_stream(out + c0 + 4 * (j * kThreads + t), a);  // (non-temporal: 1 GiB 375 -> 362 us, tools/copyprobe.hip)
    }
  } else {
    for (int64_t i = c0 + t; i < n; i += kThreads) out[i] = DIV ? x[i] / p : x[i];
  }
}

size_t decode_ws_bytes(int64_t n) {  // tile index for the smallest tile (1024 outputs)
  return (size_t)(cdiv(n < 1 ? 1 : n, (int64_t)kThreads * 4) + 1) * sizeof(unsigned);
}

template <int MODE>
int launch_decode_wave(const int32_t* idx, const float* val, const uint8_t* codes, int64_t k, float scale, int levels,
                       const float* norm, int64_t n, float weight, int accumulate, float* out, void* ws,
                       size_t ws_bytes, hipStream_t st, const char* name) {
  const int64_t ntiles = cdiv(n, (int64_t)1024);
  const size_t need = (size_t)(ntiles + 1) * sizeof(unsigned);
  if (!ws || ws_bytes < need) return fail(FLC_EWORKSPACE, "%s: workspace %zu < %zu", name, ws_bytes, need);
  if (!aligned16(out)) return fail(FLC_EINVAL, "%s: out must be 16-B aligned", name);
  unsigned* tile_start = static_cast<unsigned*>(ws);
  const unsigned gi = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(k + 1, kThreads), 2048));
  FLC_LAUNCH("tile_index", tile_index_kernel<10>, dim3(gi), dim3(kThreads), 0, st, idx, (long long)k,
             (long long)ntiles, tile_start);
  const double step = levels > 0 ? 1.0 / (double)levels : 0.0;
  if (accumulate)
    FLC_LAUNCH(name, (sparse_decode_wave_kernel<MODE, true>), dim3((unsigned)ntiles), dim3(kWave), 0, st, idx, val,
               codes, scale, levels, step, norm, n, weight, out, tile_start, (unsigned)k);
  else
    FLC_LAUNCH(name, (sparse_decode_wave_kernel<MODE, false>), dim3((unsigned)ntiles), dim3(kWave), 0, st, idx, val,
               codes, scale, levels, step, norm, n, weight, out, tile_start, (unsigned)k);
  return FLC_OK;
}

// decode over given 1024-output tile pointers (no tile_index pass): one wave per two tiles, or, when
// accumulating, one wave per tile (its slice of `out` read first)
template <int MODE>
int launch_decode_tiles(const int32_t* idx, const float* val, const uint8_t* codes, int64_t k, float scale, int levels,
                        const float* norm, int64_t n, float weight, int accumulate, float* out,
                        const unsigned* tile_start, hipStream_t st, const char* name) {
  if (!aligned16(out)) return fail(FLC_EINVAL, "%s: out must be 16-B aligned", name);
  if (k >= (1ll << 31)) return fail(FLC_EINVAL, "%s: k must be < 2^31", name);
  const int64_t ntiles = cdiv(n, (int64_t)FLC_TILE);
  const double step = levels > 0 ? 1.0 / (double)levels : 0.0;
  if (accumulate)
    FLC_LAUNCH(name, (sparse_decode_wave_kernel<MODE, true>), dim3((unsigned)ntiles), dim3(kWave), 0, st, idx, val,
               codes, scale, levels, step, norm, n, weight, out, tile_start, (unsigned)k);
  else {
    // The tile order alternates from call to call (ascending, then descending, ...): a decode then starts on the
    // lines the previous one wrote last, which are still in the 256 MiB memory-side cache, when consecutive decodes
    // write the same output (the server's accumulator, a step loop): 179.0 -> 176.5 us per 1 GiB decode, step
    // 386.9 -> 384.9 us (profiles/r05/r05r_alt_ab.txt).  Every tile is still written by exactly one wave: the output
    // does not depend on the order.  FLC_DECODE_ALT=0 keeps the ascending order.
    static const bool alt = !getenv("FLC_DECODE_ALT") || atoi(getenv("FLC_DECODE_ALT")) != 0;
    static std::atomic<int> parity{0};
    const int rev = alt ? (parity.fetch_xor(1, std::memory_order_relaxed) ^ 1) : 0;
    FLC_LAUNCH(name, (sparse_decode_wave2_kernel<MODE, 2>), dim3((unsigned)cdiv(ntiles, 2)), dim3(kWave), 0, st, idx,
               val, codes, scale, levels, step, norm, n, weight, out, tile_start, ntiles, (unsigned)k, rev);
  }
  return FLC_OK;
}

template <int MODE, int NT>
int launch_decode_wave2(const int32_t* idx, const float* val, const uint8_t* codes, int64_t k, float scale, int levels,
                        const float* norm, int64_t n, float weight, int accumulate, float* out, void* ws,
                        size_t ws_bytes, hipStream_t st, const char* name) {
  if (accumulate) return launch_decode_wave<MODE>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out,
                                                  ws, ws_bytes, st, name);
  const int64_t ntiles = cdiv(n, (int64_t)1024);
  const size_t need = (size_t)(ntiles + 1) * sizeof(unsigned);
  if (!ws || ws_bytes < need) return fail(FLC_EWORKSPACE, "%s: workspace %zu < %zu", name, ws_bytes, need);
  if (!aligned16(out)) return fail(FLC_EINVAL, "%s: out must be 16-B aligned", name);
  unsigned* tile_start = static_cast<unsigned*>(ws);
  const unsigned gi = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(k + 1, kThreads), 2048));
  FLC_LAUNCH("tile_index", tile_index_kernel<10>, dim3(gi), dim3(kThreads), 0, st, idx, (long long)k,
             (long long)ntiles, tile_start);
  const double step = levels > 0 ? 1.0 / (double)levels : 0.0;
  FLC_LAUNCH(name, (sparse_decode_wave2_kernel<MODE, NT>), dim3((unsigned)cdiv(ntiles, NT)), dim3(kWave), 0, st, idx,
             val, codes, scale, levels, step, norm, n, weight, out, tile_start, ntiles, (unsigned)k, 0);
  return FLC_OK;
}

template <int MODE>
int launch_decode(const int32_t* idx, const float* val, const uint8_t* codes, int64_t k, float scale, int levels,
                  const float* norm, int64_t n, float weight, int accumulate, float* out, void* ws, size_t ws_bytes,
                  hipStream_t st, const char* name) {
  return launch_decode_wave2<MODE, 2>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out, ws, ws_bytes,
                                      st, name);
}

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

size_t flc_sparse_decode_workspace_size(int64_t n) { return decode_ws_bytes(n); }

int flc_tile_index(const int32_t* idx, int64_t k, int64_t n, uint32_t* tiles, void* stream) {
  if (!tiles || n <= 0 || k < 0 || (k > 0 && !idx)) return fail(FLC_EINVAL, "flc_tile_index: bad arguments");
  if (n >= (1ll << 31)) return fail(FLC_EINVAL, "flc_tile_index: n must be < 2^31");
  const int64_t ntiles = cdiv(n, (int64_t)FLC_TILE);
  const unsigned gi = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(k + 1, kThreads), 2048));
  static_assert(FLC_TILE == 1024, "tile_index_kernel<10>");
  FLC_LAUNCH("tile_index", tile_index_kernel<10>, dim3(gi), dim3(kThreads), 0, as_stream(stream), idx, (long long)k,
             (long long)ntiles, tiles);
  return FLC_OK;
}

int flc_sparse_decode_tiled(const int32_t* idx, const float* val, int64_t k, float scale, int64_t n, float weight,
                            int accumulate, float* out, const uint32_t* tiles, void* stream) {
  if (!out || !tiles || n <= 0 || k < 0 || (k > 0 && (!idx || !val)))
    return fail(FLC_EINVAL, "flc_sparse_decode_tiled: bad arguments");
  if (n >= (1ll << 31)) return fail(FLC_EINVAL, "flc_sparse_decode_tiled: n must be < 2^31");
  return launch_decode_tiles<0>(idx, val, nullptr, k, scale, 0, nullptr, n, weight, accumulate, out, tiles,
                                as_stream(stream), "sparse_decode");
}

int flc_stacked_decode_tiled(const int32_t* idx, const uint8_t* codes, int64_t k, int levels, const float* norm,
                             int64_t n, float weight, int accumulate, float* out, const uint32_t* tiles, void* stream) {
  if (!out || !norm || !tiles || n <= 0 || k < 0 || (k > 0 && (!idx || !codes)))
    return fail(FLC_EINVAL, "flc_stacked_decode_tiled: bad arguments");
  if (n >= (1ll << 31)) return fail(FLC_EINVAL, "flc_stacked_decode_tiled: n must be < 2^31");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_stacked_decode_tiled: levels must be in [1, 127]");
  return launch_decode_tiles<1>(idx, nullptr, codes, k, 1.0f, levels, norm, n, weight, accumulate, out, tiles,
                                as_stream(stream), "stacked_decode");
}

int flc_sparse_decode(const int32_t* idx, const float* val, int64_t k, float scale, int64_t n, float weight,
                      int accumulate, float* out, void* ws, size_t ws_bytes, void* stream) {
  if (!out || n <= 0 || k < 0 || (k > 0 && (!idx || !val))) return fail(FLC_EINVAL, "flc_sparse_decode: bad arguments");
  if (n >= (1ll << 31)) return fail(FLC_EINVAL, "flc_sparse_decode: n must be < 2^31");
  return launch_decode<0>(idx, val, nullptr, k, scale, 0, nullptr, n, weight, accumulate, out, ws, ws_bytes,
                          as_stream(stream), "sparse_decode");
}

int flc_stacked_decode(const int32_t* idx, const uint8_t* codes, int64_t k, int levels, const float* norm, int64_t n,
                       float weight, int accumulate, float* out, void* ws, size_t ws_bytes, void* stream) {
  if (!out || !norm || n <= 0 || k < 0 || (k > 0 && (!idx || !codes)))
    return fail(FLC_EINVAL, "flc_stacked_decode: bad arguments");
  if (n >= (1ll << 31)) return fail(FLC_EINVAL, "flc_stacked_decode: n must be < 2^31");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_stacked_decode: levels must be in [1, 127]");
  return launch_decode<1>(idx, nullptr, codes, k, 1.0f, levels, norm, n, weight, accumulate, out, ws, ws_bytes,
                          as_stream(stream), "stacked_decode");
}

int flc_copy(const float* x, int64_t n, float* out, void* stream) {
  if (!x || !out || n < 0) return fail(FLC_EINVAL, "flc_copy: bad arguments");
  if (n == 0) return FLC_OK;
  if (!aligned16(x) || !aligned16(out)) return fail(FLC_EINVAL, "flc_copy: 16-B aligned buffers required");
  hipStream_t st = as_stream(stream);
  if (cdiv(n, kCopyChunk) >= (1ll << 31)) return fail(FLC_EINVAL, "flc_copy: n too large");
  FLC_LAUNCH("copy", stream_kernel<false>, dim3((unsigned)cdiv(n, kCopyChunk)), dim3(kThreads), 0, st, x, n, 1.0f, out);
  return FLC_OK;
}

int flc_scale_div(const float* x, int64_t n, float p, float* out, void* stream) {
  if (!x || !out || n < 0) return fail(FLC_EINVAL, "flc_scale_div: bad arguments");
  if (n == 0) return FLC_OK;
  if (!aligned16(x) || !aligned16(out)) return fail(FLC_EINVAL, "flc_scale_div: 16-B aligned buffers required");
  hipStream_t st = as_stream(stream);
  if (cdiv(n, kCopyChunk) >= (1ll << 31)) return fail(FLC_EINVAL, "flc_scale_div: n too large");
  FLC_LAUNCH("scale_div", stream_kernel<true>, dim3((unsigned)cdiv(n, kCopyChunk)), dim3(kThreads), 0, st, x, n, p,
             out);
  return FLC_OK;
}

int flc_randk_keys(int64_t n, uint64_t seed, uint64_t counter, float* keys, void* stream) {
  if (!keys || n <= 0 || n >= (int64_t(1) << 31)) return fail(FLC_EINVAL, "flc_randk_keys: bad arguments");
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(cdiv(n, 4), kThreads), 256 * 16);
  FLC_LAUNCH("randk_keys", randk_keys_kernel, dim3(grid), dim3(kThreads), 0, st, n, seed, counter, keys);
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

