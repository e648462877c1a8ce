// sparse.hip — dense decoders of the sparse wires and the elementwise compressors, for gfx950
// (reference: fl_sim/compressors/compressors.py:273-296).
//
//   tile_index      tile_start[t] = first kept entry of output tile t (one thread per kept entry).
//   sparse_decode   dense output, one block per 1024-output tile: the tile is zero-filled in LDS, its
//                   slice of the ascending index stream scattered into it, and it is streamed out with
//                   one 16-B store per thread (the store shape that reaches ~7 TB/s on MI355X, see
//                   tools/bwprobe.hip).
//                   Algorithmic bytes: 4 per output element + 8 (top-k: idx+val) or 5 (stacked:
//                   idx+code) per kept entry.  Optionally fused with the aggregation: out = fmaf(w, v, out).
//   randk_scatter   out[idx[j]] = fp32(D/K) * x[idx[j]] after a zero fill (compressors.py:289-291).
//   elementwise     identical (+x) and lazy (x / p) (compressors.py:273-283).
#include <hip/hip_runtime.h>
#include <math.h>

#include <stdlib.h>

#include <algorithm>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kThreads = 256;
constexpr int kDecodeVariant = 302;  // see launch_decode: 302 = one wave per two 1024-output tiles

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

// one block per output tile of TILE = 256 * V floats: zero the tile in LDS, scatter the tile's kept
// entries (tile_start[t] .. tile_start[t+1]), stream it out with V 16-B stores per thread.
//   MODE 0: v = scale * val[j];  MODE 1: v = dithering decode of codes[j] (s = levels, norm)
// XCD-aware tile order: the dispatcher deals consecutive blocks round-robin to the 8 XCDs; remapping
// block b to tile (b % 8) * (T / 8) + b / 8 makes each XCD write one contiguous eighth of the output
// (1 GiB of zero-dominated stores: 162 vs 175 us at 4096-output tiles, tools/bwprobe4.hip)
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t nb) {
  const int64_t per = nb >> 3;
  return b < (per << 3) ? (b & 7) * per + (b >> 3) : b;
}

template <int MODE, bool ACC, int V, bool EARLY, bool XCD>
__global__ __launch_bounds__(kThreads) void sparse_decode_kernel(const int* __restrict__ idx, const float* __restrict__ val,
                                                                 const uint8_t* __restrict__ codes, float scale,
                                                                 int levels, double step, const float* __restrict__ norm_ptr,
                                                                 int64_t n, float weight, float* __restrict__ out,
                                                                 const unsigned* __restrict__ tile_start) {
  constexpr int TILE = kThreads * 4 * V;
  __shared__ __attribute__((aligned(16))) float s_tile[TILE];
  const int64_t tile = XCD ? xcd_tile(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  const int64_t t0 = tile * TILE;
  const bool full = t0 + TILE <= n;
  // EARLY: the zero stores of a full, non-accumulating tile leave before any load returns; the few
  // float4s that hold kept entries are stored again below (same thread, program order)
  if (EARLY && !ACC && full) {
#pragma unroll
    for (int u = 0; u < V; ++u)
      *reinterpret_cast<float4*>(out + t0 + 4 * (int64_t)(threadIdx.x + u * kThreads)) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const unsigned lo = tile_start[tile], hi = tile_start[tile + 1];
  float4* tile4 = reinterpret_cast<float4*>(s_tile);
#pragma unroll
  for (int u = 0; u < V; ++u) tile4[threadIdx.x + u * kThreads] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  float nrm = 0.f;
  if (MODE == 1) nrm = *norm_ptr;
  for (unsigned j = lo + threadIdx.x; j < hi; j += kThreads) {
    float v;
    if (MODE == 0) {
      v = scale * val[j];
    } else {
      const uint32_t code = codes[j];
      if (!(nrm > 0.0f && nrm <= 3.402823466e38f)) {
        v = code == 0u ? 0.0f : __uint_as_float(0x7fc00000u);
      } else {
        const float lv = (float)level_value<0>((int)(code & 127u), levels, step);
        v = ((code >> 7) ? -lv : lv) * nrm;  // compressors.py:357
      }
    }
    const unsigned long long off = (unsigned long long)((long long)(unsigned)idx[j] - (long long)t0);
    if (off < (unsigned long long)TILE) s_tile[off] = v;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const int q = threadIdx.x + u * kThreads;
    const int64_t e = t0 + 4 * (int64_t)q;
    float4 v = tile4[q];
    if (e + 4 <= n) {
      if (ACC) {
        const float4 p = *reinterpret_cast<const float4*>(out + e);
        v = make_float4(fmaf(weight, v.x, p.x), fmaf(weight, v.y, p.y), fmaf(weight, v.z, p.z), fmaf(weight, v.w, p.w));
      } else if (weight != 1.0f) {
        v = make_float4(weight * v.x, weight * v.y, weight * v.z, weight * v.w);
      }
      const bool nz = __float_as_uint(v.x) | __float_as_uint(v.y) | __float_as_uint(v.z) | __float_as_uint(v.w);
      if (!(EARLY && !ACC && full) || nz) *reinterpret_cast<float4*>(out + e) = v;
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

// Streaming decode: persistent blocks, block b owns the contiguous tiles [b * tpb, (b + 1) * tpb) of
// kStreamTile outputs.  While tile t is assembled in LDS and stored, the first kept entry per thread of
// tile t + 1 (and, accumulating, its slice of `out`) is already in flight, so no store waits on a
// dependent load chain.  Tiles with more than 256 kept entries take the rest straight from memory.
constexpr int kStreamTile = kThreads * 16;  // 4096 outputs, 4 float4 per thread
constexpr int kMaxTilesPerBlock = 512;

template <int MODE, bool ACC>
__global__ __launch_bounds__(kThreads) void sparse_decode_stream_kernel(
    const int* __restrict__ idx, const float* __restrict__ val, const uint8_t* __restrict__ codes, float scale,
    int levels, double step, const float* __restrict__ norm_ptr, int64_t n, float weight, float* __restrict__ out,
    const unsigned* __restrict__ tile_start, int64_t ntiles, int tpb) {
  __shared__ __attribute__((aligned(16))) float s_tile[kStreamTile];
  __shared__ unsigned s_ts[kMaxTilesPerBlock + 1];
  const int tid = threadIdx.x;
  const int64_t tb = (int64_t)blockIdx.x * tpb;
  const int64_t te = tb + tpb < ntiles ? tb + tpb : ntiles;
  if (tb >= te) return;
  const int nt = (int)(te - tb);
  for (int i = tid; i <= nt; i += kThreads) s_ts[i] = tile_start[tb + i];
  float4* tile4 = reinterpret_cast<float4*>(s_tile);
#pragma unroll
  for (int u = 0; u < 4; ++u) tile4[tid + u * kThreads] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float nrm = MODE == 1 ? *norm_ptr : 0.0f;
  __syncthreads();
  // prefetch of tile tb: raw words only, consumed one tile later (no use before the next barrier)
  unsigned p_idx = 0xffffffffu;
  uint32_t p_raw = 0u;
  {
    const unsigned j = s_ts[0] + tid;
    if (j < s_ts[1]) {
      p_idx = (unsigned)idx[j];
      p_raw = entry_raw<MODE>(val, codes, j);
    }
  }
  float4 p_acc[4];
  if (ACC) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = tb * kStreamTile + 4 * (int64_t)(tid + u * kThreads);
      p_acc[u] = e + 4 <= n ? *reinterpret_cast<const float4*>(out + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  for (int i = 0; i < nt; ++i) {
    const int64_t t0 = (tb + i) * kStreamTile;
    const unsigned lo = s_ts[i], hi = s_ts[i + 1];
    // issue the next tile's loads first
    unsigned n_idx = 0xffffffffu;
    uint32_t n_raw = 0u;
    float4 n_acc[4];
    if (i + 1 < nt) {
      const unsigned j = hi + tid;
      if (j < s_ts[i + 2]) {
        n_idx = (unsigned)idx[j];
        n_raw = entry_raw<MODE>(val, codes, j);
      }
      if (ACC) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t e = t0 + kStreamTile + 4 * (int64_t)(tid + u * kThreads);
          n_acc[u] = e + 4 <= n ? *reinterpret_cast<const float4*>(out + e) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
    // scatter this tile's entries
    if (p_idx != 0xffffffffu) {
      const int64_t off = (int64_t)p_idx - t0;
      if (off >= 0 && off < kStreamTile) s_tile[off] = entry_value<MODE>(p_raw, scale, levels, step, nrm);
    }
    for (unsigned j = lo + kThreads + tid; j < hi; j += kThreads) {
      const int64_t off = (int64_t)(unsigned)idx[j] - t0;
      if (off >= 0 && off < kStreamTile)
        s_tile[off] = entry_value<MODE>(entry_raw<MODE>(val, codes, j), scale, levels, step, nrm);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + u * kThreads;
      const int64_t e = t0 + 4 * (int64_t)q;
      float4 v = tile4[q];
      tile4[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e + 4 <= n) {
        if (ACC) {
          const float4 pa = p_acc[u];
          v = make_float4(fmaf(weight, v.x, pa.x), fmaf(weight, v.y, pa.y), fmaf(weight, v.z, pa.z),
                          fmaf(weight, v.w, pa.w));
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
    __syncthreads();
    p_idx = n_idx;
    p_raw = n_raw;
    if (ACC) {
#pragma unroll
      for (int u = 0; u < 4; ++u) p_acc[u] = n_acc[u];
    }
  }
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
                                                                   const unsigned* __restrict__ tile_start, int dbg) {
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
  if (dbg == 3) {  // calibration: the store stream alone
#pragma unroll
    for (int u = 0; u < 4; ++u)
      *reinterpret_cast<float4*>(out + t0 + 4 * (int64_t)(lane + u * kWave)) = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  unsigned lo = 0, hi = 0;
  if (dbg != 1) { lo = tile_start[blockIdx.x]; hi = tile_start[blockIdx.x + 1]; }
  if (dbg == 2) hi = lo;
  float4* tile4 = reinterpret_cast<float4*>(s_tile);
#pragma unroll
  for (int u = 0; u < 4; ++u) tile4[lane + u * kWave] = make_float4(0.f, 0.f, 0.f, 0.f);
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
                                                                    int64_t ntiles, int64_t chunk) {
  constexpr int TILE = 1024;
  __shared__ __attribute__((aligned(16))) float s_tile[NT * TILE];
  const int lane = threadIdx.x;
  // XCD-chunked order: the dispatcher deals workgroups round-robin to the 8 XCDs; within every run of
  // 8 chunks, XCD x takes chunk x, so each XCD writes whole contiguous chunks (chunk = 0: plain order)
  int64_t g = blockIdx.x;
  if (chunk > 0) {
    const int64_t sup = 8 * chunk, full = (int64_t)gridDim.x / sup * sup;
    if (g < full) {
      const int64_t x = g & 7, j = g >> 3;
      g = (j / chunk) * sup + x * chunk + (j % chunk);
    }
  }
  const int64_t tb = g * NT;
  const int64_t t0 = tb * TILE;
  unsigned ts[NT + 1];
#pragma unroll
  for (int i = 0; i <= NT; ++i) ts[i] = tile_start[tb + i < ntiles ? tb + i : ntiles];
  float4* tile4 = reinterpret_cast<float4*>(s_tile);
#pragma unroll
  for (int u = 0; u < 4 * NT; ++u) tile4[lane + u * kWave] = make_float4(0.f, 0.f, 0.f, 0.f);
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
      *reinterpret_cast<float4*>(out + e) = v;
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int c = 0; c < 4 && e + c < n; ++c) out[e + c] = weight != 1.0f ? weight * vv[c] : vv[c];
    }
  }
}

// Grid-stride pipelined decode: G resident blocks, block b assembles tiles b, b + G, b + 2G, ... of
// TILE = 1024 V outputs.  The whole grid's stores of one iteration cover ONE contiguous window (the write
// order HBM3E takes at full rate, tools/bwprobe4.hip), and each block's dependent load chain
// (tile_start -> kept entries) runs ahead of its stores: tile i + 2's range and tile i + 1's entries
// (and, accumulating, its slice of `out`) are in flight while tile i is scattered and stored.  Two LDS
// tiles alternate, so one barrier per tile suffices; the barrier is LDS-only (lds_barrier), so the
// prefetches stay in flight across it.  Tiles with more than 256 kept entries take the rest straight
// from memory.  The loop is unrolled by two with explicit A/B register sets: no loop-carried copies
// of loaded registers, which would make the compiler wait for the prefetch it just issued.
template <int V>
struct GsRegs {
  unsigned e_idx;
  uint32_t e_raw;
  float4 acc[V];
};

template <int MODE, bool ACC, int V>
__device__ __forceinline__ void gs_tile(const int* __restrict__ idx, const float* __restrict__ val,
                                        const uint8_t* __restrict__ codes, float scale, int levels, double step,
                                        float nrm, int64_t n, float weight, float* __restrict__ out,
                                        const unsigned* __restrict__ tile_start, int64_t ntiles, int64_t t, int64_t G,
                                        float* tl, unsigned& lo0, unsigned& hi0, unsigned& lo1, unsigned& hi1,
                                        const GsRegs<V>& cur, GsRegs<V>& nxt) {
  constexpr int TILE = kThreads * 4 * V;
  const int tid = threadIdx.x;
  const int64_t t0 = t * TILE;
  nxt.e_idx = 0xffffffffu;
  nxt.e_raw = 0u;
  if (lo1 + tid < hi1) {
    nxt.e_idx = (unsigned)idx[lo1 + tid];
    nxt.e_raw = entry_raw<MODE>(val, codes, lo1 + tid);
  }
  unsigned lo2 = 0, hi2 = 0;
  if (t + 2 * G < ntiles) {
    lo2 = tile_start[t + 2 * G];
    hi2 = tile_start[t + 2 * G + 1];
  }
  if (ACC) {
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int64_t e = (t + G) * TILE + 4 * (int64_t)(tid + u * kThreads);
      nxt.acc[u] = (t + G < ntiles && e + 4 <= n) ? *reinterpret_cast<const float4*>(out + e)
                                                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  if (cur.e_idx != 0xffffffffu) {
    const int64_t off = (int64_t)cur.e_idx - t0;
    if (off >= 0 && off < TILE) tl[off] = entry_value<MODE>(cur.e_raw, scale, levels, step, nrm);
  }
  for (unsigned j = lo0 + kThreads + tid; j < hi0; j += kThreads) {
    const int64_t off = (int64_t)(unsigned)idx[j] - t0;
    if (off >= 0 && off < TILE) tl[off] = entry_value<MODE>(entry_raw<MODE>(val, codes, j), scale, levels, step, nrm);
  }
  lds_barrier();
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const int q = tid + u * kThreads;
    const int64_t e = t0 + 4 * (int64_t)q;
    float4 v = reinterpret_cast<float4*>(tl)[q];
    reinterpret_cast<float4*>(tl)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e + 4 <= n) {
      if (ACC) {
        v = make_float4(fmaf(weight, v.x, cur.acc[u].x), fmaf(weight, v.y, cur.acc[u].y),
                        fmaf(weight, v.z, cur.acc[u].z), fmaf(weight, v.w, cur.acc[u].w));
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
  lo0 = lo1;
  hi0 = hi1;
  lo1 = lo2;
  hi1 = hi2;
}

template <int MODE, bool ACC, int V>
__global__ __launch_bounds__(kThreads) void sparse_decode_gs_kernel(
    const int* __restrict__ idx, const float* __restrict__ val, const uint8_t* __restrict__ codes, float scale,
    int levels, double step, const float* __restrict__ norm_ptr, int64_t n, float weight, float* __restrict__ out,
    const unsigned* __restrict__ tile_start, int64_t ntiles) {
  constexpr int TILE = kThreads * 4 * V;
  __shared__ __attribute__((aligned(16))) float s_tile[2][TILE];
  const int tid = threadIdx.x;
  const int64_t G = gridDim.x;
  const float nrm = MODE == 1 ? *norm_ptr : 0.0f;
#pragma unroll
  for (int u = 0; u < V; ++u) {
    reinterpret_cast<float4*>(s_tile[0])[tid + u * kThreads] = make_float4(0.f, 0.f, 0.f, 0.f);
    reinterpret_cast<float4*>(s_tile[1])[tid + u * kThreads] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  int64_t t = blockIdx.x;
  unsigned lo0 = 0, hi0 = 0, lo1 = 0, hi1 = 0;
  if (t < ntiles) { lo0 = tile_start[t]; hi0 = tile_start[t + 1]; }
  if (t + G < ntiles) { lo1 = tile_start[t + G]; hi1 = tile_start[t + G + 1]; }
  GsRegs<V> A, B;
  A.e_idx = 0xffffffffu;
  A.e_raw = 0u;
  if (lo0 + tid < hi0) { A.e_idx = (unsigned)idx[lo0 + tid]; A.e_raw = entry_raw<MODE>(val, codes, lo0 + tid); }
  if (ACC) {
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int64_t e = t * TILE + 4 * (int64_t)(tid + u * kThreads);
      A.acc[u] = (t < ntiles && e + 4 <= n) ? *reinterpret_cast<const float4*>(out + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();
  while (t < ntiles) {
    gs_tile<MODE, ACC, V>(idx, val, codes, scale, levels, step, nrm, n, weight, out, tile_start, ntiles, t, G, s_tile[0],
                          lo0, hi0, lo1, hi1, A, B);
    t += G;
    if (t >= ntiles) break;
    gs_tile<MODE, ACC, V>(idx, val, codes, scale, levels, step, nrm, n, weight, out, tile_start, ntiles, t, G, s_tile[1],
                          lo0, hi0, lo1, hi1, B, A);
    t += G;
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

size_t decode_ws_bytes(int64_t n) {  // tile index for the smallest tile (1024 outputs)
  return (size_t)(cdiv(n < 1 ? 1 : n, (int64_t)kThreads * 4) + 1) * sizeof(unsigned);
}

template <int MODE, int V, bool EARLY, bool XCD>
int launch_decode_v(const int32_t* idx, const float* val, const uint8_t* codes, int64_t k, float scale, int levels,
                    const float* norm, int64_t n, float weight, int accumulate, float* out, void* ws, size_t ws_bytes,
                    hipStream_t st, const char* name) {
  constexpr int TILE = kThreads * 4 * V;
  constexpr int TILE_LOG = V == 1 ? 10 : (V == 2 ? 11 : (V == 4 ? 12 : 13));
  const int64_t ntiles = cdiv(n, TILE);
  const size_t need = (size_t)(ntiles + 1) * sizeof(unsigned);
  if (!ws || ws_bytes < need) return fail(FLC_EWORKSPACE, "%s: workspace %zu < %zu", name, ws_bytes, need);
  if (!aligned16(out)) return fail(FLC_EINVAL, "%s: out must be 16-B aligned", name);
  unsigned* tile_start = static_cast<unsigned*>(ws);
  const unsigned gi = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(k + 1, kThreads), 2048));
  FLC_LAUNCH("tile_index", tile_index_kernel<TILE_LOG>, dim3(gi), dim3(kThreads), 0, st, idx, (long long)k,
             (long long)ntiles, tile_start);
  const double step = levels > 0 ? 1.0 / (double)levels : 0.0;
  if (accumulate)
    FLC_LAUNCH(name, (sparse_decode_kernel<MODE, true, V, EARLY, XCD>), dim3((unsigned)ntiles), dim3(kThreads), 0, st, idx,
               val, codes, scale, levels, step, norm, n, weight, out, tile_start);
  else
    FLC_LAUNCH(name, (sparse_decode_kernel<MODE, false, V, EARLY, XCD>), dim3((unsigned)ntiles), dim3(kThreads), 0, st, idx,
               val, codes, scale, levels, step, norm, n, weight, out, tile_start);
  return FLC_OK;
}

int64_t decode_stream_blocks() {  // persistent grid: FLC_DECODE_BLOCKS or 8 blocks per CU
  const char* e = getenv("FLC_DECODE_BLOCKS");
  if (e && atoi(e) > 0) return atoi(e);
  int dev = 0, cu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || cu <= 0)
    cu = 256;
  return (int64_t)cu * 8;
}

template <int MODE>
int launch_decode_stream(const int32_t* idx, const float* val, const uint8_t* codes, int64_t k, float scale,
                         int levels, const float* norm, int64_t n, float weight, int accumulate, float* out, void* ws,
                         size_t ws_bytes, hipStream_t st, const char* name) {
  constexpr int TILE_LOG = 12;
  static_assert((1 << TILE_LOG) == kStreamTile, "tile index granularity");
  const int64_t ntiles = cdiv(n, kStreamTile);
  const size_t need = (size_t)(ntiles + 1) * sizeof(unsigned);
  if (!ws || ws_bytes < need) return fail(FLC_EWORKSPACE, "%s: workspace %zu < %zu", name, ws_bytes, need);
  if (!aligned16(out)) return fail(FLC_EINVAL, "%s: out must be 16-B aligned", name);
  unsigned* tile_start = static_cast<unsigned*>(ws);
  const unsigned gi = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(k + 1, kThreads), 2048));
  FLC_LAUNCH("tile_index", tile_index_kernel<TILE_LOG>, dim3(gi), dim3(kThreads), 0, st, idx, (long long)k,
             (long long)ntiles, tile_start);
  int64_t grid = std::min<int64_t>(ntiles, decode_stream_blocks());
  int64_t tpb = cdiv(ntiles, grid);
  if (tpb > kMaxTilesPerBlock) tpb = kMaxTilesPerBlock;
  grid = cdiv(ntiles, tpb);
  const double step = levels > 0 ? 1.0 / (double)levels : 0.0;
  if (accumulate)
    FLC_LAUNCH(name, (sparse_decode_stream_kernel<MODE, true>), dim3((unsigned)grid), dim3(kThreads), 0, st, idx, val,
               codes, scale, levels, step, norm, n, weight, out, tile_start, ntiles, (int)tpb);
  else
    FLC_LAUNCH(name, (sparse_decode_stream_kernel<MODE, false>), dim3((unsigned)grid), dim3(kThreads), 0, st, idx,
               val, codes, scale, levels, step, norm, n, weight, out, tile_start, ntiles, (int)tpb);
  return FLC_OK;
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
  const int dbg = getenv("FLC_DECODE_DBG") ? atoi(getenv("FLC_DECODE_DBG")) : 0;
  if (accumulate)
    FLC_LAUNCH(name, (sparse_decode_wave_kernel<MODE, true>), dim3((unsigned)ntiles), dim3(kWave), 0, st, idx, val,
               codes, scale, levels, step, norm, n, weight, out, tile_start, dbg);
  else
    FLC_LAUNCH(name, (sparse_decode_wave_kernel<MODE, false>), dim3((unsigned)ntiles), dim3(kWave), 0, st, idx, val,
               codes, scale, levels, step, norm, n, weight, out, tile_start, dbg);
  return FLC_OK;
}

int64_t decode_chunk() {  // calibration knob FLC_DECODE_CHUNK (workgroups per XCD chunk; 0: plain order)
  const char* e = getenv("FLC_DECODE_CHUNK");
  return e ? atoll(e) : 0;
}

// decode over given 1024-output tile pointers (no tile_index pass): one wave per two tiles, or, when
// accumulating, one wave per tile (its slice of `out` read first)
template <int MODE>
int launch_decode_tiles(const int32_t* idx, const float* val, const uint8_t* codes, float scale, int levels,
                        const float* norm, int64_t n, float weight, int accumulate, float* out,
                        const unsigned* tile_start, hipStream_t st, const char* name) {
  if (!aligned16(out)) return fail(FLC_EINVAL, "%s: out must be 16-B aligned", name);
  const int64_t ntiles = cdiv(n, (int64_t)FLC_TILE);
  const double step = levels > 0 ? 1.0 / (double)levels : 0.0;
  if (accumulate)
    FLC_LAUNCH(name, (sparse_decode_wave_kernel<MODE, true>), dim3((unsigned)ntiles), dim3(kWave), 0, st, idx, val,
               codes, scale, levels, step, norm, n, weight, out, tile_start, 0);
  else
    FLC_LAUNCH(name, (sparse_decode_wave2_kernel<MODE, 2>), dim3((unsigned)cdiv(ntiles, 2)), dim3(kWave), 0, st, idx,
               val, codes, scale, levels, step, norm, n, weight, out, tile_start, ntiles, decode_chunk());
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
             val, codes, scale, levels, step, norm, n, weight, out, tile_start, ntiles, decode_chunk());
  return FLC_OK;
}

int64_t decode_gs_blocks() {  // resident grid: FLC_DECODE_BLOCKS or 8 blocks of 256 threads per CU
  const char* e = getenv("FLC_DECODE_BLOCKS");
  if (e && atoi(e) > 0) return atoi(e);
  int dev = 0, cu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || cu <= 0)
    cu = 256;
  return (int64_t)cu * 8;
}

template <int MODE, int V>
int launch_decode_gs(const int32_t* idx, const float* val, const uint8_t* codes, int64_t k, float scale, int levels,
                     const float* norm, int64_t n, float weight, int accumulate, float* out, void* ws, size_t ws_bytes,
                     hipStream_t st, const char* name) {
  constexpr int TILE = kThreads * 4 * V;
  constexpr int TILE_LOG = V == 1 ? 10 : (V == 2 ? 11 : 12);
  static_assert((1 << TILE_LOG) == TILE, "tile index granularity");
  const int64_t ntiles = cdiv(n, TILE);
  const size_t need = (size_t)(ntiles + 1) * sizeof(unsigned);
  if (!ws || ws_bytes < need) return fail(FLC_EWORKSPACE, "%s: workspace %zu < %zu", name, ws_bytes, need);
  if (!aligned16(out)) return fail(FLC_EINVAL, "%s: out must be 16-B aligned", name);
  unsigned* tile_start = static_cast<unsigned*>(ws);
  const unsigned gi = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(k + 1, kThreads), 2048));
  FLC_LAUNCH("tile_index", tile_index_kernel<TILE_LOG>, dim3(gi), dim3(kThreads), 0, st, idx, (long long)k,
             (long long)ntiles, tile_start);
  const int64_t grid = std::min<int64_t>(ntiles, decode_gs_blocks());
  const double step = levels > 0 ? 1.0 / (double)levels : 0.0;
  if (accumulate)
    FLC_LAUNCH(name, (sparse_decode_gs_kernel<MODE, true, V>), dim3((unsigned)grid), dim3(kThreads), 0, st, idx, val,
               codes, scale, levels, step, norm, n, weight, out, tile_start, ntiles);
  else
    FLC_LAUNCH(name, (sparse_decode_gs_kernel<MODE, false, V>), dim3((unsigned)grid), dim3(kThreads), 0, st, idx, val,
               codes, scale, levels, step, norm, n, weight, out, tile_start, ntiles);
  return FLC_OK;
}

int decode_variant() {
  const char* e = getenv("FLC_DECODE_VARIANT");
  return e ? atoi(e) : kDecodeVariant;
}

template <int MODE>
int launch_decode(const int32_t* idx, const float* val, const uint8_t* codes, int64_t k, float scale, int levels,
                  const float* norm, int64_t n, float weight, int accumulate, float* out, void* ws, size_t ws_bytes,
                  hipStream_t st, const char* name) {
#define FLC_DV(V, E, X) return launch_decode_v<MODE, V, E, X>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out, ws, ws_bytes, st, name)
  const int dv = decode_variant();
  if (dv == 90) return launch_decode_stream<MODE>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out,
                                                  ws, ws_bytes, st, name);
  switch (dv) {
    case 301: return launch_decode_wave2<MODE, 1>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out, ws, ws_bytes, st, name);
    case 302: return launch_decode_wave2<MODE, 2>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out, ws, ws_bytes, st, name);
    case 304: return launch_decode_wave2<MODE, 4>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out, ws, ws_bytes, st, name);
    case 300: return launch_decode_wave<MODE>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out, ws, ws_bytes, st, name);
    case 201: return launch_decode_gs<MODE, 1>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out, ws, ws_bytes, st, name);
    case 202: return launch_decode_gs<MODE, 2>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out, ws, ws_bytes, st, name);
    case 204: return launch_decode_gs<MODE, 4>(idx, val, codes, k, scale, levels, norm, n, weight, accumulate, out, ws, ws_bytes, st, name);
    case 10: FLC_DV(1, false, false);
    case 11: FLC_DV(1, true, false);
    case 20: FLC_DV(2, false, false);
    case 40: FLC_DV(4, false, false);
    case 41: FLC_DV(4, true, false);
    case 80: FLC_DV(8, false, false);
    case 110: FLC_DV(1, false, true);
    case 111: FLC_DV(1, true, true);
    case 120: FLC_DV(2, false, true);
    case 140: FLC_DV(4, false, true);
    case 141: FLC_DV(4, true, true);
    default: FLC_DV(8, true, false);
  }
#undef FLC_DV
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
  return launch_decode_tiles<0>(idx, val, nullptr, scale, 0, nullptr, n, weight, accumulate, out, tiles,
                                as_stream(stream), "sparse_decode");
}

int flc_stacked_decode_tiled(const int32_t* idx, const uint8_t* codes, int64_t k, int levels, const float* norm,
                             int64_t n, float weight, int accumulate, float* out, const uint32_t* tiles, void* stream) {
  if (!out || !norm || !tiles || n <= 0 || k < 0 || (k > 0 && (!idx || !codes)))
    return fail(FLC_EINVAL, "flc_stacked_decode_tiled: bad arguments");
  if (n >= (1ll << 31)) return fail(FLC_EINVAL, "flc_stacked_decode_tiled: n must be < 2^31");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_stacked_decode_tiled: levels must be in [1, 127]");
  return launch_decode_tiles<1>(idx, nullptr, codes, 1.0f, levels, norm, n, weight, accumulate, out, tiles,
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

