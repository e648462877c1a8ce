// topk.hip — exact top-k selection and the stacked top-k -> 8-bit dithering encoder, for gfx950
// (reference: fl_sim/compressors/compressors.py:293-296 and 327-365).
//
// Selection contract (compressors.py:294-295, `out[np.argsort(out)[:-K]] = 0`): keep the k largest
// *signed* values; -0 == +0; NaN is largest; among elements equal to the k-th largest value the
// highest indices are kept (stable ascending argsort order; the reference's own argsort is unstable,
// so any tie choice satisfies it — see DESIGN.md).
//
// Pipeline: ONE streaming read of x; every later pass touches only the ~1.2 k candidates.
//   sample_gather  128 blocks: 32 K strided keys of x (order-preserving uint32 keys).
//   sample_select  1 block, keys in registers: radix select with range-adaptive digits over
//                  [min, max] of the sample -> candidate floor t_lo with count(key >= t_lo) ~ k + 4 sigma
//                  (k/n = 1 %: ~1.22 k candidates).
//   filter         the HBM pass: each wave owns a contiguous run of x and appends its candidates in
//                  index order to a private staging region (ballot/popcount compaction: no atomics,
//                  no inter-wave sync).  Algorithmic bytes 4 per element.
//   round x3       radix select over the candidates, 2048 bins per round over the live key range
//                  (round 1: [t_lo, max key] -> 3 rounds always resolve the exact threshold).  Round 1
//                  also scans the region counts in LDS (every block; no separate scan launch) and
//                  gathers the staged regions into one ordered SoA candidate array.  C < k switches
//                  every later kernel to "fallback" mode, in which they read x itself (always correct).
//                  LDS histograms with wave-aggregated atomics (a wave of equal keys = one atomic),
//                  global atomics, the XCD-sharded last arriving block picks the digit.
//   count          per-block strict / tie counts of the threshold; the last arriver scans them.
//   compact        ordered compaction of the kept set into idx[k] / val[k] or, stacked, idx[k] /
//                  codes[k] with the dithering fused in (the norm of the kept set is
//                  max(|max key|, |k-th key|), known before compaction).
// Cross-block hand-offs inside a launch go only through memory-side atomics (histogram adds, arrival
// tickets, RMW reads by the last arriver) and write-through (sc1) stores, so no L2 write-back fence
// is needed; everything else crosses a kernel boundary.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kSample = 32768;
constexpr int kSelectThreads = 1024;
constexpr int kSamplePerThread = kSample / kSelectThreads;  // 32
constexpr int kThreads = 256;
constexpr int kNW = kThreads / kWave;
constexpr int kStep = 1024;         // elements per wave step in the filter (4 x float4 per lane)
constexpr int kSelBlocks = 1024;    // grid of the round / count / compact kernels (multiple of 8)
constexpr int kHistBits = 11;
constexpr int kHistBins = 1 << kHistBits;
constexpr int kShards = 8;          // XCD shards of the arrival counters
constexpr int kMaxRegions = 8192;
constexpr int kRegionsPerThread = kMaxRegions / kThreads;  // 32 (round-1 LDS scan)

struct TopkParams {
  unsigned t_lo;       // candidate floor (sample)
  unsigned fallback;   // 1: candidates = all of x
  long long C;         // candidates
  unsigned maxkey;
  unsigned lo;         // select: low end of the live key range
  int shift;           // select: log2 keys per bin of the next round
  int done;            // select: threshold resolved
  unsigned long long width;  // select: keys in the live range [lo, lo + width)
  long long rem;       // select: rank still to find (from the top) inside the live range
  unsigned T;          // the k-th largest key
  unsigned err;
  long long need;      // elements equal to T that are kept
  long long ties_total;
  long long strict_total;
  long long k;
};

struct TopkWs {
  TopkParams* p;
  unsigned* tickets;            // [4][kShards + 1]: rounds 0..2, count
  unsigned* hist;               // [3][kHistBins]
  unsigned* sample;             // [kSample]
  unsigned* region_cnt;         // [R]
  unsigned* region_max;         // [R]
  unsigned long long* blk_cnt;  // [kSelBlocks]  strict << 32 | tie
  unsigned long long* blk_off;  // [kSelBlocks]
  unsigned* cand_idx;           // [n]  ordered by index
  unsigned* cand_raw;           // [n]  raw fp32 bits
  uint2* stage;                 // [R * region_cap]  (idx, raw) per wave region
  long long region_cap;
};

struct TopkGeom {
  int64_t blocks;      // filter blocks
  int64_t wave_chunk;  // elements per wave region (multiple of kStep)
  int64_t regions;     // blocks * 4  (<= kMaxRegions)
};

TopkGeom geometry(int64_t n) {
  TopkGeom g;
  int64_t blocks = cdiv(n, 4 * kStep * 8);  // >= 8 steps per wave
  if (blocks > kMaxRegions / 4) blocks = kMaxRegions / 4;
  if (blocks < 1) blocks = 1;
  g.wave_chunk = (int64_t)align_up((size_t)cdiv(n, blocks * 4), kStep);
  g.regions = cdiv(n, g.wave_chunk);
  g.blocks = cdiv(g.regions, 4);
  g.regions = g.blocks * 4;
  return g;
}

TopkWs carve_topk(void* ws, size_t bytes, int64_t n, size_t* need) {
  const TopkGeom g = geometry(n);
  Carver c(ws, bytes);
  TopkWs w;
  w.p = c.take<TopkParams>(1);
  w.tickets = c.take<unsigned>(4 * (kShards + 1));
  w.hist = c.take<unsigned>(3 * kHistBins);
  w.sample = c.take<unsigned>(kSample);
  w.region_cnt = c.take<unsigned>(g.regions);
  w.region_max = c.take<unsigned>(g.regions);
  w.blk_cnt = c.take<unsigned long long>(kSelBlocks);
  w.blk_off = c.take<unsigned long long>(kSelBlocks);
  w.cand_idx = c.take<unsigned>((size_t)n + 4);
  w.cand_raw = c.take<unsigned>((size_t)n + 4);
  w.region_cap = g.wave_chunk;
  w.stage = c.take<uint2>((size_t)g.regions * g.wave_chunk);
  *need = c.off;
  return w;
}

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------

// One wave: histogram h[NB] (LDS) and a rank `rem` (1-based, from the top) -> the bin holding that
// rank and the rank inside it.  The lane that finds it writes *digit / *new_rem.
template <int NB>
__device__ void wave_select_from_top(const unsigned* h, long long rem, unsigned* digit, long long* new_rem,
                                     unsigned* err) {
  constexpr int B = NB / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  long long ls = 0;
#pragma unroll
  for (int i = 0; i < B; ++i) ls += h[lane * B + i];
  const long long incl = wave_incl_scan(ls);
  const long long total = __shfl(incl, kWave - 1, kWave);
  const long long above = total - incl;  // bins of higher lanes
  const bool hit = above < rem && rem <= above + ls;
  const unsigned long long m = __ballot(hit);
  if (m == 0) {
    if (lane == 0) {
      *digit = 0;
      *new_rem = 1;
      *err |= 1u;
    }
    return;
  }
  if (lane == __ffsll((long long)m) - 1) {
    long long cum = above;
    for (int i = B - 1; i >= 0; --i) {
      const long long c = h[lane * B + i];
      if (cum + c >= rem) {
        *digit = (unsigned)(lane * B + i);
        *new_rem = rem - cum;
        break;
      }
      cum += c;
    }
  }
}

// LDS histogram add with wave aggregation: when every active lane hits the same bin (ties, narrow
// key ranges) the wave issues ONE atomic instead of a 64-way conflicting one.
__device__ __forceinline__ void hist_add(unsigned* h, unsigned bin, bool valid) {
  const unsigned long long act = __ballot(valid);
  if (act == 0ull) return;
  const int first = __ffsll((long long)act) - 1;
  const unsigned b0 = __shfl(bin, first, kWave);
  const unsigned long long same = __ballot(valid && bin == b0);
  if (same == act) {
    if ((int)(threadIdx.x & (kWave - 1)) == first) atomicAdd(&h[b0], (unsigned)__popcll(act));
  } else if (valid) {
    atomicAdd(&h[bin], 1u);
  }
}

// shift so that a key range of `width` keys maps onto at most 2^bits bins
__device__ __forceinline__ int range_shift(unsigned long long width, int bits) {
  if (width <= 1ull) return 0;
  const int len = 64 - __clzll((long long)(width - 1ull));
  return len > bits ? len - bits : 0;
}

// XCD-sharded last-arriver: true in exactly one block, after every block called it.  Call from all
// threads (contains __syncthreads()).  Every wave must have drained its atomics / sc1 stores
// (drain_stores) before; the winner reads the payload with memory-side RMWs (ld_mem).
__device__ bool last_arriver(unsigned* counters /* kShards + 1 */) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nb = gridDim.x, shard = blockIdx.x % kShards;
    const unsigned shard_size = (nb - shard + kShards - 1) / kShards;
    const unsigned active_shards = nb < (unsigned)kShards ? nb : (unsigned)kShards;
    int last = 0;
    if (__hip_atomic_fetch_add(&counters[shard], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == shard_size - 1)
      last = __hip_atomic_fetch_add(&counters[kShards], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             active_shards - 1;
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

// memory-side reads of words other blocks updated with atomics / sc1 stores in this launch
__device__ __forceinline__ unsigned ld_mem(unsigned* p) {
  return __hip_atomic_fetch_add(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_mem(unsigned long long* p) {
  return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// contiguous candidate range of this block (a multiple of 4 long, identical in every select kernel)
__device__ __forceinline__ void block_range(long long C, long long* v0, long long* v1) {
  long long per = (C + gridDim.x - 1) / gridDim.x;
  per = (per + 3) & ~3ll;
  const long long a = (long long)blockIdx.x * per;
  *v0 = a < C ? a : C;
  *v1 = a + per < C ? a + per : C;
}

// last r in [0, R) with off[r] <= c (off in LDS, nondecreasing, off[R] > c)
__device__ __forceinline__ int lds_region_search(const unsigned* off, int R, unsigned c) {
  int lo = 0, hi = R;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= c) lo = mid;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int lds_region_advance(const unsigned* off, int R, int r, unsigned c) {
  if (off[r + 1] > c) return r;
  int lo = r + 1, step = 1, hi;
  for (;;) {
    hi = lo + step;
    if (hi >= R) {
      hi = R;
      break;
    }
    if (off[hi] > c) break;
    lo = hi;
    step <<= 1;
  }
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= c) lo = mid;
    else hi = mid;
  }
  return lo;
}

// four consecutive candidate keys (raw bits) starting at c0 (a multiple of 4), from x in fallback mode
__device__ __forceinline__ void load4_raw(const float* __restrict__ x, const TopkWs& w, bool fb, long long c0,
                                          long long v1, unsigned raw[4]) {
  if (c0 + 4 <= v1) {
    if (fb) {
      const float4 v = *reinterpret_cast<const float4*>(x + c0);
      raw[0] = __float_as_uint(v.x); raw[1] = __float_as_uint(v.y);
      raw[2] = __float_as_uint(v.z); raw[3] = __float_as_uint(v.w);
    } else {
      const uint4 v = *reinterpret_cast<const uint4*>(w.cand_raw + c0);
      raw[0] = v.x; raw[1] = v.y; raw[2] = v.z; raw[3] = v.w;
    }
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      raw[u] = (c0 + u < v1) ? (fb ? __float_as_uint(x[c0 + u]) : w.cand_raw[c0 + u]) : 0u;
  }
}

// ------------------------------------------------------------------------------------------------
// sample -> candidate floor
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void topk_sample_gather_kernel(const float* __restrict__ x, int64_t n, int S,
                                                                      TopkWs w) {
  const int j = blockIdx.x * kThreads + threadIdx.x;
  if (j >= S) return;
  const int64_t pos = (S == n) ? (int64_t)j : (int64_t)(((double)j + 0.5) * (double)n / (double)S);
  w.sample[j] = order_key(__float_as_uint(x[pos < n ? pos : n - 1]));
}

__global__ __launch_bounds__(kSelectThreads) void topk_sample_select_kernel(int S, long long rank_lo, int take_all,
                                                                            TopkWs w) {
  __shared__ unsigned s_hist[256];
  __shared__ unsigned s_mm[2][kSelectThreads / kWave];
  __shared__ unsigned s_digit;
  __shared__ long long s_rem;
  __shared__ unsigned s_err;
  if (take_all) {
    if (threadIdx.x == 0) w.p->t_lo = 0u;
    return;
  }
  unsigned keys[kSamplePerThread];
  unsigned kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
  for (int i = 0; i < kSamplePerThread; ++i) {
    const int j = threadIdx.x + i * kSelectThreads;
    keys[i] = j < S ? w.sample[j] : 0u;
    if (j < S) {
      kmin = keys[i] < kmin ? keys[i] : kmin;
      kmax = keys[i] > kmax ? keys[i] : kmax;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned a = __shfl_xor(kmin, o, kWave), b = __shfl_xor(kmax, o, kWave);
    kmin = a < kmin ? a : kmin;
    kmax = b > kmax ? b : kmax;
  }
  if ((threadIdx.x & 63) == 0) {
    s_mm[0][threadIdx.x >> 6] = kmin;
    s_mm[1][threadIdx.x >> 6] = kmax;
  }
  if (threadIdx.x == 0) s_err = 0;
  __syncthreads();
  kmin = 0xffffffffu;
  kmax = 0u;
  for (int i = 0; i < kSelectThreads / kWave; ++i) {
    kmin = s_mm[0][i] < kmin ? s_mm[0][i] : kmin;
    kmax = s_mm[1][i] > kmax ? s_mm[1][i] : kmax;
  }
  unsigned lo = kmin;
  unsigned long long width = (unsigned long long)kmax - kmin + 1ull;  // live range [lo, lo + width)
  int shift = range_shift(width, 8);
  long long rem = rank_lo;
  for (int pass = 0; pass < 5; ++pass) {
    if (threadIdx.x < 256) s_hist[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kSamplePerThread; ++i) {
      const int j = threadIdx.x + i * kSelectThreads;
      const unsigned key = keys[i];
      const unsigned long long rel = (unsigned long long)key - lo;
      const bool valid = j < S && key >= lo && rel < width;
      hist_add(s_hist, (unsigned)(rel >> shift), valid);
    }
    __syncthreads();
    if (threadIdx.x < kWave) wave_select_from_top<256>(s_hist, rem, &s_digit, &s_rem, &s_err);
    __syncthreads();
    lo += s_digit << shift;
    rem = s_rem;
    __syncthreads();
    if (shift == 0) break;
    width = 1ull << shift;
    shift = shift > 8 ? shift - 8 : 0;
  }
  if (threadIdx.x == 0) w.p->t_lo = lo;
}

// ------------------------------------------------------------------------------------------------
// streaming filter (the one HBM pass over x)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void topk_filter_kernel(const float* __restrict__ x, int64_t n,
                                                               int64_t wave_chunk, TopkWs w) {
  const unsigned t_lo = w.p->t_lo;
  if (blockIdx.x == 0) {  // reset the select state of this call (read by the next kernels)
    for (int i = threadIdx.x; i < 3 * kHistBins; i += kThreads) w.hist[i] = 0u;
    if (threadIdx.x < 4 * (kShards + 1)) w.tickets[threadIdx.x] = 0u;
    if (threadIdx.x == 0) {
      w.p->done = 0;
      w.p->err = 0u;
    }
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t r = (int64_t)blockIdx.x * kNW + (threadIdx.x >> 6);
  const int64_t e_begin = r * wave_chunk;
  const int64_t e_end = e_begin + wave_chunk < n ? e_begin + wave_chunk : n;
  uint2* __restrict__ out = w.stage + r * w.region_cap;
  const unsigned long long lt = (1ull << lane) - 1ull;
  unsigned cnt = 0, mx = 0;
  for (int64_t base = e_begin; base < e_end; base += kStep) {
    float4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t e = base + 256 * q + 4 * lane;
      if (e + 4 <= e_end) {
        v[q] = ld_stream(x + e);
      } else {
        v[q].x = e + 0 < e_end ? x[e + 0] : 0.f;
        v[q].y = e + 1 < e_end ? x[e + 1] : 0.f;
        v[q].z = e + 2 < e_end ? x[e + 2] : 0.f;
        v[q].w = e + 3 < e_end ? x[e + 3] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t e = base + 256 * q + 4 * lane;
      const unsigned b0 = __float_as_uint(v[q].x), b1 = __float_as_uint(v[q].y), b2 = __float_as_uint(v[q].z),
                     b3 = __float_as_uint(v[q].w);
      const unsigned k0 = order_key(b0), k1 = order_key(b1), k2 = order_key(b2), k3 = order_key(b3);
      const bool in0 = e + 0 < e_end, in1 = e + 1 < e_end, in2 = e + 2 < e_end, in3 = e + 3 < e_end;
      const bool f0 = in0 && k0 >= t_lo, f1 = in1 && k1 >= t_lo, f2 = in2 && k2 >= t_lo, f3 = in3 && k3 >= t_lo;
      unsigned m = 0;
      m = in0 && k0 > m ? k0 : m;
      m = in1 && k1 > m ? k1 : m;
      m = in2 && k2 > m ? k2 : m;
      m = in3 && k3 > m ? k3 : m;
      mx = m > mx ? m : mx;
      const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1), m2 = __ballot(f2), m3 = __ballot(f3);
      if ((m0 | m1 | m2 | m3) != 0ull) {
        unsigned pos = cnt + __popcll(m0 & lt) + __popcll(m1 & lt) + __popcll(m2 & lt) + __popcll(m3 & lt);
        if (f0) out[pos++] = make_uint2((unsigned)(e + 0), b0);
        if (f1) out[pos++] = make_uint2((unsigned)(e + 1), b1);
        if (f2) out[pos++] = make_uint2((unsigned)(e + 2), b2);
        if (f3) out[pos++] = make_uint2((unsigned)(e + 3), b3);
        cnt += __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
      }
    }
  }
  mx = wave_max_u32(mx);
  if (lane == 0) {
    w.region_cnt[r] = e_begin < n ? cnt : 0u;
    w.region_max[r] = mx;
  }
}

// ------------------------------------------------------------------------------------------------
// radix-select rounds over the candidates: 2048 bins over the live key range per round
// ------------------------------------------------------------------------------------------------
template <bool FIRST>
__global__ __launch_bounds__(kThreads) void topk_round_kernel(const float* __restrict__ x, TopkWs w, int round, int R,
                                                              long long k, int64_t n) {
  __shared__ unsigned s_hist[kHistBins];
  __shared__ unsigned s_off[FIRST ? kMaxRegions + 1 : 1];
  __shared__ unsigned long long s_red[kNW];
  __shared__ unsigned s_mx[kNW];
  __shared__ unsigned s_digit;
  __shared__ long long s_rem;
  long long C, rem = 0;
  bool fb;
  unsigned lo, maxkey = 0;
  unsigned long long width;
  int shift;
  if (FIRST) {
    // region scan in LDS, redone by every block (32 KiB of L2-resident counts): offsets, C, max key
    const int r0 = threadIdx.x * kRegionsPerThread;
    unsigned loc[kRegionsPerThread];
    unsigned long long sum = 0;
    unsigned mx = 0;
#pragma unroll
    for (int i = 0; i < kRegionsPerThread; i += 4) {
      if (r0 + i < R) {  // R is a multiple of 4
        const uint4 c = *reinterpret_cast<const uint4*>(w.region_cnt + r0 + i);
        const uint4 m = *reinterpret_cast<const uint4*>(w.region_max + r0 + i);
        loc[i] = c.x; loc[i + 1] = c.y; loc[i + 2] = c.z; loc[i + 3] = c.w;
        mx = max(mx, max(max(m.x, m.y), max(m.z, m.w)));
      } else {
        loc[i] = loc[i + 1] = loc[i + 2] = loc[i + 3] = 0u;
      }
      sum += (unsigned long long)loc[i] + loc[i + 1] + loc[i + 2] + loc[i + 3];
    }
    unsigned long long tot;
    unsigned long long run = block_excl_scan<unsigned long long, kNW>(sum, s_red, &tot);
#pragma unroll
    for (int i = 0; i < kRegionsPerThread; ++i) {
      if (r0 + i < R) s_off[r0 + i] = (unsigned)run;
      run += loc[i];
    }
    mx = wave_max_u32(mx);
    if ((threadIdx.x & 63) == 0) s_mx[threadIdx.x >> 6] = mx;
    if (threadIdx.x == 0) s_off[R] = (unsigned)tot;
    __syncthreads();
    for (int i = 0; i < kNW; ++i) maxkey = s_mx[i] > maxkey ? s_mx[i] : maxkey;
    fb = (long long)tot < k;
    C = fb ? (long long)n : (long long)tot;
    lo = fb ? 0u : w.p->t_lo;
    width = (unsigned long long)maxkey - lo + 1ull;
    shift = range_shift(width, kHistBits);
    rem = k;
  } else {
    if (w.p->done) return;
    C = w.p->C;
    fb = w.p->fallback != 0;
    lo = w.p->lo;
    width = w.p->width;
    shift = w.p->shift;
  }
  long long v0, v1;
  block_range(C, &v0, &v1);
  for (int i = threadIdx.x; i < kHistBins; i += kThreads) s_hist[i] = 0u;
  __syncthreads();

  int r = (FIRST && !fb && v0 + 4 * (long long)threadIdx.x < v1)
              ? lds_region_search(s_off, R, (unsigned)(v0 + 4 * threadIdx.x)) : 0;
  for (long long c0 = v0 + 4 * threadIdx.x; c0 < v1; c0 += 4 * kThreads) {
    unsigned raw[4];
    if (FIRST && !fb) {
      unsigned id[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long c = c0 + u;
        if (c < v1) {
          r = lds_region_advance(s_off, R, r, (unsigned)c);
          const uint2 e = w.stage[(long long)r * w.region_cap + (c - s_off[r])];
          id[u] = e.x;
          raw[u] = e.y;
        } else {
          id[u] = 0u;
          raw[u] = 0u;
        }
      }
      if (c0 + 4 <= v1) {
        *reinterpret_cast<uint4*>(w.cand_idx + c0) = make_uint4(id[0], id[1], id[2], id[3]);
        *reinterpret_cast<uint4*>(w.cand_raw + c0) = make_uint4(raw[0], raw[1], raw[2], raw[3]);
      } else {
        for (int u = 0; u < 4; ++u)
          if (c0 + u < v1) {
            w.cand_idx[c0 + u] = id[u];
            w.cand_raw[c0 + u] = raw[u];
          }
      }
    } else {
      load4_raw(x, w, fb, c0, v1, raw);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned key = order_key(raw[u]);
      const unsigned long long rel = (unsigned long long)key - lo;
      const bool valid = c0 + u < v1 && key >= lo && rel < width;
      hist_add(s_hist, (unsigned)(rel >> shift), valid);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHistBins; i += kThreads)
    if (s_hist[i]) atomicAdd(&w.hist[round * kHistBins + i], s_hist[i]);
  drain_stores();
  if (!last_arriver(&w.tickets[round * (kShards + 1)])) return;
  for (int i = threadIdx.x; i < kHistBins; i += kThreads) s_hist[i] = ld_mem(&w.hist[round * kHistBins + i]);
  if (!FIRST && threadIdx.x == 0) s_rem = w.p->rem;
  __syncthreads();
  if (!FIRST) rem = s_rem;
  __syncthreads();
  if (threadIdx.x < kWave) wave_select_from_top<kHistBins>(s_hist, rem, &s_digit, &s_rem, &w.p->err);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nlo = lo + (s_digit << shift);
    if (FIRST) {
      w.p->C = C;
      w.p->fallback = fb ? 1u : 0u;
      w.p->maxkey = maxkey;
      w.p->k = k;
    }
    if (shift == 0) {
      w.p->T = nlo;
      w.p->need = s_rem;
      w.p->done = 1;
    } else {
      w.p->lo = nlo;
      w.p->width = 1ull << shift;
      w.p->shift = shift > kHistBits ? shift - kHistBits : 0;
      w.p->rem = s_rem;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// per-block strict / tie counts + scan by the last arriver
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void topk_count_kernel(const float* __restrict__ x, TopkWs w) {
  __shared__ unsigned long long s_red[kNW];
  const long long C = w.p->C;
  const bool fb = w.p->fallback != 0;
  const unsigned T = w.p->T;
  long long v0, v1;
  block_range(C, &v0, &v1);
  unsigned long long cnt = 0;  // strict << 32 | tie
  for (long long c0 = v0 + 4 * threadIdx.x; c0 < v1; c0 += 4 * kThreads) {
    unsigned raw[4];
    load4_raw(x, w, fb, c0, v1, raw);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned key = order_key(raw[u]);
      if (c0 + u < v1) cnt += (key > T ? (1ull << 32) : 0ull) + (key == T ? 1ull : 0ull);
    }
  }
  const unsigned long long both = block_sum<unsigned long long, kNW>(cnt, s_red);
  if (threadIdx.x == 0) st_sc1(&w.blk_cnt[blockIdx.x], both);
  drain_stores();
  if (!last_arriver(&w.tickets[3 * (kShards + 1)])) return;
  // blocks 4t .. 4t+3 per thread (gridDim.x == kSelBlocks == 4 * kThreads)
  unsigned long long v[4], s = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int b = 4 * threadIdx.x + u;
    v[u] = b < (int)gridDim.x ? ld_mem(&w.blk_cnt[b]) : 0ull;
    s += v[u];
  }
  unsigned long long tot;
  unsigned long long run = block_excl_scan<unsigned long long, kNW>(s, s_red, &tot);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int b = 4 * threadIdx.x + u;
    if (b < (int)gridDim.x) w.blk_off[b] = run;
    run += v[u];
  }
  if (threadIdx.x == 0) {
    const long long st = (long long)(tot >> 32), ti = (long long)(tot & 0xffffffffull);
    w.p->strict_total = st;
    w.p->ties_total = ti;
    if (st + w.p->need != w.p->k || w.p->need > ti) w.p->err |= 2u;
  }
}

// ------------------------------------------------------------------------------------------------
// ordered compaction of the kept set (plain top-k, or the stacked codec with fused dithering)
// ------------------------------------------------------------------------------------------------
template <bool STACKED>
__global__ __launch_bounds__(kThreads) void topk_compact_kernel(const float* __restrict__ x, TopkWs w,
                                                                int* __restrict__ idx_out, float* __restrict__ val_out,
                                                                uint8_t* __restrict__ code_out, float* __restrict__ norm_out,
                                                                int levels, double step, uint64_t seed, uint64_t counter) {
  __shared__ unsigned long long s_red[kNW];
  const long long C = w.p->C;
  const bool fb = w.p->fallback != 0;
  const unsigned T = w.p->T;
  const long long skip = w.p->ties_total - w.p->need;  // ties with rank < skip are dropped
  const long long kk = w.p->k;
  long long v0, v1;
  block_range(C, &v0, &v1);
  const unsigned long long off = w.blk_off[blockIdx.x];
  long long run_s = (long long)(off >> 32), run_t = (long long)(off & 0xffffffffull);
  float nrm = 0.0f;
  if (STACKED) {
    const float a = fabsf(key_value(w.p->maxkey)), b = fabsf(key_value(T));
    nrm = (isnan(a) || isnan(b)) ? __uint_as_float(0x7fc00000u) : (a > b ? a : b);
    if (blockIdx.x == 0 && threadIdx.x == 0) *norm_out = nrm;
  }
  for (long long base = v0; base < v1; base += 4 * kThreads) {
    const long long c0 = base + 4 * threadIdx.x;
    unsigned raw[4], id[4];
    load4_raw(x, w, fb, c0, v1, raw);
    if (fb) {
#pragma unroll
      for (int u = 0; u < 4; ++u) id[u] = (unsigned)(c0 + u);
    } else if (c0 + 4 <= v1) {
      const uint4 t = *reinterpret_cast<const uint4*>(w.cand_idx + c0);
      id[0] = t.x; id[1] = t.y; id[2] = t.z; id[3] = t.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) id[u] = c0 + u < v1 ? w.cand_idx[c0 + u] : 0u;
    }
    bool is_s[4], is_t[4];
    unsigned long long cnt = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned key = order_key(raw[u]);
      const bool in = c0 + u < v1;
      is_s[u] = in && key > T;
      is_t[u] = in && key == T;
      cnt += (is_s[u] ? (1ull << 32) : 0ull) + (is_t[u] ? 1ull : 0ull);
    }
    unsigned long long tot;
    const unsigned long long ex = block_excl_scan<unsigned long long, kNW>(cnt, s_red, &tot);
    long long s_before = run_s + (long long)(ex >> 32), t_before = run_t + (long long)(ex & 0xffffffffull);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool keep = is_s[u] || (is_t[u] && t_before >= skip);
      const long long pos = s_before + (t_before > skip ? t_before - skip : 0);
      if (keep && pos >= 0 && pos < kk) {
        idx_out[pos] = (int)id[u];
        if (STACKED) {
          const float v = __uint_as_float(raw[u]);
          uint32_t code = 0u;
          if (v != 0.0f) {
            if (!(nrm > 0.0f && nrm <= 3.402823466e38f)) {
              code = 1u;
            } else {
              const float y = fabsf(v) / nrm;  // compressors.py:344
              const int j = level_lower_bound<0>(y, levels, step);
              const int sl = j > 0 ? j - 1 : 0;
              const double lo = level_value<0>(sl, levels, step), hi = level_value<0>(sl + 1, levels, step);
              const double p = ((double)y - hi) / (lo - hi);  // compressors.py:348
              const U4 r4 = philox_group((uint64_t)id[u] >> 2, seed, counter);
              const double uu = u01(pick(r4, (int)(id[u] & 3u)));
              const int lvl = (uu < p) ? sl : sl + 1;
              code = ((raw[u] >> 31) << 7) | (uint32_t)lvl;
            }
          }
          code_out[pos] = (uint8_t)code;
        } else {
          val_out[pos] = __uint_as_float(raw[u]);
        }
      }
      s_before += is_s[u] ? 1 : 0;
      t_before += is_t[u] ? 1 : 0;
    }
    run_s += (long long)(tot >> 32);
    run_t += (long long)(tot & 0xffffffffull);
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
struct SampleSetup {
  int S;
  long long rank_lo;
  int take_all;
};

SampleSetup sample_setup(int64_t n, int64_t k) {
  SampleSetup s;
  s.S = (int)(n < kSample ? n : kSample);
  const double m = (double)s.S * (double)k / (double)n;
  const double r = ceil(m + 4.0 * sqrt(m) + 16.0);
  s.rank_lo = (long long)r;
  s.take_all = (s.rank_lo >= s.S) ? 1 : 0;
  if (s.take_all) s.rank_lo = s.S;
  return s;
}

int launch_select(const float* x, int64_t n, int64_t k, const TopkWs& w, hipStream_t st) {
  const TopkGeom g = geometry(n);
  const SampleSetup ss = sample_setup(n, k);
  const int R = (int)g.regions;
  if (!ss.take_all)
    FLC_LAUNCH("topk_sample_gather", topk_sample_gather_kernel, dim3((unsigned)cdiv(ss.S, kThreads)), dim3(kThreads), 0,
               st, x, n, ss.S, w);
  FLC_LAUNCH("topk_sample_select", topk_sample_select_kernel, dim3(1), dim3(kSelectThreads), 0, st, ss.S, ss.rank_lo,
             ss.take_all, w);
  FLC_LAUNCH("topk_filter", topk_filter_kernel, dim3((unsigned)g.blocks), dim3(kThreads), 0, st, x, n, g.wave_chunk, w);
  FLC_LAUNCH("topk_round", topk_round_kernel<true>, dim3(kSelBlocks), dim3(kThreads), 0, st, x, w, 0, R, (long long)k, n);
  FLC_LAUNCH("topk_round", topk_round_kernel<false>, dim3(kSelBlocks), dim3(kThreads), 0, st, x, w, 1, R, (long long)k, n);
  FLC_LAUNCH("topk_round", topk_round_kernel<false>, dim3(kSelBlocks), dim3(kThreads), 0, st, x, w, 2, R, (long long)k, n);
  FLC_LAUNCH("topk_count", topk_count_kernel, dim3(kSelBlocks), dim3(kThreads), 0, st, x, w);
  return FLC_OK;
}

int check_topk(const float* x, int64_t n, int64_t k, const char* who) {
  if (!x || n <= 0) return fail(FLC_EINVAL, "%s: bad arguments", who);
  if (n >= (1ll << 31)) return fail(FLC_EINVAL, "%s: n must be < 2^31", who);
  if (k <= 0 || k >= n) return fail(FLC_EINVAL, "%s: need 0 < k < n (got k=%lld, n=%lld)", who, (long long)k, (long long)n);
  if (!aligned16(x)) return fail(FLC_EINVAL, "%s: x must be 16-B aligned", who);
  return FLC_OK;
}

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

size_t flc_topk_workspace_size(int64_t n, int64_t k) {
  (void)k;
  size_t need = 0;
  (void)carve_topk(nullptr, 0, n < 1 ? 1 : n, &need);
  return need;
}

int flc_topk_encode(const float* x, int64_t n, int64_t k, int32_t* idx, float* val, void* ws, size_t ws_bytes,
                    void* stream) {
  if (int rc = check_topk(x, n, k, "flc_topk_encode")) return rc;
  if (!idx || !val) return fail(FLC_EINVAL, "flc_topk_encode: null output");
  size_t need = 0;
  TopkWs w = carve_topk(ws, ws_bytes, n, &need);
  if (!ws || need > ws_bytes) return fail(FLC_EWORKSPACE, "flc_topk_encode: workspace %zu < %zu", ws_bytes, need);
  hipStream_t st = as_stream(stream);
  if (int rc = launch_select(x, n, k, w, st)) return rc;
  FLC_LAUNCH("topk_compact", topk_compact_kernel<false>, dim3(kSelBlocks), dim3(kThreads), 0, st, x, w, idx, val,
             (uint8_t*)nullptr, (float*)nullptr, 0, 0.0, (uint64_t)0, (uint64_t)0);
  return FLC_OK;
}

int flc_stacked_encode(const float* x, int64_t n, int64_t k, int levels, uint64_t seed, uint64_t counter,
                       const double* compat_u, int32_t* idx, uint8_t* codes, float* norm, void* ws, size_t ws_bytes,
                       void* stream) {
  if (int rc = check_topk(x, n, k, "flc_stacked_encode")) return rc;
  if (!idx || !codes || !norm) return fail(FLC_EINVAL, "flc_stacked_encode: null output");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_stacked_encode: levels must be in [1, 127]");
  if (compat_u)
    return fail(FLC_EUNSUPPORTED,
                "flc_stacked_encode: compat RNG is composed by the caller (flc_topk_encode + flc_quant_encode)");
  size_t need = 0;
  TopkWs w = carve_topk(ws, ws_bytes, n, &need);
  if (!ws || need > ws_bytes) return fail(FLC_EWORKSPACE, "flc_stacked_encode: workspace %zu < %zu", ws_bytes, need);
  hipStream_t st = as_stream(stream);
  if (int rc = launch_select(x, n, k, w, st)) return rc;
  FLC_LAUNCH("stacked_compact", topk_compact_kernel<true>, dim3(kSelBlocks), dim3(kThreads), 0, st, x, w, idx,
             (float*)nullptr, codes, norm, levels, 1.0 / (double)levels, seed, counter);
  return FLC_OK;
}

}  // extern "C"
