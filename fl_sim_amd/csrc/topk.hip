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
//   sample_select  1 block, keys in registers: radix select (2048-bin digits over the live range of
//                  the sample) -> candidate floor t_lo with count(key >= t_lo) ~ k + 4 sigma
//                  (k/n = 1 %: ~1.22 k candidates).
//   filter         the HBM pass: each wave owns a contiguous run of x and appends its candidates in
//                  index order to a private staging region (ballot/mbcnt compaction: no atomics, no
//                  inter-wave sync).  Algorithmic bytes 4 per element.
//   select         ONE persistent launch, one 1024-thread block per CU, five phases separated by
//                  XCD-sharded grid barriers whose last arriver ("leader") does the serial step:
//                    P0  region offsets in LDS (every block), candidate count C, max key;
//                    P1  gather the staged candidates into an ordered SoA array + radix round 1;
//                    P2  radix rounds 2-3 (2048 bins over the live key range; 3 rounds always resolve
//                        the exact k-th largest key T);
//                    P3  per-block strict / tie counts, scanned by the leader;
//                    P4  ordered compaction into idx[k] / val[k], or, stacked, idx[k] / codes[k] with
//                        the dithering fused in (norm of the kept set = max(|max key|, |T|)).
//                  C < k switches every phase to "fallback" mode, reading x itself (always correct).
// Cross-block hand-offs inside a launch go through memory-side atomics only (histogram adds, arrival
// counters, RMW reads, atomic exchanges of the published state); candidates are re-read only by the
// thread that wrote them.  Spins are bounded (error flag), and the host serialises the persistent
// launches of different streams so two of them never compete for residency.
#include <hip/hip_runtime.h>
#include <math.h>

#include <stdlib.h>

#include <algorithm>
#include <mutex>

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
constexpr int kSelThreads = 1024;   // persistent select: one block of 16 waves per CU
constexpr int kSelNW = kSelThreads / kWave;
constexpr int kMaxSelBlocks = 1024;
constexpr int kHistBits = 11;
constexpr int kHistBins = 1 << kHistBits;
constexpr int kShards = 8;          // XCD shards of the arrival counters
constexpr int kMaxRegions = 8192;
constexpr int kRegionsPerThread = kMaxRegions / kSelThreads;  // 8 (P0 LDS scan)

struct TopkParams {
  unsigned t_lo;       // candidate floor (sample_select -> filter, select)
  unsigned pad;
};

// state published by the grid-barrier leaders of the select launch (64-bit words, memory-side
// atomics only); zeroed per call by the filter
struct SelState {
  unsigned long long gen;     // barrier generation
  unsigned long long lo;      // live key range [lo, lo + width), log2 keys per bin, rank left
  unsigned long long width;
  unsigned long long shift;
  unsigned long long rem;
  unsigned long long done;    // threshold resolved
  unsigned long long T;       // the k-th largest key
  unsigned long long need;    // elements equal to T that are kept
  unsigned long long ties;
  unsigned long long strict;
  unsigned long long err;     // 1: digit not found, 2: count mismatch, 4: barrier spin timeout
  unsigned long long C;       // diagnostics
  unsigned long long fallback;
  unsigned long long maxkey;
};

struct TopkWs {
  TopkParams* p;
  SelState* st;
  unsigned* bar;                // [kShards + 1] grid-barrier arrival counters (monotonic per call)
  unsigned* hist;               // [3][kHistBins]
  unsigned* sample;             // [kSample]
  unsigned* region_cnt;         // [R]
  unsigned* region_max;         // [R]
  unsigned long long* blk_cnt;  // [kMaxSelBlocks]  strict << 32 | tie
  unsigned long long* blk_off;  // [kMaxSelBlocks]
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
  w.st = c.take<SelState>(1);
  w.bar = c.take<unsigned>(kShards + 1);
  w.hist = c.take<unsigned>(3 * kHistBins);
  w.sample = c.take<unsigned>(kSample);
  w.region_cnt = c.take<unsigned>(g.regions);
  w.region_max = c.take<unsigned>(g.regions);
  w.blk_cnt = c.take<unsigned long long>(kMaxSelBlocks);
  w.blk_off = c.take<unsigned long long>(kMaxSelBlocks);
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

// memory-side reads of words other blocks updated with atomics / sc1 stores in this launch
__device__ __forceinline__ unsigned ld_mem(unsigned* p) {
  return __hip_atomic_fetch_add(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_mem(unsigned long long* p) {
  return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  __shared__ unsigned s_hist[kHistBins];
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
  int shift = range_shift(width, kHistBits);
  long long rem = rank_lo;
  for (int pass = 0; pass < 4; ++pass) {
    for (int i = threadIdx.x; i < kHistBins; i += kSelectThreads) s_hist[i] = 0;
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
    if (threadIdx.x < kWave) wave_select_from_top<kHistBins>(s_hist, rem, &s_digit, &s_rem, &s_err);
    __syncthreads();
    lo += s_digit << shift;
    rem = s_rem;
    __syncthreads();
    if (shift == 0) break;
    width = 1ull << shift;
    shift = shift > kHistBits ? shift - kHistBits : 0;
  }
  if (threadIdx.x == 0) w.p->t_lo = lo;
}

// ------------------------------------------------------------------------------------------------
// streaming filter (the one HBM pass over x)
// ------------------------------------------------------------------------------------------------
// candidate test on values: key(v) >= t_lo  <=>  v >= t_lo_value  or  v is NaN (NaN is the largest
// key; -0 == +0 holds for the float compare as for the keys)
__device__ __forceinline__ float floor_value(unsigned t_lo) {
  return t_lo <= 0x007fffffu ? -__builtin_inff() : key_value(t_lo);  // keys below -inf: negative NaNs
}

// one 1024-element step of a wave: 4 x float4 per lane (q-major: lane l, q -> elements 256q + 4l + c)
template <bool TAIL>
__device__ __forceinline__ void filter_step(const float* __restrict__ x, int64_t base, int64_t e_end, float tf,
                                            uint2* __restrict__ out, unsigned& cnt, float& vmax, bool& saw_nan,
                                            int lane) {
  float4 v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t e = base + 256 * q + 4 * lane;
    if (!TAIL) {
      v[q] = ld_stream(x + e);
    } else {
      v[q].x = e + 0 < e_end ? x[e + 0] : -__builtin_inff();
      v[q].y = e + 1 < e_end ? x[e + 1] : -__builtin_inff();
      v[q].z = e + 2 < e_end ? x[e + 2] : -__builtin_inff();
      v[q].w = e + 3 < e_end ? x[e + 3] : -__builtin_inff();
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a0 = v[q].x, a1 = v[q].y, a2 = v[q].z, a3 = v[q].w;
    vmax = fmaxf(vmax, fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)));  // fmaxf ignores NaN; NaN tracked apart
    const bool n0 = a0 != a0, n1 = a1 != a1, n2 = a2 != a2, n3 = a3 != a3;
    saw_nan |= n0 | n1 | n2 | n3;
    // tail padding is -inf, which passes only when tf == -inf: exclude it explicitly there
    const int64_t e = base + 256 * q + 4 * lane;
    const bool f0 = (a0 >= tf || n0) && (!TAIL || e + 0 < e_end);
    const bool f1 = (a1 >= tf || n1) && (!TAIL || e + 1 < e_end);
    const bool f2 = (a2 >= tf || n2) && (!TAIL || e + 2 < e_end);
    const bool f3 = (a3 >= tf || n3) && (!TAIL || e + 3 < e_end);
    const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1), m2 = __ballot(f2), m3 = __ballot(f3);
    if ((m0 | m1 | m2 | m3) == 0ull) continue;
    unsigned pos = cnt;
    pos = __builtin_amdgcn_mbcnt_hi((unsigned)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m0, pos));
    pos = __builtin_amdgcn_mbcnt_hi((unsigned)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m1, pos));
    pos = __builtin_amdgcn_mbcnt_hi((unsigned)(m2 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m2, pos));
    pos = __builtin_amdgcn_mbcnt_hi((unsigned)(m3 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m3, pos));
    if (f0 | f1 | f2 | f3) {
      if (f0) out[pos++] = make_uint2((unsigned)(e + 0), __float_as_uint(a0));
      if (f1) out[pos++] = make_uint2((unsigned)(e + 1), __float_as_uint(a1));
      if (f2) out[pos++] = make_uint2((unsigned)(e + 2), __float_as_uint(a2));
      if (f3) out[pos++] = make_uint2((unsigned)(e + 3), __float_as_uint(a3));
    }
    cnt += __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
  }
}

__global__ __launch_bounds__(kThreads) void topk_filter_kernel(const float* __restrict__ x, int64_t n,
                                                               int64_t wave_chunk, TopkWs w) {
  const float tf = floor_value(w.p->t_lo);
  if (blockIdx.x == 0) {  // reset the select state of this call (read by the next launch)
    for (int i = threadIdx.x; i < 3 * kHistBins; i += kThreads) w.hist[i] = 0u;
    if (threadIdx.x < kShards + 1) w.bar[threadIdx.x] = 0u;
    if (threadIdx.x < (int)(sizeof(SelState) / 8)) reinterpret_cast<unsigned long long*>(w.st)[threadIdx.x] = 0ull;
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t r = (int64_t)blockIdx.x * kNW + (threadIdx.x >> 6);
  const int64_t e_begin = r * wave_chunk;
  const int64_t e_end = e_begin + wave_chunk < n ? e_begin + wave_chunk : n;
  uint2* __restrict__ out = w.stage + r * w.region_cap;
  unsigned cnt = 0;
  float vmax = -__builtin_inff();
  bool saw_nan = false;
  int64_t base = e_begin;
  for (; base + kStep <= e_end; base += kStep) filter_step<false>(x, base, e_end, tf, out, cnt, vmax, saw_nan, lane);
  if (base < e_end) filter_step<true>(x, base, e_end, tf, out, cnt, vmax, saw_nan, lane);
  unsigned mx = order_key(__float_as_uint(vmax));
  mx = __ballot(saw_nan) ? 0xffffffffu : mx;
  mx = wave_max_u32(mx);
  if (lane == 0) {
    w.region_cnt[r] = e_begin < n ? cnt : 0u;
    w.region_max[r] = e_begin < n ? mx : 0u;
  }
}

// ------------------------------------------------------------------------------------------------
// persistent select: P0 scan | P1 gather + round 1 | rounds 2-3 | counts | compaction
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long ld_mem64(unsigned long long* p) {
  return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_mem64(unsigned long long* p, unsigned long long v) {
  (void)__hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the per-block copy of the leader-published state
struct SelView {
  unsigned lo;
  unsigned long long width;
  int shift;
  long long rem;
  int done;
  unsigned T;
  long long need, ties;
};

// Grid barrier: every block arrives on its XCD shard counter, the last of each shard on the top
// counter; the last arriver overall runs `lead` (all of its threads) and then bumps the generation
// word the others poll (relaxed agent-scope loads + s_sleep, bounded).  Counters are monotonic within
// a call, so barrier number `nbar` waits for (nbar + 1) full sets of arrivals.
template <typename F>
__device__ void grid_barrier(const TopkWs& w, unsigned nbar, F&& lead) {
  __shared__ int s_lead;
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nb = gridDim.x, shard = blockIdx.x % kShards;
    const unsigned shard_size = (nb - shard + kShards - 1) / kShards;
    const unsigned active = nb < (unsigned)kShards ? nb : (unsigned)kShards;
    int l = 0;
    if (__hip_atomic_fetch_add(&w.bar[shard], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        shard_size * (nbar + 1) - 1)
      l = __hip_atomic_fetch_add(&w.bar[kShards], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
          active * (nbar + 1) - 1;
    s_lead = l;
  }
  __syncthreads();
  if (s_lead) {
    lead();
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0) st_mem64(&w.st->gen, nbar + 1);
  } else if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(&w.st->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nbar + 1ull) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 24)) {  // ~1 s: a block never arrived; flag it and let the launch drain
        __hip_atomic_fetch_or(&w.st->err, 4ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

__device__ void read_view(const TopkWs& w, SelView* v) {
  if (threadIdx.x == 0) {
    v->lo = (unsigned)ld_mem64(&w.st->lo);
    v->width = ld_mem64(&w.st->width);
    v->shift = (int)ld_mem64(&w.st->shift);
    v->rem = (long long)ld_mem64(&w.st->rem);
    v->done = (int)ld_mem64(&w.st->done);
    v->T = (unsigned)ld_mem64(&w.st->T);
    v->need = (long long)ld_mem64(&w.st->need);
    v->ties = (long long)ld_mem64(&w.st->ties);
  }
  __syncthreads();
}

// leader step of a radix round: digit of the rank `rem` in the global histogram of round r
__device__ void lead_pick(const TopkWs& w, int r, const SelView& cur, unsigned* s_hist) {
  __shared__ unsigned s_digit;
  __shared__ long long s_rem;
  __shared__ unsigned s_err;
  for (int i = threadIdx.x; i < kHistBins; i += kSelThreads) s_hist[i] = ld_mem(&w.hist[r * kHistBins + i]);
  if (threadIdx.x == 0) s_err = 0;
  __syncthreads();
  if (threadIdx.x < kWave) wave_select_from_top<kHistBins>(s_hist, cur.rem, &s_digit, &s_rem, &s_err);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nlo = cur.lo + (s_digit << cur.shift);
    if (s_err) __hip_atomic_fetch_or(&w.st->err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur.shift == 0) {
      st_mem64(&w.st->T, nlo);
      st_mem64(&w.st->need, (unsigned long long)s_rem);
      st_mem64(&w.st->ties, s_hist[s_digit]);
      st_mem64(&w.st->done, 1ull);
    } else {
      st_mem64(&w.st->lo, nlo);
      st_mem64(&w.st->width, 1ull << cur.shift);
      st_mem64(&w.st->shift, (unsigned long long)(cur.shift > kHistBits ? cur.shift - kHistBits : 0));
      st_mem64(&w.st->rem, (unsigned long long)s_rem);
    }
  }
}

template <bool STACKED>
__global__ __launch_bounds__(kSelThreads) void topk_select_kernel(const float* __restrict__ x, TopkWs w, int R,
                                                                  long long k, int64_t n, int* __restrict__ idx_out,
                                                                  float* __restrict__ val_out,
                                                                  uint8_t* __restrict__ code_out,
                                                                  float* __restrict__ norm_out, int levels, double step,
                                                                  uint64_t seed, uint64_t counter) {
  __shared__ unsigned s_off[kMaxRegions + 1];
  __shared__ unsigned s_hist[kHistBins];
  __shared__ unsigned long long s_red[kSelNW];
  __shared__ unsigned s_mx[kSelNW];
  __shared__ SelView s_view;
  const int tid = threadIdx.x;

  // ---- P0: region offsets in LDS, candidate count, max key (identical in every block)
  {
    const int r0 = tid * kRegionsPerThread;
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
    unsigned long long run = block_excl_scan<unsigned long long, kSelNW>(sum, s_red, &tot);
#pragma unroll
    for (int i = 0; i < kRegionsPerThread; ++i) {
      if (r0 + i < R) s_off[r0 + i] = (unsigned)run;
      run += loc[i];
    }
    mx = wave_max_u32(mx);
    if ((tid & 63) == 0) s_mx[tid >> 6] = mx;
    if (tid == 0) {
      s_off[R] = (unsigned)tot;
      s_red[0] = tot;
    }
    __syncthreads();
  }
  const unsigned long long c_cand = s_red[0];
  unsigned maxkey = 0;
  for (int i = 0; i < kSelNW; ++i) maxkey = s_mx[i] > maxkey ? s_mx[i] : maxkey;
  const bool fb = (long long)c_cand < k;
  const long long C = fb ? (long long)n : (long long)c_cand;
  long long per = (C + gridDim.x - 1) / gridDim.x;
  per = (per + 3) & ~3ll;
  const long long v0 = min((long long)blockIdx.x * per, C), v1 = min(v0 + per, C);

  SelView cur;
  cur.lo = fb ? 0u : w.p->t_lo;
  cur.width = (unsigned long long)maxkey - cur.lo + 1ull;
  cur.shift = range_shift(cur.width, kHistBits);
  cur.rem = k;
  cur.done = 0;
  unsigned nbar = 0;

  // ---- P1 + rounds: histogram of the live range, leader picks the digit
  for (int round = 0; round < 3; ++round) {
    for (int i = tid; i < kHistBins; i += kSelThreads) s_hist[i] = 0u;
    __syncthreads();
    int r = 0;
    if (round == 0 && !fb && v0 + 4 * (long long)tid < v1) r = lds_region_search(s_off, R, (unsigned)(v0 + 4 * tid));
    for (long long c0 = v0 + 4 * tid; c0 < v1; c0 += 4 * kSelThreads) {
      unsigned raw[4];
      if (fb) {
        if (c0 + 4 <= v1) {
          const float4 v = *reinterpret_cast<const float4*>(x + c0);
          raw[0] = __float_as_uint(v.x); raw[1] = __float_as_uint(v.y);
          raw[2] = __float_as_uint(v.z); raw[3] = __float_as_uint(v.w);
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) raw[u] = c0 + u < v1 ? __float_as_uint(x[c0 + u]) : 0u;
        }
      } else if (round == 0) {
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
      } else if (c0 + 4 <= v1) {  // re-read what this thread wrote in round 0
        const uint4 t = *reinterpret_cast<const uint4*>(w.cand_raw + c0);
        raw[0] = t.x; raw[1] = t.y; raw[2] = t.z; raw[3] = t.w;
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) raw[u] = c0 + u < v1 ? w.cand_raw[c0 + u] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const unsigned key = order_key(raw[u]);
        const unsigned long long rel = (unsigned long long)key - cur.lo;
        const bool valid = c0 + u < v1 && key >= cur.lo && rel < cur.width;
        hist_add(s_hist, (unsigned)(rel >> cur.shift), valid);
      }
    }
    __syncthreads();
    for (int i = tid; i < kHistBins; i += kSelThreads)
      if (s_hist[i]) atomicAdd(&w.hist[round * kHistBins + i], s_hist[i]);
    grid_barrier(w, nbar++, [&] { lead_pick(w, round, cur, s_hist); });
    read_view(w, &s_view);
    cur = s_view;
    __syncthreads();
    if (cur.done) break;
  }

  // ---- counts: strict / ties of T per block, scanned by the leader
  const unsigned T = cur.T;
  {
    unsigned long long cnt = 0;  // strict << 32 | tie
    for (long long c0 = v0 + 4 * tid; c0 < v1; c0 += 4 * kSelThreads) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long c = c0 + u;
        if (c < v1) {
          const unsigned key = order_key(fb ? __float_as_uint(x[c]) : w.cand_raw[c]);
          cnt += (key > T ? (1ull << 32) : 0ull) + (key == T ? 1ull : 0ull);
        }
      }
    }
    const unsigned long long both = block_sum<unsigned long long, kSelNW>(cnt, s_red);
    if (tid == 0) st_mem64(&w.blk_cnt[blockIdx.x], both);
  }
  grid_barrier(w, nbar++, [&] {
    const unsigned long long v = tid < (int)gridDim.x ? ld_mem64(&w.blk_cnt[tid]) : 0ull;
    unsigned long long tot;
    const unsigned long long ex = block_excl_scan<unsigned long long, kSelNW>(v, s_red, &tot);
    if (tid < (int)gridDim.x) st_mem64(&w.blk_off[tid], ex);
    if (tid == 0) {
      const long long st = (long long)(tot >> 32), ti = (long long)(tot & 0xffffffffull);
      st_mem64(&w.st->strict, (unsigned long long)st);
      st_mem64(&w.st->ties, (unsigned long long)ti);
      st_mem64(&w.st->C, (unsigned long long)C);
      st_mem64(&w.st->fallback, fb ? 1ull : 0ull);
      st_mem64(&w.st->maxkey, maxkey);
      if (st + cur.need != k || cur.need > ti)
        __hip_atomic_fetch_or(&w.st->err, 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  });
  __shared__ unsigned long long s_off_blk, s_ties;
  if (tid == 0) {
    s_off_blk = ld_mem64(&w.blk_off[blockIdx.x]);
    s_ties = ld_mem64(&w.st->ties);
  }
  __syncthreads();

  // ---- ordered compaction of the kept set
  const long long skip = (long long)s_ties - cur.need;  // ties with rank < skip are dropped
  long long run_s = (long long)(s_off_blk >> 32), run_t = (long long)(s_off_blk & 0xffffffffull);
  float nrm = 0.0f;
  if (STACKED) {
    const float a = fabsf(key_value(maxkey)), b = fabsf(key_value(T));
    nrm = (isnan(a) || isnan(b)) ? __uint_as_float(0x7fc00000u) : (a > b ? a : b);
    if (blockIdx.x == 0 && tid == 0) *norm_out = nrm;
  }
  const bool nrm_ok = nrm > 0.0f && nrm <= 3.402823466e38f;
  for (long long base = v0; base < v1; base += 4 * kSelThreads) {
    const long long c0 = base + 4 * tid;
    unsigned raw[4], id[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long c = c0 + u;
      const bool in = c < v1;
      raw[u] = in ? (fb ? __float_as_uint(x[c]) : w.cand_raw[c]) : 0u;
      id[u] = in ? (fb ? (unsigned)c : w.cand_idx[c]) : 0u;
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
    const unsigned long long ex = block_excl_scan<unsigned long long, kSelNW>(cnt, s_red, &tot);
    long long s_before = run_s + (long long)(ex >> 32), t_before = run_t + (long long)(ex & 0xffffffffull);
    // dithering of the 4 values first, branch-free, so the 4 chains overlap
    uint32_t code[4];
    if (STACKED) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float v = __uint_as_float(raw[u]);
        const float y = nrm_ok ? fabsf(v) / nrm : 0.0f;  // compressors.py:344
        const int j = level_lower_bound<0>(y, levels, step);
        const int sl = j > 0 ? j - 1 : 0;
        const double lo = level_value<0>(sl, levels, step), hi = level_value<0>(sl + 1, levels, step);
        const double p = ((double)y - hi) / (lo - hi);  // compressors.py:348
        const U4 r4 = philox_group((uint64_t)id[u] >> 2, seed, counter);
        const double uu = u01(pick(r4, (int)(id[u] & 3u)));
        const uint32_t lvl = (uint32_t)((uu < p) ? sl : sl + 1);
        const uint32_t c = nrm_ok ? (((raw[u] >> 31) << 7) | lvl) : 1u;
        code[u] = (v != 0.0f) ? c : 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool keep = is_s[u] || (is_t[u] && t_before >= skip);
      const long long pos = s_before + (t_before > skip ? t_before - skip : 0);
      if (keep && pos >= 0 && pos < k) {
        idx_out[pos] = (int)id[u];
        if (STACKED) code_out[pos] = (uint8_t)code[u];
        else val_out[pos] = __uint_as_float(raw[u]);
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

// one persistent select launch per device at a time: launches on different streams are ordered with an
// event chain (stream-ordered, no host blocking), so two never compete for co-residency
struct SelectGate {
  std::mutex mu;
  hipEvent_t last[64] = {};
  int grid[64] = {};
};
SelectGate& gate() {
  static SelectGate g;
  return g;
}

int select_grid(int dev) {
  SelectGate& g = gate();
  if (g.grid[dev] == 0) {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cu <= 0) cu = 256;
    g.grid[dev] = cu < kMaxSelBlocks ? cu : kMaxSelBlocks;
  }
  return g.grid[dev];
}

template <bool STACKED>
int launch_topk(const float* x, int64_t n, int64_t k, const TopkWs& w, hipStream_t st, int* idx, float* val,
                uint8_t* codes, float* norm, int levels, uint64_t seed, uint64_t counter) {
  const TopkGeom g = geometry(n);
  const SampleSetup ss = sample_setup(n, k);
  const int R = (int)g.regions;
  if (!ss.take_all)
    FLC_LAUNCH("topk_sample_gather", topk_sample_gather_kernel, dim3((unsigned)cdiv(ss.S, kThreads)), dim3(kThreads), 0,
               st, x, n, ss.S, w);
  FLC_LAUNCH("topk_sample_select", topk_sample_select_kernel, dim3(1), dim3(kSelectThreads), 0, st, ss.S, ss.rank_lo,
             ss.take_all, w);
  FLC_LAUNCH("topk_filter", topk_filter_kernel, dim3((unsigned)g.blocks), dim3(kThreads), 0, st, x, n, g.wave_chunk, w);
  int dev = 0;
  FLC_CHECK_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return fail(FLC_EUNSUPPORTED, "device index %d", dev);
  const int grid = select_grid(dev);
  SelectGate& gt = gate();
  std::lock_guard<std::mutex> lk(gt.mu);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  FLC_CHECK_HIP(hipStreamIsCapturing(st, &cs));
  const bool gated = cs == hipStreamCaptureStatusNone;
  if (gated) {
    if (!gt.last[dev]) FLC_CHECK_HIP(hipEventCreateWithFlags(&gt.last[dev], hipEventDisableTiming));
    else FLC_CHECK_HIP(hipStreamWaitEvent(st, gt.last[dev], 0));
  }
  const double step = levels > 0 ? 1.0 / (double)levels : 0.0;
  FLC_LAUNCH(STACKED ? "stacked_select" : "topk_select", topk_select_kernel<STACKED>, dim3((unsigned)grid),
             dim3(kSelThreads), 0, st, x, w, R, (long long)k, n, idx, val, codes, norm, levels, step, seed, counter);
  if (gated) FLC_CHECK_HIP(hipEventRecord(gt.last[dev], st));
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
  return launch_topk<false>(x, n, k, w, as_stream(stream), idx, val, nullptr, nullptr, 0, 0, 0);
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
  return launch_topk<true>(x, n, k, w, as_stream(stream), idx, nullptr, codes, norm, levels, seed, counter);
}

}  // extern "C"
