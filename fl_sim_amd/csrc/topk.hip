// topk.hip — exact top-k sparsifier, the stacked top-k -> 8-bit dithering codec, and the sparse
// decoders, for gfx950 (reference: fl_sim/compressors/compressors.py:284-296 and 327-365).
//
// Selection contract (compressors.py:294-295, `out[np.argsort(out)[:-K]] = 0`): keep the k largest
// *signed* values; -0 == +0; NaN is largest; among elements equal to the k-th largest value the
// highest indices are kept (stable ascending argsort order; the reference's own argsort is unstable,
// so any tie choice satisfies it — see DESIGN.md).
//
// Pipeline (one HBM read of x; every later pass touches only the ~1.2 k candidates):
//   topk_sample   1 block: 32 K strided keys -> LDS radix select -> candidate floor t_lo, chosen so
//                 that count(key >= t_lo) ~ k + 4 sigma with high probability.
//   topk_filter   one streaming read of x: each wave owns a contiguous run of x and appends its
//                 candidates (key >= t_lo) in index order to a private staging region (ballot/mbcnt
//                 compaction, no atomics, no inter-wave sync).  Algorithmic bytes 4/element.
//   topk_scan     1 block: region offsets, candidate count C, max key; C < k -> fallback mode in which
//                 every later pass reads x itself instead of the candidate list (always correct).
//   topk_round x3 radix select (11/11/10-bit digits) over the candidates; LDS histograms, global
//                 atomics, XCD-sharded last-arriver picks the digit.  Round 1 also gathers the staged
//                 regions into one ordered candidate array.
//   topk_count    per-block strict/tie counts, last arriver scans them.
//   topk_compact  ordered compaction of the kept set into idx[k] / val[k] (or, stacked, into
//                 idx[k] / codes[k] with the dithering fused in: the norm of the kept set is
//                 max(|max|, |k-th largest|), known before compaction).
//   sparse_decode dense output tile by tile: 64-ary wave search of the tile's slice of idx, LDS tile
//                 zero-fill + scatter, 16-B streaming stores.  Algorithmic bytes 4/element + 5..8/kept.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kSample = 32768;      // sample keys (128 KiB of LDS)
constexpr int kSampleThreads = 1024;
constexpr int kThreads = 256;
constexpr int kNW = kThreads / kWave;
constexpr int kStep = 1024;         // elements per wave step in the filter (4 x float4 per lane)
constexpr int kSelBlocks = 256;     // grid of the select / count / compact kernels (multiple of 8)
constexpr int kHistBins = 2048;
constexpr int kTile = 8192;         // decode tile (32 KiB of LDS)
constexpr int kShards = 8;          // XCD shards of the arrival counters

struct TopkParams {
  unsigned t_lo;
  unsigned fallback;
  long long C;
  unsigned maxkey;
  unsigned prefix;
  long long rem;
  unsigned T;
  unsigned err;
  long long need;
  long long ties_total;
  long long strict_total;
  long long k;
  float norm;
};

struct TopkWs {
  TopkParams* p;
  unsigned* tickets;          // [4][kShards + 1]
  unsigned* hist;             // [3][kHistBins]
  unsigned* region_cnt;       // [R]
  unsigned* region_max;       // [R]
  long long* region_off;      // [R + 1]
  unsigned* blk_strict;       // [kSelBlocks]
  unsigned* blk_tie;          // [kSelBlocks]
  long long* blk_strict_off;  // [kSelBlocks]
  long long* blk_tie_off;     // [kSelBlocks]
  uint2* cand;                // [cand_cap]  (idx, raw bits), ordered by idx
  uint2* stage;               // [R * region_cap]
  long long region_cap;
  long long cand_cap;
};

struct TopkGeom {
  int64_t blocks;      // filter blocks
  int64_t wave_chunk;  // elements per wave region (multiple of kStep)
  int64_t regions;     // blocks * 4
};

TopkGeom geometry(int64_t n) {
  TopkGeom g;
  int64_t blocks = cdiv(n, 4 * kStep * 8);  // >= 8 steps per wave
  if (blocks > 2048) blocks = 2048;
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
  w.region_cnt = c.take<unsigned>(g.regions);
  w.region_max = c.take<unsigned>(g.regions);
  w.region_off = c.take<long long>(g.regions + 1);
  w.blk_strict = c.take<unsigned>(kSelBlocks);
  w.blk_tie = c.take<unsigned>(kSelBlocks);
  w.blk_strict_off = c.take<long long>(kSelBlocks);
  w.blk_tie_off = c.take<long long>(kSelBlocks);
  w.region_cap = g.wave_chunk;
  w.cand_cap = n;
  w.cand = c.take<uint2>((size_t)n);
  w.stage = c.take<uint2>((size_t)g.regions * g.wave_chunk);
  *need = c.off;
  return w;
}

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------

// One wave: given a histogram h[NB] in LDS and a rank `rem` (1-based, counted from the top),
// find the bin holding that rank and the rank within it.  Lane 0 writes *digit / *new_rem.
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

// XCD-sharded last-arriver: returns true in exactly one block, after every block called it.
// Call from all threads; contains __syncthreads().  Every storing wave must have drained before.
__device__ bool last_arriver(unsigned* counters /* kShards + 1 */) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nb = gridDim.x, shard = blockIdx.x % kShards;
    const unsigned shard_size = (nb - shard + kShards - 1) / kShards;
    const unsigned active_shards = nb < (unsigned)kShards ? nb : (unsigned)kShards;
    int last = 0;
    if (arrive(&counters[shard]) == shard_size - 1) {
      acquire_agent();
      last = arrive(&counters[kShards]) == active_shards - 1;
    }
    s_last = last;
  }
  __syncthreads();
  if (s_last) {
    if (threadIdx.x == 0) acquire_agent();
    __syncthreads();
  }
  return s_last != 0;
}

__device__ __forceinline__ unsigned ld_mem(unsigned* p) {
  return __hip_atomic_fetch_add(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------
// K0: sample -> candidate floor
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kSampleThreads) void topk_sample_kernel(const float* __restrict__ x, int64_t n, int S,
                                                                     long long rank_lo, int take_all, TopkWs w) {
  extern __shared__ __attribute__((aligned(16))) unsigned s_keys[];  // [S]
  __shared__ unsigned s_hist[256];
  __shared__ unsigned s_digit;
  __shared__ long long s_rem;
  __shared__ unsigned s_err;
  if (take_all) {
    if (threadIdx.x == 0) w.p->t_lo = 0u;
    return;
  }
  for (int j = threadIdx.x; j < S; j += kSampleThreads) {
    const int64_t pos = (S == n) ? (int64_t)j : (int64_t)(((double)j + 0.5) * (double)n / (double)S);
    s_keys[j] = order_key(__float_as_uint(x[pos < n ? pos : n - 1]));
  }
  unsigned prefix = 0;
  long long rem = rank_lo;
  if (threadIdx.x == 0) s_err = 0;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    if (threadIdx.x < 256) s_hist[threadIdx.x] = 0;
    __syncthreads();
    for (int j = threadIdx.x; j < S; j += kSampleThreads) {
      const unsigned key = s_keys[j];
      if (pass == 0 || (key >> (shift + 8)) == prefix) atomicAdd(&s_hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kWave) wave_select_from_top<256>(s_hist, rem, &s_digit, &s_rem, &s_err);
    __syncthreads();
    prefix = (prefix << 8) | s_digit;
    rem = s_rem;
    __syncthreads();
  }
  if (threadIdx.x == 0) w.p->t_lo = prefix;
}

// ------------------------------------------------------------------------------------------------
// K1: streaming filter
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void topk_filter_kernel(const float* __restrict__ x, int64_t n,
                                                               int64_t wave_chunk, TopkWs w) {
  const unsigned t_lo = w.p->t_lo;
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
      const unsigned any = (unsigned)((m0 | m1 | m2 | m3) != 0ull);
      if (any) {
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
// K1.5: region scan (1 block)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void topk_scan_kernel(int64_t regions, int64_t n, long long k, TopkWs w) {
  __shared__ long long s_red[16];
  __shared__ unsigned s_max[16];
  long long running = 0;
  unsigned mx = 0;
  for (int64_t base = 0; base < regions; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const long long v = i < regions ? (long long)w.region_cnt[i] : 0;
    if (i < regions) mx = w.region_max[i] > mx ? w.region_max[i] : mx;
    long long tot;
    const long long ex = block_excl_scan<long long, 16>(v, s_red, &tot);
    if (i < regions) w.region_off[i] = running + ex;
    running += tot;
  }
  mx = wave_max_u32(mx);
  if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = mx;
  // zero the select state (histograms, tickets) for this call
  for (int i = threadIdx.x; i < 3 * kHistBins; i += 1024) w.hist[i] = 0u;
  if (threadIdx.x < 4 * (kShards + 1)) w.tickets[threadIdx.x] = 0u;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned m = 0;
    for (int i = 0; i < 16; ++i) m = s_max[i] > m ? s_max[i] : m;
    w.region_off[regions] = running;
    const unsigned fb = running < k ? 1u : 0u;
    w.p->fallback = fb;
    w.p->C = fb ? (long long)n : running;
    w.p->maxkey = m;
    w.p->prefix = 0u;
    w.p->rem = k;
    w.p->k = k;
    w.p->err = 0u;
  }
}


// 64-ary search by one wave: last r in [0, R) with off[r] <= v (off nondecreasing, off[R] > v)
__device__ long long wave_region_search(const long long* __restrict__ off, long long R, long long v) {
  const int lane = threadIdx.x & (kWave - 1);
  long long lo = 0, hi = R;
  while (hi - lo > 1) {
    const long long stride = (hi - lo + kWave - 1) / kWave;
    const long long p = lo + (long long)lane * stride;
    const bool le = p < hi && off[p] <= v;
    const int cnt = __popcll(__ballot(le));
    const long long nlo = lo + (long long)(cnt - 1) * stride;
    hi = nlo + stride < hi ? nlo + stride : hi;
    lo = nlo;
  }
  return lo;
}

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
// K2: radix-select rounds over the candidates (3 x {11, 11, 10} bits)
// ------------------------------------------------------------------------------------------------
template <int SHIFT, int BITS, bool FIRST, bool LAST>
__global__ __launch_bounds__(kThreads) void topk_round_kernel(const float* __restrict__ x, TopkWs w, int round,
                                                              long long regions) {
  __shared__ unsigned s_hist[kHistBins];
  __shared__ long long s_r0;
  __shared__ unsigned s_digit;
  __shared__ long long s_rem;
  constexpr unsigned kMask = (1u << BITS) - 1u;
  const long long C = w.p->C;
  const bool fb = w.p->fallback != 0;
  const unsigned prefix = FIRST ? 0u : w.p->prefix;
  const long long per = (C + gridDim.x - 1) / gridDim.x;
  const long long v0 = (long long)blockIdx.x * per;
  const long long v1 = v0 + per < C ? v0 + per : C;
  for (int i = threadIdx.x; i < (1 << BITS); i += kThreads) s_hist[i] = 0u;
  if (FIRST && !fb && threadIdx.x < kWave && v0 < v1) {
    const long long r0 = wave_region_search(w.region_off, regions, v0);
    if (threadIdx.x == 0) s_r0 = r0;
  }
  __syncthreads();

  if (fb) {
    for (long long c = v0 + threadIdx.x; c < v1; c += kThreads) {
      const unsigned key = order_key(__float_as_uint(x[c]));
      if (FIRST || ((unsigned long long)key >> (SHIFT + BITS)) == prefix) atomicAdd(&s_hist[(key >> SHIFT) & kMask], 1u);
    }
  } else if (FIRST) {
    long long r = s_r0;
    for (long long c = v0 + threadIdx.x; c < v1; c += kThreads) {
      while (w.region_off[r + 1] <= c) ++r;
      const uint2 e = w.stage[r * w.region_cap + (c - w.region_off[r])];
      w.cand[c] = e;
      const unsigned key = order_key(e.y);
      atomicAdd(&s_hist[(key >> SHIFT) & kMask], 1u);
    }
  } else {
    for (long long c = v0 + threadIdx.x; c < v1; c += kThreads) {
      const unsigned key = order_key(w.cand[c].y);
      if (((unsigned long long)key >> (SHIFT + BITS)) == prefix) atomicAdd(&s_hist[(key >> SHIFT) & kMask], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < (1 << BITS); i += kThreads)
    if (s_hist[i]) atomicAdd(&w.hist[round * kHistBins + i], s_hist[i]);
  drain_stores();
  if (!last_arriver(&w.tickets[round * (kShards + 1)])) return;
  for (int i = threadIdx.x; i < (1 << BITS); i += kThreads) s_hist[i] = ld_mem(&w.hist[round * kHistBins + i]);
  __syncthreads();
  if (threadIdx.x < kWave) wave_select_from_top<(1 << BITS)>(s_hist, w.p->rem, &s_digit, &s_rem, &w.p->err);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned np = (prefix << BITS) | s_digit;
    w.p->prefix = np;
    w.p->rem = s_rem;
    if (LAST) {
      w.p->T = np;
      w.p->need = s_rem;
      w.p->ties_total = s_hist[s_digit];
    }
  }
}

__device__ __forceinline__ uint2 source_entry(const float* __restrict__ x, const TopkWs& w, bool fb, long long c) {
  if (fb) return make_uint2((unsigned)c, __float_as_uint(x[c]));
  return w.cand[c];
}

// ------------------------------------------------------------------------------------------------
// K3: per-block strict / tie counts + scan by the last arriver
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void topk_count_kernel(const float* __restrict__ x, TopkWs w) {
  __shared__ long long s_red[kNW];
  const long long C = w.p->C;
  const bool fb = w.p->fallback != 0;
  const unsigned T = w.p->T;
  const long long per = (C + gridDim.x - 1) / gridDim.x;
  const long long v0 = (long long)blockIdx.x * per;
  const long long v1 = v0 + per < C ? v0 + per : C;
  long long st = 0, ti = 0;
  for (long long c = v0 + threadIdx.x; c < v1; c += kThreads) {
    const unsigned key = order_key(source_entry(x, w, fb, c).y);
    st += key > T;
    ti += key == T;
  }
  // pack both counts in one scan value: strict in the high 32 bits (counts < 2^31)
  const long long both = block_sum<long long, kNW>((st << 32) | ti, s_red);
  if (threadIdx.x == 0) {
    st_sc1(&w.blk_strict[blockIdx.x], (unsigned)(both >> 32));
    st_sc1(&w.blk_tie[blockIdx.x], (unsigned)(both & 0xffffffffll));
  }
  drain_stores();
  if (!last_arriver(&w.tickets[3 * (kShards + 1)])) return;
  // gridDim.x == kSelBlocks == kThreads: one block per thread
  const long long vs = threadIdx.x < (int)gridDim.x ? (long long)ld_mem(&w.blk_strict[threadIdx.x]) : 0;
  const long long vt = threadIdx.x < (int)gridDim.x ? (long long)ld_mem(&w.blk_tie[threadIdx.x]) : 0;
  long long tot_s, tot_t;
  const long long es = block_excl_scan<long long, kNW>(vs, s_red, &tot_s);
  const long long et = block_excl_scan<long long, kNW>(vt, s_red, &tot_t);
  if (threadIdx.x < (int)gridDim.x) {
    w.blk_strict_off[threadIdx.x] = es;
    w.blk_tie_off[threadIdx.x] = et;
  }
  if (threadIdx.x == 0) {
    w.p->strict_total = tot_s;
    w.p->ties_total = tot_t;
    if (tot_s + w.p->need != w.p->k || w.p->need > tot_t) w.p->err |= 2u;
  }
}

// ------------------------------------------------------------------------------------------------
// K4: ordered compaction of the kept set (plain top-k, or fused 8-bit dithering for the stack)
// ------------------------------------------------------------------------------------------------
template <bool STACKED>
__global__ __launch_bounds__(kThreads) void topk_compact_kernel(const float* __restrict__ x, TopkWs w,
                                                                int* __restrict__ idx_out, float* __restrict__ val_out,
                                                                uint8_t* __restrict__ code_out, float* __restrict__ norm_out,
                                                                int levels, double step, uint64_t seed, uint64_t counter) {
  __shared__ unsigned s_ws[2][kNW], s_wt[2][kNW];
  const long long C = w.p->C;
  const bool fb = w.p->fallback != 0;
  const unsigned T = w.p->T;
  const long long skip = w.p->ties_total - w.p->need;  // ties with rank < skip are dropped
  const long long kk = w.p->k;
  const long long per = (C + gridDim.x - 1) / gridDim.x;
  const long long v0 = (long long)blockIdx.x * per;
  const long long v1 = v0 + per < C ? v0 + per : C;
  long long run_s = w.blk_strict_off[blockIdx.x];
  long long run_t = w.blk_tie_off[blockIdx.x];
  float nrm = 0.0f;
  if (STACKED) {
    const float a = fabsf(key_value(w.p->maxkey)), b = fabsf(key_value(T));
    nrm = (isnan(a) || isnan(b)) ? __uint_as_float(0x7fc00000u) : (a > b ? a : b);
    if (blockIdx.x == 0 && threadIdx.x == 0) *norm_out = nrm;
  }
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int par = 0;
  for (long long base = v0; base < v1; base += kThreads, par ^= 1) {
    const long long c = base + threadIdx.x;
    const bool in = c < v1;
    const uint2 e = in ? source_entry(x, w, fb, c) : make_uint2(0u, 0u);
    const unsigned key = order_key(e.y);
    const bool is_s = in && key > T, is_t = in && key == T;
    const unsigned long long ms = __ballot(is_s), mt = __ballot(is_t);
    if (lane == 0) {
      s_ws[par][wid] = (unsigned)__popcll(ms);
      s_wt[par][wid] = (unsigned)__popcll(mt);
    }
    __syncthreads();
    long long ws_before = 0, wt_before = 0, tot_s = 0, tot_t = 0;
#pragma unroll
    for (int q = 0; q < kNW; ++q) {
      ws_before += q < wid ? s_ws[par][q] : 0u;
      wt_before += q < wid ? s_wt[par][q] : 0u;
      tot_s += s_ws[par][q];
      tot_t += s_wt[par][q];
    }
    const long long s_before = run_s + ws_before + __popcll(ms & lt);
    const long long t_before = run_t + wt_before + __popcll(mt & lt);
    const bool keep = is_s || (is_t && t_before >= skip);
    const long long pos = s_before + (t_before > skip ? t_before - skip : 0);
    if (keep && pos >= 0 && pos < kk) {
      idx_out[pos] = (int)e.x;
      if (STACKED) {
        const float v = __uint_as_float(e.y);
        uint32_t code = 0u;
        if (v != 0.0f) {
          if (!(nrm > 0.0f && nrm <= 3.402823466e38f)) {
            code = 1u;
          } else {
            const float y = fabsf(v) / nrm;
            const int j = level_lower_bound<0>(y, levels, step);
            const int sl = j > 0 ? j - 1 : 0;
            const double lo = level_value<0>(sl, levels, step), hi = level_value<0>(sl + 1, levels, step);
            const double p = ((double)y - hi) / (lo - hi);
            const U4 r4 = philox_group((uint64_t)e.x >> 2, seed, counter);
            const double u = u01(pick(r4, (int)(e.x & 3u)));
            const int lvl = (u < p) ? sl : sl + 1;
            code = ((e.y >> 31) << 7) | (uint32_t)lvl;
          }
        }
        code_out[pos] = (uint8_t)code;
      } else {
        val_out[pos] = __uint_as_float(e.y);
      }
    }
    run_s += tot_s;
    run_t += tot_t;
  }
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

bool g_sample_attr_set = false;

int launch_select(const float* x, int64_t n, int64_t k, const TopkWs& w, hipStream_t st) {
  const TopkGeom g = geometry(n);
  const SampleSetup ss = sample_setup(n, k);
  const size_t lds = (size_t)ss.S * sizeof(unsigned);
  if (!g_sample_attr_set) {
    FLC_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(topk_sample_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kSample * sizeof(unsigned))));
    g_sample_attr_set = true;
  }
  FLC_LAUNCH("topk_sample", topk_sample_kernel, dim3(1), dim3(kSampleThreads), lds, st, x, n, ss.S, ss.rank_lo,
             ss.take_all, w);
  FLC_LAUNCH("topk_filter", topk_filter_kernel, dim3((unsigned)g.blocks), dim3(kThreads), 0, st, x, n, g.wave_chunk, w);
  FLC_LAUNCH("topk_scan", topk_scan_kernel, dim3(1), dim3(1024), 0, st, g.regions, n, (long long)k, w);
  FLC_LAUNCH("topk_round", (topk_round_kernel<21, 11, true, false>), dim3(kSelBlocks), dim3(kThreads), 0, st, x, w, 0,
             (long long)g.regions);
  FLC_LAUNCH("topk_round", (topk_round_kernel<10, 11, false, false>), dim3(kSelBlocks), dim3(kThreads), 0, st, x, w, 1,
             (long long)g.regions);
  FLC_LAUNCH("topk_round", (topk_round_kernel<0, 10, false, true>), dim3(kSelBlocks), dim3(kThreads), 0, st, x, w, 2,
             (long long)g.regions);
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
