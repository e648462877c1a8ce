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
//   sample_select  1 block, keys in registers: two fixed 11-bit digit passes locate the sample
//                  quantiles at ranks m + 4 sqrt(m) + 16 and m - 4 sqrt(m) - 16 (m = k S / n): the
//                  candidate floor t_lo (count(key >= t_lo) ~ k + 4 sigma, so ~1.22 k candidates at
//                  k/n = 1 %) and a ceiling t_hi that very likely lies above the k-th largest key.
//   filter         the HBM pass: one-shot 64 KB blocks (4 waves x 16 float4 per lane, all loads in
//                  flight at once); each block appends its candidates in index order to a private
//                  staging region (ballot/mbcnt compaction, one LDS exchange of wave counts, no
//                  atomics).  Algorithmic bytes: 4 per element.
//   select         ONE persistent launch, one 1024-thread block per CU:
//                    P0  region offsets in LDS (every block) and the candidate count C;
//                    rounds  gather the staged candidates (round 0) into an index-ordered array and an
//                        LDS key cache (and reduce the max key), then 2048-bin radix rounds over the
//                        live key range (round 0: [t_lo, t_hi), keys above it counted apart) until
//                        the exact k-th largest key T is resolved (usually 2 rounds);
//                    counts  strict / tie counts per block come from the resolving round's local
//                        histogram (no extra pass), scanned by the barrier leader;
//                    compaction  ordered write of idx[k] / val[k], or, stacked, idx[k] / codes[k]
//                        with the dithering fused in (norm of the kept set = max(|max key|, |T|)).
//                  Rounds are separated by grid barriers: every block raises its own arrival flag,
//                  block 0 polls them, runs the serial "leader" step and publishes a generation word.
//                  C < k switches every phase to "fallback" mode, reading x itself (always correct).
// Cross-block hand-offs inside a launch go through memory-side atomics only (histogram adds, flag
// and state exchanges, RMW reads); candidates are re-read only by the thread that wrote them.  Spins
// are bounded (error flag), and the host serialises the persistent launches of different streams so
// two of them never compete for residency.
#include <hip/hip_runtime.h>
#include <math.h>

#include <stdlib.h>

#include <algorithm>
#include <mutex>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

#ifndef FLC_FILTER_VARIANT
#define FLC_FILTER_VARIANT 0  // != 0 only in calibration builds (tools/calib_variants.sh): results invalid
#endif

constexpr int kSample = 32768;
constexpr int kSelectThreads = 1024;
constexpr int kSamplePerThread = kSample / kSelectThreads;  // 32
constexpr int kThreads = 256;
constexpr int kFNW = kThreads / kWave;       // filter: 4 waves per block
constexpr int kStepF4 = 8;                   // float4 per lane per wave step
constexpr int kWaveSpan = kStepF4 * 256;     // 2048 elements per wave step (8 KB)
constexpr int kBlockSpan = kFNW * kWaveSpan; // 8192 elements: filter chunks are multiples of this
constexpr int kSelThreads = 1024;            // persistent select: one block of 16 waves per CU
constexpr int kSelNW = kSelThreads / kWave;
constexpr int kMaxSelBlocks = 1024;
constexpr int kHistBits = 11;
constexpr int kHistBins = 1 << kHistBits;
constexpr int kHistStride = kHistBins + 64;  // a round's bins + its "above the range" counter
constexpr int kMaxRounds = 6;
#ifndef FLC_MAX_REGIONS
#define FLC_MAX_REGIONS 16384
#endif
constexpr int kMaxRegions = FLC_MAX_REGIONS; // filter blocks = staging regions
constexpr int kRegionsPerThread = kMaxRegions / kSelThreads;  // 16 (P0 LDS scan)
constexpr int kKeyCache = 14336;             // candidates per select block kept in LDS
constexpr int kWcCap = 512;                  // block regions whose wave counts a select block keeps in LDS
constexpr int kFlagStride = 16;              // one 64-B line per barrier arrival flag

struct TopkParams {
  unsigned t_lo;             // candidate floor (sample_select -> filter, select)
  unsigned pad;
  unsigned long long t_hi;   // likely ceiling of the k-th largest key (<= 2^32)
};

// state published by the barrier leader of the select launch (64-bit words, memory-side atomics
// only); zeroed per call by the filter
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
  unsigned long long rounds;
};

struct TopkWs {
  TopkParams* p;
  SelState* st;
  unsigned* flags;              // [kMaxSelBlocks * kFlagStride] barrier arrival flags
  unsigned* hist;               // [kMaxRounds][kHistStride]
  unsigned* sample;             // [kSample]
  unsigned* region_cnt;         // [R]      candidates per filter block
  unsigned* wave_cnt;           // [4 R]    candidates per wave quarter of a block
  unsigned long long* blk_cnt;  // [kMaxSelBlocks]  strict << 32 | tie
  unsigned long long* blk_off;  // [kMaxSelBlocks]
  unsigned* cand_idx;           // [n]  ordered by index
  unsigned* cand_raw;           // [n]  raw fp32 bits (only when the LDS key cache is too small)
  uint2* stage;                 // [4 R * dcap]  (idx, raw): the first dcap candidates of each wave, dense
  uint2* spill;                 // [4 R * qc]    the rest (worst case, rarely touched)
  long long dcap;               // dense staging entries per wave (~2x the expected candidates)
  long long qc;                 // elements per wave quarter of a filter block (chunk / 4)
  unsigned long long* stamps;   // [16] diagnostic build only (FLC_SELECT_STAMPS)
  unsigned long long* trace;    // [kMaxRounds * 8] leader's per-round record (diagnostics)
};

struct TopkGeom {
  int64_t chunk;    // elements per filter block (multiple of kBlockSpan)
  int64_t regions;  // filter blocks launched, a multiple of 4 (trailing blocks may be empty)
};

TopkGeom geometry(int64_t n) {
  TopkGeom g;
  int64_t blocks = cdiv(n, kBlockSpan);
  if (blocks > kMaxRegions) blocks = kMaxRegions;
  if (blocks < 1) blocks = 1;
  g.chunk = (int64_t)align_up((size_t)cdiv(n, blocks), kBlockSpan);
  g.regions = (int64_t)align_up((size_t)cdiv(n, g.chunk), 4);
  return g;
}

struct SampleSetup {
  int S;
  long long rank_lo, rank_hi;
  int take_all;
};

SampleSetup sample_setup(int64_t n, int64_t k) {
  SampleSetup s;
  s.S = (int)(n < kSample ? n : kSample);
  const double m = (double)s.S * (double)k / (double)n;
  s.rank_lo = (long long)ceil(m + 4.0 * sqrt(m) + 16.0);
  const double rh = floor(m - 4.0 * sqrt(m) - 16.0);
  s.rank_hi = rh >= 1.0 ? (long long)rh : 0;
  s.take_all = (s.rank_lo >= s.S) ? 1 : 0;
  if (s.take_all) s.rank_lo = s.S;
  return s;
}

// dense staging per wave: twice the expected candidate count (the sample's floor admits ~rank_lo / S of
// the elements) plus slack; waves with more candidates continue in their worst-case spill region.
// Keeping the common case dense keeps the appends of all active waves inside a few MB (TLB / DRAM
// page locality); a worst-case-sized region per wave made the staging writes 3-4x slower.
int64_t dense_cap(int64_t n, int64_t k) {
  const TopkGeom g = geometry(n);
  const int64_t qc = g.chunk / kFNW;
  const SampleSetup ss = sample_setup(n, k < 1 ? 1 : k);
  if (ss.take_all) return qc;
  const double frac = std::min(1.0, (double)ss.rank_lo / (double)ss.S);
  const int64_t cap = (int64_t)align_up((size_t)(2.0 * frac * (double)qc) + 64, 32);
  return cap < qc ? cap : qc;
}

TopkWs carve_topk(void* ws, size_t bytes, int64_t n, int64_t k, size_t* need) {
  const TopkGeom g = geometry(n);
  Carver c(ws, bytes);
  TopkWs w;
  w.p = c.take<TopkParams>(1);
  w.stamps = c.take<unsigned long long>(16);
  w.st = c.take<SelState>(1);
  w.trace = c.take<unsigned long long>(kMaxRounds * 8);
  w.flags = c.take<unsigned>((size_t)kMaxSelBlocks * kFlagStride);
  w.hist = c.take<unsigned>((size_t)kMaxRounds * kHistStride);
  w.sample = c.take<unsigned>(kSample);
  w.region_cnt = c.take<unsigned>(g.regions);
  w.wave_cnt = c.take<unsigned>(4 * g.regions);
  w.blk_cnt = c.take<unsigned long long>(kMaxSelBlocks);
  w.blk_off = c.take<unsigned long long>(kMaxSelBlocks);
  w.cand_idx = c.take<unsigned>((size_t)n + 4);
  w.cand_raw = c.take<unsigned>((size_t)n + 4);
  // region stride = chunk + a 2304-B skew: with a power-of-two stride every block's appends would land
  // on the same HBM channel (measured: 34 us instead of 8 us of staging writes on 1 GiB)
  w.qc = g.chunk / kFNW;
  w.dcap = dense_cap(n, k);
  w.stage = c.take<uint2>((size_t)g.regions * kFNW * w.dcap);
  w.spill = c.take<uint2>((size_t)g.regions * kFNW * w.qc);
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

// memory-side reads / writes of words other blocks update with atomics in this launch
__device__ __forceinline__ unsigned ld_mem(unsigned* p) {
  return __hip_atomic_fetch_add(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_mem64(unsigned long long* p) {
  return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_mem64(unsigned long long* p, unsigned long long v) {
  (void)__hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
// sample -> candidate floor and ceiling
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void topk_sample_gather_kernel(const float* __restrict__ x, int64_t n, int S,
                                                                      TopkWs w) {
  const int j = blockIdx.x * kThreads + threadIdx.x;
  if (j >= S) return;
  const int64_t pos = (S == n) ? (int64_t)j : (int64_t)(((double)j + 0.5) * (double)n / (double)S);
  w.sample[j] = order_key(__float_as_uint(x[pos < n ? pos : n - 1]));
}

// Two fixed digit passes (key bits 31..21, then 20..10) per target rank.  Only the count guarantees
// matter: every sample key in or above the floor's bin is >= t_lo (so >= rank_lo of them), and fewer
// than rank_hi sample keys are >= t_hi (the end of the ceiling's bin).
__global__ __launch_bounds__(kSelectThreads) void topk_sample_select_kernel(int S, long long rank_lo,
                                                                            long long rank_hi, int take_all,
                                                                            TopkWs w) {
  __shared__ unsigned s_hist[2][kHistBins];
  __shared__ unsigned s_digit[2];
  __shared__ long long s_rem[2];
  __shared__ unsigned s_err;
  const int tid = threadIdx.x, wid = tid >> 6;
  if (take_all) {
    if (tid == 0) {
      w.p->t_lo = 0u;
      w.p->t_hi = 1ull << 32;
    }
    return;
  }
  const bool two = rank_hi > 0;
  unsigned keys[kSamplePerThread];
#pragma unroll
  for (int i = 0; i < kSamplePerThread; ++i) {
    const int j = tid + i * kSelectThreads;
    keys[i] = j < S ? w.sample[j] : 0u;
  }
  for (int i = tid; i < 2 * kHistBins; i += kSelectThreads) (&s_hist[0][0])[i] = 0u;
  if (tid == 0) s_err = 0;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kSamplePerThread; ++i) hist_add(s_hist[0], keys[i] >> 21, tid + i * kSelectThreads < S);
  __syncthreads();
  if (wid == 0) wave_select_from_top<kHistBins>(s_hist[0], rank_lo, &s_digit[0], &s_rem[0], &s_err);
  else if (wid == 1 && two) wave_select_from_top<kHistBins>(s_hist[0], rank_hi, &s_digit[1], &s_rem[1], &s_err);
  __syncthreads();
  const unsigned d0 = s_digit[0], d1 = two ? s_digit[1] : 0u;
  const long long r0 = s_rem[0], r1 = two ? s_rem[1] : 0;
  for (int i = tid; i < 2 * kHistBins; i += kSelectThreads) (&s_hist[0][0])[i] = 0u;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kSamplePerThread; ++i) {
    const bool in = tid + i * kSelectThreads < S;
    const unsigned hi = keys[i] >> 21, bin = (keys[i] >> 10) & (kHistBins - 1);
    hist_add(s_hist[0], bin, in && hi == d0);
    if (two) hist_add(s_hist[1], bin, in && hi == d1);
  }
  __syncthreads();
  if (wid == 0) wave_select_from_top<kHistBins>(s_hist[0], r0, &s_digit[0], &s_rem[0], &s_err);
  else if (wid == 1 && two) wave_select_from_top<kHistBins>(s_hist[1], r1, &s_digit[1], &s_rem[1], &s_err);
  __syncthreads();
  if (tid == 0) {
    unsigned t_lo = (d0 << 21) | (s_digit[0] << 10);
    unsigned long long t_hi = two ? (unsigned long long)((d1 << 21) | (s_digit[1] << 10)) + 1024ull : 1ull << 32;
    if (s_err) {  // cannot happen for 0 < rank <= S; stay correct anyway: everything is a candidate
      t_lo = 0u;
      t_hi = 1ull << 32;
    }
    w.p->t_lo = t_lo;
    w.p->t_hi = t_hi;
  }
}

// ------------------------------------------------------------------------------------------------
// streaming filter (the one HBM pass over x)
// ------------------------------------------------------------------------------------------------
// candidate test on values: key(v) >= t_lo  <=>  v >= t_lo_value  or  v is NaN (NaN is the largest
// key; -0 == +0 holds for the float compare as for the keys)
__device__ __forceinline__ float floor_value(unsigned t_lo) {
  return t_lo <= 0x007fffffu ? -__builtin_inff() : key_value(t_lo);  // keys below -inf: negative NaNs
}

// key(v) >= t_lo as one unordered compare: true for v >= tf and for NaN
__device__ __forceinline__ bool is_cand(float a, float tf) { return !(a < tf); }

// one wave's 4096-element span of a block step: 16 float4 per lane (q-major: lane l, step q ->
// elements 256q + 4l + c).  A partial span (the last block only) clamps each float4 to the last one
// holding valid data (16-B aligned, so it never crosses a page); `lim` masks everything past b_end.
template <bool FULL>
__device__ __forceinline__ void filter_load(const float* __restrict__ x, int64_t wb, int64_t b_end, int lane,
                                            float4 (&v)[kStepF4]) {
  if (FULL) {
#pragma unroll
    for (int q = 0; q < kStepF4; ++q) v[q] = ld_stream(x + wb + 256 * q + 4 * lane);
  } else {
    const int64_t last4 = (b_end - 1) & ~(int64_t)3;
#pragma unroll
    for (int q = 0; q < kStepF4; ++q) {
      const int64_t e = wb + 256 * q + 4 * lane;
      v[q] = *reinterpret_cast<const float4*>(x + (e < last4 ? e : last4));
    }
  }
}

template <bool FULL>
__device__ __forceinline__ bool in_span(int o, int lim) { return FULL || o < lim; }

template <bool FULL>
__device__ __forceinline__ void cand4(const float4& v, float tf, int o, int lim, bool& f0, bool& f1, bool& f2,
                                      bool& f3) {
  f0 = is_cand(v.x, tf) && in_span<FULL>(o + 0, lim);
  f1 = is_cand(v.y, tf) && in_span<FULL>(o + 1, lim);
  f2 = is_cand(v.z, tf) && in_span<FULL>(o + 2, lim);
  f3 = is_cand(v.w, tf) && in_span<FULL>(o + 3, lim);
}

// the wave's candidate count: one compare per element into a wave mask, scalar popcounts
template <bool FULL>
__device__ __forceinline__ unsigned filter_count(const float4 (&v)[kStepF4], float tf, int lim, int lane) {
  unsigned cnt = 0;
#pragma unroll
  for (int q = 0; q < kStepF4; ++q) {
    bool f0, f1, f2, f3;
    cand4<FULL>(v[q], tf, 256 * q + 4 * lane, lim, f0, f1, f2, f3);
    cnt += __popcll(__ballot(f0)) + __popcll(__ballot(f1)) + __popcll(__ballot(f2)) + __popcll(__ballot(f3));
  }
  return cnt;
}

#ifndef FLC_STAGE_NT
#define FLC_STAGE_NT 0
#endif
__device__ __forceinline__ void st_stage(uint2* dst, unsigned idx, float v) {
  if (FLC_STAGE_NT) {
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    u32x2 t = {idx, __float_as_uint(v)};
    __builtin_nontemporal_store(t, reinterpret_cast<u32x2*>(dst));
  } else {
    *dst = make_uint2(idx, __float_as_uint(v));
  }
}

// ordered append from position `pos` (element order within a step q: lane-major, then the 4 components)
template <bool FULL>
__device__ __forceinline__ void filter_write(const float4 (&v)[kStepF4], float tf, int lim, int lane, unsigned wbu,
                                             unsigned pos, uint2* __restrict__ out, uint2* __restrict__ spill,
                                             unsigned dcap) {
#pragma unroll
  for (int q = 0; q < kStepF4; ++q) {
    bool f0, f1, f2, f3;
    cand4<FULL>(v[q], tf, 256 * q + 4 * lane, lim, f0, f1, f2, f3);
    const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1), m2 = __ballot(f2), m3 = __ballot(f3);
    if ((m0 | m1 | m2 | m3) != 0ull) {
      unsigned p = pos;
      p = __builtin_amdgcn_mbcnt_hi((unsigned)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m0, p));
      p = __builtin_amdgcn_mbcnt_hi((unsigned)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m1, p));
      p = __builtin_amdgcn_mbcnt_hi((unsigned)(m2 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m2, p));
      p = __builtin_amdgcn_mbcnt_hi((unsigned)(m3 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m3, p));
      if (f0 | f1 | f2 | f3) {
        const unsigned e = wbu + (unsigned)(256 * q + 4 * lane);
        if (f0) { st_stage(p < dcap ? out + p : spill + (p - dcap), e + 0u, v[q].x); ++p; }
        if (f1) { st_stage(p < dcap ? out + p : spill + (p - dcap), e + 1u, v[q].y); ++p; }
        if (f2) { st_stage(p < dcap ? out + p : spill + (p - dcap), e + 2u, v[q].z); ++p; }
        if (f3) st_stage(p < dcap ? out + p : spill + (p - dcap), e + 3u, v[q].w);
      }
      pos += __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
    }
  }
}

// one wave step (2048 elements, already loaded into v): count, append in order after the wave's
// earlier candidates
template <bool FULL>
__device__ __forceinline__ void filter_process(const float4 (&v)[kStepF4], int64_t wb, int64_t q_end, float tf,
                                               uint2* __restrict__ out, uint2* __restrict__ spill, unsigned dcap,
                                               unsigned& run) {
  const int lane = threadIdx.x & (kWave - 1);
  const int lim = FULL ? kWaveSpan : (int)(q_end > wb ? (q_end - wb < kWaveSpan ? q_end - wb : kWaveSpan) : 0);
  const unsigned wcnt = filter_count<FULL>(v, tf, lim, lane);
#if FLC_FILTER_VARIANT == 2  // calibration only: loads + count, no append
  run += wcnt;
  return;
#endif
  // re-derive the masks rather than keep them live across the count (an opaque copy of the floor
  // stops the compiler from reusing the count pass's compares)
  float tf2 = tf;
  asm volatile("" : "+v"(tf2));
  if (wcnt != 0u) filter_write<FULL>(v, tf2, lim, lane, (unsigned)wb, run, out, spill, dcap);
  run += wcnt;
}

// Each wave owns a contiguous quarter of its block's chunk and appends to its own quarter of the
// block's staging region: no barrier between the waves.  The block total (for the select's region
// scan) is formed by the last wave to finish, via one 64-bit LDS ticket (waves done << 32 | count).
__global__ __launch_bounds__(kThreads) void topk_filter_kernel(const float* __restrict__ x, int64_t n, int64_t chunk,
                                                               int sel_grid, TopkWs w) {
  __shared__ unsigned long long s_tick;
  const float tf = floor_value(w.p->t_lo);
  if (threadIdx.x == 0) s_tick = 0ull;
  if (blockIdx.x == 0) {  // reset the select state of this call (read by the next launch)
    for (int i = threadIdx.x; i < kMaxRounds * kHistStride; i += kThreads) w.hist[i] = 0u;
    for (int i = threadIdx.x; i < sel_grid; i += kThreads) w.flags[i * kFlagStride] = 0u;
    if (threadIdx.x < (int)(sizeof(SelState) / 8)) reinterpret_cast<unsigned long long*>(w.st)[threadIdx.x] = 0ull;
  }
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x >> 6;
  const int64_t qc = chunk / kFNW;
  const int64_t q_begin = (int64_t)blockIdx.x * chunk + wid * qc;
  const int64_t q_end = q_begin + qc < n ? q_begin + qc : n;
  const int64_t wave_id = (int64_t)blockIdx.x * kFNW + wid;
  uint2* __restrict__ out = w.stage + wave_id * w.dcap;
  uint2* __restrict__ spill = w.spill + wave_id * qc;
  const unsigned dcap = (unsigned)w.dcap;
  unsigned run = 0;
  // software pipeline over the wave's full steps: step i + 1 is in flight while step i is processed
  const int64_t nfull = q_end > q_begin ? (q_end - q_begin) / kWaveSpan : 0;
  int64_t s = q_begin, i = 0;
  float4 va[kStepF4], vb[kStepF4];
  if (nfull > 0) filter_load<true>(x, s, q_end, lane, va);
  for (; i + 2 <= nfull; i += 2) {
    filter_load<true>(x, s + kWaveSpan, q_end, lane, vb);
    filter_process<true>(va, s, q_end, tf, out, spill, dcap, run);
    s += kWaveSpan;
    if (i + 2 < nfull) filter_load<true>(x, s + kWaveSpan, q_end, lane, va);
    filter_process<true>(vb, s, q_end, tf, out, spill, dcap, run);
    s += kWaveSpan;
  }
  if (i < nfull) {
    filter_process<true>(va, s, q_end, tf, out, spill, dcap, run);
    s += kWaveSpan;
  }
  if (s < q_end) {
    filter_load<false>(x, s, q_end, lane, va);
    filter_process<false>(va, s, q_end, tf, out, spill, dcap, run);
  }
  if (lane == 0) {
    w.wave_cnt[blockIdx.x * kFNW + wid] = run;
    const unsigned long long old = atomicAdd(&s_tick, (1ull << 32) | run);
    if ((old >> 32) == (unsigned long long)(kFNW - 1)) w.region_cnt[blockIdx.x] = (unsigned)old + run;
  }
}

// ------------------------------------------------------------------------------------------------
// persistent select: P0 scan | radix rounds | counts | compaction
// ------------------------------------------------------------------------------------------------

// the per-block copy of the leader-published state
struct SelView {
  unsigned lo;
  unsigned long long width;
  int shift;
  long long rem;
  int done;
  unsigned T;
  long long need;
  unsigned maxkey;
};

// Grid barrier: every block but 0 raises its arrival flag (one 64-B line each, no contended
// counter); block 0 polls all flags in parallel, runs `lead` (all of its threads) and bumps the
// generation word the others poll (relaxed agent-scope loads + s_sleep, bounded).
template <typename F>
__device__ void grid_barrier(const TopkWs& w, unsigned nbar, F&& lead) {
  const unsigned target = nbar + 1;
  drain_stores();
  __syncthreads();
  if (blockIdx.x == 0) {
    const int tid = threadIdx.x;
    if (tid > 0 && tid < (int)gridDim.x) {
      unsigned* f = w.flags + (size_t)tid * kFlagStride;
      unsigned spins = 0;
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 24)) {  // ~1 s: a block never arrived; flag it and let the launch drain
          __hip_atomic_fetch_or(&w.st->err, 4ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    lead();
    drain_stores();
    __syncthreads();
    if (tid == 0) st_mem64(&w.st->gen, target);
  } else if (threadIdx.x == 0) {
    (void)__hip_atomic_exchange(w.flags + (size_t)blockIdx.x * kFlagStride, target, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(&w.st->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned long long)target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 24)) {
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
    v->maxkey = (unsigned)ld_mem64(&w.st->maxkey);
  }
  __syncthreads();
}

// leader step of a radix round.  `rem` is the rank (from the top) of the k-th largest key among all
// keys >= lo, so it stays k; the round's `A` keys above the live range come first: if A >= rem the
// key lies above the range (re-range to [lo + width, top)), otherwise pick the bin of rank rem - A in
// the global histogram of round r and narrow the range to it.
__device__ void lead_pick(const TopkWs& w, int r, const SelView& cur, unsigned* s_ghist) {
  __shared__ unsigned s_digit;
  __shared__ long long s_rem;
  __shared__ unsigned s_err;
  __shared__ long long s_above;
  unsigned* h = w.hist + (size_t)r * kHistStride;
  for (int i = threadIdx.x; i < kHistBins; i += kSelThreads) s_ghist[i] = ld_mem(&h[i]);
  __shared__ unsigned s_maxkey;
  if (threadIdx.x == 0) {
    s_err = 0;
    s_above = (long long)ld_mem(&h[kHistBins]);
    s_maxkey = r == 0 ? ld_mem(&w.hist[kHistBins + 1]) : cur.maxkey;
    if (r == 0) st_mem64(&w.st->maxkey, s_maxkey);
    st_mem64(&w.st->rounds, (unsigned long long)r + 1ull);
  }
  __syncthreads();
  const long long A = s_above;
  if (A >= cur.rem) {  // the k-th largest key is above the range (block-uniform branch)
    if (threadIdx.x == 0) {
      const unsigned long long nlo = (unsigned long long)cur.lo + cur.width;
      const unsigned long long top = (unsigned long long)s_maxkey + 1ull;
      const unsigned long long nw = top > nlo ? top - nlo : 0ull;
      if (nw == 0ull) __hip_atomic_fetch_or(&w.st->err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      st_mem64(&w.st->lo, nlo);
      st_mem64(&w.st->width, nw);
      st_mem64(&w.st->shift, (unsigned long long)range_shift(nw, kHistBits));
      st_mem64(&w.st->rem, (unsigned long long)cur.rem);
    }
    return;
  }
  if (threadIdx.x < kWave) wave_select_from_top<kHistBins>(s_ghist, cur.rem - A, &s_digit, &s_rem, &s_err);
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long* tr = w.trace + r * 8;
    tr[0] = cur.lo; tr[1] = cur.width; tr[2] = (unsigned long long)cur.shift; tr[3] = (unsigned long long)cur.rem;
    tr[4] = (unsigned long long)A; tr[5] = s_digit; tr[6] = (unsigned long long)s_rem; tr[7] = s_ghist[s_digit];
    const unsigned nlo = cur.lo + (s_digit << cur.shift);
    if (s_err) __hip_atomic_fetch_or(&w.st->err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur.shift == 0) {
      st_mem64(&w.st->T, nlo);
      st_mem64(&w.st->need, (unsigned long long)s_rem);
      st_mem64(&w.st->done, 1ull);
    } else {
      const unsigned long long nw = 1ull << cur.shift;
      st_mem64(&w.st->lo, nlo);
      st_mem64(&w.st->width, nw);
      st_mem64(&w.st->shift, (unsigned long long)range_shift(nw, kHistBits));
      st_mem64(&w.st->rem, (unsigned long long)cur.rem);  // rank from the top among keys >= lo: unchanged
    }
  }
}

#ifdef FLC_SELECT_STAMPS
#define STAMP(i)                                                                                 \
  do {                                                                                           \
    if (blockIdx.x == 0 && threadIdx.x == 0) w.stamps[i] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)
#else
#define STAMP(i) do { } while (0)
#endif

template <bool STACKED>
__global__ __launch_bounds__(kSelThreads) void topk_select_kernel(const float* __restrict__ x, TopkWs w, int R,
                                                                  long long k, int64_t n, int* __restrict__ idx_out,
                                                                  float* __restrict__ val_out,
                                                                  uint8_t* __restrict__ code_out,
                                                                  float* __restrict__ norm_out, int levels, double step,
                                                                  uint64_t seed, uint64_t counter) {
  __shared__ unsigned s_off[kMaxRegions + 1];
  __shared__ __attribute__((aligned(16))) unsigned s_keys[kKeyCache];
  __shared__ unsigned s_hist[kHistBins];
  __shared__ unsigned s_ghist[kHistBins];
  __shared__ uint4 s_wc[kWcCap];
  __shared__ unsigned long long s_red[kSelNW];
  __shared__ unsigned s_mx[kSelNW];
  __shared__ SelView s_view;
  const int tid = threadIdx.x;
  STAMP(0);

  // ---- P0: region offsets in LDS and the candidate count (identical in every block)
  {
    const int r0 = tid * kRegionsPerThread;
    unsigned loc[kRegionsPerThread];
    unsigned long long sum = 0;
#pragma unroll
    for (int i = 0; i < kRegionsPerThread; i += 4) {
      if (r0 + i < R) {  // R is a multiple of 4
        const uint4 c = *reinterpret_cast<const uint4*>(w.region_cnt + r0 + i);
        loc[i] = c.x; loc[i + 1] = c.y; loc[i + 2] = c.z; loc[i + 3] = c.w;
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
    if (tid == 0) {
      s_off[R] = (unsigned)tot;
      s_red[0] = tot;
    }
    __syncthreads();
  }
  const unsigned long long c_cand = s_red[0];
  __syncthreads();  // s_red is reused below
  const bool fb = (long long)c_cand < k;
  const long long C = fb ? (long long)n : (long long)c_cand;
  long long per = (C + gridDim.x - 1) / gridDim.x;
  per = (per + 3) & ~3ll;
  const long long v0 = min((long long)blockIdx.x * per, C), v1 = min(v0 + per, C);
  const bool cached = per <= kKeyCache;  // grid-uniform

  // round 0 covers [t_lo, t_hi) (fallback: every key); keys above it are counted apart
  SelView cur;
  cur.lo = fb ? 0u : w.p->t_lo;
  unsigned long long hi_end = fb ? (1ull << 32) : w.p->t_hi;
  if (hi_end <= (unsigned long long)cur.lo || hi_end > (1ull << 32)) hi_end = 1ull << 32;
  cur.width = hi_end - cur.lo;
  cur.shift = range_shift(cur.width, kHistBits);
  cur.rem = k;
  cur.done = 0;
  cur.T = 0;
  cur.need = 0;
  cur.maxkey = 0;
  SelView prev = cur;
  unsigned long long a_blk = 0;  // keys above the live range in this block (last round)
  unsigned nbar = 0;
  STAMP(1);

  // ---- radix rounds: histogram of the live range (+ count above it), leader picks the digit
  for (int round = 0; round < kMaxRounds; ++round) {
    for (int i = tid; i < kHistBins; i += kSelThreads) s_hist[i] = 0u;
    __syncthreads();
    unsigned above = 0, mk = 0;
    int r = 0, r_cur = -1, r_first = 0;
    bool wc_lds = false;
    uint4 wc = make_uint4(0u, 0u, 0u, 0u);
    if (round == 0 && !fb) {
      // wave counts of the block regions this select block gathers from, staged in LDS when they fit
      if (v0 < v1) {
        r_first = lds_region_search(s_off, R, (unsigned)v0);
        const int r_last = lds_region_search(s_off, R, (unsigned)(v1 - 1));
        wc_lds = r_last - r_first + 1 <= kWcCap;
        if (wc_lds)
          for (int i = tid; i <= r_last - r_first; i += kSelThreads)
            s_wc[i] = *reinterpret_cast<const uint4*>(w.wave_cnt + (size_t)(r_first + i) * kFNW);
      }
      __syncthreads();
      if (v0 + 4 * (long long)tid < v1) r = lds_region_search(s_off, R, (unsigned)(v0 + 4 * tid));
    }
    for (long long c0 = v0 + 4 * tid; c0 < v1; c0 += 4 * kSelThreads) {
      unsigned raw[4];
      if (round == 0) {
        if (fb) {
          if (c0 + 4 <= v1) {
            const float4 v = *reinterpret_cast<const float4*>(x + c0);
            raw[0] = __float_as_uint(v.x); raw[1] = __float_as_uint(v.y);
            raw[2] = __float_as_uint(v.z); raw[3] = __float_as_uint(v.w);
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) raw[u] = c0 + u < v1 ? __float_as_uint(x[c0 + u]) : 0u;
          }
        } else {
          unsigned id[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const long long c = c0 + u;
            if (c < v1) {
              r = lds_region_advance(s_off, R, r, (unsigned)c);
              if (r != r_cur) {
                r_cur = r;
                wc = wc_lds ? s_wc[r - r_first] : *reinterpret_cast<const uint4*>(w.wave_cnt + (size_t)r * kFNW);
              }
              // candidate -> (block region, wave quarter, offset): the quarters are in index order
              unsigned loc = (unsigned)(c - s_off[r]);
              long long q = 0;
              if (loc >= wc.x) { loc -= wc.x; q = 1;
                if (loc >= wc.y) { loc -= wc.y; q = 2;
                  if (loc >= wc.z) { loc -= wc.z; q = 3; } } }
              const long long wv = (long long)r * kFNW + q;
              const uint2 e = loc < (unsigned)w.dcap ? w.stage[wv * w.dcap + loc] : w.spill[wv * w.qc + (loc - w.dcap)];
              id[u] = e.x;
              raw[u] = e.y;
            } else {
              id[u] = 0u;
              raw[u] = 0u;
            }
          }
          if (c0 + 4 <= v1) {
            *reinterpret_cast<uint4*>(w.cand_idx + c0) = make_uint4(id[0], id[1], id[2], id[3]);
            if (!cached) *reinterpret_cast<uint4*>(w.cand_raw + c0) = make_uint4(raw[0], raw[1], raw[2], raw[3]);
          } else {
            for (int u = 0; u < 4; ++u)
              if (c0 + u < v1) {
                w.cand_idx[c0 + u] = id[u];
                if (!cached) w.cand_raw[c0 + u] = raw[u];
              }
          }
        }
        if (cached) *reinterpret_cast<uint4*>(s_keys + (c0 - v0)) = make_uint4(raw[0], raw[1], raw[2], raw[3]);
      } else if (cached) {  // re-read what this thread cached in round 0
        const uint4 t = *reinterpret_cast<const uint4*>(s_keys + (c0 - v0));
        raw[0] = t.x; raw[1] = t.y; raw[2] = t.z; raw[3] = t.w;
      } else if (fb) {
#pragma unroll
        for (int u = 0; u < 4; ++u) raw[u] = c0 + u < v1 ? __float_as_uint(x[c0 + u]) : 0u;
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
        const bool in = c0 + u < v1 && key >= cur.lo;
        if (round == 0) mk = (c0 + u < v1 && key > mk) ? key : mk;
        above += (in && rel >= cur.width) ? 1u : 0u;
        hist_add(s_hist, (unsigned)(rel >> cur.shift), in && rel < cur.width);
      }
    }
    __syncthreads();
    unsigned* h = w.hist + (size_t)round * kHistStride;
    for (int i = tid; i < kHistBins; i += kSelThreads)
      if (s_hist[i]) atomicAdd(&h[i], s_hist[i]);
    a_blk = block_sum<unsigned long long, kSelNW>((unsigned long long)above, s_red);
    if (tid == 0 && a_blk) atomicAdd(&h[kHistBins], (unsigned)a_blk);
    if (round == 0) {  // the max key (norm of the stacked codec, top of a re-range)
      mk = wave_max_u32(mk);
      if ((tid & 63) == 0) s_mx[tid >> 6] = mk;
      __syncthreads();
      if (tid == 0) {
        unsigned m = 0;
        for (int i = 0; i < kSelNW; ++i) m = s_mx[i] > m ? s_mx[i] : m;
        if (v0 < v1) atomicMax(&h[kHistBins + 1], m);
      }
    }
    STAMP(2 + 2 * round);
    prev = cur;
    grid_barrier(w, nbar++, [&] { lead_pick(w, round, cur, s_ghist); });
    STAMP(3 + 2 * round);
    read_view(w, &s_view);
    cur = s_view;
    __syncthreads();
    if (cur.done) break;
  }
  if (!cur.done && blockIdx.x == 0 && tid == 0)
    __hip_atomic_fetch_or(&w.st->err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  // ---- counts from the resolving round's local histogram: strict = above + bins past T's bin
  const unsigned T = cur.T;
  {
    const unsigned d = T - prev.lo;  // the resolving round has shift 0: bin = key - lo
    unsigned long long cnt = 0;      // strict << 32 | tie
    for (int i = tid; i < kHistBins; i += kSelThreads) {
      const unsigned hv = s_hist[i];
      cnt += ((unsigned)i > d ? ((unsigned long long)hv << 32) : 0ull) + ((unsigned)i == d ? hv : 0ull);
    }
    const unsigned long long both = block_sum<unsigned long long, kSelNW>(cnt, s_red) + (a_blk << 32);
    if (tid == 0) st_mem64(&w.blk_cnt[blockIdx.x], both);
  }
  STAMP(14);
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
      if (st + cur.need != k || cur.need > ti)
        __hip_atomic_fetch_or(&w.st->err, 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  });
  STAMP(15);
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
    const float a = fabsf(key_value(cur.maxkey)), b = fabsf(key_value(T));
    nrm = (isnan(a) || isnan(b)) ? __uint_as_float(0x7fc00000u) : (a > b ? a : b);
    if (blockIdx.x == 0 && tid == 0) *norm_out = nrm;
  }
  const bool nrm_ok = nrm > 0.0f && nrm <= 3.402823466e38f;
  for (long long base = v0; base < v1; base += 4 * kSelThreads) {
    const long long c0 = base + 4 * tid;
    unsigned raw[4], id[4];
    if (cached) {
      const uint4 t = *reinterpret_cast<const uint4*>(s_keys + (c0 < v1 ? c0 - v0 : 0));
      raw[0] = t.x; raw[1] = t.y; raw[2] = t.z; raw[3] = t.w;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long c = c0 + u;
      const bool in = c < v1;
      if (!cached) raw[u] = in ? (fb ? __float_as_uint(x[c]) : w.cand_raw[c]) : 0u;
      raw[u] = in ? raw[u] : 0u;
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
        const U4 r4 = philox_group((uint64_t)id[u] >> 2, seed, counter);
        const double uu = u01(pick(r4, (int)(id[u] & 3u)));
        const uint32_t lvl = (uint32_t)dither_level<0>(y, levels, step, uu);  // compressors.py:346-353
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
  STAMP(13);
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
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
  std::lock_guard<std::mutex> lk(g.mu);
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
  int dev = 0;
  FLC_CHECK_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return fail(FLC_EUNSUPPORTED, "device index %d", dev);
  const int grid = select_grid(dev);
  if (!ss.take_all)
    FLC_LAUNCH("topk_sample_gather", topk_sample_gather_kernel, dim3((unsigned)cdiv(ss.S, kThreads)), dim3(kThreads), 0,
               st, x, n, ss.S, w);
  FLC_LAUNCH("topk_sample_select", topk_sample_select_kernel, dim3(1), dim3(kSelectThreads), 0, st, ss.S, ss.rank_lo,
             ss.rank_hi, ss.take_all, w);
  FLC_LAUNCH("topk_filter", topk_filter_kernel, dim3((unsigned)R), dim3(kThreads), 0, st, x, n, g.chunk, grid, w);
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
  (void)carve_topk(nullptr, 0, n < 1 ? 1 : n, k, &need);
  return need;
}

int flc_topk_encode(const float* x, int64_t n, int64_t k, int32_t* idx, float* val, void* ws, size_t ws_bytes,
                    void* stream) {
  if (int rc = check_topk(x, n, k, "flc_topk_encode")) return rc;
  if (!idx || !val) return fail(FLC_EINVAL, "flc_topk_encode: null output");
  size_t need = 0;
  TopkWs w = carve_topk(ws, ws_bytes, n, k, &need);
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
  TopkWs w = carve_topk(ws, ws_bytes, n, k, &need);
  if (!ws || need > ws_bytes) return fail(FLC_EWORKSPACE, "flc_stacked_encode: workspace %zu < %zu", ws_bytes, need);
  return launch_topk<true>(x, n, k, w, as_stream(stream), idx, nullptr, codes, norm, levels, seed, counter);
}

}  // extern "C"
