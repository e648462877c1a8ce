// topk.hip — exact top-k selection and the stacked top-k -> 8-bit dithering encoder for gfx950
// (reference: fl_sim/compressors/compressors.py:293-296 and 327-365).
//
// Selection contract (compressors.py:294-295, `out[np.argsort(out)[:-K]] = 0`): keep the k largest
// *signed* values; -0 == +0; NaN is largest; among elements equal to the k-th largest value the
// highest indices are kept (stable ascending argsort order; the reference's own argsort is unstable,
// so any tie choice satisfies it — see DESIGN.md).
//
// Two launches (the default, "fused" path); block b of the encode owns the element range [b M, (b + 1) M):
//   sample   32 K strided keys of x (order-preserving uint32 keys).
//   encode   one block of 1024 threads per CU (topk_select_kernel<STACKED, FUSED = true>), in two phases:
//     filter phase (filter_phase): every block derives, identically, from the sample a candidate floor t_lo
//            (count(key >= t_lo) ~ k + 4 sigma: ~1.27 k candidates at k/n = 1 %) and a likely ceiling t_hi of the
//            k-th largest key; then the one HBM pass over its range (4 B/element): 16 waves stream 16 K-element
//            block steps (4 float4 per lane, the next step in flight), one float compare per element,
//            ballot/mbcnt compaction, the step's 16 wave counts exchanged through LDS so that the block's
//            candidates land in index order in LDS (past its 16 K LDS slots, in an HBM overflow area);
//            candidates in [t_lo, t_hi) are binned into a 2048-bin LDS histogram on the fly.  At the end the
//            histogram, above-the-band count, max key and candidate count are added to global memory
//            (memory-side atomics), followed by ONE grid exchange.
//     select phase: the summed histogram picks the bin holding the k-th largest key; every block publishes its
//            candidates inside that bin (~3 each at the headline) and its count above it; after one more exchange
//            every block resolves the exact k-th largest key T among those keys and its own output offset
//            locally, then writes its slice of the kept entries in index order from LDS: idx[k] + val[k] or
//            idx[k] + codes[k] with the dithering fused, and the tile pointers.  Rare paths (a list overflow, a
//            re-range, a floor that admitted fewer than k elements — then every block reads its x range directly)
//            fall back to histogram rounds, each one exchange.
// Calibration builds keep the earlier split form (FLC_TOPK_SPLIT=1: a separate filter kernel staging the
// candidates through HBM, the kernel boundary as the hand-off).  (A paired pass — blocks 2j and 2j + 1 streaming their
// joint range from both ends, claiming the middle steps at run time — measured no faster and was removed in round 5:
// DESIGN.md §8.)  The batched encoders (flc_stacked_encode_batch*) run one fused select per client on its share of the
// CUs, in one launch.
// An exchange: the block drains its stores/atomics, raises its own flag to the exchange's epoch
// (call * 32 + phase, from a call counter in the workspace), one wave polls all flags.  The histograms
// are zeroed by the select at the end of each call; the workspace is zero-initialised once by its
// owner.  Select launches on different streams of one device are serialised by an event chain, so two
// never compete for co-residency; spins are bounded (error flag).
#include <hip/hip_runtime.h>
#include <math.h>

#include <stddef.h>
#include <stdlib.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kET = 1024;                     // threads per block of the filter / select kernels (one per CU)
constexpr int kENW = kET / kWave;             // 16 waves
constexpr int kStepF4 = 4;                    // float4 per lane per wave step
constexpr int kWaveSpan = kStepF4 * 256;      // 1024 elements per wave step
constexpr int kBlockStep = kENW * kWaveSpan;  // 16384 elements per block step
constexpr int kCap = 16384;                   // candidates per block kept in LDS
constexpr int kSample = 32768;
constexpr int kSPT = kSample / kET;           // 32 sample keys per thread
constexpr int kTopPer = 8;                    // compact sample: the 8 largest keys of each 64-key wave of the sample ...
constexpr int kSampTop = kSample / 64 * kTopPer;  // ... 4096 keys, 4 per encode thread (single-client calls)
constexpr int kHistBits = 11;
constexpr int kHistBins = 1 << kHistBits;
constexpr int kHistStride = kHistBins + 64;   // bins, [kHistBins] above-the-range count, [+1] max key
// copies of the round-0 histogram: block b adds into copy b % kHistCopies (slot 0, then slots kMaxSlots ..), so each
// bin's word takes G / kHistCopies of the G blocks' atomics instead of all of them; readers sum the copies
constexpr int kHistCopies = 8;
constexpr int kMaxSlots = 12;                 // histogram rounds per call (normal + fallback pass)
constexpr int kEpochStride = 32;              // exchanges per call < 32
constexpr int kMaxBlocks = 1024;              // <= kET (per-block words are read one per thread)
constexpr int kInbin = 32;                    // in-bin keys a block may publish (more: histogram rounds) ...
constexpr int kInbinMax = 256;                //   ... or up to kInbinAll / blocks when a select has few blocks
constexpr int kInbinAll = 1024;               // in-bin keys of all blocks resolved locally
constexpr int kTile = FLC_TILE;               // outputs per tile of the CSR tile pointers
constexpr int kTileLog = 10;
static_assert((1 << kTileLog) == kTile, "tile size");
constexpr int kFlagStride = 16;               // workspace words reserved per block for flags

// diagnostics and the call counter (64-bit words, memory-side atomics only)
struct EncState {
  unsigned long long call;   // calls completed on this workspace (epoch base)
  unsigned long long err;    // 1: digit not found, 2: count mismatch, 4: exchange spin timeout
  unsigned long long C;      // candidates (floor admitted)
  unsigned long long fallback;
  unsigned long long T;      // the k-th largest key
  unsigned long long maxkey;
  unsigned long long rounds;
  unsigned long long t_lo, t_hi;
  unsigned long long need, ties, strict;
  unsigned long long sample_path;  // 0 fast, 1 general radix, 2 take-all
  unsigned long long pad[3];
};

// workspace layout: fixed offsets from one base pointer (every region 256-B aligned; only the staging
// area at the end depends on n), so a kernel carries one pointer instead of a struct of them
constexpr size_t al256(size_t v) { return (v + 255) / 256 * 256; }
constexpr size_t kOffSt = 0;
constexpr size_t kOffFlags = al256(kOffSt + 128);
constexpr size_t kOffHist = al256(kOffFlags + (size_t)kMaxBlocks * kFlagStride * 4);
constexpr size_t kOffAcc = kOffHist + (size_t)(kMaxSlots + kHistCopies - 1) * kHistStride * 4;  // contiguous with hist (zeroed together)
constexpr size_t kOffBlk = al256(kOffAcc + 64);
constexpr size_t kOffStamps = al256(kOffBlk + (size_t)kMaxBlocks * 8);
constexpr size_t kOffBlkT = al256(kOffStamps + 128);   // [kMaxBlocks][4] per-block times (diagnostic build)
constexpr size_t kOffSample = al256(kOffBlkT + (size_t)kMaxBlocks * 32);
constexpr size_t kOffSampTop = al256(kOffSample + (size_t)kSample * 4);
constexpr size_t kOffInbin = al256(kOffSampTop + (size_t)kSampTop * 4);
constexpr size_t kOffBlkC = al256(kOffInbin + (size_t)kMaxBlocks * kInbin * 4);
constexpr size_t kOffStage = al256(kOffBlkC + (size_t)kMaxBlocks * 4);  // + G * kCap * 8 (keys, then indices)
static_assert(kOffAcc % 8 == 0 && kOffHist % 8 == 0 && (kHistStride * 4) % 8 == 0, "acc / total words are 64-bit");
static_assert(sizeof(EncState) <= 128, "state block");

// A batched call (flc_stacked_encode_batch) runs one independent select per client in one launch: client g owns
// blocks [g * nb, (g + 1) * nb) and its own header (st ... blkC, at base + g * kOffStage) and staging / overflow
// area (at var + g * vstride); `bid` / `nb` are the block's index and the block count of its own select (for a
// single call: blockIdx.x and gridDim.x).  Every select ORs its error bits into `errp` (group 0's word).
struct EncWs {
  char* base;     // the header (fixed offsets kOffSt .. kOffStage)
  char* var;      // staging area, then the overflow area
  int64_t M;      // elements per block range (multiple of kBlockStep)
  size_t off_ovf; // byte offset from `var` of the candidate overflow area: per block 2 * ovf words (keys, indices)
  unsigned ovf;   // candidates per block kept in HBM beyond the LDS's kCap (0: none)
  int bid, nb;    // this block's index in its select, the blocks of its select (set in the kernel prologue)
  size_t vstride; // batched: bytes between two clients' staging / overflow areas
  int compact;    // the sample kernel wrote the compact sample (samptop): the floor / ceiling start from it
  unsigned long long* errp;
  __device__ EncState* st() const { return reinterpret_cast<EncState*>(base + kOffSt); }
  __device__ unsigned* flags() const { return reinterpret_cast<unsigned*>(base + kOffFlags); }
  __device__ unsigned* hist() const { return reinterpret_cast<unsigned*>(base + kOffHist); }
  __device__ unsigned long long* acc() const { return reinterpret_cast<unsigned long long*>(base + kOffAcc); }
  __device__ unsigned long long* blk_cnt() const { return reinterpret_cast<unsigned long long*>(base + kOffBlk); }
  __device__ unsigned long long* stamps() const { return reinterpret_cast<unsigned long long*>(base + kOffStamps); }
  __device__ unsigned long long* blkt() const { return reinterpret_cast<unsigned long long*>(base + kOffBlkT); }
  __device__ unsigned* sample() const { return reinterpret_cast<unsigned*>(base + kOffSample); }
  __device__ unsigned* samptop() const { return reinterpret_cast<unsigned*>(base + kOffSampTop); }
  __device__ unsigned* inbin() const { return reinterpret_cast<unsigned*>(base + kOffInbin); }
  __device__ unsigned* blk_c() const { return reinterpret_cast<unsigned*>(base + kOffBlkC); }  // candidates / block
  __device__ unsigned* stage_key(int b) const { return reinterpret_cast<unsigned*>(var) + (size_t)b * 2 * kCap; }
  __device__ unsigned* stage_idx(int b) const { return stage_key(b) + kCap; }
  __device__ unsigned* ovf_key(int b) const {
    return reinterpret_cast<unsigned*>(var + off_ovf) + (size_t)b * 2 * ovf;
  }
  __device__ unsigned* ovf_idx(int b) const { return ovf_key(b) + ovf; }
};

struct EncGeom {
  int G;
  int64_t M;
};

EncGeom enc_geometry(int64_t n, int cus) {
  EncGeom g;
  int64_t G0 = std::min<int64_t>(std::min<int64_t>(cus, kMaxBlocks), cdiv(n, kBlockStep));
  if (G0 < 1) G0 = 1;
  g.M = (int64_t)align_up((size_t)cdiv(n, G0), kBlockStep);
  g.G = (int)cdiv(n, g.M);
  return g;
}

struct SampleSetup {
  int S;
  long long rank_lo, rank_hi;
  int take_all;
};

// s_max: the sample size cap (kSample; a batched call of small clients takes fewer keys per client, because its
// sample gathers cost one HBM line per key for every client while the floor / ceiling runs per client in parallel)
SampleSetup sample_setup(int64_t n, int64_t k, int s_max = kSample) {
  SampleSetup s;
  s.S = (int)(n < s_max ? n : s_max);
  const double m = (double)s.S * (double)k / (double)n;
  s.rank_lo = (long long)ceil(m + 4.0 * sqrt(m) + 16.0);
  // the ceiling: 4 sigma + 16 below m, or (small m: a batched client's 4 K-key sample at k = 1 % has m = 41) just
  // 4 sigma — without a ceiling the band reaches the top of the key range and its bins are too coarse for the in-bin
  // lists (histogram rounds follow); a ceiling that admits k keys or more only costs those rounds
  double rh = floor(m - 4.0 * sqrt(m) - 16.0);
  if (rh < 1.0) rh = floor(m - 4.0 * sqrt(m));
  s.rank_hi = rh >= 1.0 ? (long long)rh : 0;
  s.take_all = (s.rank_lo >= s.S) ? 1 : 0;
  if (s.take_all) s.rank_lo = s.S;
  return s;
}

// Candidates beyond a block's LDS (kCap) go to an HBM overflow area sized from the expected count: the floor
// admits about rank_lo / S of the elements, so a block holds ~(rank_lo / S) * M candidates; twice that (for skew)
// beyond kCap, capped at kMaxOvf.  Blocks past kCap + ovf re-read their range instead (x-mode).  At k = 1 % the
// area is empty up to 1 GiB inputs (M = 1 Mi: ~13 K candidates per block) and lets 2-8 GiB inputs keep their
// candidates instead of re-reading x.
constexpr int64_t kMaxOvf = 1ll << 17;
SampleSetup sample_setup(int64_t n, int64_t k, int s_max);
unsigned ovf_capacity(int64_t n, int64_t k, int64_t M, int s_max = kSample) {
  const SampleSetup ss = sample_setup(n, k, s_max);
  const double frac = ss.take_all ? 1.0 : std::min(1.0, (double)ss.rank_lo / (double)ss.S);
  int64_t want = (int64_t)std::ceil(2.0 * frac * (double)M) + 4096 - kCap;
  want = std::min<int64_t>(std::min<int64_t>(want, kMaxOvf), M);
  return want > 0 ? (unsigned)align_up((size_t)want, 64) : 0u;
}

// staging + overflow bytes of one select over n elements with `cus` blocks at most
size_t enc_var_bytes(int64_t n, int64_t k, int cus, EncGeom* geo, unsigned* ovf, size_t* off_ovf,
                     int s_max = kSample) {
  const EncGeom g = enc_geometry(n, cus);
  const unsigned o = ovf_capacity(n, k, g.M, s_max);
  const size_t oo = al256((size_t)g.G * kCap * 8);
  if (geo) *geo = g;
  if (ovf) *ovf = o;
  if (off_ovf) *off_ovf = oo;
  return al256(oo + (size_t)g.G * o * 8);
}

EncWs carve_enc(void* ws, int64_t n, int64_t k, int cus, size_t* need) {
  EncWs w;
  w.base = static_cast<char*>(ws);
  w.var = w.base + kOffStage;
  EncGeom g;
  const size_t vb = enc_var_bytes(n, k, cus, &g, &w.ovf, &w.off_ovf);
  w.M = g.M;
  w.bid = 0;
  w.nb = g.G;
  w.vstride = 0;
  w.compact = 0;
  w.errp = reinterpret_cast<unsigned long long*>(w.base + kOffSt + offsetof(EncState, err));
  *need = kOffStage + vb;
  return w;
}
constexpr int kZeroWords = (kMaxSlots + kHistCopies - 1) * kHistStride + 16;  // hist + acc, as 32-bit words

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------

// Histogram select: a histogram h[2048] (LDS) and a rank r (1-based, from the top) -> the bin holding
// that rank and the rank inside it.
// Block-wide (all kET threads call it; contains barriers): thread t holds the adjacent bins below
// 2047 - BPT t (no LDS bank conflicts), one block scan from the top gives each thread the count above
// its bins, and the thread holding rank r[j] writes digit[j] / new_rem[j].  (A wave-wide select reading
// 32 bins per lane at a 128-B lane stride hits one bank 64 ways.)
template <int NR>
__device__ __forceinline__ void block_select_from_top(const unsigned* h, const long long (&r)[NR], unsigned* digit,
                                      long long* new_rem, unsigned* err, unsigned long long* s_red) {
  constexpr int BPT = kHistBins / kET;  // bins per thread, highest first
  static_assert(BPT * kET == kHistBins, "bins per thread");
  const int t = threadIdx.x;
  const int top = kHistBins - 1 - BPT * t;
  unsigned c[BPT];
  unsigned long long sum = 0;
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    c[i] = h[top - i];
    sum += c[i];
  }
  unsigned long long tot;
  const long long ex = (long long)block_excl_scan_lds<unsigned long long, kENW>(sum, s_red, &tot);
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const long long rj = r[j];
    if (rj <= 0) continue;
    long long above = ex;
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      if (above < rj && rj <= above + (long long)c[i]) {
        digit[j] = (unsigned)(top - i);
        new_rem[j] = rj - above;
      }
      above += c[i];
    }
    if (t == 0 && (long long)tot < rj) {
      digit[j] = 0u;
      new_rem[j] = 1;
      *err |= 1u;
    }
  }
  lds_barrier();
}

// block-wide sums of N 64-bit values per thread in one LDS round (s_buf: kENW * N words)
template <int N>
__device__ __forceinline__ void block_sum_n(unsigned long long (&v)[N], unsigned long long* s_buf) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = wave_sum(v[i]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) s_buf[wid * N + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    unsigned long long t = 0;
    for (int w = 0; w < kENW; ++w) t += s_buf[w * N + i];
    v[i] = t;
  }
  __syncthreads();
}

// LDS histogram add with wave aggregation: when every active lane hits the same bin (ties, narrow
// key ranges) the wave issues ONE atomic instead of a 64-way conflicting one.
__device__ __forceinline__ void hist_add(unsigned* h, unsigned bin, bool valid) {
  const unsigned long long act = __ballot(valid);
  if (act == 0ull) return;
  const int first = __ffsll((long long)act) - 1;
  const unsigned b0 = (unsigned)__builtin_amdgcn_readlane((int)bin, first);  // (uniform lane: no LDS shuffle)
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

__device__ __forceinline__ int64_t cdiv_dev(int64_t a, int64_t b) { return (a + b - 1) / b; }

// coherent (agent-scope) reads / writes of words other blocks update in this launch: relaxed atomic
// loads, not read-modify-writes, so that all G blocks reading one word do not serialise on it
__device__ __forceinline__ unsigned ld_mem(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_mem64(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_mem64(unsigned long long* p, unsigned long long v) {
  (void)__hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// candidate test on values: key(v) >= t_lo  <=>  v >= t_lo_value  or  v is NaN.  Exact for
// t_lo <= key(+inf) (the host-side clamp below): below key(-inf) every value qualifies.
__device__ __forceinline__ float floor_value(unsigned t_lo) {
  return t_lo <= 0x007fffffu ? -__builtin_inff() : key_value(t_lo);
}
__device__ __forceinline__ bool is_cand(float a, float tf) { return !(a < tf); }

// ------------------------------------------------------------------------------------------------
// sample -> candidate floor and ceiling, computed identically by every block
// ------------------------------------------------------------------------------------------------
struct SampleLds {
  unsigned hist2[kHistBins];
  unsigned wmin[kENW];
  unsigned wmax[kENW];
  unsigned digit[2];
  long long rem[2];
  unsigned err;
  unsigned bad;  // compact sample: some wave of the sample holds more keys above the floor than its 8 listed
};

// sample index of a thread's key slot i: 16-B runs, so the coherent read is 8 x 16 B per thread
__device__ __forceinline__ int sample_j(int i) { return 4 * (int)threadIdx.x + 4 * kET * (i >> 2) + (i & 3); }

// a thread's kSPT sample keys (coherent-enough plain loads: the sample kernel finished before this one)
__device__ __forceinline__ void load_sample_keys(const unsigned* sample, int S, unsigned (&keys)[kSPT]) {
  if (S == kSample) {  // all eight 16-B groups in flight together
    uint4 t[kSPT / 4];
#pragma unroll
    for (int i = 0; i < kSPT; i += 4) t[i / 4] = *reinterpret_cast<const uint4*>(sample + sample_j(i));
#pragma unroll
    for (int i = 0; i < kSPT; i += 4) {
      keys[i] = t[i / 4].x; keys[i + 1] = t[i / 4].y; keys[i + 2] = t[i / 4].z; keys[i + 3] = t[i / 4].w;
    }
  } else {  // small n: S = n keys
#pragma unroll
    for (int i = 0; i < kSPT; ++i) keys[i] = sample_j(i) < S ? sample[sample_j(i)] : 0u;  // 0: below every key
  }
}

// Fast path (rank_lo <= kET): B = the smallest lane maximum, so at least kET >= rank_lo sample keys are
// >= B (one per lane); typically B sits near the 80th percentile.  An 11-bit histogram of the keys in
// [B, max] (plain LDS atomics, from registers) locates the bins of ranks rank_lo and rank_hi; a target
// bin holding more than a few sample keys (clustered values, ties) is refined by a second pass inside
// it.  The floor is the floor of rank_lo's bin (>= rank_lo sample keys at or above it) and the ceiling
// the end of rank_hi's bin (fewer than rank_hi sample keys at or above it).
// Two halves: the histogram (the keys' last use in registers: the caller issues the second HBM step
// in their place) and the pick (the rare refinement re-reads the keys).
// N = kSPT: the full sample (slot i valid when sample_j(i) < S); N = 4: the compact sample (every slot valid)
template <int N>
__device__ __forceinline__ bool sample_slot_valid(int i, int S) { return N != kSPT || sample_j(i) < S; }

template <int N>
__device__ __forceinline__ void sample_fast_hist(const unsigned (&keys)[N], int S, SampleLds& L, unsigned* s_hist,
                                                 unsigned* B_out, int* sh_out) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid >> 6;
  unsigned m = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) m = keys[i] > m ? keys[i] : m;  // invalid slots hold key 0
  const unsigned wmn = wave_min_u32(m), wmx = wave_max_u32(m);
  if (lane == 0) {
    L.wmin[wid] = wmn;
    L.wmax[wid] = wmx;
  }
  if (tid == 0) {
    L.err = 0;
    L.bad = 0;
  }
  for (int i = tid; i < kHistBins; i += kET) {
    s_hist[i] = 0u;
    L.hist2[i] = 0u;
  }
  lds_barrier();
  unsigned B = 0xffffffffu, mx = 0;
#pragma unroll
  for (int w = 0; w < kENW; ++w) {
    B = L.wmin[w] < B ? L.wmin[w] : B;
    mx = L.wmax[w] > mx ? L.wmax[w] : mx;
  }
  const int sh = range_shift((unsigned long long)mx - B + 1ull, kHistBits);
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (sample_slot_valid<N>(i, S) && keys[i] >= B) atomicAdd(&s_hist[(keys[i] - B) >> sh], 1u);
  *B_out = B;
  *sh_out = sh;
}

// (N = 4: `sample` is the compact sample, the refinement re-reads the thread's 4 keys of it)
template <int N>
__device__ __forceinline__ bool sample_fast_pick(const unsigned* sample, int S, long long rank_lo, long long rank_hi,
                                                 unsigned B, int sh, SampleLds& L, unsigned* s_hist,
                                                 unsigned long long* s_red, unsigned* t_lo_out,
                                                 unsigned long long* t_hi_out) {
  const int tid = threadIdx.x;
  lds_barrier();
  const bool two = rank_hi > 0;
  const long long rk[2] = {rank_lo, two ? rank_hi : 0};
  block_select_from_top<2>(s_hist, rk, L.digit, L.rem, &L.err, s_red);
  if (L.err) return false;  // block-uniform
  const unsigned d0 = L.digit[0], d1 = two ? L.digit[1] : 0u;
  unsigned lo0 = B + (d0 << sh), lo1 = B + (d1 << sh);
  int sh_hi = sh;
  const bool ref0 = sh > 0 && s_hist[d0] > 8u, ref1 = two && sh > 0 && s_hist[d1] > 8u;  // block-uniform
  if (ref0 || ref1) {
    unsigned keys[N];
    if constexpr (N == kSPT) {
      load_sample_keys(sample, S, keys);
    } else {
      static_assert(N == 4, "compact sample: 4 keys per thread");
      const uint4 t4 = *reinterpret_cast<const uint4*>(sample + 4 * tid);
      keys[0] = t4.x; keys[1] = t4.y; keys[2] = t4.z; keys[3] = t4.w;
    }
    const long long r0 = L.rem[0], r1 = two ? L.rem[1] : 0;
    const int sh2 = sh > kHistBits ? sh - kHistBits : 0;
    const unsigned long long bw = 1ull << sh;
    lds_barrier();
    for (int i = tid; i < kHistBins; i += kET) s_hist[i] = 0u;
    lds_barrier();
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if (!sample_slot_valid<N>(i, S)) continue;
      const unsigned long long rel0 = (unsigned long long)keys[i] - lo0, rel1 = (unsigned long long)keys[i] - lo1;
      if (ref0 && keys[i] >= lo0 && rel0 < bw) atomicAdd(&s_hist[(unsigned)(rel0 >> sh2)], 1u);
      if (ref1 && keys[i] >= lo1 && rel1 < bw) atomicAdd(&L.hist2[(unsigned)(rel1 >> sh2)], 1u);
    }
    lds_barrier();
    const long long ra[1] = {ref0 ? r0 : 0}, rb[1] = {ref1 ? r1 : 0};
    block_select_from_top<1>(s_hist, ra, &L.digit[0], &L.rem[0], &L.err, s_red);
    block_select_from_top<1>(L.hist2, rb, &L.digit[1], &L.rem[1], &L.err, s_red);
    if (L.err) return false;
    if (ref0) lo0 += L.digit[0] << sh2;
    if (ref1) { lo1 += L.digit[1] << sh2; sh_hi = sh2; }
  }
  *t_lo_out = lo0;
  *t_hi_out = two ? (unsigned long long)lo1 + (1ull << sh_hi) : (1ull << 32);
  return true;
}

// General path (any rank): two fixed 11-bit digit passes (key bits 31..21, then 20..10) per target.
// The keys are re-read from the sample (L2) in each pass, 16 B at a time: the caller holds the first
// two HBM steps in registers here, and a 32-key array on top of them would spill.
__device__ __forceinline__ uint4 sample_group(const unsigned* sample, int S, int g) {
  const int j = sample_j(4 * g);
  if (S == kSample) return *reinterpret_cast<const uint4*>(sample + j);
  uint4 t;
  t.x = j < S ? sample[j] : 0u;
  t.y = j + 1 < S ? sample[j + 1] : 0u;
  t.z = j + 2 < S ? sample[j + 2] : 0u;
  t.w = j + 3 < S ? sample[j + 3] : 0u;
  return t;
}

__device__ __forceinline__ void sample_general(const unsigned* sample, int S, long long rank_lo, long long rank_hi,
                                               SampleLds& L, unsigned* s_hist, unsigned long long* s_red,
                                               unsigned* t_lo_out, unsigned long long* t_hi_out) {
  const int tid = threadIdx.x;
  const bool two = rank_hi > 0;
  lds_barrier();
  for (int i = tid; i < kHistBins; i += kET) {
    s_hist[i] = 0u;
    L.hist2[i] = 0u;
  }
  if (tid == 0) L.err = 0;
  lds_barrier();
#pragma unroll 2
  for (int g = 0; g < kSPT / 4; ++g) {
    const uint4 t = sample_group(sample, S, g);
    const int j = sample_j(4 * g);
    hist_add(s_hist, t.x >> 21, j < S);
    hist_add(s_hist, t.y >> 21, j + 1 < S);
    hist_add(s_hist, t.z >> 21, j + 2 < S);
    hist_add(s_hist, t.w >> 21, j + 3 < S);
  }
  lds_barrier();
  {
    const long long rk[2] = {rank_lo, two ? rank_hi : 0};
    block_select_from_top<2>(s_hist, rk, L.digit, L.rem, &L.err, s_red);
  }
  const unsigned d0 = L.digit[0], d1 = two ? L.digit[1] : 0u;
  const long long r0 = L.rem[0], r1 = two ? L.rem[1] : 0;
  for (int i = tid; i < kHistBins; i += kET) s_hist[i] = 0u;
  lds_barrier();
#pragma unroll 2
  for (int g = 0; g < kSPT / 4; ++g) {
    const uint4 t = sample_group(sample, S, g);
    const int j = sample_j(4 * g);
    const unsigned kk[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bool in = j + c < S;
      const unsigned hi = kk[c] >> 21, bin = (kk[c] >> 10) & (kHistBins - 1);
      hist_add(s_hist, bin, in && hi == d0);
      if (two) hist_add(L.hist2, bin, in && hi == d1);
    }
  }
  lds_barrier();
  {
    const long long ra[1] = {r0}, rb[1] = {two ? r1 : 0};
    block_select_from_top<1>(s_hist, ra, &L.digit[0], &L.rem[0], &L.err, s_red);
    block_select_from_top<1>(L.hist2, rb, &L.digit[1], &L.rem[1], &L.err, s_red);
  }
  unsigned t_lo = (d0 << 21) | (L.digit[0] << 10);
  unsigned long long t_hi = two ? (unsigned long long)((d1 << 21) | (L.digit[1] << 10)) + 1024ull : 1ull << 32;
  if (L.err) {  // cannot happen for 0 < rank <= S; stay correct anyway: everything is a candidate
    t_lo = 0u;
    t_hi = 1ull << 32;
  }
  *t_lo_out = t_lo;
  *t_hi_out = t_hi;
}

// ------------------------------------------------------------------------------------------------
// filter
// ------------------------------------------------------------------------------------------------
// Sources of the filter's elements.  A wave step covers SF * 256 elements: SF float4 per lane, q-major (lane l,
// step slot q -> elements 256q + 4l + c).  FlatSrc reads one fp32 vector; DeltaSrc forms the client delta
// local - global of a list of parameter tensors on the fly (FedOptClient.communicate, _fedopt.py:294-297, fused
// into the encode's read: nothing is written), two float4 per slot, so it runs SF = 2 to keep the same
// registers and bytes in flight per wave as FlatSrc's SF = 4.
struct FlatSrc {
  static constexpr int SF = 4;
  const float* x;
  struct Step {
    float4 v[SF];
    __device__ __forceinline__ float4 val(int q) const { return v[q]; }
  };
  struct Cursor {};
  __device__ __forceinline__ float get(int64_t e) const { return x[e]; }
  // a partial step (the last block only) clamps each float4 to the last one holding valid data (16-B aligned, so it
  // never crosses a page); `lim` masks everything past the range end
  template <bool FULL>
  __device__ __forceinline__ void load(Cursor&, int64_t wb, int64_t end, int lane, Step& st) const {
    if (FULL) {
#pragma unroll
      for (int q = 0; q < SF; ++q) st.v[q] = ld_stream(x + wb + 256 * q + 4 * lane);
    } else {
      const int64_t last4 = (end - 1) & ~(int64_t)3;
#pragma unroll
      for (int q = 0; q < SF; ++q) {
        const int64_t e = wb + 256 * q + 4 * lane;
        st.v[q] = *reinterpret_cast<const float4*>(x + (e < last4 ? e : (last4 >= 0 ? last4 : 0)));
      }
    }
  }
};

// device-side table of DeltaSrc's tensors (in the workspace): off[t] = first flat index of tensor t,
// off[nseg] = n; lp / gp = the tensors' local / global parameter pointers
struct SegTab {
  const long long* off;
  const float* const* lp;
  const float* const* gp;
  int nseg;
};
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));  // 4-B aligned 16-B access

struct DeltaSrc {
  static constexpr int SF = 2;
  SegTab t;
  struct Step {
    float4 l[SF], g[SF];
    __device__ __forceinline__ float4 val(int q) const {  // local - global, one rounding (torch add_(alpha=-1))
      return make_float4(l[q].x - g[q].x, l[q].y - g[q].y, l[q].z - g[q].z, l[q].w - g[q].w);
    }
  };
  // the wave's current tensor (wave-uniform: kept in SGPRs)
  struct Cursor {
    long long lo = 1, hi = 0;
    const float* l = nullptr;
    const float* g = nullptr;
  };
  __device__ __forceinline__ int seg_of(int64_t e) const {  // off[s] <= e < off[s + 1]
    int lo = 0, hi = t.nseg;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (t.off[mid] <= e) lo = mid;
      else hi = mid;
    }
    return lo;
  }
  __device__ __forceinline__ float get(int64_t e) const {
    const int sg = seg_of(e);
    const int64_t r = e - t.off[sg];
    return t.lp[sg][r] - t.gp[sg][r];
  }
  // (every cursor field through readfirstlane: wave-uniform values the compiler would otherwise keep in VGPRs)
  static __device__ __forceinline__ long long rfl64(long long v) {
    return (long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v) |
           ((long long)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32);
  }
  __device__ __forceinline__ void seek(Cursor& c, int64_t wb) const {
    if (wb >= c.lo && wb < c.hi) return;
    const int sg = __builtin_amdgcn_readfirstlane(seg_of(wb));
    c.lo = rfl64(t.off[sg]);
    c.hi = rfl64(t.off[sg + 1]);
    c.l = reinterpret_cast<const float*>(rfl64(reinterpret_cast<long long>(t.lp[sg])));
    c.g = reinterpret_cast<const float*>(rfl64(reinterpret_cast<long long>(t.gp[sg])));
  }
  template <bool FULL>
  __device__ __forceinline__ void load(Cursor& c, int64_t wb, int64_t end, int lane, Step& st) const {
    seek(c, wb);
    const int64_t span_end = wb + 256 * SF;
    if ((FULL || span_end <= end) && span_end <= c.hi) {  // the whole wave step inside one tensor (wave-uniform)
      const float* l = c.l + (wb - c.lo) + 4 * lane;
      const float* g = c.g + (wb - c.lo) + 4 * lane;
#pragma unroll
      for (int q = 0; q < SF; ++q) {
#if FLC_DELTA_A16  // calibration only (assumes 16-B aligned operands): the pass with dwordx4 loads
        const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(l + 256 * q));
        const f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g + 256 * q));
#else
        const f32x4u a = __builtin_nontemporal_load(reinterpret_cast<const f32x4u*>(l + 256 * q));
        const f32x4u b = __builtin_nontemporal_load(reinterpret_cast<const f32x4u*>(g + 256 * q));
#endif
        st.l[q] = make_float4(a.x, a.y, a.z, a.w);
        st.g[q] = make_float4(b.x, b.y, b.z, b.w);
      }
    } else {  // a tensor boundary or the range end inside the step: element by element
#pragma unroll
      for (int q = 0; q < SF; ++q) {
        float a[4], b[4];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          const int64_t e = wb + 256 * q + 4 * lane + cc;
          a[cc] = 0.0f;
          b[cc] = 0.0f;
          if (e < end) {
            const int sg = seg_of(e);
            const int64_t r = e - t.off[sg];
            a[cc] = t.lp[sg][r];
            b[cc] = t.gp[sg][r];
          }
        }
        st.l[q] = make_float4(a[0], a[1], a[2], a[3]);
        st.g[q] = make_float4(b[0], b[1], b[2], b[3]);
      }
    }
  }
};

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

template <bool FULL, class Step, int SF>
__device__ __forceinline__ unsigned step_count(const Step& v, float tf, int lim, int lane) {
  unsigned cnt = 0;
#pragma unroll
  for (int q = 0; q < SF; ++q) {
    bool f0, f1, f2, f3;
    cand4<FULL>(v.val(q), tf, 256 * q + 4 * lane, lim, f0, f1, f2, f3);
    cnt += __popcll(__ballot(f0)) + __popcll(__ballot(f1)) + __popcll(__ballot(f2)) + __popcll(__ballot(f3));
  }
  return cnt;
}

struct FilterCtx {
  unsigned* s_key;
  unsigned* s_idx;
  unsigned* g_key;  // the block's HBM overflow (candidates kCap .. kCap + gcap - 1)
  unsigned* g_idx;
  unsigned gcap;
  unsigned* s_hist;
  unsigned t_lo;
  unsigned long long width0;  // t_hi - t_lo
  int sh0;
  unsigned above;         // per thread: candidates >= t_hi
  unsigned mk;            // per thread: max candidate key
  unsigned swept;         // (block-uniform) LDS candidates [0, swept) already in the band histogram
};

// one LDS candidate into the band histogram / above count / max key
__device__ __forceinline__ void band_bin(FilterCtx& c, unsigned p) {
  const unsigned key = order_key(c.s_key[p]);
  const unsigned long long rel = (unsigned long long)(key - c.t_lo);
  if (rel >= c.width0) ++c.above;
  else atomicAdd(&c.s_hist[(unsigned)(rel >> c.sh0)], 1u);
  c.mk = key > c.mk ? key : c.mk;
}

// a candidate into the block's LDS arrays; the band histogram, above count and max key of the stored
// candidates are formed after the pass in one dense sweep over LDS (every lane busy), only candidates
// beyond the LDS capacity are binned here (and kept in the HBM overflow while it has room)
// (OVF = false: the caller has checked that the whole step lands below kCap — the hot path, LDS stores only)
template <bool OVF>
__device__ __forceinline__ void emit(FilterCtx& c, unsigned q, unsigned e, float v) {
  const unsigned raw = __float_as_uint(v);
  const unsigned p = q;
  if (!OVF || p < (unsigned)kCap) {
    c.s_key[p] = raw;
    c.s_idx[p] = e;
  } else {
    if (p - (unsigned)kCap < c.gcap) {
      c.g_key[p - kCap] = raw;
      c.g_idx[p - kCap] = e;
    }
    const unsigned key = order_key(raw);
    const unsigned long long rel = (unsigned long long)(key - c.t_lo);
    if (rel >= c.width0) ++c.above;
    else atomicAdd(&c.s_hist[(unsigned)(rel >> c.sh0)], 1u);
    c.mk = key > c.mk ? key : c.mk;
  }
}

// ordered append from position `pos` (within a q: lane-major, then the 4 components)
template <bool FULL, class Step, int SF, bool OVF>
__device__ __forceinline__ void step_write(const Step& st, float tf, int lim, int lane, unsigned wbu,
                                           unsigned pos, FilterCtx& c) {
#pragma unroll
  for (int q = 0; q < SF; ++q) {
    bool f0, f1, f2, f3;
    const float4 vq = st.val(q);
    cand4<FULL>(vq, tf, 256 * q + 4 * lane, lim, f0, f1, f2, f3);
    const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1), m2 = __ballot(f2), m3 = __ballot(f3);
    if ((m0 | m1 | m2 | m3) != 0ull) {
      unsigned p = pos;
      p = __builtin_amdgcn_mbcnt_hi((unsigned)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m0, p));
      p = __builtin_amdgcn_mbcnt_hi((unsigned)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m1, p));
      p = __builtin_amdgcn_mbcnt_hi((unsigned)(m2 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m2, p));
      p = __builtin_amdgcn_mbcnt_hi((unsigned)(m3 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m3, p));
      if (f0 | f1 | f2 | f3) {
        const unsigned e = wbu + (unsigned)(256 * q + 4 * lane);
        if (f0) { emit<OVF>(c, p, e + 0u, vq.x); ++p; }
        if (f1) { emit<OVF>(c, p, e + 1u, vq.y); ++p; }
        if (f2) { emit<OVF>(c, p, e + 2u, vq.z); ++p; }
        if (f3) emit<OVF>(c, p, e + 3u, vq.w);
      }
      pos += __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
    }
  }
}

// one block step: count, exchange the 16 wave counts through LDS, append in index order
template <bool FULL, class Step, int SF>
__device__ __forceinline__ void step_process(const Step& v, int64_t wb, int64_t end, float tf,
                                             unsigned (&s_wc)[2][kENW], int par, unsigned& base, FilterCtx& c) {
  constexpr int span = SF * 256;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x >> 6;
  const int lim = FULL ? span : (int)(end > wb ? (end - wb < span ? end - wb : span) : 0);
  const unsigned cnt = step_count<FULL, Step, SF>(v, tf, lim, lane);
  if (lane == 0) s_wc[par][wid] = cnt;
  lds_barrier();
#if !FLC_BAND_AFTER_PASS
  {  // the band histogram of the earlier steps' LDS candidates (their writes are visible after this barrier),
     // binned while this step's loads are in flight: the post-pass sweep is left with the last step's
    const unsigned s1 = base < (unsigned)kCap ? base : (unsigned)kCap;
    for (unsigned p = c.swept + threadIdx.x; p < s1; p += kET) band_bin(c, p);
    c.swept = s1;
  }
#endif
  unsigned pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kENW; ++w) {
    const unsigned cw = s_wc[par][w];
    pre += w < wid ? cw : 0u;
    tot += cw;
  }
  // re-derive the masks rather than keep them live across the count (an opaque copy of the floor
  // stops the compiler from reusing the count pass's compares)
  float tf2 = tf;
  asm volatile("" : "+v"(tf2));
  if (cnt != 0u) {
    if (base + tot <= (unsigned)kCap)  // (block-uniform) the step lands in LDS: no overflow code on the hot path
      step_write<FULL, Step, SF, false>(v, tf2, lim, lane, (unsigned)wb, base + pre, c);
    else
      step_write<FULL, Step, SF, true>(v, tf2, lim, lane, (unsigned)wb, base + pre, c);
  }
  base += tot;
}

// ------------------------------------------------------------------------------------------------
// exchanges and the per-block view of the selection state
// ------------------------------------------------------------------------------------------------
// Exchange (grid barrier with data): the block's prior atomics / stores drained, its own flag raised to
// `ep` (packed flags, one word per block), then one wave polls all G flags (each lane a few words per
// round, relaxed agent-scope loads, a wave-wide vote, sleep between rounds).  No leader and no
// contended counter: 256 arrivals on ONE word serialise at the memory-side atomic unit (measured ~5 us).
// every block's flag at `ep` or later: all of a lane's flag loads issued together (no short-circuit, so one
// round trip per poll rather than one per flag), then one wave-wide vote
__device__ __forceinline__ bool all_arrived(const EncWs& w, unsigned ep) {
  const int tid = threadIdx.x & (kWave - 1), G = w.nb;
  bool ok = true;
#pragma unroll
  for (int i = 0; i < kMaxBlocks / kWave; ++i) {
    const int b = tid + i * kWave;
    if (i * kWave >= G) break;  // (uniform)
    const unsigned f = __hip_atomic_load(w.flags() + (b < G ? b : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ok &= b >= G || (int)(f - ep) >= 0;
  }
  return __ballot(!ok) == 0ull;
}

__device__ __forceinline__ void exchange(const EncWs& w, unsigned ep) {
  drain_stores();
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid == 0) __hip_atomic_store(w.flags() + w.bid, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid < kWave) {
    unsigned spins = 0;
    for (;;) {
      if (all_arrived(w, ep)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {  // ~1 s: a block never arrived; flag it and let the launch drain
        if (tid == 0) __hip_atomic_fetch_or(w.errp, 4ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// Exchange with work: wave 0 raises the flag and polls as in exchange(); waves 1.. run `work()` (one
// bounded chunk per call; false = nothing left) until wave 0 reports the exchange complete, finish the
// chunk in hand and drain its stores.  Used to move per-candidate Philox words into the waits.
template <typename F>
__device__ __forceinline__ void exchange_work(const EncWs& w, unsigned ep, unsigned* s_xdone, F&& work) {
  const int tid = threadIdx.x;
  if (tid == 0) *s_xdone = 0u;
  drain_stores();
  __syncthreads();
  if (tid == 0) __hip_atomic_store(w.flags() + w.bid, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid < kWave) {
    unsigned spins = 0;
    for (;;) {
      if (all_arrived(w, ep)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {  // ~1 s: a block never arrived; flag it and let the launch drain
        if (tid == 0) __hip_atomic_fetch_or(w.errp, 4ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    if (tid == 0) __hip_atomic_store(s_xdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    while (__hip_atomic_load(s_xdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
      if (!work()) break;
    drain_stores();
  }
  __syncthreads();
}

struct SelState {
  unsigned lo;
  unsigned long long width;
  int shift;
  long long rem;
  int done;
  int narrowed;    // the last pick narrowed the range to one bin (need = rank inside it, from the top)
  unsigned T;
  long long need;
};

// copy c of the round-0 histogram
__device__ __forceinline__ unsigned* hist_copy(const EncWs& w, int c) {
  return w.hist() + (size_t)(c == 0 ? 0 : kMaxSlots + c - 1) * kHistStride;
}
// copy c's share of the candidate total (64-bit, after the above count and the max key)
__device__ __forceinline__ unsigned long long* hist_total(const EncWs& w, int c) {
  return reinterpret_cast<unsigned long long*>(hist_copy(w, c) + kHistBins + 2);
}

// after the exchange of round slot r: the summed histogram, its above-the-range count and max key (and,
// for round 0, the candidate total) read into LDS in one batch of coherent loads (one round trip)
__device__ __forceinline__ void load_hist(const EncWs& w, int r, unsigned* s_ghist, unsigned long long* s_ex,
                                          bool with_total) {
  constexpr int BPT = kHistBins / kET;
  unsigned* h = w.hist() + (size_t)r * kHistStride;
  const int tid = threadIdx.x;
  unsigned v[BPT];
  unsigned long long e = 0;
  if (r == 0) {  // round 0: the sum of the copies (all loads issued together)
    unsigned u[kHistCopies][BPT];
#pragma unroll
    for (int c = 0; c < kHistCopies; ++c)
#pragma unroll
      for (int i = 0; i < BPT; ++i) u[c][i] = ld_mem(&hist_copy(w, c)[tid + i * kET]);
    unsigned long long x[kHistCopies];
    if (tid < 2) {  // above count (summed), max key (the largest)
#pragma unroll
      for (int c = 0; c < kHistCopies; ++c) x[c] = ld_mem(&hist_copy(w, c)[kHistBins + tid]);
    } else if (tid == 2 && with_total) {  // the candidate total (summed)
#pragma unroll
      for (int c = 0; c < kHistCopies; ++c) x[c] = ld_mem64(hist_total(w, c));
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      v[i] = 0u;
#pragma unroll
      for (int c = 0; c < kHistCopies; ++c) v[i] += u[c][i];
    }
    if (tid < 3) {
      unsigned long long a = 0u;
#pragma unroll
      for (int c = 0; c < kHistCopies; ++c) a = tid != 1 ? a + x[c] : (x[c] > a ? x[c] : a);
      e = tid == 2 && !with_total ? 0ull : a;
    }
  } else {
#pragma unroll
    for (int i = 0; i < BPT; ++i) v[i] = ld_mem(&h[tid + i * kET]);
    if (tid < 2) e = ld_mem(&h[kHistBins + tid]);  // above count, max key
    else if (tid == 2 && with_total) e = ld_mem64(hist_total(w, 0));  // (never: only round 0 has a total)
  }
#pragma unroll
  for (int i = 0; i < BPT; ++i) s_ghist[tid + i * kET] = v[i];
  if (tid < 3) s_ex[tid] = e;
  __syncthreads();
}

// pick (identically in every block) from the loaded histogram; `cur` lives in LDS (block-uniform state
// kept out of registers: at 1024 threads a wave has 128 VGPRs, and the filter's live set left none).  `rem` is the rank (from the top) of
// the k-th largest key among keys >= lo, so it stays k; the round's `A` keys above the live range
// come first: if A >= rem the key lies above the range (re-range to [lo + width, max + 1)), otherwise
// pick the bin of rank rem - A and narrow to it.
__device__ __forceinline__ void pick_digit(const EncWs& w, SelState& cur, long long A, unsigned maxkey, const unsigned* s_ghist,
                           unsigned* s_err, unsigned long long* s_red) {
  __shared__ unsigned s_digit;
  __shared__ long long s_rem;
  if (threadIdx.x == 0) *s_err = 0;
  __syncthreads();
  // (the new state is written field by field by thread 0: a whole-struct copy lands in scratch)
  if (A >= cur.rem) {  // the k-th largest key is above the range (block-uniform branch)
    const unsigned long long nlo = (unsigned long long)cur.lo + cur.width;
    const unsigned long long top = (unsigned long long)maxkey + 1ull;
    const unsigned long long nw = top > nlo ? top - nlo : 0ull;
    if (nw == 0ull && threadIdx.x == 0)
      __hip_atomic_fetch_or(w.errp, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (threadIdx.x == 0) {
      cur.narrowed = 0;
      cur.lo = (unsigned)nlo;
      cur.width = nw ? nw : 1ull;
      cur.shift = range_shift(nw ? nw : 1ull, kHistBits);
    }
    __syncthreads();
    return;
  }
  {
    const long long rk[1] = {cur.rem - A};
    block_select_from_top<1>(s_ghist, rk, &s_digit, &s_rem, s_err, s_red);
  }
  const unsigned d = s_digit;
  const long long rr = s_rem;
  if (*s_err && threadIdx.x == 0) __hip_atomic_fetch_or(w.errp, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned nlo = cur.lo + (d << cur.shift);
  const int csh = cur.shift;
  __syncthreads();  // every thread has read cur, s_digit, s_rem
  if (threadIdx.x == 0) {
    cur.narrowed = 0;
    if (csh == 0) {
      cur.T = nlo;
      cur.need = rr;
      cur.done = 1;
    } else {
      cur.lo = nlo;
      cur.width = 1ull << csh;
      cur.shift = range_shift(1ull << csh, kHistBits);
      cur.narrowed = 1;
      cur.need = rr;
    }
  }
  __syncthreads();
}

// candidate p of this block: its LDS array, or (fallback, or more candidates than kCap) the block's x
// range itself — every element, since no later phase keeps an element below the floor anyway
template <class Src>
struct CandSrc {
  const unsigned* s_key;  // LDS candidates in index order (a reverse block's: offset by kCap - C)
  const unsigned* s_idx;
  unsigned* g_key;  // the HBM overflow: candidates kCap.. (gmode)
  unsigned* g_idx;
  Src x;
  int64_t b0;
  bool xmode;
  bool gmode;       // more candidates than LDS holds, all of them in LDS + the overflow
};
template <class Src>
__device__ __forceinline__ void cand_get(const CandSrc<Src>& c, unsigned p, unsigned& raw, unsigned& id) {
  if (c.xmode) {
    raw = __float_as_uint(c.x.get(c.b0 + p));
    id = (unsigned)(c.b0 + p);
  } else if (!c.gmode || p < (unsigned)kCap) {
    raw = c.s_key[p];
    id = c.s_idx[p];
  } else {  // (written by this block's waves in the filter pass, before the exchange that followed it)
    raw = ld_mem(c.g_key + (p - kCap));
    id = ld_mem(c.g_idx + (p - kCap));
  }
}

#ifdef FLC_SELECT_STAMPS
// phase stamps of block 0, kept in LDS and written out at the end (slots: filter 0-4, select 5-15;
// s_memrealtime, 100 MHz)
__device__ __forceinline__ unsigned long long* stamp_lds() {
  __shared__ unsigned long long s_stamp[16];
  return s_stamp;
}
#define STAMP(i)                                                                                 \
  do {                                                                                           \
    if (blockIdx.x == 0 && threadIdx.x == 0) stamp_lds()[i] = __builtin_amdgcn_s_memrealtime();  \
  } while (0)
#define STAMP_INIT()                                                                             \
  do {                                                                                           \
    if (threadIdx.x < 16) stamp_lds()[threadIdx.x] = 0ull;                                       \
    __syncthreads();                                                                             \
  } while (0)
#define STAMP_OUT(lo, hi)                                                                        \
  if (blockIdx.x == 0 && (int)threadIdx.x >= (lo) && (int)threadIdx.x < (hi))                    \
  w.stamps()[threadIdx.x] = stamp_lds()[threadIdx.x]
#define BLKT(i)                                                                                  \
  do {                                                                                           \
    if (threadIdx.x == 0) w.blkt()[blockIdx.x * 4 + (i)] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)
#else
#define STAMP(i) do { } while (0)
#define STAMP_INIT() do { } while (0)
#define STAMP_OUT(lo, hi) do { } while (0)
#define BLKT(i) do { } while (0)
#endif

// ------------------------------------------------------------------------------------------------
// sample kernel
// ------------------------------------------------------------------------------------------------
template <class Src>
__device__ __forceinline__ unsigned sample_one(const Src& x, int64_t n, int S, const EncWs& w, int j) {
  if (j >= S) return 0u;
  const int64_t pos = (S == n) ? (int64_t)j : (int64_t)(((double)j + 0.5) * (double)n / (double)S);
  const unsigned key = order_key(__float_as_uint(x.get(pos < n ? pos : n - 1)));
  w.sample()[j] = key;
  return key;
}

template <class Src>
__global__ __launch_bounds__(256) void topk_sample_kernel(Src x, int64_t n, int S, EncWs w) {
#ifdef FLC_SELECT_STAMPS  // diagnostic timeline: each sample block's start and end (blkt rows 512 + b)
  if (threadIdx.x == 0 && blockIdx.x < 256) w.blkt()[(512 + blockIdx.x) * 4] = __builtin_amdgcn_s_memrealtime();
#endif
  const int j = blockIdx.x * 256 + threadIdx.x;
  unsigned key = sample_one(x, n, S, w, j);
  if (w.compact) {  // (S == kSample: every lane holds a key) the wave's 8 largest keys, descending: the compact sample
    const int lane = (int)(threadIdx.x & (kWave - 1));
    unsigned mine = 0u;
#pragma unroll
    for (int r = 0; r < kTopPer; ++r) {
      const unsigned m = wave_max_u32(key);
      if (lane == r) mine = m;
      const unsigned long long at = __ballot(key == m);
      if (lane == __ffsll((long long)at) - 1) key = 0u;  // one instance of it leaves the wave's set
    }
    if (lane < kTopPer) w.samptop()[(j >> 6) * kTopPer + lane] = mine;
  }
#ifdef FLC_SELECT_STAMPS
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x < 256) w.blkt()[(512 + blockIdx.x) * 4 + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}

// one client of a batched call (flc_stacked_encode_batch[_delta]): its input, Philox seed and outputs.  `x` is the
// client's flat delta, or (delta batch) its table of local parameter pointers; the kernel's source argument is the
// prototype (the delta batch: offsets and global pointers shared by every client)
struct BatchEntry {
  const void* x;
  uint64_t seed;
  int* idx;
  uint8_t* codes;
  float* norm;
  unsigned* tiles;
  float* val;  // plain top-k batch (flc_topk_encode_batch): the kept values
};

// batched: every client's header state, flags and histograms ([0, kOffBlk) of each kOffStage header) zeroed in one
// launch at the start of a call (grid: blocks per header x headers) — except header 0's error word (EncState::err,
// the one every client ORs into and flc_topk_status reads), which stays sticky across calls until a reset
static_assert(offsetof(EncState, call) == 0 && offsetof(EncState, err) == 8, "the error word is bytes 8-15");
__global__ __launch_bounds__(256) void zero_headers_kernel(char* base, int n_words16) {
  uint4* p = reinterpret_cast<uint4*>(base + (size_t)blockIdx.y * kOffStage);
  for (int i = (int)blockIdx.x * 256 + (int)threadIdx.x; i < n_words16; i += (int)gridDim.x * 256) {
    if (i == 0 && blockIdx.y == 0) {
      reinterpret_cast<unsigned long long*>(p)[0] = 0ull;  // the call counter only
      continue;
    }
    p[i] = make_uint4(0u, 0u, 0u, 0u);
  }
}

// client g's element source from the prototype and its batch entry
__device__ __forceinline__ FlatSrc batch_src(const FlatSrc&, const BatchEntry& e) {
  return FlatSrc{static_cast<const float*>(e.x)};
}
__device__ __forceinline__ DeltaSrc batch_src(const DeltaSrc& proto, const BatchEntry& e) {
  DeltaSrc d = proto;
  d.t.lp = static_cast<const float* const*>(e.x);
  return d;
}

// batched: `per` blocks sample each client into its own header (and zero the client's header for its select: the
// state, the flags of its nb blocks, the histograms and accumulators — the `per` blocks of a client each take a
// slice; the sample keys lie past kOffBlk)
template <class Src>
__global__ __launch_bounds__(256) void topk_sample_batch_kernel(Src proto, const BatchEntry* __restrict__ tab,
                                                                int64_t n, int S, EncWs w, int per) {
  const int g = (int)blockIdx.x / per, sub = (int)blockIdx.x - g * per;
  w.base += (size_t)g * kOffStage;
  {
    constexpr int kW0 = (int)(kOffFlags / 16), kWH = (int)(kOffHist / 16), kWE = (int)(kOffBlk / 16);
    const int wf = (int)((size_t)w.nb * kFlagStride * 4 + 15) / 16;  // the select's flags
    const int nz = kW0 + wf + (kWE - kWH);
    uint4* p = reinterpret_cast<uint4*>(w.base);
    for (int i = sub * 256 + (int)threadIdx.x; i < nz; i += per * 256) {
      const int q = i < kW0 + wf ? i : kWH + (i - kW0 - wf);
      if (q == 0 && g == 0) {  // header 0: the call counter only — its error word (errp) stays sticky
        reinterpret_cast<unsigned long long*>(p)[0] = 0ull;
        continue;
      }
      p[q] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  (void)sample_one(batch_src(proto, tab[g]), n, S, w, sub * 256 + (int)threadIdx.x);
}

// ------------------------------------------------------------------------------------------------
// filter kernel: floor / ceiling from the sample, the HBM pass, staging + round-0 histogram
// ------------------------------------------------------------------------------------------------
struct FilterOut {
  unsigned C_b;            // candidates of this block (<= kCap of them in s_key / s_idx)
  unsigned t_lo;           // floor key
  unsigned long long t_hi; // ceiling key (exclusive)
  int64_t b0, b1;          // the block's element range
};

// floor / ceiling from the sample, the HBM pass into the block's LDS candidate arrays, the round-0 band
// histogram and counts; STAGE: also the staging copy of the candidates for a separate select kernel
// (SINGLE: a single-client select, which may take the compact sample; the batched selects do not)
template <bool STAGE, class Src, bool SINGLE = false>
__device__ __forceinline__ FilterOut filter_phase(const Src& x, int64_t n, const EncWs& w, int S,
                                                  long long rank_lo, long long rank_hi, int take_all,
                                                  unsigned* s_key, unsigned* s_idx, unsigned* s_hist,
                                                  unsigned (&s_wc)[2][kENW], unsigned long long* s_red,
                                                  unsigned* s_mx) {
  SampleLds& SL = *reinterpret_cast<SampleLds*>(s_key);  // the sample phase precedes every candidate write
  static_assert(sizeof(SampleLds) <= sizeof(unsigned) * kCap, "sample scratch must fit the key array");
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid >> 6;
  int64_t b0 = (int64_t)w.bid * w.M;
  int64_t b1 = b0 + w.M < n ? b0 + w.M : n;
  constexpr int SF = Src::SF;
  constexpr int64_t kWS = SF * 256;         // elements per wave step
  constexpr int64_t kBS = kENW * kWS;       // elements per block step (M is a multiple of it)
  using Step = typename Src::Step;
  const int nsteps = (int)cdiv_dev(b1 - b0, kBS);
  STAMP(0);

  // ---- floor / ceiling (identical in every block); the first step of the HBM pass is already in flight
  // meanwhile (issued after the sample keys, so waiting for the keys does not wait for it)
  Step va, vb;
  typename Src::Cursor cur;
  // (the wave's offset through readfirstlane: wave-uniform, so every step address and the DeltaSrc cursor stay scalar)
  const int64_t woff = (int64_t)__builtin_amdgcn_readfirstlane(wid) * kWS;
  const int64_t wb0 = b0 + woff;
  const int nfull = (int)((b1 - b0) / kBS);
  unsigned t_lo;
  unsigned long long t_hi;
  if (take_all) {
    t_lo = 0u;
    t_hi = 1ull << 32;
    if (w.bid == 0 && tid == 0) w.st()->sample_path = 2ull;
  } else {
    bool ok = false;
    const bool fast = rank_lo <= kET;  // grid-uniform
    if (SINGLE && w.compact && fast) {  // (single-client selects only; the batched ones skip the code)
      // The compact sample (the 8 largest keys of each 64-key wave of the sample, 4096 keys: 4 per thread, one 16-B
      // load instead of eight): the floor and the ceiling from it, both HBM steps issued right behind that load.
      // The floor's rank among the compact keys is a lower bound of its rank in the full sample; the two agree when
      // no wave of the sample has its 8th largest key at or above the floor (else, rarely — clustered inputs — the
      // general pick over the full sample runs).  Either way the floor only sets how many candidates are kept.
      const uint4 c4 = *reinterpret_cast<const uint4*>(w.samptop() + 4 * tid);
      x.template load<false>(cur, wb0, b1, lane, va);
      x.template load<false>(cur, wb0 + kBS, b1, lane, vb);
      unsigned keys[4] = {c4.x, c4.y, c4.z, c4.w};
      unsigned B = 0;
      int shB = 0;
      sample_fast_hist<4>(keys, S, SL, s_hist, &B, &shB);
      STAMP(1);
      ok = sample_fast_pick<4>(w.samptop(), S, rank_lo, rank_hi, B, shB, SL, s_hist, s_red, &t_lo, &t_hi);
      if (ok && (tid & 1) && c4.w >= t_lo) SL.bad = 1u;  // (odd threads hold keys 4-7 of a wave: .w its 8th largest)
      lds_barrier();
      ok = ok && SL.bad == 0u;
    } else {
      unsigned keys[kSPT];
      load_sample_keys(w.sample(), S, keys);
      // the first two steps stream while the floor / ceiling are picked (unconditional, clamped
      // in-range loads, so no wait is merged in): the first right away, the second in the registers the
      // keys leave free after the histogram
      x.template load<false>(cur, wb0, b1, lane, va);
      unsigned B = 0;
      int shB = 0;
      if (fast) sample_fast_hist<kSPT>(keys, S, SL, s_hist, &B, &shB);
      STAMP(1);
      x.template load<false>(cur, wb0 + kBS, b1, lane, vb);
      if (fast) ok = sample_fast_pick<kSPT>(w.sample(), S, rank_lo, rank_hi, B, shB, SL, s_hist, s_red, &t_lo, &t_hi);
    }
    if (!ok) sample_general(w.sample(), S, rank_lo, rank_hi, SL, s_hist, s_red, &t_lo, &t_hi);
    if (w.bid == 0 && tid == 0) w.st()->sample_path = ok ? 0ull : 1ull;
  }
  // the float predicate !(v < key_value(t_lo)) equals key >= t_lo for t_lo <= key(+inf)
  if (t_lo > 0xff800000u) t_lo = 0xff800000u;
  if (t_hi <= (unsigned long long)t_lo || t_hi > (1ull << 32)) t_hi = 1ull << 32;
  if (w.bid == 0 && tid == 0) {
    w.st()->t_lo = t_lo;
    w.st()->t_hi = t_hi;
  }
  lds_barrier();  // sample scratch (aliases s_key) dead from here (LDS-only: the prefetched steps stay in flight)
  for (int i = tid; i < kHistBins; i += kET) s_hist[i] = 0u;
  lds_barrier();
  STAMP(2);
  BLKT(0);

  // ---- the HBM pass
  const float tf = floor_value(t_lo);
  FilterCtx fc;
  fc.s_key = s_key;
  fc.s_idx = s_idx;
  fc.gcap = STAGE ? 0u : w.ovf;  // (the split path stages LDS only)
  fc.g_key = w.ovf_key(w.bid);
  fc.g_idx = w.ovf_idx(w.bid);
  fc.s_hist = s_hist;
  fc.t_lo = t_lo;
  fc.width0 = t_hi - t_lo;
  fc.sh0 = range_shift(fc.width0, kHistBits);
  fc.above = 0;
  fc.mk = 0;
  fc.swept = 0;
  unsigned base = 0;
  {
    // full block steps in a two-deep software pipeline; every load in the loop body is unconditional
    // (a conditional prefetch makes the compiler copy the loaded registers on a side path, and the copy
    // waits for the load), and the partial tail step is peeled off
    int s = 0;
    if (take_all && nfull > 0) x.template load<true>(cur, wb0, b1, lane, va);
    if (!take_all && nfull >= 3) {  // peeled first iteration: steps 0 and 1 are in flight already
      step_process<true, Step, SF>(va, wb0, b1, tf, s_wc, 0, base, fc);
      x.template load<true>(cur, wb0 + 2 * kBS, b1, lane, va);
      step_process<true, Step, SF>(vb, wb0 + kBS, b1, tf, s_wc, 1, base, fc);
      s = 2;
    }
    for (; s + 3 <= nfull; s += 2) {
      const int64_t wa = wb0 + (int64_t)s * kBS, wbn = wa + kBS;
      x.template load<true>(cur, wbn, b1, lane, vb);
      step_process<true, Step, SF>(va, wa, b1, tf, s_wc, 0, base, fc);
      x.template load<true>(cur, wbn + kBS, b1, lane, va);
      step_process<true, Step, SF>(vb, wbn, b1, tf, s_wc, 1, base, fc);
    }
    if (s + 2 == nfull) {
      const int64_t wa = wb0 + (int64_t)s * kBS, wbn = wa + kBS;
      x.template load<true>(cur, wbn, b1, lane, vb);
      step_process<true, Step, SF>(va, wa, b1, tf, s_wc, 0, base, fc);
      step_process<true, Step, SF>(vb, wbn, b1, tf, s_wc, 1, base, fc);
      s += 2;
    } else if (s + 1 == nfull) {
      step_process<true, Step, SF>(va, wb0 + (int64_t)s * kBS, b1, tf, s_wc, 0, base, fc);
      ++s;
    }
    if (s < nsteps) {  // the partial last step of the last block
      const int64_t wa = wb0 + (int64_t)s * kBS;
      x.template load<false>(cur, wa, b1, lane, va);
      step_process<false, Step, SF>(va, wa, b1, tf, s_wc, s & 1, base, fc);
    }
  }
  const unsigned C_b = base;
  __syncthreads();
  STAMP(3);
  BLKT(1);
  {  // band histogram / above / max of the stored candidates
    const unsigned nst = C_b < (unsigned)kCap ? C_b : (unsigned)kCap;
    for (unsigned p = fc.swept + tid; p < nst; p += kET) band_bin(fc, p);
    __syncthreads();
  }

  // ---- staging (16-B stores; split path only) and the round-0 histogram / counts
  if (STAGE) {
    const unsigned nst = C_b < (unsigned)kCap ? C_b : (unsigned)kCap;
    uint4* dk = reinterpret_cast<uint4*>(w.stage_key(w.bid));
    uint4* di = reinterpret_cast<uint4*>(w.stage_idx(w.bid));
    const uint4* sk = reinterpret_cast<const uint4*>(s_key);
    const uint4* si = reinterpret_cast<const uint4*>(s_idx);
    for (unsigned q = tid; q < (nst + 3u) / 4u; q += kET) {
      dk[q] = sk[q];
      di[q] = si[q];
    }
  }
  unsigned* h = hist_copy(w, w.bid % kHistCopies);
  for (int i = tid; i < kHistBins; i += kET)
    if (s_hist[i]) atomicAdd(&h[i], s_hist[i]);
  const unsigned long long ab = block_sum<unsigned long long, kENW>((unsigned long long)fc.above, s_red);
  const unsigned mkw = wave_max_u32(fc.mk);
  if (lane == 0) s_mx[wid] = mkw;
  __syncthreads();
  if (tid == 0) {
    unsigned m = 0;
    for (int i = 0; i < kENW; ++i) m = s_mx[i] > m ? s_mx[i] : m;
    if (ab) atomicAdd(&h[kHistBins], (unsigned)ab);
    atomicMax(&h[kHistBins + 1], m);
    atomicAdd(hist_total(w, w.bid % kHistCopies), (unsigned long long)C_b);
    if (STAGE) w.blk_c()[w.bid] = C_b;
  }
  STAMP(4);
  BLKT(2);
  FilterOut o;
  o.C_b = C_b;
  o.t_lo = t_lo;
  o.t_hi = t_hi;
  o.b0 = b0;
  o.b1 = b1;
  return o;
}

template <class Src>
__global__ __launch_bounds__(kET) void topk_filter_kernel(Src x, int64_t n, EncWs w, int S,
                                                          long long rank_lo, long long rank_hi, int take_all) {
  __shared__ __attribute__((aligned(16))) unsigned s_key[kCap];
  __shared__ __attribute__((aligned(16))) unsigned s_idx[kCap];
  __shared__ unsigned s_hist[kHistBins];
  __shared__ unsigned s_wc[2][kENW];
  __shared__ unsigned long long s_red[kENW];
  __shared__ unsigned s_mx[kENW];
  STAMP_INIT();
  w.bid = (int)blockIdx.x;
  w.nb = (int)gridDim.x;
  (void)filter_phase<true>(x, n, w, S, rank_lo, rank_hi, take_all, s_key, s_idx, s_hist, s_wc, s_red, s_mx);
  STAMP_OUT(0, 5);
}

// ------------------------------------------------------------------------------------------------
// select kernel: the k-th largest key, the block offsets, the ordered compaction
// ------------------------------------------------------------------------------------------------
// FUSED: the filter phase runs first in the same kernel (one exchange after it): the candidates stay in
// LDS, so the staging round trip through HBM and a kernel boundary are gone
// BATCH (stacked, fused, flat input only): blocks [g * w.nb, (g + 1) * w.nb) run client g's select with its own
// header, staging area, input, seed and outputs (tab[g]); the selects never exchange with each other
template <bool STACKED, bool FUSED, class Src, bool BATCH = false>
__global__ __launch_bounds__(kET) void topk_select_kernel(Src x, int64_t n, long long k, EncWs w,
                                                          int* __restrict__ idx_out, float* __restrict__ val_out,
                                                          uint8_t* __restrict__ code_out, float* __restrict__ norm_out,
                                                          int levels, double step, uint64_t seed, uint64_t counter,
                                                          unsigned* __restrict__ tile_out, int S, long long rank_lo,
                                                          long long rank_hi, int take_all,
                                                          const BatchEntry* __restrict__ tab = nullptr) {
  if constexpr (BATCH) {
    static_assert(FUSED, "batched selects are the fused encode");
    const int g = (int)blockIdx.x / w.nb;  // (w.nb: blocks per client, set by the host)
    w.bid = (int)blockIdx.x - g * w.nb;
    w.base += (size_t)g * kOffStage;
    w.var += (size_t)g * w.vstride;
    const BatchEntry e = tab[g];
    x = batch_src(x, e);
    seed = e.seed;
    idx_out = e.idx;
    code_out = e.codes;
    val_out = e.val;
    norm_out = e.norm;
    tile_out = e.tiles;
  } else {
    w.bid = (int)blockIdx.x;
    w.nb = (int)gridDim.x;
  }
  __shared__ __attribute__((aligned(16))) unsigned s_key[kCap];
  __shared__ __attribute__((aligned(16))) unsigned s_idx[kCap];
  __shared__ unsigned s_hh[2 * kHistBins];  // the round / global histograms
  unsigned* const s_hist = s_hh;
  unsigned* const s_ghist = s_hh + kHistBins;
  __shared__ unsigned long long s_red[kENW];
  __shared__ unsigned s_mx[kENW];
  __shared__ unsigned s_err;
  __shared__ unsigned long long s_glob[4];
  __shared__ unsigned long long s_ex[3];
  __shared__ SelState s_cur, s_prev;
  __shared__ unsigned long long s_sum[kENW * 6];
#ifdef FLC_SELECT_STAMPS  // diagnostic timeline: each block's first instruction (blkt rows 256 + b)
  if (threadIdx.x == 0 && blockIdx.x < 256) w.blkt()[(256 + blockIdx.x) * 4] = __builtin_amdgcn_s_memrealtime();
#endif
  STAMP_INIT();
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid >> 6;
  int64_t b0 = (int64_t)w.bid * w.M;
  int64_t b1 = b0 + w.M < n ? b0 + w.M : n;
  unsigned* hist = w.hist();
  unsigned C_b;
  unsigned ep;
  const unsigned* s_keyl = s_key;  // the block's LDS candidates in index order
  const unsigned* s_idxl = s_idx;
  // Philox words of the candidates (stacked), precomputed in exchange waits into the block's staging
  // area (unused by the fused path; the split path has copied its staged candidates to LDS by then):
  // chunk c = wave range c % kENW, its 64 candidates of iteration c / kENW; chunks [0, s_rnext) are
  // complete after the exchange that ran them
  __shared__ unsigned s_rnext, s_xdone;
  unsigned* const rnd = w.stage_key(w.bid);
  unsigned rnd_n = 0;  // candidates covered by the chunk map (0: none)
  auto rnd_work = [&]() -> bool {
    unsigned c = 0;
    if (lane == 0) c = atomicAdd(&s_rnext, 1u);
    c = (unsigned)__builtin_amdgcn_readlane((int)c, 0);  // (lane 0 claimed: a readlane, not an LDS shuffle)
    const unsigned Qn = ((rnd_n + kENW - 1) / kENW + kWave - 1) / kWave * kWave;
    if (c >= (Qn / kWave) * (unsigned)kENW) return false;
    const unsigned wr = c % kENW, it = c / kENW;
    const unsigned r0 = wr * Qn < rnd_n ? wr * Qn : rnd_n, r1 = r0 + Qn < rnd_n ? r0 + Qn : rnd_n;
    const unsigned p = r0 + it * kWave + lane;
    if (p < r1) {
      const unsigned id = s_idxl[p];
      rnd[p] = pick(philox_group((uint64_t)id >> 2, seed, counter), (int)(id & 3u));
    }
    return true;
  };
  if (FUSED) {
    __shared__ unsigned s_wc[2][kENW];
    if (tid == 0) s_glob[2] = ld_mem64(&w.st()->call);  // (read before any exchange of this call)
    const FilterOut fo =
        filter_phase<false, Src, !BATCH>(x, n, w, S, rank_lo, rank_hi, take_all, s_key, s_idx, s_hist, s_wc, s_red,
                                         s_mx);
    C_b = fo.C_b;
    b0 = fo.b0;
    b1 = fo.b1;
    if (tid == 0) {
      s_glob[0] = fo.t_lo;
      s_glob[1] = fo.t_hi;
    }
    ep = (unsigned)s_glob[2] * kEpochStride;  // (s_glob[2] was written before the filter's barriers)
    if (tid == 0) s_rnext = 0u;
    if (STACKED) {  // (x-mode blocks, C_b > kCap, have no chunks; if the call falls back, none is used)
      rnd_n = C_b <= (unsigned)kCap ? C_b : 0u;
      exchange_work(w, ++ep, &s_xdone, rnd_work);  // every block's round-0 histogram, counts, max are in
    } else {
      exchange(w, ++ep);
    }
    STAMP(5);
  } else {
    // ---- one batch of loads: this block's candidates (staging), the round-0 histogram and counts
    STAMP(5);
    C_b = w.blk_c()[w.bid];
    const unsigned nst = C_b < (unsigned)kCap ? C_b : (unsigned)kCap;
    {
      const uint4* sk = reinterpret_cast<const uint4*>(w.stage_key(w.bid));
      const uint4* si = reinterpret_cast<const uint4*>(w.stage_idx(w.bid));
      uint4* dk = reinterpret_cast<uint4*>(s_key);
      uint4* di = reinterpret_cast<uint4*>(s_idx);
      for (unsigned q = tid; q < (nst + 3u) / 4u; q += kET) {
        dk[q] = sk[q];
        di[q] = si[q];
      }
    }
    if (tid == 0) {
      s_glob[0] = w.st()->t_lo;
      s_glob[1] = w.st()->t_hi;
      s_glob[2] = ld_mem64(&w.st()->call);
    }
    ep = 0;  // set below, after the barrier
    if (tid == 0) s_rnext = 0u;
  }
  load_hist(w, 0, s_ghist, s_ex, true);  // (ends in a barrier)
  const unsigned t_lo = (unsigned)s_glob[0];
  const unsigned long long t_hi = s_glob[1];
  const unsigned call = (unsigned)s_glob[2];
  if (!FUSED) ep = call * kEpochStride;
  const unsigned long long C_tot = s_ex[2];
  const bool fb = (long long)C_tot < k;  // grid-uniform
  unsigned maxkey = (unsigned)s_ex[1];
  long long A_cur = (long long)s_ex[0];
  int slot = 0;
  unsigned long long a_blk = 0;
  STAMP(6);

  SelState& cur = s_cur;
  SelState& prev = s_prev;
  if (tid == 0) {
    cur.lo = t_lo;
    cur.width = t_hi - t_lo;
    cur.shift = range_shift(cur.width, kHistBits);
    cur.rem = k;
    cur.done = 0;
    cur.narrowed = 0;
    cur.T = 0;
    cur.need = 0;
    prev = cur;
  }
  CandSrc<Src> src;
  src.s_key = s_keyl;
  src.s_idx = s_idxl;
  src.x = x;
  src.b0 = b0;
  src.g_key = w.ovf_key(w.bid);
  src.g_idx = w.ovf_idx(w.bid);
  const unsigned gcap = FUSED ? w.ovf : 0u;
  src.xmode = fb || C_b > (unsigned)kCap + gcap;  // block-uniform
  src.gmode = !src.xmode && C_b > (unsigned)kCap;
  const unsigned ncand = src.xmode ? (unsigned)(b1 - b0) : C_b;

  auto flush = [&](int sl, unsigned above_t, unsigned mk_t) {
    unsigned* h = hist + (size_t)sl * kHistStride;
    for (int i = tid; i < kHistBins; i += kET)
      if (s_hist[i]) atomicAdd(&h[i], s_hist[i]);
    const unsigned long long ab = block_sum<unsigned long long, kENW>((unsigned long long)above_t, s_red);
    const unsigned mkw = wave_max_u32(mk_t);
    if (lane == 0) s_mx[wid] = mkw;
    __syncthreads();
    if (tid == 0) {
      unsigned m = 0;
      for (int i = 0; i < kENW; ++i) m = s_mx[i] > m ? s_mx[i] : m;
      if (ab) atomicAdd(&h[kHistBins], (unsigned)ab);
      atomicMax(&h[kHistBins + 1], m);
    }
    return ab;
  };

  if (fb) {
    // fallback pass: every element is a candidate; a round over the full key range from x
    if (tid == 0) {
      cur.lo = 0u;
      cur.width = 1ull << 32;
      cur.shift = range_shift(cur.width, kHistBits);
    }
    slot = 1;
    for (int i = tid; i < kHistBins; i += kET) s_hist[i] = 0u;
    __syncthreads();
    unsigned mk = 0;
    const int sh = cur.shift;
    for (unsigned p0 = 0; p0 < ncand; p0 += kET) {
      const unsigned p = p0 + tid;
      unsigned raw = 0, id = 0;
      if (p < ncand) cand_get(src, p, raw, id);
      const unsigned key = order_key(raw);
      mk = (p < ncand && key > mk) ? key : mk;
      hist_add(s_hist, key >> sh, p < ncand);
    }
    __syncthreads();
    a_blk = flush(slot, 0u, mk);
    exchange(w, ++ep);
    load_hist(w, slot, s_ghist, s_ex, false);
    maxkey = (unsigned)s_ex[1];
    A_cur = (long long)s_ex[0];
  }
  // pick on the histogram just summed
  __syncthreads();
  if (tid == 0) prev = cur;
  pick_digit(w, cur, A_cur, maxkey, s_ghist, &s_err, s_red);
  STAMP(7);
  unsigned long long pre = 0, tot = 0;
  bool counted = false, wave_counted = false;
  // the compaction's wave ranges: wave `wid` owns candidates [cq0, cq1) of this block
  const unsigned cQ = ((ncand + kENW - 1) / kENW + kWave - 1) / kWave * kWave;
  const unsigned cq0 = (unsigned)wid * cQ < ncand ? (unsigned)wid * cQ : ncand;
  const unsigned cq1 = cq0 + cQ < ncand ? cq0 + cQ : ncand;
  __shared__ unsigned long long s_wcnt[kENW];  // per wave range: strict << 32 | ties
  if (!fb && cur.narrowed && slot == 0) {
    // ---- in-bin exchange: every block publishes its candidates inside the chosen bin (~3 per block at
    // the headline) and its count of candidates above the bin; one exchange later every block resolves T
    // among those keys and forms its own prefix locally: no second histogram round and no separate
    // count exchange.  Falls through to the histogram rounds if any list overflows.
    __shared__ unsigned s_nl;
    __shared__ unsigned s_mykey[kInbinMax], s_mywv[kInbinMax];
    if (tid == 0) s_nl = 0u;
    __syncthreads();
    const unsigned lo0 = cur.lo;
    const unsigned long long wd0 = cur.width;
    // a block's list slots: 32, or more when the select has few blocks (a batched client's 2-4: its in-bin keys per
    // block are many more, and the gathered list still holds kInbinAll)
    const unsigned cap = (unsigned)max(kInbin, min(kInbinMax, kInbinAll / max(w.nb, 1)));
    unsigned* my_list = w.inbin() + (size_t)w.bid * cap;
    // scanned in the compaction's wave ranges: the count above the bin per wave range plus the wave of
    // each of my in-bin keys give the compaction its per-wave strict / tie counts once T is known
    unsigned gtw = 0;
    auto scan_one = [&](const unsigned p, const unsigned raw) {
      const unsigned key = order_key(raw);
      const unsigned long long rel = (unsigned long long)key - lo0;
      const bool valid = p < cq1 && key >= lo0 && key >= t_lo;  // (x-mode: below the floor never counts)
      gtw += (unsigned)__popcll(__ballot(valid && rel >= wd0));
      const bool f = valid && rel < wd0;
      const unsigned long long bm = __ballot(f);
      if (bm) {
        unsigned base_l = 0;
        if (lane == 0) base_l = atomicAdd(&s_nl, (unsigned)__popcll(bm));
        base_l = (unsigned)__builtin_amdgcn_readlane((int)base_l, 0);
        const unsigned q = base_l + __builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
        if (f && q < cap) {  // write-through: read by other XCDs after the exchange
          __hip_atomic_store(my_list + q, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_mykey[q] = key;
          s_mywv[q] = (unsigned)wid;
        }
      }
    };
    if (!src.xmode && !src.gmode) {
      // LDS candidates: 4 rounds of reads at clamped indices issued together, then scanned
      const unsigned wq0 = (unsigned)__builtin_amdgcn_readfirstlane((int)cq0);
      const unsigned wq1 = (unsigned)__builtin_amdgcn_readfirstlane((int)cq1);
      const unsigned pl = wq1 > 0u ? wq1 - 1u : 0u;
      for (unsigned p00 = wq0; p00 < wq1; p00 += 4u * kWave) {
        unsigned r4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned p = p00 + (unsigned)(j * kWave) + lane;
          r4[j] = src.s_key[p < wq1 ? p : pl];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) scan_one(p00 + (unsigned)(j * kWave) + lane, r4[j]);
      }
    } else {
      for (unsigned p0 = cq0; p0 < cq1; p0 += kWave) {
        const unsigned p = p0 + lane;
        unsigned raw = 0, id = 0;
        if (p < cq1) cand_get(src, p, raw, id);
        scan_one(p, raw);
      }
    }
    if (lane == 0) s_wcnt[wid] = (unsigned long long)gtw << 32;
    lds_barrier();  // (the list stores drain in the exchange)
    if (tid == 0) {
      unsigned long long gt = 0;
      for (int v2 = 0; v2 < kENW; ++v2) gt += s_wcnt[v2] >> 32;
      st_mem64(&w.blk_cnt()[w.bid], ((unsigned long long)s_nl << 32) | (gt & 0xffffffffull));
    }
    STAMP(8);
    if (STACKED) {
      if (!FUSED) rnd_n = src.xmode ? 0u : ncand;
      exchange_work(w, ++ep, &s_xdone, rnd_work);
    } else {
      exchange(w, ++ep);
    }
    STAMP(9);
    // all-gather in ONE batch of coherent loads: every block's list size and count above the bin, and
    // all list slots (sizes are checked afterwards)
    unsigned* s_lkey = s_ghist;               // <= kInbinAll keys
    unsigned* s_lblk = s_ghist + kInbinAll;   // their blocks
    static_assert(2 * kInbinAll <= kHistBins, "in-bin list fits the histogram buffer");
    __shared__ unsigned s_nb[kMaxBlocks];
    __shared__ unsigned s_ovf, s_nall;
    constexpr int kLW = 8;  // list words per thread per batch (G <= 256: one batch)
    const int words = w.nb * (int)cap;
    unsigned long long meta = 0;
    unsigned lw[kLW];
    if (tid < w.nb) meta = ld_mem64(&w.blk_cnt()[tid]);
#pragma unroll
    for (int i = 0; i < kLW; ++i) {
      const int j = i * kET + tid;
      lw[i] = j < words ? ld_mem(w.inbin() + j) : 0u;
    }
    if (tid == 0) { s_ovf = 0u; s_nall = 0u; }
    __syncthreads();
    unsigned long long my_gt = 0, pre_gt = 0;
    if (tid < w.nb) {
      const unsigned nb = (unsigned)(meta >> 32);
      s_nb[tid] = nb;
      my_gt = meta & 0xffffffffull;
      pre_gt = tid < w.bid ? my_gt : 0ull;
      if (nb > cap) atomicOr(&s_ovf, 1u);
    }
    __syncthreads();
    if (s_ovf == 0u) {
      for (int c0 = 0; c0 < words; c0 += kLW * kET) {
        if (c0 > 0) {  // more than 256 blocks: further batches
#pragma unroll
          for (int i = 0; i < kLW; ++i) {
            const int j = c0 + i * kET + tid;
            lw[i] = j < words ? ld_mem(w.inbin() + j) : 0u;
          }
        }
#pragma unroll
        for (int i = 0; i < kLW; ++i) {
          const int j = c0 + i * kET + tid;
          const int bb = j / (int)cap;
          const bool v = j < words && (unsigned)(j % (int)cap) < s_nb[bb < w.nb ? bb : 0];
          const unsigned long long bm = __ballot(v);
          if (bm) {
            unsigned base_l = 0;
            if (lane == 0) base_l = atomicAdd(&s_nall, (unsigned)__popcll(bm));
            base_l = (unsigned)__builtin_amdgcn_readlane((int)base_l, 0);
            const unsigned q = base_l + __builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
            if (v && q < (unsigned)kInbinAll) {
              s_lkey[q] = lw[i];
              s_lblk[q] = (unsigned)bb;
            }
          }
        }
      }
      __syncthreads();
      STAMP(10);
      if (s_nall <= (unsigned)kInbinAll) {  // block-uniform
        const unsigned nall = s_nall;
        // exact k-th largest among the in-bin keys: rank cur.need from the top, local radix passes
        unsigned lo = lo0;
        unsigned long long width = wd0;
        long long r = cur.need;
        __shared__ unsigned s_d;
        __shared__ long long s_r;
        for (int pass = 0; pass < 4; ++pass) {
          const int sh = range_shift(width, kHistBits);
          for (int i = tid; i < kHistBins; i += kET) s_hist[i] = 0u;
          __syncthreads();
          for (unsigned p0 = 0; p0 < ((nall + 63u) & ~63u); p0 += kET) {
            const unsigned p = p0 + tid;
            const unsigned key = p < nall ? s_lkey[p] : lo;
            const unsigned long long rel = (unsigned long long)key - lo;
            hist_add(s_hist, (unsigned)(rel >> sh), p < nall && key >= lo && rel < width);
          }
          __syncthreads();
          {
            const long long rk[1] = {r};
            block_select_from_top<1>(s_hist, rk, &s_d, &s_r, &s_err, s_red);
          }
          lo += s_d << sh;
          r = s_r;
          width = 1ull << sh;
          __syncthreads();
          if (sh == 0) break;
        }
        if (tid == 0) {
          cur.T = lo;
          cur.need = r;
          cur.done = 1;
        }
        STAMP(11);
        // strict / tie counts: above-the-bin counts + in-bin keys > T / == T, by block
        const unsigned T0 = lo;
        unsigned long long ps = 0, pt = 0, as = 0, at = 0;
        for (unsigned p = tid; p < nall; p += kET) {
          const unsigned key = s_lkey[p], bb = s_lblk[p];
          const unsigned long long s1 = key > T0 ? 1ull : 0ull, t1 = key == T0 ? 1ull : 0ull;
          as += s1;
          at += t1;
          if (bb < w.bid) { ps += s1; pt += t1; }
        }
        // the four in-bin counts are <= kInbinAll: 16-bit fields of one word
        static_assert(kInbinAll < 65536, "16-bit count fields");
        unsigned long long sums[3] = {as | (at << 16) | (ps << 32) | (pt << 48), my_gt, pre_gt};
        block_sum_n<3>(sums, s_sum);
        const unsigned long long A_s = sums[0] & 0xffffull, A_t = (sums[0] >> 16) & 0xffffull;
        const unsigned long long P_s = (sums[0] >> 32) & 0xffffull, P_t = sums[0] >> 48;
        pre = ((sums[2] + P_s) << 32) | P_t;
        tot = ((sums[1] + A_s) << 32) | A_t;
        counted = true;
        // (T0 >= t_lo: every key > T0 or == T0 passed the floor test of the scan above)
        if (T0 >= t_lo && tid < (int)s_nl) {
          const unsigned key = s_mykey[tid];
          atomicAdd(&s_wcnt[s_mywv[tid]], (key > T0 ? (1ull << 32) : 0ull) + (key == T0 ? 1ull : 0ull));
        }
        wave_counted = T0 >= t_lo;
      }
    }
    __syncthreads();
    STAMP(12);
  }
  // histogram rounds over the block's candidates until T is resolved (rare paths)
  if (!counted && cur.narrowed && !fb && slot == 0) {
    // the round-0 local histogram is not kept by this kernel: nothing to reuse, start a round
  }
  for (int guard = 0; !cur.done && guard < kMaxSlots && slot + 1 < kMaxSlots; ++guard) {
    ++slot;
    for (int i = tid; i < kHistBins; i += kET) s_hist[i] = 0u;
    __syncthreads();
    const unsigned lo = cur.lo;
    const unsigned long long wd = cur.width;
    const int sh = cur.shift;
    unsigned above = 0;
    const unsigned pend = (ncand + kET - 1) / kET * kET;
    for (unsigned p0 = 0; p0 < pend; p0 += kET) {
      const unsigned p = p0 + tid;
      unsigned raw = 0, id = 0;
      if (p < ncand) cand_get(src, p, raw, id);
      const unsigned key = order_key(raw);
      const unsigned long long rel = (unsigned long long)key - lo;
      const bool in = p < ncand && key >= lo;
      above += (in && rel >= wd) ? 1u : 0u;
      hist_add(s_hist, (unsigned)(rel >> sh), in && rel < wd);
    }
    __syncthreads();
    a_blk = flush(slot, above, 0u);
    exchange(w, ++ep);
    load_hist(w, slot, s_ghist, s_ex, false);
    if (tid == 0) prev = cur;
    pick_digit(w, cur, (long long)s_ex[0], maxkey, s_ghist, &s_err, s_red);
  }
  __syncthreads();
  if (!cur.done && w.bid == 0 && tid == 0)
    __hip_atomic_fetch_or(w.errp, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned T = cur.T;
  const long long need = cur.need;
  if (!counted) {
    // ---- counts from the resolving round's local histogram: strict = above + bins past T's bin
    // (the round-0 band resolving directly has no local histogram here: count from the candidates)
    unsigned long long cnt = 0;  // strict << 32 | tie
    if (slot == 0) {
      const unsigned pend = (ncand + kET - 1) / kET * kET;
      for (unsigned p0 = 0; p0 < pend; p0 += kET) {
        const unsigned p = p0 + tid;
        unsigned raw = 0, id = 0;
        if (p < ncand) cand_get(src, p, raw, id);
        const unsigned key = order_key(raw);
        cnt += (p < ncand && key > T) ? (1ull << 32) : 0ull;
        cnt += (p < ncand && key == T) ? 1ull : 0ull;
      }
    } else {
      const unsigned d = T - prev.lo;  // the resolving round has shift 0: bin = key - lo
      for (int i = tid; i < kHistBins; i += kET) {
        const unsigned hv = s_hist[i];
        cnt += ((unsigned)i > d ? ((unsigned long long)hv << 32) : 0ull) + ((unsigned)i == d ? hv : 0ull);
      }
    }
    const unsigned long long both = block_sum<unsigned long long, kENW>(cnt, s_red) + (slot == 0 ? 0ull : (a_blk << 32));
    if (tid == 0) st_mem64(&w.blk_cnt()[w.bid], both);
    exchange(w, ++ep);
    const unsigned long long v = tid < w.nb ? ld_mem64(&w.blk_cnt()[tid]) : 0ull;
    unsigned long long t_all;
    const unsigned long long ex = block_excl_scan<unsigned long long, kENW>(v, s_red, &t_all);
    if (tid == w.bid) s_glob[3] = ex;
    __syncthreads();
    pre = s_glob[3];
    tot = t_all;
  }
  STAMP(13);
  const long long strict_tot = (long long)(tot >> 32), ties_tot = (long long)(tot & 0xffffffffull);
  // every hist / acc read of this call happened before the last exchange: zero them for the next call
  // (my slice), and the call counter advances
  {
    unsigned* z = hist;
    const int per = (kZeroWords + w.nb - 1) / w.nb;
    const int z0 = w.bid * per, z1 = z0 + per < kZeroWords ? z0 + per : kZeroWords;
    for (int i = z0 + tid; i < z1; i += kET) z[i] = 0u;
  }
  if (w.bid == 0 && tid == 0) {
    (void)__hip_atomic_fetch_add(&w.st()->call, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    EncState* st = w.st();
    st->C = C_tot;
    st->fallback = fb ? 1ull : 0ull;
    st->T = T;
    st->maxkey = maxkey;
    st->rounds = (unsigned long long)slot + 1ull;
    st->need = (unsigned long long)need;
    st->ties = (unsigned long long)ties_tot;
    st->strict = (unsigned long long)strict_tot;
    if (strict_tot + need != k || need > ties_tot)
      __hip_atomic_fetch_or(w.errp, 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- ordered compaction: wave `wid` owns candidates [wid * Q, (wid + 1) * Q) of this block
  const long long skip = ties_tot - need;  // ties with global tie rank < skip are dropped
  float nrm = 0.0f;
  if (STACKED) {
    const float a = fabsf(key_value(maxkey)), b = fabsf(key_value(T));
    nrm = (isnan(a) || isnan(b)) ? __uint_as_float(0x7fc00000u) : (a > b ? a : b);
    if (w.bid == 0 && tid == 0) *norm_out = nrm;
  }
  const bool nrm_ok = nrm > 0.0f && nrm <= 3.402823466e38f;
  // tile pointers (CSR over FLC_TILE-output tiles): kept entries per tile of this block, counted in the
  // compaction, scanned afterwards (block ranges are whole tiles: M is a multiple of kBlockStep)
  // Tile pointers (CSR over FLC_TILE-output tiles) straight from the compaction, no block scan: wave w owns
  // the tiles whose first element lies in (lo_w, hi_w], the ids just below its first candidate and at
  // its last one (block edges at b0 - 1 and b1 - 1), and gives each the position of the first kept entry
  // at or after the tile's start: a kept entry fills the tiles that start after the previous kept entry,
  // and the wave's last kept entry's successor position fills the rest up to hi_w.
#if FLC_CALIB_NOTILES  // calibration builds only: results invalid
  const bool tiled = false;
#else
  const bool tiled = tile_out != nullptr;
#endif
  const unsigned q0 = cq0, q1 = cq1;
  const bool tile_owner = tiled && (q0 < q1 || (ncand == 0u && wid == 0));  // (wave-uniform)
  int64_t tile_prev = -1, tile_hi = -1;  // element ids
  if (tile_owner) {
    unsigned r0 = 0, i0 = 0, r1 = 0, i1 = 0;
    if (q0 > 0u) cand_get(src, q0 - 1u, r0, i0);
    if (q1 > 0u && q1 < ncand) cand_get(src, q1 - 1u, r1, i1);
    tile_prev = q0 == 0u ? b0 - 1 : (int64_t)i0;
    tile_hi = q1 >= ncand ? b1 - 1 : (int64_t)i1;
  }
  if (!wave_counted) {  // pass 1: this wave's strict / tie counts (the in-bin path counted them already)
    unsigned ws = 0, wt = 0;
    for (unsigned p0 = q0; p0 < q1; p0 += kWave) {
      const unsigned p = p0 + lane;
      unsigned raw = 0, id = 0;
      if (p < q1) cand_get(src, p, raw, id);
      const unsigned key = order_key(raw);
      ws += __popcll(__ballot(p < q1 && key > T));
      wt += __popcll(__ballot(p < q1 && key == T));
    }
    __syncthreads();
    if (lane == 0) s_wcnt[wid] = ((unsigned long long)ws << 32) | wt;
  }
  lds_barrier();  // (LDS-only: the histogram zeroing stores need no wait)
  long long s_before = (long long)(pre >> 32), t_before = (long long)(pre & 0xffffffffull);
  for (int v2 = 0; v2 < wid; ++v2) {
    s_before += (long long)(s_wcnt[v2] >> 32);
    t_before += (long long)(s_wcnt[v2] & 0xffffffffull);
  }
  // pass 2: keep decisions, then the writes
  // chunks whose Philox words were precomputed in the exchange waits (wave-uniform test per iteration)
  const unsigned rdone = (STACKED && !src.xmode && rnd_n == ncand) ? s_rnext : 0u;
#ifdef FLC_SELECT_STAMPS  // diagnostic: Philox chunks precomputed / chunks of the block
  if (tid == 0) w.blkt()[blockIdx.x * 4 + 2] = ((unsigned long long)((cQ / kWave) * kENW) << 32) | rdone;
#endif
  // Philox words kRnd rounds ahead (a load from L2 takes longer than one round): kRnd register slots,
  // the rounds unrolled by kRnd so each slot is a fixed register; loads at a clamped address,
  // unconditional, so no wait is merged in
#ifndef FLC_KRND
  constexpr int kRnd = 4;
#else
  constexpr int kRnd = FLC_KRND;
#endif
  // the code byte of a kept candidate (stacked): compressors.py:344-353 on |v| / norm
  // No division on the common path: t' = |v| * fp32(s / norm) and u = fp32(word) * 2^-32 decide whenever
  // they clear the margins of quant.hip's encode (1e-4 from a level, 5e-5 between u and p; valid for s <= 127,
  // the argument written there); the rest take the exact fp64 rule on fp32(|v| / norm).
  const bool fast_ok = nrm_ok && levels <= 127;
  const float rs = fast_ok ? (float)levels / nrm : 0.0f;
  auto code_of = [&](const unsigned raw, const unsigned id, const bool have, const unsigned rw) -> unsigned {
#if FLC_CALIB_NOCODE  // calibration builds only: results invalid
    return (raw >> 24) ^ rw;
#endif
    const float v = __uint_as_float(raw);
#if FLC_CALIB_NOPHILOX  // calibration builds only (tools/calib_select.sh): results invalid
    const uint32_t r = 0x80000000u;
#else
    uint32_t r;
    if (have) r = rw;
    else r = pick(philox_group((uint64_t)id >> 2, seed, counter), (int)(id & 3u));
#endif
    uint32_t lvl;
    const float t = fabsf(v) * rs;
    const float jf = ceilf(t);
    const float pf = jf - t;
    const float uf = (float)r * 2.3283064365386963e-10f;
    if (fast_ok && (pf > 1e-4f) & (t - (jf - 1.0f) > 1e-4f) & (fabsf(uf - pf) > 5e-5f)) {
      lvl = (uint32_t)(int)jf - (uf < pf ? 1u : 0u);
    } else {
      const float y = nrm_ok ? fabsf(v) / nrm : 0.0f;  // compressors.py:344
      lvl = (uint32_t)dither_level<0>(y, levels, step, u01(r));  // compressors.py:346-353
    }
    const uint32_t c = nrm_ok ? (((raw >> 31) << 7) | lvl) : 1u;
    return (v != 0.0f) ? c : 0u;
  };
  // tiles starting after the previous kept entry (lane - 1's id by a DPP wave shift; lane 0: `tile_prev`)
  // and at or before this one get this entry's position: the first kept entry at or after such a tile's
  // start.  Every candidate between two kept entries is dropped, so kept entries alone define the tiles.
  auto tiles_of = [&](const bool v, const unsigned id, const long long pos) {
    const unsigned prev_lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(tile_prev < 0 ? 0 : tile_prev));
    const unsigned pid = (unsigned)__builtin_amdgcn_update_dpp((int)prev_lo, (int)id, 0x138, 0xf, 0xf, false);  // wave_shr:1
    const int64_t prev = lane == 0 ? tile_prev : (int64_t)pid;
    if (v)
      for (int64_t t = (prev >> kTileLog) + 1; t <= ((int64_t)id >> kTileLog); ++t) tile_out[t] = (unsigned)pos;
    const unsigned long long im = __ballot(v);
    if (im) {
      const int hl = 63 - __clzll(im);  // (wave-uniform)
      tile_prev = (int64_t)(unsigned)__builtin_amdgcn_readlane((int)id, hl);
    }
  };
  const unsigned plast = q1 > 0u ? q1 - 1u : 0u;
  if (!src.xmode && !src.gmode) {
    // LDS candidates: pass 2 touches no memory but LDS and the Philox words.  Kept entries are staged in
    // place, wave range order (a kept entry's slot q0 + (kept before it in the range) <= its own index, and
    // the next round's candidates, read before this round's slots are written, lie past them), then
    // written out with the tile pointers in a second loop: no stores in the decision loop, so the
    // Philox-word loads kRnd rounds ahead keep counted waits instead of draining every store each round.
    const unsigned wq0 = (unsigned)__builtin_amdgcn_readfirstlane((int)q0);
    const unsigned wq1 = (unsigned)__builtin_amdgcn_readfirstlane((int)q1);
    const long long kept0 = s_before + (t_before > skip ? t_before - skip : 0);  // position of my first kept entry
    unsigned nk = 0;  // kept entries staged (wave-uniform)
    unsigned* const st_id = const_cast<unsigned*>(src.s_idx);
    unsigned* const st_cw = const_cast<unsigned*>(src.s_key);
    unsigned rq[kRnd];
#pragma unroll
    for (int j = 0; j < kRnd; ++j) {
      const unsigned pa = wq0 + (unsigned)(j * kWave) + lane;
#if FLC_CALIB_NORQ  // calibration builds only: results invalid
      rq[j] = pa;
#else
      rq[j] = STACKED ? ld_mem(rnd + (pa < (unsigned)kCap ? pa : kCap - 1)) : 0u;
#endif
    }
    unsigned c_raw = 0, c_id = 0;
    {
      const unsigned pc = wq0 + lane < wq1 ? wq0 + lane : plast;
      c_raw = src.s_key[pc];
      c_id = src.s_idx[pc];
    }
    for (unsigned p00 = wq0; p00 < wq1; p00 += kRnd * kWave) {
#pragma unroll
      for (int j = 0; j < kRnd; ++j) {  // (rounds past q1: no lane in, nothing kept)
        const unsigned p0 = p00 + (unsigned)(j * kWave);
        const unsigned rw = rq[j];
        if (STACKED) {
          const unsigned pa = p0 + (unsigned)(kRnd * kWave) + lane;
#if FLC_CALIB_NORQ
          rq[j] = pa;
#else
          rq[j] = ld_mem(rnd + (pa < (unsigned)kCap ? pa : kCap - 1));
#endif
        }
        const unsigned pn = p0 + kWave + lane < wq1 ? p0 + kWave + lane : plast;
        const unsigned n_raw = src.s_key[pn], n_id = src.s_idx[pn];
        const unsigned p = p0 + lane;
        const bool in = p < wq1;
        const unsigned key = order_key(c_raw);
        const bool is_s = in && key > T, is_t = in && key == T;
        const unsigned long long ms = __ballot(is_s), mt = __ballot(is_t);
        const long long tb = t_before + __builtin_amdgcn_mbcnt_hi((unsigned)(mt >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mt, 0u));
        const bool keep = is_s || (is_t && tb >= skip);
        const unsigned long long km = __ballot(keep);
        if (keep) {
          const unsigned slot = wq0 + nk + __builtin_amdgcn_mbcnt_hi((unsigned)(km >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)km, 0u));
          const bool have = ((p0 - wq0) / kWave * kENW + (unsigned)wid) < rdone;
          st_id[slot] = c_id;
          st_cw[slot] = STACKED ? code_of(c_raw, c_id, have, rw) : c_raw;
        }
        nk += (unsigned)__popcll(km);
        s_before += __popcll(ms);
        t_before += __popcll(mt);
        c_raw = n_raw;
        c_id = n_id;
      }
    }
    STAMP(14);
    // write-out: positions kept0 + i, i < nk, contiguous per wave
    for (unsigned i0 = 0; i0 < nk; i0 += kWave) {
      const unsigned i = i0 + lane;
      const bool v = i < nk;
      const unsigned id = v ? st_id[wq0 + i] : 0u, cw = v ? st_cw[wq0 + i] : 0u;
      const long long pos = kept0 + (long long)i;
#if !FLC_CALIB_NOWRITE
      if (v && pos >= 0 && pos < k) {
        idx_out[pos] = (int)id;
        if (STACKED) code_out[pos] = (uint8_t)cw;
        else val_out[pos] = __uint_as_float(cw);
      }
#endif
      if (tile_owner) tiles_of(v, id, pos);
    }
  } else {
    // x-mode (fallback, or more candidates than LDS + the HBM overflow hold: candidates from x) and g-mode (LDS +
    // overflow): candidates through cand_get, writes in the loop
    unsigned rq[kRnd];
#pragma unroll
    for (int j = 0; j < kRnd; ++j) rq[j] = 0u;
    auto round = [&](const unsigned p0, const unsigned rw, const unsigned raw, const unsigned id) {
      const unsigned p = p0 + lane;
      const bool in = p < q1;
      const unsigned key = order_key(raw);
      const bool is_s = in && key > T, is_t = in && key == T;
      const unsigned long long ms = __ballot(is_s), mt = __ballot(is_t);
      const long long sb = s_before + __builtin_amdgcn_mbcnt_hi((unsigned)(ms >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)ms, 0u));
      const long long tb = t_before + __builtin_amdgcn_mbcnt_hi((unsigned)(mt >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mt, 0u));
      const bool keep = is_s || (is_t && tb >= skip);
      const long long pos = sb + (tb > skip ? tb - skip : 0);
#if FLC_CALIB_NOWRITE  // calibration builds only: results invalid
      if (keep && pos == -5) {
#else
      if (keep && pos >= 0 && pos < k) {
#endif
        idx_out[pos] = (int)id;
        if (STACKED) code_out[pos] = (uint8_t)code_of(raw, id, false, rw);
        else val_out[pos] = __uint_as_float(raw);
      }
      if (tile_owner) tiles_of(in, id, pos);  // (pos of a dropped candidate: the kept entries before it)
      s_before += __popcll(ms);
      t_before += __popcll(mt);
    };
    // the next round's candidates are read while this one is processed (clamped index: unconditional)
    unsigned c_raw = 0, c_id = 0;
    if (q0 < q1) cand_get(src, q0 + lane < q1 ? q0 + lane : plast, c_raw, c_id);
    for (unsigned p0 = q0; p0 < q1; p0 += kWave) {
      unsigned n_raw, n_id;
      const unsigned pn = p0 + kWave + lane;
      cand_get(src, pn < q1 ? pn : plast, n_raw, n_id);
      round(p0, rq[0], c_raw, c_id);
      c_raw = n_raw;
      c_id = n_id;
    }
    STAMP(14);
  }
  if (tile_owner) {  // tiles after the wave's last kept entry: the next kept position
    const long long nxt = s_before + (t_before > skip ? t_before - skip : 0);
    for (int64_t t = (tile_prev >> kTileLog) + 1 + lane; t <= (tile_hi >> kTileLog); t += kWave) tile_out[t] = (unsigned)nxt;
    if (w.bid == w.nb - 1 && q1 >= ncand && lane == 0) tile_out[cdiv_dev(n, kTile)] = (unsigned)k;
  }
  STAMP(15);
  BLKT(3);
  STAMP_OUT(FUSED ? 0 : 5, 16);
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
template <bool STACKED, class Src>
int launch_topk(const Src& x, int64_t n, int64_t k, void* ws, size_t ws_bytes, hipStream_t st, int* idx, float* val,
                uint8_t* codes, float* norm, int levels, uint64_t seed, uint64_t counter, unsigned* tiles,
                const char* who) {
  int dev = 0;
  const int cus = stream_cus(st, &dev);
  size_t need = 0;
  EncWs w = carve_enc(ws, n, k, cus, &need);
  if (!ws || need > ws_bytes) return fail(FLC_EWORKSPACE, "%s: workspace %zu < %zu", who, ws_bytes, need);
  const EncGeom g = enc_geometry(n, cus);
  const SampleSetup ss = sample_setup(n, k);
#if defined(FLC_CALIB) || defined(FLC_SELECT_STAMPS)  // calibration builds: FLC_TOPK_SPLIT=1 times the two-kernel path
  static const bool split = getenv("FLC_TOPK_SPLIT") && atoi(getenv("FLC_TOPK_SPLIT")) != 0;
#else
  constexpr bool split = false;
#endif
  // the compact sample when the full 32 K keys are taken (FLC_COMPACT_SAMPLE=0: calibration A/B only)
  static const bool compact_on = !getenv("FLC_COMPACT_SAMPLE") || atoi(getenv("FLC_COMPACT_SAMPLE")) != 0;
  w.compact = (compact_on && !ss.take_all && ss.S == kSample) ? 1 : 0;
  if (!ss.take_all)
    FLC_LAUNCH("topk_sample", topk_sample_kernel<Src>, dim3((unsigned)cdiv(ss.S, 256)), dim3(256), 0, st, x, n, ss.S, w);
  if (split)
    FLC_LAUNCH("topk_filter", topk_filter_kernel<Src>, dim3((unsigned)g.G), dim3(kET), 0, st, x, n, w, ss.S, ss.rank_lo,
               ss.rank_hi, ss.take_all);
  Coresident co(st, dev);
  if (co.status()) return co.status();
  const double step = levels > 0 ? 1.0 / (double)levels : 0.0;
  if (split)
    FLC_LAUNCH_CO(co, STACKED ? "stacked_select" : "topk_select", (topk_select_kernel<STACKED, false, Src>), dim3((unsigned)g.G),
               dim3(kET), 0, st, x, n, (long long)k, w, idx, val, codes, norm, levels, step, seed, counter,
               tiles, ss.S, ss.rank_lo, ss.rank_hi, ss.take_all, (const BatchEntry*)nullptr);
  else
    FLC_LAUNCH_CO(co, STACKED ? "stacked_encode" : "topk_encode", (topk_select_kernel<STACKED, true, Src>), dim3((unsigned)g.G),
               dim3(kET), 0, st, x, n, (long long)k, w, idx, val, codes, norm, levels, step, seed, counter,
               tiles, ss.S, ss.rank_lo, ss.rank_hi, ss.take_all, (const BatchEntry*)nullptr);
  return co.finish();
}

// Batched stacked encode: the clients in chunks of at most `cus` (one select of cus / chunk blocks each, all in one
// launch, so every block of the launch is co-resident: one per CU); chunks run one after another on the stream.
// Workspace: [chunk headers of kOffStage][chunk staging / overflow areas of vstride][the entry table]; the headers'
// state, flags and histograms are zeroed at the start of every call.
struct BatchGeom {
  int chunk;       // clients per launch
  EncGeom g;       // one client's select geometry
  unsigned ovf;
  size_t off_ovf;  // from the client's staging area
  size_t vstride;
  size_t table_off, extra_off, need;
};

// keys per client of a batched call's sample: n / 256 rounded down to a power of two, within [4096, kSample]
// (a 1 M-element client samples 4 K keys; 8 M and more the full 32 K)
int batch_sample_cap(int64_t n) {
  int s = 4096;
  while (s < kSample && (int64_t)s * 2 * 128 <= n) s *= 2;
  return s;
}

// extra_bytes: the delta batch's tensor tables, after the entry table (at extra_off)
BatchGeom batch_geometry(int64_t n, int64_t k, int n_clients, int cus, size_t extra_bytes = 0) {
  BatchGeom b;
  b.chunk = std::max(1, std::min(n_clients, cus));
  b.vstride = enc_var_bytes(n, k, std::max(1, cus / b.chunk), &b.g, &b.ovf, &b.off_ovf, batch_sample_cap(n));
  b.table_off = (size_t)b.chunk * (kOffStage + b.vstride);
  b.extra_off = b.table_off + al256((size_t)std::max(n_clients, 1) * sizeof(BatchEntry));
  b.need = b.extra_off + al256(extra_bytes);
  return b;
}

// Pinned staging of the host-built tables (batch entries, delta pointer tables): a ring of slots per device, each
// reused only after the last stream operation reading it has completed.  An event is recorded after every kEvery-th
// slot's use only (each record put a ≈ 5.6 µs gap before the stream's next kernel); reusing slot s waits for the event
// of slot q = s | (kEvery - 1), used after s in the previous lap — with kRing slots that is a call ≥ kRing - kEvery calls
// back, normally long complete.  A copy from pageable memory goes through the runtime's own staging and can hold the
// host until the device reaches it.  The batch entry table is not copied at all: pinned memory is mapped into the
// device's address space, and each block reads its client's entry once, in place (one PCIe read at the kernel's
// start instead of a copy and the dispatch gap behind it: ≈ 10 µs per call, §3.1b).
//
// The bookkeeping (RingBook, pure host logic: flc_ring_selftest drives it without a device) records at STAGE time
// that a slot is in use and in which lap, and clears its event mark; table_done then records the stream and, every
// kEvery-th slot, the event.  q's event covers s only when q was staged and done in the same lap as s (after s) on
// the same stream: a stage that never reached table_done (an error return between the two), or a recorded event from
// an earlier lap, cannot stand for s.  Otherwise the reuse drains the ring's device (made current for the call).
// Under stream capture the ring is not used at all (a captured graph reads a host slot at replay time, laps later):
// the tables go into the device workspace through kernel arguments (fill_table), see stage_or_fill.
constexpr int kRing = 32, kEvery = 8;
static_assert(kRing % kEvery == 0 && (kEvery & (kEvery - 1)) == 0, "event slots");
struct RingBook {
  enum Wait { kNone = 0, kEvent = 1, kDrain = 2 };
  unsigned long long lap_of[kRing] = {};  // lap of the slot's latest stage (valid when used)
  const void* st_of[kRing] = {};          // stream of its latest use (set by done; null: not done)
  bool used[kRing] = {};                  // staged, and not yet known complete
  bool rec[kRing] = {};                   // an event was recorded after its latest use (set by done)
  unsigned long long lap = 0;
  int next = 0;
  // the next slot to stage into and how to make it free: *wait_slot = the slot whose event to wait for (kEvent)
  int stage(Wait* how, int* wait_slot) {
    const int s = next, q = s | (kEvery - 1);
    *how = kNone;
    *wait_slot = -1;
    if (used[s]) {
      if (rec[q] && used[q] && lap_of[q] == lap_of[s] && st_of[s] != nullptr && st_of[q] == st_of[s]) {
        *how = kEvent;
        *wait_slot = q;
      } else {
        *how = kDrain;
      }
    }
    return s;
  }
  // the wait for slot s is done (or none was needed): s is staged in the current lap
  void staged(int s, Wait how) {
    if (how == kDrain)  // the whole device drained: every earlier use is complete
      for (int i = 0; i < kRing; ++i) used[i] = false;
    used[s] = true;
    lap_of[s] = lap;
    st_of[s] = nullptr;
    rec[s] = false;
    next = (s + 1) % kRing;
    if (next == 0) ++lap;
  }
  // the last stream operation reading slot s is enqueued on `st`; returns true when an event is to be recorded
  bool done(int s, const void* st) {
    st_of[s] = st;
    rec[s] = (s & (kEvery - 1)) == kEvery - 1;
    return rec[s];
  }
};
struct TableRing {
  std::mutex mu;
  RingBook book;
  char* buf[kRing] = {};
  char* dptr[kRing] = {};  // the slot's device address
  size_t cap[kRing] = {};
  hipEvent_t ev[kRing] = {};
};
TableRing& table_ring(int dev) {
  static TableRing rings[64];
  return rings[dev < 0 || dev >= 64 ? 0 : dev];
}
// run `f` with `dev` current (the ring's slots, events and drains belong to that device, not to the calling
// thread's current one), restoring the previous device
template <class F>
hipError_t on_device(int dev, F&& f) {
  int cur = -1;
  hipError_t e = hipGetDevice(&cur);
  if (e != hipSuccess) return e;
  if (cur != dev && (e = hipSetDevice(dev)) != hipSuccess) return e;
  const hipError_t r = f();
  const hipError_t e2 = cur != dev ? hipSetDevice(cur) : hipSuccess;
  return r != hipSuccess ? r : e2;
}
// `bytes` of `src` into the next pinned slot: *dev_ptr = its device address; table_done() after the last launch or copy
// that reads it
int stage_table(int dev, const void* src, size_t bytes, char** dev_ptr, char** host_ptr, int* slot) {
  TableRing& r = table_ring(dev);
  std::lock_guard<std::mutex> lk(r.mu);
  RingBook::Wait how;
  int q = -1;
  const int s = r.book.stage(&how, &q);
  if (how == RingBook::kEvent) FLC_CHECK_HIP(hipEventSynchronize(r.ev[q]));
  else if (how == RingBook::kDrain) FLC_CHECK_HIP(on_device(dev, [] { return hipDeviceSynchronize(); }));
  if (r.cap[s] < bytes) {
    if (r.buf[s]) FLC_CHECK_HIP(hipHostFree(r.buf[s]));
    r.buf[s] = r.dptr[s] = nullptr;
    r.cap[s] = 0;
    const size_t cap = std::max<size_t>(align_up(bytes, 4096), 16384);
    FLC_CHECK_HIP(on_device(dev, [&] {
      return hipHostMalloc(reinterpret_cast<void**>(&r.buf[s]), cap, hipHostMallocDefault);
    }));
    r.cap[s] = cap;
    void* d = nullptr;
    FLC_CHECK_HIP(hipHostGetDevicePointer(&d, r.buf[s], 0));
    r.dptr[s] = static_cast<char*>(d);
  }
  if (!r.ev[s]) FLC_CHECK_HIP(on_device(dev, [&] { return hipEventCreateWithFlags(&r.ev[s], hipEventDisableTiming); }));
  r.book.staged(s, how);
  std::memcpy(r.buf[s], src, bytes);
  *dev_ptr = r.dptr[s];
  if (host_ptr) *host_ptr = r.buf[s];
  *slot = s;
  return FLC_OK;
}
int table_done(int dev, int slot, hipStream_t st) {
  TableRing& r = table_ring(dev);
  std::lock_guard<std::mutex> lk(r.mu);
  if (r.book.done(slot, st)) FLC_CHECK_HIP(hipEventRecord(r.ev[slot], st));
  return FLC_OK;
}

// Under stream capture: `bytes` (a multiple of 4) of `src` written to the device address `dst` by kernels whose
// arguments carry the bytes (2 KB per launch), so the captured graph holds the table itself
struct TableChunk {
  unsigned w[512];
};
__global__ __launch_bounds__(256) void fill_table_kernel(unsigned* __restrict__ dst, TableChunk c, int words) {
  for (int i = (int)threadIdx.x; i < words; i += 256) dst[i] = c.w[i];
}
int fill_table(void* dst, const void* src, size_t bytes, hipStream_t st) {
  const size_t words = (bytes + 3) / 4;
  for (size_t w0 = 0; w0 < words; w0 += 512) {
    TableChunk c;
    const size_t nw = std::min<size_t>(512, words - w0);
    std::memset(&c, 0, sizeof(c));
    std::memcpy(c.w, static_cast<const char*>(src) + 4 * w0, std::min(bytes - 4 * w0, 4 * nw));
    FLC_LAUNCH("fill_table", fill_table_kernel, dim3(1), dim3(256), 0, st, static_cast<unsigned*>(dst) + w0, c, (int)nw);
  }
  return FLC_OK;
}
int capturing(hipStream_t st, bool* cap) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  FLC_CHECK_HIP(hipStreamIsCapturing(st, &cs));
  *cap = cs != hipStreamCaptureStatusNone;
  return FLC_OK;
}

// copy `bytes` from `src` to the device address `dst`, stream-ordered on `st` (of device `dev`), through a pinned slot
// (under capture: through kernel arguments)
int copy_table(int dev, void* dst, const void* src, size_t bytes, hipStream_t st) {
  bool cap = false;
  if (const int rc = capturing(st, &cap)) return rc;
  if (cap) return fill_table(dst, src, bytes, st);
  char *d = nullptr, *h = nullptr;
  int slot = 0;
  if (const int rc = stage_table(dev, src, bytes, &d, &h, &slot)) return rc;
  const hipError_t e = hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, st);
  const int rc = table_done(dev, slot, st);
  FLC_CHECK_HIP(e);
  return rc;
}

// the batched launches over the clients in chunks of bg.chunk (tab: the entry table, device-readable)
template <class Src, bool STACKED>
int launch_topk_batch_chunks(const Src& proto, const BatchEntry* tab, int C, const BatchGeom& bg, int64_t n, int64_t k,
                             int levels, uint64_t counter, char* base, hipStream_t st, int dev) {
  // each call starts its headers from zero (state, flags, histograms): no history is carried between calls, so the
  // header / staging split may move with the client count
  const SampleSetup ss = sample_setup(n, k, batch_sample_cap(n));
  const double step = levels > 0 ? 1.0 / (double)levels : 0.0;
  static_assert(kOffBlk % 16 == 0 && kOffStage % 16 == 0 && kOffFlags % 16 == 0 && kOffHist % 16 == 0,
                "16-B zeroing of the headers");
  if (ss.take_all)  // (otherwise every chunk's sample launch zeroes its clients' headers)
    FLC_LAUNCH("zero_headers", zero_headers_kernel, dim3(8, (unsigned)bg.chunk), dim3(256), 0, st, base,
               (int)(kOffBlk / 16));
  EncWs w;
  w.base = base;
  w.var = base + (size_t)bg.chunk * kOffStage;
  w.M = bg.g.M;
  w.off_ovf = bg.off_ovf;
  w.ovf = bg.ovf;
  w.bid = 0;
  w.nb = bg.g.G;
  w.vstride = bg.vstride;
  w.compact = 0;  // (the full sample: the batched sample kernel writes no compact one)
  w.errp = reinterpret_cast<unsigned long long*>(base + kOffSt + offsetof(EncState, err));
  Coresident co(st, dev);
  if (co.status()) return co.status();
  for (int c0 = 0; c0 < C; c0 += bg.chunk) {
    const int cn = std::min(bg.chunk, C - c0);
    const BatchEntry* t = tab + c0;
    if (!ss.take_all) {
      const int per = (int)cdiv(ss.S, 256);
      FLC_LAUNCH("topk_sample_batch", topk_sample_batch_kernel<Src>, dim3((unsigned)(cn * per)), dim3(256), 0, st,
                 proto, t, n, ss.S, w, per);
    }
    FLC_LAUNCH_CO(co, STACKED ? "stacked_encode_batch" : "topk_encode_batch", (topk_select_kernel<STACKED, true, Src, true>),
               dim3((unsigned)(cn * bg.g.G)),
               dim3(kET), 0, st, proto, n, (long long)k, w, nullptr, nullptr, nullptr, nullptr, levels, step, 0ull,
               counter, nullptr, ss.S, ss.rank_lo, ss.rank_hi, ss.take_all, t);
  }
  return co.finish();
}

// host: the entries read in place from a pinned slot; with `extra` (already holding device addresses inside the
// workspace) both copied into the workspace in one copy
template <class Src, bool STACKED = true>
int launch_topk_batch(const Src& proto, const std::vector<BatchEntry>& ents, const std::vector<char>& extra, int64_t n,
                      int64_t k, int levels, uint64_t counter, void* ws, size_t ws_bytes, hipStream_t st,
                      const char* who) {
  int dev = 0;
  const int cus = stream_cus(st, &dev);
  const int C = (int)ents.size();
  const BatchGeom bg = batch_geometry(n, k, C, cus, extra.size());
  if (!ws || bg.need > ws_bytes) return fail(FLC_EWORKSPACE, "%s: workspace %zu < %zu", who, ws_bytes, bg.need);
  char* base = static_cast<char*>(ws);
  const BatchEntry* tab = reinterpret_cast<const BatchEntry*>(base + bg.table_off);
  int slot = -1;  // the entries read in place from a pinned slot (no extra tables), or copied with them
  bool cap = false;
  if (const int rc = capturing(st, &cap)) return rc;
  if (extra.empty() && cap) {  // (under capture: into the workspace, through kernel arguments)
    if (const int rc = fill_table(base + bg.table_off, ents.data(), ents.size() * sizeof(BatchEntry), st)) return rc;
  } else if (extra.empty()) {
    char* d = nullptr;
    if (const int rc = stage_table(dev, ents.data(), ents.size() * sizeof(BatchEntry), &d, nullptr, &slot)) return rc;
    tab = reinterpret_cast<const BatchEntry*>(d);
  } else {  // (the delta tables are read throughout the pass: device memory)
    std::vector<char> host(bg.extra_off - bg.table_off + extra.size(), 0);
    std::memcpy(host.data(), ents.data(), ents.size() * sizeof(BatchEntry));
    std::memcpy(host.data() + (bg.extra_off - bg.table_off), extra.data(), extra.size());
    if (const int rc = copy_table(dev, base + bg.table_off, host.data(), host.size(), st)) return rc;
  }
  const int rc = launch_topk_batch_chunks<Src, STACKED>(proto, tab, C, bg, n, k, levels, counter, base, st, dev);
  if (slot >= 0) {
    const int rc2 = table_done(dev, slot, st);
    if (rc == FLC_OK) return rc2;
  }
  return rc;
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
  size_t need = 0;
  (void)carve_enc(nullptr, n < 1 ? 1 : n, k < 1 ? 1 : k, current_cus(nullptr), &need);
  return need;
}

int flc_topk_encode_tiled(const float* x, int64_t n, int64_t k, int32_t* idx, float* val, uint32_t* tiles, void* ws,
                          size_t ws_bytes, void* stream) {
  if (int rc = check_topk(x, n, k, "flc_topk_encode")) return rc;
  if (!idx || !val) return fail(FLC_EINVAL, "flc_topk_encode: null output");
  return launch_topk<false>(FlatSrc{x}, n, k, ws, ws_bytes, as_stream(stream), idx, val, nullptr, nullptr, 0, 0, 0, tiles,
                            "flc_topk_encode");
}

int flc_topk_encode(const float* x, int64_t n, int64_t k, int32_t* idx, float* val, void* ws, size_t ws_bytes,
                    void* stream) {
  return flc_topk_encode_tiled(x, n, k, idx, val, nullptr, ws, ws_bytes, stream);
}

int flc_stacked_encode_tiled(const float* x, int64_t n, int64_t k, int levels, uint64_t seed, uint64_t counter,
                             const double* compat_u, int32_t* idx, uint8_t* codes, float* norm, uint32_t* tiles,
                             void* ws, size_t ws_bytes, void* stream) {
  if (int rc = check_topk(x, n, k, "flc_stacked_encode")) return rc;
  if (!idx || !codes || !norm) return fail(FLC_EINVAL, "flc_stacked_encode: null output");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_stacked_encode: levels must be in [1, 127]");
  if (compat_u)
    return fail(FLC_EUNSUPPORTED,
                "flc_stacked_encode: compat RNG is composed by the caller (flc_topk_encode + flc_quant_encode)");
  return launch_topk<true>(FlatSrc{x}, n, k, ws, ws_bytes, as_stream(stream), idx, nullptr, codes, norm, levels, seed,
                           counter, tiles, "flc_stacked_encode");
}

int flc_stacked_encode(const float* x, int64_t n, int64_t k, int levels, uint64_t seed, uint64_t counter,
                       const double* compat_u, int32_t* idx, uint8_t* codes, float* norm, void* ws, size_t ws_bytes,
                       void* stream) {
  return flc_stacked_encode_tiled(x, n, k, levels, seed, counter, compat_u, idx, codes, norm, nullptr, ws, ws_bytes,
                                  stream);
}

// the delta encoder's tensor table sits after the encoder's own workspace
size_t delta_table_bytes(int n_tensors) { return align_up((size_t)(n_tensors + 1) * 8 + (size_t)n_tensors * 16, 256); }

size_t flc_stacked_encode_delta_workspace_size(int64_t n, int64_t k, int n_tensors) {
  return align_up(flc_topk_workspace_size(n, k), 256) + delta_table_bytes(n_tensors < 0 ? 0 : n_tensors);
}

int flc_stacked_encode_delta(const float* const* local, const float* const* global, const int64_t* sizes,
                             int n_tensors, int64_t k, int levels, uint64_t seed, uint64_t counter, int32_t* idx,
                             uint8_t* codes, float* norm, uint32_t* tiles, void* ws, size_t ws_bytes, void* stream) {
  if (n_tensors <= 0 || !local || !global || !sizes) return fail(FLC_EINVAL, "flc_stacked_encode_delta: bad arguments");
  if (!idx || !codes || !norm) return fail(FLC_EINVAL, "flc_stacked_encode_delta: null output");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_stacked_encode_delta: levels must be in [1, 127]");
  std::vector<long long> off((size_t)n_tensors + 1, 0);
  for (int t = 0; t < n_tensors; ++t) {
    if (sizes[t] < 0 || (sizes[t] > 0 && (!local[t] || !global[t])))
      return fail(FLC_EINVAL, "flc_stacked_encode_delta: bad tensor %d", t);
    if ((reinterpret_cast<uintptr_t>(local[t]) | reinterpret_cast<uintptr_t>(global[t])) & 3u)
      return fail(FLC_EINVAL, "flc_stacked_encode_delta: tensor %d is not 4-B aligned", t);
    off[t + 1] = off[t] + sizes[t];
  }
  const int64_t n = off[n_tensors];
  if (n >= (1ll << 31)) return fail(FLC_EINVAL, "flc_stacked_encode_delta: n must be < 2^31");
  if (k <= 0 || k >= n)
    return fail(FLC_EINVAL, "flc_stacked_encode_delta: need 0 < k < n (got k=%lld, n=%lld)", (long long)k, (long long)n);
  const size_t enc = align_up(flc_topk_workspace_size(n, k), 256);
  if (!ws || ws_bytes < enc + delta_table_bytes(n_tensors))
    return fail(FLC_EWORKSPACE, "flc_stacked_encode_delta: workspace %zu < %zu", ws_bytes,
                enc + delta_table_bytes(n_tensors));
  // table: off[n_tensors + 1] (int64), then the local pointers, then the global pointers
  std::vector<char> host(delta_table_bytes(n_tensors), 0);
  std::memcpy(host.data(), off.data(), off.size() * 8);
  std::memcpy(host.data() + off.size() * 8, local, (size_t)n_tensors * 8);
  std::memcpy(host.data() + off.size() * 8 + (size_t)n_tensors * 8, global, (size_t)n_tensors * 8);
  char* tab = static_cast<char*>(ws) + enc;
  hipStream_t st = as_stream(stream);
  int dev = 0;
  (void)stream_cus(st, &dev);
  if (const int rc = copy_table(dev, tab, host.data(), host.size(), st)) return rc;
  DeltaSrc src;
  src.t.off = reinterpret_cast<const long long*>(tab);
  src.t.lp = reinterpret_cast<const float* const*>(tab + off.size() * 8);
  src.t.gp = reinterpret_cast<const float* const*>(tab + off.size() * 8 + (size_t)n_tensors * 8);
  src.t.nseg = n_tensors;
  return launch_topk<true>(src, n, k, ws, enc, st, idx, nullptr, codes, norm, levels, seed, counter, tiles,
                           "flc_stacked_encode_delta");
}

size_t flc_stacked_encode_batch_workspace_size(int64_t n, int64_t k, int n_clients) {
  return batch_geometry(n < 1 ? 1 : n, k < 1 ? 1 : k, n_clients < 1 ? 1 : n_clients, current_cus(nullptr)).need;
}

int flc_stacked_encode_batch(const float* const* xs, int n_clients, int64_t n, int64_t k, int levels,
                             const uint64_t* seeds, uint64_t counter, int32_t* const* idx, uint8_t* const* codes,
                             float* const* norm, uint32_t* const* tiles, void* ws, size_t ws_bytes, void* stream) {
  const char* who = "flc_stacked_encode_batch";
  if (n_clients <= 0 || !xs || !seeds || !idx || !codes || !norm) return fail(FLC_EINVAL, "%s: bad arguments", who);
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "%s: levels must be in [1, 127]", who);
  std::vector<BatchEntry> ents((size_t)n_clients);
  for (int c = 0; c < n_clients; ++c) {
    if (int rc = check_topk(xs[c], n, k, who)) return rc;
    if (!idx[c] || !codes[c] || !norm[c]) return fail(FLC_EINVAL, "%s: null output of client %d", who, c);
    ents[c] = BatchEntry{xs[c], seeds[c], idx[c], codes[c], norm[c], tiles ? tiles[c] : nullptr, nullptr};
  }
  return launch_topk_batch(FlatSrc{nullptr}, ents, {}, n, k, levels, counter, ws, ws_bytes, as_stream(stream), who);
}

size_t flc_topk_encode_batch_workspace_size(int64_t n, int64_t k, int n_clients) {
  return flc_stacked_encode_batch_workspace_size(n, k, n_clients);
}

int flc_topk_encode_batch(const float* const* xs, int n_clients, int64_t n, int64_t k, int32_t* const* idx,
                          float* const* val, uint32_t* const* tiles, void* ws, size_t ws_bytes, void* stream) {
  const char* who = "flc_topk_encode_batch";
  if (n_clients <= 0 || !xs || !idx || !val) return fail(FLC_EINVAL, "%s: bad arguments", who);
  std::vector<BatchEntry> ents((size_t)n_clients);
  for (int c = 0; c < n_clients; ++c) {
    if (int rc = check_topk(xs[c], n, k, who)) return rc;
    if (!idx[c] || !val[c]) return fail(FLC_EINVAL, "%s: null output of client %d", who, c);
    ents[c] = BatchEntry{xs[c], 0, idx[c], nullptr, nullptr, tiles ? tiles[c] : nullptr, val[c]};
  }
  return launch_topk_batch<FlatSrc, false>(FlatSrc{nullptr}, ents, {}, n, k, 0, 0, ws, ws_bytes, as_stream(stream),
                                           who);
}

// the delta batch's tables: off[n_tensors + 1] (int64), the global pointers, then each client's local pointers
size_t delta_batch_extra_bytes(int n_tensors, int n_clients) {
  return (size_t)(n_tensors + 1) * 8 + (size_t)n_tensors * 8 + (size_t)n_clients * n_tensors * 8;
}

size_t flc_stacked_encode_delta_batch_workspace_size(int64_t n, int64_t k, int n_clients, int n_tensors) {
  n_clients = n_clients < 1 ? 1 : n_clients;
  n_tensors = n_tensors < 1 ? 1 : n_tensors;
  return batch_geometry(n < 1 ? 1 : n, k < 1 ? 1 : k, n_clients, current_cus(nullptr),
                        delta_batch_extra_bytes(n_tensors, n_clients)).need;
}

int flc_stacked_encode_delta_batch(const float* const* local, const float* const* global, const int64_t* sizes,
                                   int n_tensors, int n_clients, int64_t k, int levels, const uint64_t* seeds,
                                   uint64_t counter, int32_t* const* idx, uint8_t* const* codes, float* const* norm,
                                   uint32_t* const* tiles, void* ws, size_t ws_bytes, void* stream) {
  const char* who = "flc_stacked_encode_delta_batch";
  if (n_tensors <= 0 || n_clients <= 0 || !local || !global || !sizes || !seeds || !idx || !codes || !norm)
    return fail(FLC_EINVAL, "%s: bad arguments", who);
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "%s: levels must be in [1, 127]", who);
  std::vector<long long> off((size_t)n_tensors + 1, 0);
  for (int t = 0; t < n_tensors; ++t) {
    if (sizes[t] < 0) return fail(FLC_EINVAL, "%s: bad tensor %d", who, t);
    if (sizes[t] > 0 && (!global[t] || (reinterpret_cast<uintptr_t>(global[t]) & 3u)))
      return fail(FLC_EINVAL, "%s: global tensor %d is null or not 4-B aligned", who, t);
    for (int c = 0; c < n_clients; ++c) {
      const float* l = local[(size_t)c * n_tensors + t];
      if (sizes[t] > 0 && (!l || (reinterpret_cast<uintptr_t>(l) & 3u)))
        return fail(FLC_EINVAL, "%s: local tensor %d of client %d is null or not 4-B aligned", who, t, c);
    }
    off[t + 1] = off[t] + sizes[t];
  }
  const int64_t n = off[n_tensors];
  if (n >= (1ll << 31)) return fail(FLC_EINVAL, "%s: n must be < 2^31", who);
  if (k <= 0 || k >= n) return fail(FLC_EINVAL, "%s: need 0 < k < n (got k=%lld, n=%lld)", who, (long long)k, (long long)n);
  for (int c = 0; c < n_clients; ++c)
    if (!idx[c] || !codes[c] || !norm[c]) return fail(FLC_EINVAL, "%s: null output of client %d", who, c);
  const BatchGeom bg = batch_geometry(n, k, n_clients, current_cus(nullptr),
                                      delta_batch_extra_bytes(n_tensors, n_clients));
  if (!ws || bg.need > ws_bytes) return fail(FLC_EWORKSPACE, "%s: workspace %zu < %zu", who, ws_bytes, bg.need);
  char* dx = static_cast<char*>(ws) + bg.extra_off;  // the tables' device address
  std::vector<char> extra(delta_batch_extra_bytes(n_tensors, n_clients), 0);
  const size_t o_gp = off.size() * 8, o_lp = o_gp + (size_t)n_tensors * 8;
  std::memcpy(extra.data(), off.data(), off.size() * 8);
  std::memcpy(extra.data() + o_gp, global, (size_t)n_tensors * 8);
  std::memcpy(extra.data() + o_lp, local, (size_t)n_clients * n_tensors * 8);
  DeltaSrc proto;
  proto.t.off = reinterpret_cast<const long long*>(dx);
  proto.t.gp = reinterpret_cast<const float* const*>(dx + o_gp);
  proto.t.lp = nullptr;
  proto.t.nseg = n_tensors;
  std::vector<BatchEntry> ents((size_t)n_clients);
  for (int c = 0; c < n_clients; ++c)
    ents[c] = BatchEntry{dx + o_lp + (size_t)c * n_tensors * 8, seeds[c], idx[c], codes[c], norm[c],
                         tiles ? tiles[c] : nullptr, nullptr};
  return launch_topk_batch(proto, ents, extra, n, k, levels, counter, ws, ws_bytes, as_stream(stream), who);
}

// the pinned table ring's bookkeeping on its own (no device): ops are triples (kind, slot, stream id); kind 0 stages
// (writes the triple slot, wait kind 0 none / 1 event / 2 drain, event slot to `out`), kind 1 marks `slot` done on
// stream `stream id` (ids > 0); returns the number of triples written, or -1 on a bad op
int flc_ring_selftest(const int32_t* ops, int n_ops, int32_t* out, int n_out) {
  if (!ops || n_ops < 0 || (!out && n_out > 0)) return -1;
  RingBook b;
  int w = 0;
  for (int i = 0; i < n_ops; ++i) {
    const int32_t kind = ops[3 * i], slot = ops[3 * i + 1], sid = ops[3 * i + 2];
    if (kind == 0) {
      RingBook::Wait how;
      int q = -1;
      const int s = b.stage(&how, &q);
      b.staged(s, how);
      if (w >= n_out) return -1;
      out[3 * w] = s;
      out[3 * w + 1] = (int32_t)how;
      out[3 * w + 2] = q;
      ++w;
    } else if (kind == 1) {
      if (slot < 0 || slot >= kRing || sid <= 0) return -1;
      (void)b.done(slot, reinterpret_cast<const void*>((uintptr_t)sid));
    } else {
      return -1;
    }
  }
  return w;
}

int flc_topk_status(void* ws, uint64_t* err_out, int reset, void* stream) {
  if (!ws || !err_out) return fail(FLC_EINVAL, "flc_topk_status: null workspace or output");
  hipStream_t st = as_stream(stream);
  char* err_word = static_cast<char*>(ws) + kOffSt + offsetof(EncState, err);
  FLC_CHECK_HIP(hipMemcpyAsync(err_out, err_word, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
  if (reset) FLC_CHECK_HIP(hipMemsetAsync(err_word, 0, sizeof(uint64_t), st));
  return FLC_OK;
}

}  // extern "C"
