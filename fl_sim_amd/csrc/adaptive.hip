// adaptive.hip — the adaptive random compressor for gfx950
// (reference: fl_sim/compressors/compressors.py:297-301):
//
//   ind = np.random.choice(np.arange(D), size=1, p=np.abs(x) / np.abs(x).sum());  out[ind] = x[ind]
//
// which numpy evaluates as (numpy 2.x, legacy RandomState.choice with replace=True):
//   S   = np.abs(x).sum()       fp32: the 8192-element buffers of the reduction folded in order, each
//                               buffer summed by numpy's pairwise_sum (leaves of <= 128 with 8
//                               accumulators, splits at n/2 rounded down to a multiple of 8);
//   p   = |x| / S               fp32, correctly rounded, then cast to fp64;
//   checks: kahan_sum(p) NaN -> "probabilities contain NaN"; |sum - 1| > atol -> "do not sum to 1"
//           (atol = max(sqrt(eps64), sqrt(eps32)) = 3.4526698e-4 for an fp32 p);
//   cdf = p.cumsum()            fp64, strictly sequential: c_i = fl(c_{i-1} + p_i);
//   cdf /= cdf[-1];  u = random_sample();  ind = cdf.searchsorted(u, side='right').
//
// On a float64 x (the reference keeps it float64) the same holds with S an fp64 sum of the same buffers and trees and
// p = |x| / S an fp64 division; numpy's tolerance is then atol = sqrt(eps64) (the *_f64 entry points; every kernel
// below is a template over the element type).
//
// Every rounding above is reproduced.  The one sequential dependency, the fp64 running sum, is made parallel
// without giving up exactness.  Inside one binade [2^E, 2^(E+1)) fp64 values are the multiples m * U of
// U = 2^(E-52), and round-to-nearest-even commutes with a shift by an EVEN multiple of U.  Each chunk of kChunk
// elements is run twice from a guess g of its start (phase A: from g and from g + U, in parallel over chunks).
// When both runs and the true run stay in binade E, the chunk maps the integer m of its true start to
//     m + inc[m & 1]      (the parity picks the run whose distance to the true start is even)
// exactly.  Such maps compose (a pair of increments per input parity), so:
//   * a segmented scan composes the maps of consecutive chunks of one binade inside blocks of kPieceBlk chunks
//     ("pieces"); a chunk whose runs leave their binade, or come within kEta of its edges, is a piece of its own
//     that is special: K3b runs it from four starts G + r (the guess's grid index, r = 0..3) and records, per run,
//     its end and the largest shift d (d = 0 mod 4) under which the run shifted by d stays the run from G + r + d —
//     across one binade edge too, where the spacing doubles (a shift by a multiple of 4 spacings is an even multiple
//     of the new binade's spacing);
//   * one wave walks the pieces in order (O(1) per composed piece and per special chunk whose true start lies within
//     its run's margin; kChunk dependent adds for a chunk re-run), checking that every composed piece starts and ends
//     in its binade — which makes every chunk map in it exact;
//   * the piece holding searchsorted(u) is found among the pieces' exact starts and ends, the chunk inside it from the
//     piece's start and each chunk's exclusive prefix map (one chunk per thread), and that chunk is re-run for the index.
// If a check fails (never expected: the margins are ~100x the guesses' error) the exact chunk-by-chunk chain runs
// instead, so the result never depends on the speculation.  The guesses come from the pairwise partial sums of |x|;
// their accuracy only decides how many chunks are re-run.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <cstdlib>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kBuf = 8192;    // numpy's reduction buffer (np.getbufsize() default)
constexpr int kLeaf = 128;    // numpy PW_BLOCKSIZE
constexpr int kChunk = 256;   // elements per speculated cdf chunk (two pairwise leaves)
constexpr int kQ = kBuf / kChunk;
constexpr int kPad = kBuf + kBuf / kLeaf;  // LDS copy of one buffer, one pad word per leaf
constexpr int kPieceBlk = 1024;            // chunks per block of the piece scan
constexpr int kRecMax = 128;               // pieces per scan block (more: the sequential chain)
constexpr int kWalkBatch = 1024;           // piece records staged in LDS per step of the walk
constexpr int kMaxScanBlocks = 8192;       // ceil(2^31 / kChunk / kPieceBlk)
constexpr double kEta = 1.0 / 65536.0;     // relative margin to a binade edge for a speculated chunk
constexpr int kRecLegacy = 1024;           // chunk records staged in LDS per step of the sequential chain
constexpr int kSpecMax = 4096;             // special chunks per call (more: re-run)
constexpr int kSpecLds = 256;              // special chunks' maps staged in LDS per step of the walk

// status word (device int32) written by ar_check
constexpr int kStNan = 1, kStSum = 2;
constexpr double kAtol = 3.4526698300124393e-04;    // sqrt(finfo(float32).eps)
constexpr double kAtol64 = 1.4901161193847656e-08;  // sqrt(finfo(float64).eps)

// element type helpers: p_i = |x_i| / S in x's type (fp32: then cast to fp64), 16-B vectors of x
__device__ __forceinline__ double q_of(float v, float S) { return (double)(fabsf(v) / S); }
__device__ __forceinline__ double q_of(double v, double S) { return fabs(v) / S; }
__device__ __forceinline__ float abs_of(float v) { return fabsf(v); }
__device__ __forceinline__ double abs_of(double v) { return fabs(v); }
template <class T>
struct Vec16 {  // the elements of one 16-B load
  static constexpr int N = 16 / (int)sizeof(T);
  T e[N];
};
template <class T>
__device__ __forceinline__ Vec16<T> load16(const T* __restrict__ x, int64_t e, int64_t n) {
  Vec16<T> v;
  if (e + Vec16<T>::N <= n) {
    if constexpr (sizeof(T) == 4) {
      const float4 q = *reinterpret_cast<const float4*>(x + e);
      v.e[0] = q.x; v.e[1] = q.y; v.e[2] = q.z; v.e[3] = q.w;
    } else {
      const double2 q = *reinterpret_cast<const double2*>(x + e);
      v.e[0] = q.x; v.e[1] = q.y;
    }
  } else {  // past n: zeros, which leave a running sum unchanged
#pragma unroll
    for (int i = 0; i < Vec16<T>::N; ++i) v.e[i] = e + i < n ? x[e + i] : (T)0;
  }
  return v;
}

// A piece: chunks [first, last] of one scan block.  e >= 1: chunks of binade e whose maps compose to (inc0, inc1);
// e < 0: one chunk re-run from its exact start (inc0 / inc1 then hold its guess and the end of the run from it).
// e <= -2: a special chunk, its four-run map in spec[-2 - e] (the walk's LDS slot of it in `slot`).
struct Rec {
  long long inc0, inc1;
  int first, last, e, slot;
};

// A special chunk (K3b): runs from the grid indices G + r of binade E.  Run r ends at grid index end[r] of binade
// E + ((cross >> r) & 1); a true start m = G + r + d (d = 0 mod 4, |d| <= margin[r]) ends at end[r] + d (no crossing)
// or end[r] + d / 2 (crossed).  margin[r] < 0: run r is unusable.
struct Spec {
  long long G;
  long long end[4];
  long long margin[4];
  int E, cross;
  long long chunk;
};

struct ArWs {
  double* buf_sum;   // [nbuf] pairwise sum of |x| per reduction buffer (in x's type, stored exactly)
  double* bpre;      // [nbuf] fp64 prefix of buf_sum (guesses only)
  double* q_abs;     // [nbuf * kQ] approximate sum of |x| per chunk (guesses only)
  double* guess;     // [nq] speculated start of each chunk's running sum
  double* end_a;     // [nq] end of the run started at guess
  double* end_b;     // [nq] end of the run started at guess + U
  long long* fn;     // [2 nq] the chunk's map: increment for an even / odd start
  int* fe;           // [nq] the chunk's binade when its map is usable, else -1
  long long* pre;    // [2 nq] exclusive prefix of the maps inside the chunk's piece
  int* prec;         // [nq] the chunk's piece (index inside its scan block)
  Rec* rec;          // [nblk * kRecMax]
  int* rec_cnt;      // [nblk]
  int* rec_off;      // [nblk] global index of each scan block's first piece
  double* rec_t;     // [nblk * kRecMax] exact start of each piece (global piece index)
  double* rec_end;   // [nblk * kRecMax] exact end of each piece
  double* start;     // [nq + 1] exact running sum before each chunk; start[nq] = cdf[-1]
  double* p_part;    // [ceil(nq / 256)] partial fp64 sums of p (the "sum to 1" check)
  double* total;     // [1] S (in x's type, stored exactly)
  Spec* spec;        // [kSpecMax] special chunks (K3 appends, K3b fills)
  int32_t* nspec;    // [1] special chunks appended (may exceed kSpecMax: the rest are re-run)
  int32_t* status;   // [1]
  int32_t* fail;     // [1] 1: the speculation did not verify, the sequential chain ran
  int32_t* stats;    // [4] the walk's counts: special chunks, special maps taken, chunks re-run, sequential chain
  long long* lo;     // [1] chunk holding searchsorted(u)
};

__device__ __forceinline__ int binade(double v) {  // exponent field: one grid spacing per value
  return (int)((uint64_t)__double_as_longlong(v) >> 52);  // v >= 0 here
}
__device__ __forceinline__ double spacing(int e) {  // grid spacing of binade e (e = 0: subnormals)
  return e == 0 ? 4.9406564584124654e-324 : ldexp(1.0, e - 1075);
}
// the map of a chunk (or a composition of them) applied to the integer m of an exact start of binade e
__device__ __forceinline__ long long apply_map(long long m, long long i0, long long i1) { return m + ((m & 1) ? i1 : i0); }
__device__ __forceinline__ long long to_grid(double t, int e) { return (long long)ldexp(t, 1075 - e); }
__device__ __forceinline__ double from_grid(long long m, int e) { return ldexp((double)m, e - 1075); }
__device__ __forceinline__ bool in_binade(long long m) { return m >= (1ll << 52) && m < (1ll << 53); }
// wave-uniform copies (SGPRs) of a lane-0 value
__device__ __forceinline__ int rfl32(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {  // lane l's value (l wave-uniform)
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}
// the same two conversions as bit operations, for a normal t of binade e and m in [2^52, 2^53) (the walk's chain)
__device__ __forceinline__ long long grid_bits(double t) {
  return (long long)(((uint64_t)__double_as_longlong(t) & ((1ull << 52) - 1)) | (1ull << 52));
}
__device__ __forceinline__ double bits_grid(long long m, int e) {
  return __longlong_as_double(((long long)e << 52) | (m & ((1ll << 52) - 1)));
}

// ---- numpy's pairwise_sum on fp32 (loops_utils.h.src) ------------------------------------------------
template <class T>
__device__ T pw_leaf(const T* a, int n) {
  if (n < 8) {
    T r = 0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  T r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  }
  T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

// The partial last buffer's pairwise tree (its shape depends on its length only) as a program built on the host:
// the leaves in order, then the internal nodes in post-order, each the sum of two earlier values (value code c: leaf
// c for c < 128, node c - 128 otherwise).  <= 128 leaves and <= 127 nodes for a buffer of <= 8192 elements.
struct TailProg {
  int nleaf, nop, nlvl;
  short lf_start[128], lf_len[128];
  unsigned char op_a[128], op_b[128];
  unsigned char op_lvl[128];  // 1 + the larger of its operands' levels (leaves: 0); one level's nodes are independent
};

void tail_prog_levels(TailProg& p) {  // (host)
  p.nlvl = 0;
  for (int o = 0; o < p.nop; ++o) {
    const int la = p.op_a[o] < 128 ? 0 : p.op_lvl[p.op_a[o] - 128];
    const int lb = p.op_b[o] < 128 ? 0 : p.op_lvl[p.op_b[o] - 128];
    p.op_lvl[o] = (unsigned char)(1 + std::max(la, lb));
    p.nlvl = std::max(p.nlvl, (int)p.op_lvl[o]);
  }
}

int tail_prog_build(TailProg& p, int s0, int m) {  // (host) returns the value code of pairwise_sum(a + s0, m)
  if (m <= kLeaf) {
    p.lf_start[p.nleaf] = (short)s0;
    p.lf_len[p.nleaf] = (short)m;
    return p.nleaf++;
  }
  int n2 = m / 2;
  n2 -= n2 % 8;
  const int a = tail_prog_build(p, s0, n2);
  const int b = tail_prog_build(p, s0 + n2, m - n2);
  p.op_a[p.nop] = (unsigned char)a;
  p.op_b[p.nop] = (unsigned char)b;
  return 128 + p.nop++;
}

template <class T>
__device__ void ar_tail_sum(const T* __restrict__ x, int64_t n, const TailProg& prog, ArWs ws, T* sh);

// ---- K1: full reduction buffers (n2 splits of 8192 are a perfect tree of 64 leaves of 128); one block more for the
// partial last buffer (K1b) when there is one -----------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(256) void ar_buffer_sum_kernel(const T* __restrict__ x, int64_t n, int64_t n_full_bufs,
                                                            TailProg prog, ArWs ws) {
  constexpr int VN = Vec16<T>::N;
  __shared__ T sh[kPad];
  // (the partial buffer, when there is one, takes block 0: its serial tree starts first and hides under the others)
  const bool tail = (int64_t)gridDim.x > n_full_bufs;
  if (tail && blockIdx.x == 0) {
    ar_tail_sum(x, n, prog, ws, sh);
    return;
  }
  const int64_t b = (int64_t)blockIdx.x - (tail ? 1 : 0);
  const T* src = x + b * kBuf;
  // 256 threads x 16-B loads: coalesced, |x| written with one pad word per 128-element leaf
  for (int v = threadIdx.x; v < kBuf / VN; v += 256) {
    const Vec16<T> q = load16(src, (int64_t)VN * v, (int64_t)kBuf);
    const int i = VN * v;
    const int o = i + (i >> 7);
#pragma unroll
    for (int c = 0; c < VN; ++c) sh[o + c] = abs_of(q.e[c]);
  }
  __syncthreads();
  if (threadIdx.x >= kWave) return;
  const int l = threadIdx.x;
  const T* a = sh + l * (kLeaf + 1);  // lane l's leaf: banks l + c, conflict-free
  T r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
#pragma unroll
  for (int i = 8; i < kLeaf; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  }
  T s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  // the tree above the leaves is balanced: a butterfly over the lanes (+ is commutative)
#pragma unroll
  for (int m = 1; m < kWave; m <<= 1) {
    s += __shfl_xor(s, m);
    if (m == kChunk / kLeaf / 2 && (l & (kChunk / kLeaf - 1)) == 0)
      ws.q_abs[b * kQ + l / (kChunk / kLeaf)] = (double)s;  // a two-leaf subtree = one cdf chunk
  }
  if (l == 0) ws.buf_sum[b] = (double)s;
}

// ---- K1b: the last, partial buffer (an irregular tree; the last block of K1's launch): leaves in parallel, then the
// tree's <= 127 additions level by level (the host-built program; every addition as in the tree, so the same sum) ----
template <class T>
__device__ void ar_tail_sum(const T* __restrict__ x, int64_t n, const TailProg& prog, ArWs ws, T* sh) {
  constexpr int VN = Vec16<T>::N;
  __shared__ T lf_sum[128], op_sum[128];
  const int tid = threadIdx.x;
  const int64_t b = n / kBuf;
  const int len = (int)(n - b * kBuf);
  for (int v = tid; v * VN < len; v += 256) {
    const Vec16<T> q = load16(x + b * kBuf, (int64_t)v * VN, (int64_t)len);
#pragma unroll
    for (int c = 0; c < VN; ++c) sh[v * VN + c] = abs_of(q.e[c]);
  }
  __syncthreads();
  if (tid < prog.nleaf) lf_sum[tid] = pw_leaf(sh + prog.lf_start[tid], prog.lf_len[tid]);
  // guesses: an fp64 sum of |x| per chunk of the partial buffer (any order: eight 32-element parts per chunk)
  if (tid < kQ * 8) {
    const int c = tid >> 3, lo = c * kChunk + (tid & 7) * 32, hi = std::min(len, lo + 32);
    double s = 0.0;
    for (int i = lo; i < hi; ++i) s += (double)sh[i];
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    if ((tid & 7) == 0 && c * kChunk < len) ws.q_abs[b * kQ + c] = s;
  }
  for (int l = 1; l <= prog.nlvl; ++l) {
    __syncthreads();
    if (tid < prog.nop && prog.op_lvl[tid] == l) {
      const int a = prog.op_a[tid], c = prog.op_b[tid];
      op_sum[tid] = (a < 128 ? lf_sum[a] : op_sum[a - 128]) + (c < 128 ? lf_sum[c] : op_sum[c - 128]);
    }
  }
  __syncthreads();
  if (tid == 0) ws.buf_sum[b] = (double)(prog.nop ? op_sum[prog.nop - 1] : lf_sum[0]);
}

// ---- K2: S (buffers folded in order, in x's type) and the fp64 prefix of the buffer sums (guesses) -------------
// The fold is one dependent chain of adds: thread 0 reads the tile 16 B at a time (the reads off the chain).  Past
// nbuf the tile holds +0, which leaves S (a sum of |x|, never -0) unchanged.
template <class T>
__global__ __launch_bounds__(1024) void ar_total_kernel(int64_t nbuf, ArWs ws) {
  __shared__ __attribute__((aligned(16))) T tile[1024];
  __shared__ double scan_lds[1024 / kWave];
  const int tid = threadIdx.x;
  T S = 0;
  double carry = 0.0;
  if (tid == 0) ws.nspec[0] = 0;  // (phase A, the next kernel but one, appends the special chunks)
  for (int64_t base = 0; base < nbuf; base += 1024) {
    const int64_t i = base + tid;
    const T v = i < nbuf ? (T)ws.buf_sum[i] : (T)0;
    tile[tid] = v;
    double tot;
    const double ex = block_excl_scan<double, 1024 / kWave>((double)v, scan_lds, &tot);  // (syncs: tile ready)
    if (i < nbuf) ws.bpre[i] = carry + ex;
    carry += tot;
    if (tid == 0) {
      constexpr int VN = Vec16<T>::N;
      const int nv = (int)((std::min<int64_t>(1024, nbuf - base) + VN - 1) / VN);
#pragma unroll 8
      for (int j = 0; j < nv; ++j) {
        if constexpr (sizeof(T) == 4) {
          const float4 q = reinterpret_cast<const float4*>(tile)[j];
          S = S + q.x;
          S = S + q.y;
          S = S + q.z;
          S = S + q.w;
        } else {
          const double2 q = reinterpret_cast<const double2*>(tile)[j];
          S = S + q.x;
          S = S + q.y;
        }
      }
    }
    __syncthreads();
  }
  if (tid == 0) ws.total[0] = (double)S;
}

// ---- K3 (phase A): per chunk, the two speculative runs, the chunk's map and its sum of p ------------------
// A wave owns 64 consecutive chunks and stages them through LDS in four rounds of 64 elements each (16-B loads,
// 16 lanes per 256 B row piece); lane c then runs chunk c from its row (stride 65 words: conflict-free).
// (float64: rounds of 32 elements per row, so a lane's loads stay sixteen 16-B vectors)
template <class T>
__global__ __launch_bounds__(256) void ar_phase_a_kernel(const T* __restrict__ x, int64_t n, int64_t nq, ArWs ws) {
  constexpr int VN = Vec16<T>::N, kRowE = 16 * VN, kRow = kRowE + 1;
  __shared__ T stage[4][kWave * kRow];
  __shared__ double red[4];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x >> 6;
  const int64_t j0 = (int64_t)blockIdx.x * 256 + wid * kWave;  // the wave's first chunk (a multiple of 2 kQ)
  const int64_t j = j0 + lane;
  const T S = (T)ws.total[0];
  const double inv = 1.0 / (double)S;
  // guess = the buffer's fp64 prefix + the exclusive prefix of the chunk sums inside the buffer (32 lanes each)
  const double qa = j < nq ? ws.q_abs[j] : 0.0;
  const double incl = wave_incl_scan(qa);
  const double half = lane_bcast(incl, kQ - 1);
  const double ga = j < nq ? (ws.bpre[j / kQ] + (incl - qa - (lane >= kQ ? half : 0.0))) * inv : 0.0;
  const int E = binade(ga);
  const double gb = ga + spacing(E);
  double ca = ga, cb = gb, ps = 0.0;
  T* st = stage[wid];
  for (int r = 0; r < kChunk / kRowE; ++r) {
    Vec16<T> v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int f = i * kWave + lane, row = f >> 4, c4 = f & 15;
      v[i] = load16(x, (j0 + row) * kChunk + r * kRowE + c4 * VN, n);
    }
    __builtin_amdgcn_wave_barrier();  // the previous round's rows are read (LDS ops complete in order per wave)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int f = i * kWave + lane, row = f >> 4, c4 = f & 15;
      T* d = st + row * kRow + c4 * VN;
#pragma unroll
      for (int c = 0; c < VN; ++c) d[c] = v[i].e[c];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const T* rowp = st + lane * kRow;
#pragma unroll 16
    for (int e = 0; e < kRowE; ++e) {
      const double q = q_of(rowp[e], S);
      ca = ca + q;
      cb = cb + q;
      ps += q;
    }
  }
  if (j < nq) {
    // usable map: both runs in binade E, clear of its edges by kEta (the true start lies within ~2^-19 of ga)
    const bool ok = E >= 1 && binade(gb) == E && binade(ca) == E && binade(cb) == E &&
                    ga >= ldexp(1.0 + kEta, E - 1023) && fmax(ca, cb) <= ldexp(1.0 - kEta, E - 1022);
    long long i0 = 0, i1 = 0;
    if (ok) {
      const long long G = to_grid(ga, E);
      const long long d0 = to_grid(ca - ga, E), d1 = to_grid(cb - gb, E);
      // a start of the same parity as G is an even distance from ga: the run from ga; otherwise from ga + U
      i0 = (G & 1) ? d1 : d0;
      i1 = (G & 1) ? d0 : d1;
    }
    ws.guess[j] = ga;
    ws.end_a[j] = ca;
    ws.end_b[j] = cb;
    ws.fn[2 * j] = i0;
    ws.fn[2 * j + 1] = i1;
    int fe = ok ? E : -1;
    if (!ok && E >= 1 && E <= 2044 && binade(ca) <= E + 1) {  // crosses one edge, or near one: a special chunk
      const int idx = atomicAdd(ws.nspec, 1);
      if (idx < kSpecMax) {
        Spec* sp = ws.spec + idx;
        sp->G = to_grid(ga, E);
        sp->E = E;
        sp->chunk = j;
        fe = -2 - idx;
      }
    }
    ws.fe[j] = fe;
  }
  const double s = wave_sum(j < nq ? ps : 0.0);
  if (lane == 0) red[wid] = s;
  __syncthreads();
  if (threadIdx.x == 0) ws.p_part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---- K4: numpy's checks on p (before any uniform is drawn): block 0 of the special kernel's launch (K3b) -----------
__device__ void ar_check(int64_t nparts, double atol, ArWs ws, int32_t* status_out) {
  __shared__ double lds[256 / kWave];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < nparts; i += 256) s += ws.p_part[i];
  s = block_sum<double, 256 / kWave>(s, lds);
  if (threadIdx.x == 0) {
    int st = 0;
    if (isnan(s)) st = kStNan;
    else if (!(fabs(s - 1.0) <= atol)) st = kStSum;
    ws.status[0] = st;
    if (status_out) *status_out = st;
  }
}

// ---- K5: pieces — a segmented scan of the chunk maps inside each block of kPieceBlk chunks ---------------
// compose(f, g) = f then g: an input of parity p moves by f[p], then by g at the new parity
__device__ __forceinline__ void compose(long long f0, long long f1, long long g0, long long g1, long long* h0,
                                        long long* h1) {
  *h0 = f0 + ((f0 & 1) ? g1 : g0);
  *h1 = f1 + ((f1 & 1) ? g0 : g1);
}

__global__ __launch_bounds__(kPieceBlk) void ar_piece_kernel(int64_t nq, ArWs ws) {
  __shared__ long long s0[kPieceBlk], s1[kPieceBlk];
  __shared__ int sh[kPieceBlk], se[kPieceBlk];
  __shared__ int scan_lds[kPieceBlk / kWave];
  if (ws.status[0] != 0) return;
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * kPieceBlk + tid;
  const bool valid = j < nq;
  const int e = valid ? ws.fe[j] : -2;
  long long a0 = valid ? ws.fn[2 * j] : 0, a1 = valid ? ws.fn[2 * j + 1] : 0;
  se[tid] = e;
  __syncthreads();
  const int ep = tid > 0 ? se[tid - 1] : -3;
  // a piece starts at the block's first chunk, at a binade change, and at / after a chunk to re-run
  int head = (tid == 0 || e < 0 || ep < 0 || e != ep) ? 1 : 0;
  // Hillis-Steele segmented inclusive scan: (f, h) (+) (g, k) = (k ? g : f then g, h | k)
  int hf = head;
  s0[tid] = a0;
  s1[tid] = a1;
  sh[tid] = hf;
  __syncthreads();
  for (int d = 1; d < kPieceBlk; d <<= 1) {
    long long n0 = a0, n1 = a1;
    int nh = hf;
    if (tid >= d && !hf) {
      compose(s0[tid - d], s1[tid - d], a0, a1, &n0, &n1);
      nh = sh[tid - d];
    }
    __syncthreads();
    a0 = n0;
    a1 = n1;
    hf = hf | nh;
    s0[tid] = a0;
    s1[tid] = a1;
    sh[tid] = hf;
    __syncthreads();
  }
  // exclusive prefix inside the piece: the previous chunk's inclusive value, or the identity at a head
  const long long p0 = head ? 0 : (tid > 0 ? s0[tid - 1] : 0), p1 = head ? 0 : (tid > 0 ? s1[tid - 1] : 0);
  int nheads;
  const int hx = block_excl_scan<int, kPieceBlk / kWave>(valid ? head : 0, scan_lds, &nheads);
  const int r = hx + (valid ? head : 0) - 1;  // this chunk's piece
  if (!valid) return;
  ws.pre[2 * j] = p0;
  ws.pre[2 * j + 1] = p1;
  ws.prec[j] = r;
  if (tid == 0) ws.rec_cnt[blockIdx.x] = nheads;
  if (r >= kRecMax) return;  // (the walk sees the count and takes the sequential chain)
  Rec* rc = ws.rec + (size_t)blockIdx.x * kRecMax + r;
  if (head) {
    rc->first = (int)j;
    rc->e = e;
  }
  const bool last = tid == kPieceBlk - 1 || j + 1 == nq || se[tid + 1] < 0 || e < 0 || se[tid + 1] != e;
  if (last) {
    rc->last = (int)j;
    if (e >= 1) {
      rc->inc0 = a0;
      rc->inc1 = a1;
    } else {  // a re-run chunk: its guess and the end of the run from it (the run is exact when the start is)
      rc->inc0 = __double_as_longlong(ws.guess[j]);
      rc->inc1 = __double_as_longlong(ws.end_a[j]);
    }
  }
}

// Exact sequential run of chunk u from its exact start t by one wave (every lane ends with the same t).  The
// chunk's elements are v (4 per lane, lane-major); their p values are staged in the wave's LDS scratch qs (kChunk
// doubles) and every lane reads them in order (same address: a broadcast; the reads are off the add chain).  With
// cD > 0 each lane also returns, per element it holds, the normalised cdf test c / cD > u as a bit of *hits.
template <class T>
struct Four {
  T a, b, c, d;
};
template <class T>
__device__ __forceinline__ void stage_q(const Four<T> v, T S, double* qs) {
  const int lane = threadIdx.x & (kWave - 1);
  __builtin_amdgcn_wave_barrier();  // (this wave's earlier reads of qs come first: LDS ops complete in order)
  reinterpret_cast<double2*>(qs)[2 * lane] = make_double2(q_of(v.a, S), q_of(v.b, S));
  reinterpret_cast<double2*>(qs)[2 * lane + 1] = make_double2(q_of(v.c, S), q_of(v.d, S));
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <class T>
__device__ double wave_run(const Four<T> v, double t, T S, double* qs, double cD = 0.0, double u = 0.0,
                           unsigned* hits = nullptr) {
  const int lane = threadIdx.x & (kWave - 1);
  stage_q(v, S, qs);
  const double2* q2 = reinterpret_cast<const double2*>(qs);
  double k0 = 0.0, k1 = 0.0, k2 = 0.0, k3 = 0.0;  // (hits) this lane's own four running sums
#pragma unroll 8
  for (int L = 0; L < kWave; ++L) {
    const double2 a = q2[2 * L], b = q2[2 * L + 1];
    t = t + a.x;
    const double c0 = t;
    t = t + a.y;
    const double c1 = t;
    t = t + b.x;
    const double c2 = t;
    t = t + b.y;
    if (hits && lane == L) {
      k0 = c0;
      k1 = c1;
      k2 = c2;
      k3 = t;
    }
  }
  // (the divisions after the chain, all lanes at once, not 256 of them on it)
  if (hits) *hits = (k0 / cD > u ? 1u : 0u) | (k1 / cD > u ? 2u : 0u) | (k2 / cD > u ? 4u : 0u) | (k3 / cD > u ? 8u : 0u);
  return t;
}

// The same run from a per-lane start t, also returning the last running sum below `edge` (or the start) and the
// first at or above it (or inf).
template <class T>
__device__ double wave_run_edges(const Four<T> v, double t, T S, double* qs, double edge, double* below,
                                 double* above) {
  stage_q(v, S, qs);
  const double2* q2 = reinterpret_cast<const double2*>(qs);
  double lo = t, hi = __longlong_as_double(0x7ff0000000000000ll);
#define FLC_AR_STEP(q)    \
  t = t + (q);            \
  lo = t < edge ? t : lo; \
  hi = (t >= edge && t < hi) ? t : hi;
#pragma unroll 8
  for (int L = 0; L < kWave; ++L) {
    const double2 a = q2[2 * L], b = q2[2 * L + 1];
    FLC_AR_STEP(a.x)
    FLC_AR_STEP(a.y)
    FLC_AR_STEP(b.x)
    FLC_AR_STEP(b.y)
  }
#undef FLC_AR_STEP
  *below = lo;
  *above = hi;
  return t;
}

template <class T>
__device__ __forceinline__ Four<T> load_chunk4(const T* __restrict__ x, int64_t n, int64_t u) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t e = u * kChunk + 4 * lane;
  if (e + 4 <= n) {
    if constexpr (sizeof(T) == 4) {
      const float4 q = *reinterpret_cast<const float4*>(x + e);
      return Four<T>{q.x, q.y, q.z, q.w};
    } else {
      const double2 q0 = *reinterpret_cast<const double2*>(x + e), q1 = *reinterpret_cast<const double2*>(x + e + 2);
      return Four<T>{q0.x, q0.y, q1.x, q1.y};
    }
  }
  return Four<T>{e < n ? x[e] : (T)0, e + 1 < n ? x[e + 1] : (T)0, e + 2 < n ? x[e + 2] : (T)0, (T)0};
}

// ---- K3b: the special chunks' four runs (one wave per chunk; lane r & 3 runs from G + r) -----------------------
// Run r is the true run from G + r + d (d = 0 mod 4) when the true start is in binade E and |d| <= margin[r]:
//   * no crossing: every sum of the run shifted by d stays below the edge 2^(E+1) while it is <= margin + 2 spacings
//     from it, and round-to-nearest-even commutes with a shift by an even multiple of the spacing;
//   * one crossing: the sums before it stay below the edge (lo), the first one after it stays above (hi, in spacings
//     of E; its rounding error is at most one), and the rest stay below 2^(E+2) (top).  In binade E + 1 the shift d is
//     an even multiple of the spacing 2 U because d = 0 mod 4.
// (block 0 first runs the check, K4; the runs do not wait for it: with a failed check the select never reads them)
template <class T>
__global__ __launch_bounds__(256) void ar_special_kernel(const T* __restrict__ x, int64_t n, ArWs ws, int64_t nparts,
                                                         double atol, int32_t* status_out) {
  if (blockIdx.x == 0) ar_check(nparts, atol, ws, status_out);
  __shared__ double q_lds[256 / kWave][kChunk];
  const int nsp = min(ws.nspec[0], kSpecMax);
  const int lane = threadIdx.x & (kWave - 1), r = lane & 3;
  const T S = (T)ws.total[0];
  for (int s = blockIdx.x * (256 / kWave) + (threadIdx.x >> 6); s < nsp; s += gridDim.x * (256 / kWave)) {
    Spec* sp = ws.spec + s;
    const int E = sp->E;
    const long long G = sp->G;
    const Four<T> v = load_chunk4(x, n, sp->chunk);
    const bool valid = G + r >= (1ll << 52) && G + r < (1ll << 53);
    const double edge = ldexp(1.0, E - 1022);
    double below, above;
    const double t =
        wave_run_edges(v, from_grid(valid ? G + r : (1ll << 52), E), S, q_lds[threadIdx.x >> 6], edge, &below, &above);
    long long end = 0, margin = -1;
    int cross = 0;
    if (valid) {
      const int eb = binade(t);
      if (eb == E) {
        end = to_grid(t, E);
        margin = to_grid(edge - t, E) - 2;
      } else if (eb == E + 1) {
        cross = 1;
        end = to_grid(t, E + 1);
        const long long lo = to_grid(edge - below, E), hi = to_grid(above - edge, E), top = to_grid(2.0 * edge - t, E);
        margin = std::min(std::min(lo, hi), top) - 2;
      }
    }
    const unsigned long long cm = __ballot(cross != 0);
    if (lane < 4) {
      sp->end[r] = end;
      sp->margin[r] = margin;
    }
    if (lane == 0) sp->cross = (int)(cm & 15ull);
  }
}

// ---- K6: the walk — every piece's exact start, in order, on one wave ---------------------------------------
// Blocks 1.. of the launch write the dense output's zeros meanwhile (the walk is one wave's latency chain).
template <class T>
__global__ __launch_bounds__(1024) void ar_walk_kernel(const T* __restrict__ x, int64_t n, int64_t nq, int nblk,
                                                       int force_seq, double u, ArWs ws, T* __restrict__ out) {
  __shared__ int off[kMaxScanBlocks];
  __shared__ Rec batch[kWalkBatch];
  __shared__ Spec spec_lds[kSpecLds];
  __shared__ double t_lds[kWalkBatch], end_lds[kWalkBatch];  // the batch's piece starts / ends (written out after)
  __shared__ double q_lds[kChunk];                             // wave 0's re-run scratch
  __shared__ long long run0[kWalkBatch], run1[kWalkBatch];     // the runs' segmented map scan
  __shared__ int run_h[kWalkBatch], run_x[kWalkBatch], run_e[kWalkBatch], item_r[kWalkBatch];
  __shared__ int scan_lds[1024 / kWave];
  __shared__ int s_bad, s_total, s_taken, s_reruns, s_piece;
  __shared__ double s_t;
  if (ws.status[0] != 0) return;
  const int tid = threadIdx.x;
  if (blockIdx.x > 0) {  // out = 0 (16-B stores past a head of < 16 B; the final kernel writes out[ind] later)
    constexpr int VN = Vec16<T>::N;
    const int64_t head = std::min<int64_t>(n, (int64_t)((16 - ((uintptr_t)out & 15)) & 15) / (int64_t)sizeof(T));
    const int64_t nv = (n - head) / VN;
    const int64_t stride = (int64_t)(gridDim.x - 1) * 1024;
    uint4* o4 = reinterpret_cast<uint4*>(out + head);
    for (int64_t i = (int64_t)(blockIdx.x - 1) * 1024 + tid; i < nv; i += stride) o4[i] = make_uint4(0u, 0u, 0u, 0u);
    if (blockIdx.x == 1) {
      if (tid < head) out[tid] = (T)0;
      if (tid < n - head - nv * VN) out[head + nv * VN + tid] = (T)0;
    }
    return;
  }
#if FLC_CALIB_AR_STAMPS  // calibration builds only: the walk's phase times (10 ns ticks) replace the stats
  const uint64_t st0 = __builtin_amdgcn_s_memrealtime();
  uint64_t st1 = 0, st2 = 0, st3 = 0, st4 = 0;
#endif
  if (tid == 0) {
    s_bad = force_seq;
    s_taken = 0;
    s_reruns = 0;
    s_t = 0.0;  // cdf starts from 0: c_0 = 0 + p_0
  }
  __syncthreads();
  // the pieces' global numbering (a scan of the per-block counts)
  int carry = 0;
  for (int base = 0; base < nblk; base += 1024) {
    const int b = base + tid;
    const int c = b < nblk ? ws.rec_cnt[b] : 0;
    if (c > kRecMax) s_bad = 1;
    int tot;
    const int ex = block_excl_scan<int, 1024 / kWave>(c, scan_lds, &tot);
    if (b < nblk) {
      off[b] = carry + ex;
      ws.rec_off[b] = carry + ex;
    }
    carry += tot;
  }
  if (tid == 0) s_total = carry;
  __syncthreads();
  const int total = s_total;
#if FLC_CALIB_AR_STAMPS
  st1 = __builtin_amdgcn_s_memrealtime();
#endif
  const T S = (T)ws.total[0];
  for (int g0 = 0; g0 < total && !s_bad; g0 += kWalkBatch) {
    const int g = g0 + tid;
    const bool valid = g < total;
    Rec rc{};
    if (valid) {  // the block holding piece g: the last b with off[b] <= g
      int lo = 0, hi = nblk - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= g) lo = mid;
        else hi = mid - 1;
      }
      rc = ws.rec[(size_t)lo * kRecMax + (g - off[lo])];
    }
    // Consecutive composed pieces of one binade (split only by the scan blocks' bounds) compose further: a segmented
    // scan of their maps over the batch ("runs"), so the walk steps once per run and once per other piece.
    const bool mp = valid && rc.e >= 1;
    run_e[tid] = valid ? rc.e : -100;
    __syncthreads();
    const int ep = tid > 0 ? run_e[tid - 1] : -100, en = tid + 1 < kWalkBatch ? run_e[tid + 1] : -100;
    const bool head = mp && !(ep >= 1 && ep == rc.e), last = mp && !(en >= 1 && en == rc.e);
    long long a0 = mp ? rc.inc0 : 0, a1 = mp ? rc.inc1 : 0;
    int hf = (head || !mp) ? 1 : 0, hx = tid;  // segment flag; the run's head (its own index at a head)
    run0[tid] = a0;
    run1[tid] = a1;
    run_h[tid] = hf;
    run_x[tid] = hx;
    __syncthreads();
    for (int d = 1; d < kWalkBatch; d <<= 1) {
      long long n0 = a0, n1 = a1;
      int nh = hf, nx = hx;
      if (tid >= d && !hf) {
        compose(run0[tid - d], run1[tid - d], a0, a1, &n0, &n1);
        nh = run_h[tid - d];
        nx = run_x[tid - d];
      }
      __syncthreads();
      a0 = n0;
      a1 = n1;
      hf = hf | nh;
      hx = nx;
      run0[tid] = a0;
      run1[tid] = a1;
      run_h[tid] = hf;
      run_x[tid] = hx;
      __syncthreads();
    }
    // exclusive map inside the run (identity at its head); the walk items: every non-map piece and each run's last
    const long long x0 = (mp && !head) ? run0[tid - 1] : 0, x1 = (mp && !head) ? run1[tid - 1] : 0;
    const bool item = valid && (!mp || last);
    int nitems;
    const int ii = block_excl_scan<int, 1024 / kWave>(item ? 1 : 0, scan_lds, &nitems);
    // the batch's special chunks' maps into LDS slots (beyond kSpecLds of them: read from memory on the walk)
    const bool is_sp = valid && rc.e <= -2;
    int nsp;
    const int slot = block_excl_scan<int, 1024 / kWave>(is_sp ? 1 : 0, scan_lds, &nsp);
    if (valid) {
      rc.slot = (is_sp && slot < kSpecLds) ? slot : -1;
      if (rc.slot >= 0) spec_lds[slot] = ws.spec[-2 - rc.e];
      if (mp) {  // a run's last: the run's composed map, and its head's index in `first`
        rc.inc0 = a0;
        rc.inc1 = a1;
        rc.first = hx;
      }
      if (item) {
        batch[ii] = rc;
        item_r[ii] = tid;
      }
    }
    __syncthreads();
#if FLC_CALIB_AR_STAMPS
    if (g0 == 0) st2 = __builtin_amdgcn_s_memrealtime();
#endif
    if (tid < kWave) {  // wave 0 walks the batch's items
      // The state is t's bit pattern, wave-uniform (scalar registers), so a composed run's step is a few scalar
      // integer ops on it: grid index = mantissa | 2^52, binade = the exponent field.  Items in windows of 64: lane i
      // holds item w0 + i (one LDS read per lane per window), the step reads its fields with readlane, and lane i keeps
      // the item's start / end for one LDS store per lane after the window.
      const int cnt = nitems;
      uint64_t tb = rfl64((uint64_t)__double_as_longlong(s_t));
      bool bad = false;
      int taken = 0, reruns = 0;
      const int lane = tid;
      constexpr uint64_t kMant = (1ull << 52) - 1, kHid = 1ull << 52;
      for (int w0 = 0; w0 < cnt && !bad; w0 += kWave) {
        const int wn = std::min(kWave, cnt - w0);
        Rec mine{};
        int my_r = 0;
        if (lane < wn) {
          mine = batch[w0 + lane];
          my_r = item_r[w0 + lane];
        }
        // a special item's map in its lane's registers too (from its LDS slot, or from memory past kSpecLds)
        long long sG = 0, sEnd[4] = {0, 0, 0, 0}, sMg[4] = {-1, -1, -1, -1};
        int sE = -1, sCross = 0;
        if (lane < wn && mine.e <= -2) {
          Spec v;
          if (mine.slot >= 0) v = spec_lds[mine.slot];
          else v = ws.spec[-2 - mine.e];
          sG = v.G;
          sE = v.E;
          sCross = v.cross;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            sEnd[q] = v.end[q];
            sMg[q] = v.margin[q];
          }
        }
        uint64_t my_t = 0, my_end = 0;
        for (int i = 0; i < wn; ++i) {
          const int e = __builtin_amdgcn_readlane(mine.e, i);
          const uint64_t inc0 = rl64((uint64_t)mine.inc0, i), inc1 = rl64((uint64_t)mine.inc1, i);
          my_t = lane == i ? tb : my_t;
          if (e >= 1) {  // a composed run of binade e: its map on the grid index
            const uint64_t m = (tb & kMant) | kHid;
            const uint64_t m2 = m + ((m & 1) ? inc1 : inc0);
            if ((int)(tb >> 52) != e || m2 < kHid || m2 >= 2 * kHid) {
              bad = true;
              break;
            }
            tb = ((uint64_t)e << 52) | (m2 & kMant);
          } else {
            const int first = __builtin_amdgcn_readlane(mine.first, i);
            bool done = false;
            if (e <= -2) {  // a special chunk: its run's map when the true start is within its margin
              const int se = __builtin_amdgcn_readlane(sE, i), cross = __builtin_amdgcn_readlane(sCross, i);
              const long long m = (long long)((tb & kMant) | kHid);
              const long long G = (long long)rl64((uint64_t)sG, i);
              const int rr = (int)((m - G) & 3);
              const long long d = m - G - rr;
              const long long mgv = rr == 0 ? sMg[0] : rr == 1 ? sMg[1] : rr == 2 ? sMg[2] : sMg[3];
              const long long env = rr == 0 ? sEnd[0] : rr == 1 ? sEnd[1] : rr == 2 ? sEnd[2] : sEnd[3];
              const long long mg = (long long)rl64((uint64_t)mgv, i), end = (long long)rl64((uint64_t)env, i);
              const int cr = (cross >> rr) & 1;
              const long long m2 = end + (cr ? d / 2 : d);
              if ((int)(tb >> 52) == se && mg >= 0 && (d < 0 ? -d : d) <= mg && in_binade(m2)) {
                tb = ((uint64_t)(se + cr) << 52) | ((uint64_t)m2 & kMant);
                done = true;
                ++taken;
              }
            }
            if (!done) {
              if (tb == inc0) {
                tb = inc1;  // started at the guess: the run from it is the run
              } else {
                const double t = wave_run(load_chunk4(x, n, first), __longlong_as_double((long long)tb), S, q_lds);
                tb = rfl64((uint64_t)__double_as_longlong(t));
                ++reruns;
              }
            }
          }
          my_end = lane == i ? tb : my_end;
        }
        if (lane < wn) {  // a run's start goes to its head's slot (the write-out below needs it); ends by record
          t_lds[mine.e >= 1 ? mine.first : my_r] = __longlong_as_double((long long)my_t);
          end_lds[my_r] = __longlong_as_double((long long)my_end);
        }
      }
      const double t = __longlong_as_double((long long)tb);
      if (tid == 0) {
        s_t = t;
        if (bad) s_bad = 1;
        s_taken += taken;
        s_reruns += reruns;
#if FLC_CALIB_AR_STAMPS
        st4 = __builtin_amdgcn_s_memrealtime();
#endif
      }
    }
    __syncthreads();
    if (valid) {  // every piece's start and end (a run's pieces from its start and their maps, all in its binade)
      double ts = t_lds[tid], te = end_lds[tid];
      if (mp) {
        const long long m0 = grid_bits(t_lds[hx]);
        ts = bits_grid(apply_map(m0, x0, x1), rc.e);
        te = bits_grid(apply_map(m0, a0, a1), rc.e);
      }
      ws.rec_t[g] = ts;
      ws.rec_end[g] = te;
    }
    __syncthreads();  // (the next batch rewrites the LDS arrays)
  }
  // The chunk holding searchsorted(u, side='right'): the piece first (the normalised cdf is non-decreasing and
  // cdf[-1] / cdf[-1] = 1 > u, so exactly one piece has start <= u < end), then the chunk inside it, one per thread.
  if (!s_bad) {
    const double cD = s_t;
    if (tid == 0) s_piece = -1;
    __syncthreads();  // (and every batch's rec_t / rec_end, written by this block, are visible)
    for (int g = tid; g < total; g += 1024)
      if (ws.rec_t[g] / cD <= u && ws.rec_end[g] / cD > u) s_piece = g;
    __syncthreads();
    const int gp = s_piece;
    if (gp >= 0) {
      int lo = 0, hi = nblk - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= gp) lo = mid;
        else hi = mid - 1;
      }
      const Rec rc = ws.rec[(size_t)lo * kRecMax + (gp - off[lo])];
      const int64_t j = (int64_t)rc.first + tid;
      if (j <= rc.last) {
        const double tp = ws.rec_t[gp];
        const int e = ws.fe[j];
        double t = tp, end = ws.rec_end[gp];
        if (e >= 1) {
          const long long m = apply_map(to_grid(tp, e), ws.pre[2 * j], ws.pre[2 * j + 1]);
          t = from_grid(m, e);
          end = from_grid(apply_map(m, ws.fn[2 * j], ws.fn[2 * j + 1]), e);
        }
        if (t / cD <= u && end / cD > u) {
          ws.lo[0] = j;
          ws.start[j] = t;
        }
      }
    }
  }
  if (tid == 0) {
    ws.start[nq] = s_t;
    ws.fail[0] = s_bad;
    ws.stats[0] = ws.nspec[0];
    ws.stats[1] = s_taken;
    ws.stats[2] = s_reruns;
    ws.stats[3] = s_bad;
#if FLC_CALIB_AR_STAMPS
    st3 = __builtin_amdgcn_s_memrealtime();
    ws.stats[0] = (int)(st1 - st0);
    ws.stats[1] = (int)(st2 - st0);
    ws.stats[2] = (int)(st3 - st0);
    ws.stats[3] = (int)(st4 - st0);
#endif
  }
}

// ---- K8: the index — chunk lo re-run from its exact start; or, if the speculation failed, the exact
// chunk-by-chunk chain (phase B of the sequential design) and a binary search first ----------------------------
template <class T>
__global__ __launch_bounds__(1024) void ar_final_kernel(const T* __restrict__ x, int64_t n, int64_t nq, double u,
                                                        ArWs ws, int64_t* __restrict__ index, T* __restrict__ out) {
  __shared__ double g_s[kRecLegacy], ea_s[kRecLegacy], eb_s[kRecLegacy];
  __shared__ double q_lds[kChunk];  // wave 0's run scratch
  __shared__ long long s_lo;
  if (ws.status[0] != 0) return;  // the host raises numpy's ValueError; nothing is drawn or written
  const int tid = threadIdx.x;
  const T S = (T)ws.total[0];
  if (ws.fail[0] != 0) {
    double t = 0.0;
    for (int64_t base = 0; base < nq; base += kRecLegacy) {
      const int64_t i = base + tid;
      if (i < nq) {
        g_s[tid] = ws.guess[i];
        ea_s[tid] = ws.end_a[i];
        eb_s[tid] = ws.end_b[i];
      }
      __syncthreads();
      if (tid < kWave) {
        const int cnt = (int)std::min<int64_t>(kRecLegacy, nq - base);
        for (int r = 0; r < cnt; ++r) {
          const int64_t jj = base + r;
          if (tid == 0) ws.start[jj] = t;
          const double ga = g_s[r];
          const double d = t - ga;
          if (d == 0.0) {  // the speculated run IS the run
            t = ea_s[r];
            continue;
          }
          const int e = binade(ga);
          bool ok = e >= 1 && binade(t) == e;  // then d is exact and a multiple of U
          double cand = 0.0;
          if (ok) {
            const long long k = to_grid(d, e);
            const bool even = (k & 1) == 0;
            const double g = even ? ga : ga + spacing(e);
            const double end = even ? ea_s[r] : eb_s[r];
            cand = end + (t - g);
            ok = binade(g) == e && binade(end) == e && binade(cand) == e;
          }
          t = ok ? cand : wave_run(load_chunk4(x, n, jj), t, S, q_lds);
        }
      }
      __syncthreads();
    }
    if (tid == 0) {
      ws.start[nq] = t;
      const double cD = t;
      int64_t lo = 0, hi = nq - 1;  // first chunk whose last normalised cdf value exceeds u
      while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        const double end = mid + 1 < nq ? ws.start[mid + 1] : cD;
        if (end / cD > u) hi = mid;
        else lo = mid + 1;
      }
      s_lo = lo;
    }
    __syncthreads();
  } else if (tid == 0) {
    s_lo = ws.lo[0];
  }
  __syncthreads();
  if (tid >= kWave) return;
  const int64_t lo = s_lo;
  const double cD = ws.start[nq];
  unsigned hits = 0;
  (void)wave_run(load_chunk4(x, n, lo), ws.start[lo], S, q_lds, cD, u, &hits);
  // the first element of the chunk whose normalised cdf exceeds u (the chunk's end does: some element qualifies;
  // elements past n add 0 and never come first)
  const unsigned long long any = __ballot(hits != 0);
  const int L = __builtin_ctzll(any);
  const unsigned hl = (unsigned)__builtin_amdgcn_readlane((int)hits, L);
  const int64_t ind = std::min<int64_t>(n - 1, lo * kChunk + 4 * L + __builtin_ctz(hl));
  if (tid == 0) {
    index[0] = ind;
    out[ind] = x[ind];
  }
}

ArWs carve(void* base, int64_t n, size_t* bytes) {
  const int64_t nbuf = cdiv(n, kBuf), nq = cdiv(n, kChunk), nblk = cdiv(nq, kPieceBlk), npa = cdiv(nq, 256);
  Carver c(base, base ? ~size_t(0) : 0);
  ArWs w;
  w.buf_sum = c.take<double>(nbuf);
  w.bpre = c.take<double>(nbuf);
  w.q_abs = c.take<double>(nbuf * kQ);
  w.guess = c.take<double>(nq);
  w.end_a = c.take<double>(nq);
  w.end_b = c.take<double>(nq);
  w.fn = c.take<long long>(2 * nq);
  w.fe = c.take<int>(nq);
  w.pre = c.take<long long>(2 * nq);
  w.prec = c.take<int>(nq);
  w.rec = c.take<Rec>(nblk * kRecMax);
  w.rec_cnt = c.take<int>(nblk);
  w.rec_off = c.take<int>(nblk);
  w.rec_t = c.take<double>(nblk * kRecMax);
  w.rec_end = c.take<double>(nblk * kRecMax);
  w.start = c.take<double>(nq + 1);
  w.p_part = c.take<double>(npa);
  w.total = c.take<double>(1);
  w.spec = c.take<Spec>(kSpecMax);
  w.nspec = c.take<int32_t>(1);
  w.status = c.take<int32_t>(1);
  w.fail = c.take<int32_t>(1);
  w.stats = c.take<int32_t>(4);
  w.lo = c.take<long long>(1);
  if (bytes) *bytes = c.off;
  return w;
}

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

size_t flc_adaptive_workspace_size(int64_t n) {
  if (n <= 0) return 0;
  size_t b = 0;
  carve(nullptr, n, &b);
  return b;
}

}  // extern "C"

namespace {
template <class T>
int adaptive_prepare(const T* x, int64_t n, int32_t* status, void* ws, size_t ws_bytes, void* stream, double atol,
                     const char* who) {
  if (!x || n <= 0 || n >= (int64_t(1) << 31) || !ws) return fail(FLC_EINVAL, "%s: bad arguments", who);
  if (ws_bytes < flc_adaptive_workspace_size(n)) return fail(FLC_EWORKSPACE, "%s: workspace too small", who);
  if (!aligned16(x)) return fail(FLC_EINVAL, "%s: x must be 16-byte aligned", who);
  hipStream_t st = as_stream(stream);
  ArWs w = carve(ws, n, nullptr);
  const int64_t nfull = n / kBuf, nbuf = cdiv(n, kBuf), nq = cdiv(n, kChunk), npa = cdiv(nq, 256);
  TailProg prog{};
  if (nbuf > nfull) {
    (void)tail_prog_build(prog, 0, (int)(n - nfull * kBuf));
    tail_prog_levels(prog);
  }
  FLC_LAUNCH("adaptive_buffer_sum", ar_buffer_sum_kernel<T>, dim3((unsigned)nbuf), dim3(256), 0, st, x, n, nfull, prog, w);
  FLC_LAUNCH("adaptive_total", ar_total_kernel<T>, dim3(1), dim3(1024), 0, st, nbuf, w);
  FLC_LAUNCH("adaptive_phase_a", ar_phase_a_kernel<T>, dim3((unsigned)npa), dim3(256), 0, st, x, n, nq, w);
  FLC_LAUNCH("adaptive_special", ar_special_kernel<T>, dim3(64), dim3(256), 0, st, x, n, w, npa, atol, status);
  return FLC_OK;
}

template <class T>
int adaptive_select(const T* x, int64_t n, double u, int64_t* index, T* out, void* ws, size_t ws_bytes, void* stream,
                    const char* who) {
  if (!x || n <= 0 || n >= (int64_t(1) << 31) || !ws || !index || !out || !(u >= 0.0 && u < 1.0))
    return fail(FLC_EINVAL, "%s: bad arguments", who);
  if (ws_bytes < flc_adaptive_workspace_size(n)) return fail(FLC_EWORKSPACE, "%s: workspace too small", who);
  hipStream_t st = as_stream(stream);
  ArWs w = carve(ws, n, nullptr);
  const int64_t nq = cdiv(n, kChunk);
  const int nblk = (int)cdiv(nq, kPieceBlk);
  // FLC_ADAPTIVE_SEQUENTIAL=1: skip the speculation's result and run the exact chunk-by-chunk chain (tests)
  const char* fs = getenv("FLC_ADAPTIVE_SEQUENTIAL");
  const int force_seq = (fs && atoi(fs) != 0) ? 1 : 0;
  FLC_LAUNCH("adaptive_piece", ar_piece_kernel, dim3((unsigned)nblk), dim3(kPieceBlk), 0, st, nq, w);
  // (block 0 walks; the other blocks write the output's zeros on the other CUs meanwhile)
#if FLC_CALIB_AR_NOZERO  // calibration builds only (tools/adaptive_probe.py): no zero blocks, results invalid
  const unsigned zb = 0;
#else
  const unsigned zb = (unsigned)std::min<int64_t>(255, std::max<int64_t>(1, cdiv(n * (int64_t)sizeof(T), 256 * 1024)));
#endif
  FLC_LAUNCH("adaptive_walk", ar_walk_kernel<T>, dim3(1 + zb), dim3(1024), 0, st, x, n, nq, nblk, force_seq, u, w,
             out);
  FLC_LAUNCH("adaptive_final", ar_final_kernel<T>, dim3(1), dim3(1024), 0, st, x, n, nq, u, w, index, out);
  return FLC_OK;
}
}  // namespace

extern "C" {

int flc_adaptive_prepare(const float* x, int64_t n, int32_t* status, void* ws, size_t ws_bytes, void* stream) {
  return adaptive_prepare(x, n, status, ws, ws_bytes, stream, kAtol, "flc_adaptive_prepare");
}

int flc_adaptive_select(const float* x, int64_t n, double u, int64_t* index, float* out, void* ws, size_t ws_bytes,
                        void* stream) {
  return adaptive_select(x, n, u, index, out, ws, ws_bytes, stream, "flc_adaptive_select");
}

int flc_adaptive_prepare_f64(const double* x, int64_t n, int32_t* status, void* ws, size_t ws_bytes, void* stream) {
  return adaptive_prepare(x, n, status, ws, ws_bytes, stream, kAtol64, "flc_adaptive_prepare_f64");
}

int flc_adaptive_select_f64(const double* x, int64_t n, double u, int64_t* index, double* out, void* ws,
                            size_t ws_bytes, void* stream) {
  return adaptive_select(x, n, u, index, out, ws, ws_bytes, stream, "flc_adaptive_select_f64");
}

int flc_adaptive_stats(const void* ws, size_t ws_bytes, int64_t n, int32_t* stats, void* stream) {
  if (!ws || !stats || n <= 0 || n >= (int64_t(1) << 31)) return fail(FLC_EINVAL, "flc_adaptive_stats: bad arguments");
  if (ws_bytes < flc_adaptive_workspace_size(n)) return fail(FLC_EWORKSPACE, "flc_adaptive_stats: workspace too small");
  ArWs w = carve(const_cast<void*>(ws), n, nullptr);
  FLC_CHECK_HIP(hipMemcpyAsync(stats, w.stats, 4 * sizeof(int32_t), hipMemcpyDeviceToDevice, as_stream(stream)));
  return FLC_OK;
}

}  // extern "C"
