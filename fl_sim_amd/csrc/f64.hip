// f64.hip — the codec on float64 inputs, for gfx950
// (reference: fl_sim/compressors/compressors.py:267-410, which runs every compressor on whatever dtype x has:
// ``np.zeros_like(x)``, ``x / P``, ``D / K * x[i]``, ``math.log2(abs(x[i]))``, ``np.linalg.norm(x, p)`` and the
// level arithmetic all stay in float64 when x is float64).
//
// The float64 forms are separate kernels, not templates of the float32 ones: the float32 codec reproduces the
// reference's mixed fp32 / fp64 arithmetic (fp32 divisions and products, fp64 level brackets), while on a float64
// vector every step is one fp64 operation, so these kernels are shorter and share none of those rules.
//
//   copy / scale_div / randk_apply   IDENTICAL (+x), LAZY (x / P), RANDK (out[i] = D / K * x[i]) in fp64
//   natural                          alpha = log2|x|, down = floor, up = ceil, pt = (2^up - |x|) / 2^down,
//                                    sign * 2^down iff u < pt else sign * 2^up (compressors.py:306-318)
//   quant_norm                       max |x| (p = inf, exact) or sqrt of an fp64 sum of squares (p = 2, fixed order)
//   quant                            y = |x| / norm, the first bracket lv(s) <= y <= lv(s+1), p = (y - lv(s+1)) /
//                                    (lv(s) - lv(s+1)), lower level iff u < p, value lv * sign * norm
//                                    (compressors.py:339-357, 376-393); 8-bit codes sign << 7 | level
//   topk_dense                       out = x on the K largest (ties: the highest indices, as the float32 encoder),
//                                    0 elsewhere (compressors.py:293-296): a band around the K-th largest key from
//                                    a sample, one filter pass into per-chunk candidate segments, the exact key
//                                    from the band's bin, a tiled dense write (below); an exact radix select over
//                                    x whenever the band misses
// Uniforms: compat mode takes u[r] for the r-th consumer in index order (the reference's random.random() calls);
// philox mode the word of the element's own index (the float32 codec's stream).  Every kernel streams its input
// with 16-B loads (two doubles per load); all are HBM-bound element-wise or counting passes (no MFMA).
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kT = 256;                 // threads per block
constexpr int kNW = kT / kWave;
constexpr int kE = 4;                   // consecutive elements per thread per iteration (two 16-B loads)
constexpr int kIt = 8;                  // iterations per chunk
constexpr int kChunk = kT * kE * kIt;   // 8192 elements per chunk (one block)

__device__ __forceinline__ void load4(const double* __restrict__ x, int64_t e0, int64_t n, double v[kE]) {
  if (e0 + kE <= n) {
    const double2 a = *reinterpret_cast<const double2*>(x + e0);
    const double2 b = *reinterpret_cast<const double2*>(x + e0 + 2);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  } else {
#pragma unroll
    for (int j = 0; j < kE; ++j) v[j] = e0 + j < n ? x[e0 + j] : 0.0;
  }
}

__device__ __forceinline__ void store4(double* __restrict__ out, int64_t e0, int64_t n, const double v[kE]) {
  if (e0 + kE <= n) {
    *reinterpret_cast<double2*>(out + e0) = make_double2(v[0], v[1]);
    *reinterpret_cast<double2*>(out + e0 + 2) = make_double2(v[2], v[3]);
  } else {
    for (int j = 0; j < kE && e0 + j < n; ++j) out[e0 + j] = v[j];
  }
}

// philox-mode uniform of element e (the float32 codec's stream: word e & 3 of group e >> 2)
__device__ __forceinline__ double philox_u(int64_t e, uint64_t seed, uint64_t counter) {
  return u01(pick(philox_group((uint64_t)e >> 2, seed, counter), (int)(e & 3)));
}

// ------------------------------------------------------------------------------------------------
// element-wise forms
// ------------------------------------------------------------------------------------------------
template <bool DIV>
__global__ __launch_bounds__(kT) void ew_kernel(const double* __restrict__ x, int64_t n, double p,
                                                double* __restrict__ out) {
  const int64_t n2 = n >> 1;
  const double2* x2 = reinterpret_cast<const double2*>(x);
  double2* o2 = reinterpret_cast<double2*>(out);
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n2; i += (int64_t)gridDim.x * kT) {
    double2 v = x2[i];
    if (DIV) v = make_double2(v.x / p, v.y / p);
    o2[i] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) out[n - 1] = DIV ? x[n - 1] / p : x[n - 1];
}

__global__ __launch_bounds__(kT) void randk_scatter64_kernel(const double* __restrict__ x, const int* __restrict__ idx,
                                                             long long k, double scale, double* __restrict__ out) {
  for (long long j = (long long)blockIdx.x * kT + threadIdx.x; j < k; j += (long long)gridDim.x * kT) {
    const int i = idx[j];
    out[i] = scale * x[i];  // compressors.py:290: D / K * x[i] (a Python float times an fp64 element)
  }
}

// ------------------------------------------------------------------------------------------------
// consumers (compat mode): per-chunk counts, one-block scan, and the in-chunk order inside the encoders
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool norm_ok64(double nrm) { return nrm > 0.0 && nrm <= 1.7976931348623157e308; }

// the reference draws random.random() for x[i] (natural: every nonzero element; dithering: every nonzero element
// whose y = |x| / norm is not NaN, i.e. every nonzero one unless the norm is 0, inf or NaN)
template <int MODE>  // 0: natural, 1: dithering
__device__ __forceinline__ bool consumes64(double v, double nrm) {
  if (v == 0.0) return false;
  if (MODE == 0 || norm_ok64(nrm)) return true;
  return !isnan(fabs(v) / nrm);
}

template <int MODE>
__global__ __launch_bounds__(kT) void count64_kernel(const double* __restrict__ x, int64_t n,
                                                     const double* __restrict__ norm, int* __restrict__ counts) {
  __shared__ int s_red[kNW];
  const double nrm = MODE == 1 ? *norm : 0.0;
  int cnt = 0;
  for (int it = 0; it < kIt; ++it) {
    const int64_t e0 = (int64_t)blockIdx.x * kChunk + ((int64_t)it * kT + threadIdx.x) * kE;
    if (e0 >= n) break;
    double v[kE];
    load4(x, e0, n, v);
#pragma unroll
    for (int j = 0; j < kE; ++j) cnt += (e0 + j < n && consumes64<MODE>(v[j], nrm)) ? 1 : 0;
  }
  const int tot = block_sum<int, kNW>(cnt, s_red);
  if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

// offsets[c] = consumers before chunk c; offsets[nchunks] = total
__global__ __launch_bounds__(1024) void scan64_kernel(const int* __restrict__ counts, long long* __restrict__ offsets,
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
  if (threadIdx.x == 0) offsets[nchunks] = running;
}

// the uniforms of one iteration's kE elements (block-wide: contains barriers in compat mode)
template <int MODE, bool COMPAT>
__device__ __forceinline__ void uniforms64(const double v[kE], int64_t e0, int64_t n, double nrm, uint64_t seed,
                                           uint64_t counter, const double* __restrict__ compat_u, long long& running,
                                           long long* s_scan, double u[kE]) {
  if (COMPAT) {
    int c[kE], cnt = 0;
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      c[j] = (e0 + j < n && consumes64<MODE>(v[j], nrm)) ? 1 : 0;
      cnt += c[j];
    }
    long long tot;
    long long r = running + block_excl_scan<long long, kNW>((long long)cnt, s_scan, &tot);
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      u[j] = c[j] ? compat_u[r] : 0.0;
      r += c[j];
    }
    running += tot;
  } else {
#pragma unroll
    for (int j = 0; j < kE; ++j) u[j] = philox_u(e0 + j, seed, counter);
  }
}

// ------------------------------------------------------------------------------------------------
// natural compression (compressors.py:302-318) on fp64: code = sign << 15 | (e + 1075), e in [-1074, 1024]
// (0 = zero, 0x7fff = NaN; inf keeps its sign, e = 1025; the reference raises on both)
// ------------------------------------------------------------------------------------------------
constexpr int kNatBias = 1075;

__device__ __forceinline__ uint32_t natural64_code(double xv, double u) {
  if (xv == 0.0) return 0u;
  if (isnan(xv)) return 0x7fffu;
  const uint32_t sign = signbit(xv) ? 1u : 0u;
  const double a = fabs(xv);
  if (isinf(a)) return (sign << 15) | (uint32_t)(1025 + kNatBias);
  // math.log2 / floor / ceil of the reference, in fp64 (a power of two gives down == up and pt = 0).  Away from a
  // power of two floor / ceil of the rounded log2 are the exponent f and f + 1: a = m * 2^f, m in [1, 2), and
  // log2 a = f + log2 m lies at least ~1.44 (m - 1) above f and 0.72 (2 - m) below f + 1, far more than the half ulp of
  // a number near f (<= (|f| + 1) * 2^-53).  Only mantissas within W = (|f| + 2) * 2^-48 of 1 or 2 (a generous
  // margin) take the log2, whose rounding onto an integer decides them as it does in the reference.
  int f;
  const double m = 2.0 * frexp(a, &f);  // a = m * 2^(f - 1), m in [1, 2)
  f -= 1;
  const double W = (double)(abs(f) + 2) * 3.552713678800501e-15;  // 2^-48
  int down, up;
  if (m - 1.0 > W && 2.0 - m > W) {
    down = f;
    up = f + 1;
  } else {
    const double alpha = log2(a);
    down = (int)floor(alpha);
    up = (int)ceil(alpha);
  }
  const double pt = (ldexp(1.0, up) - a) / ldexp(1.0, down);
  const int e = (u < pt) ? down : up;
  return (sign << 15) | (uint32_t)(e + kNatBias);
}

__device__ __forceinline__ double natural64_value(uint32_t code) {
  if (code == 0u) return 0.0;
  if (code == 0x7fffu) return __longlong_as_double(0x7ff8000000000000ll);
  const int e = (int)(code & 0x7fffu) - kNatBias;
  const double v = e > 1024 ? __longlong_as_double(0x7ff0000000000000ll) : ldexp(1.0, e);
  return (code >> 15) ? -v : v;
}

template <bool COMPAT>
__global__ __launch_bounds__(kT) void natural64_kernel(const double* __restrict__ x, int64_t n, uint64_t seed,
                                                       uint64_t counter, const double* __restrict__ compat_u,
                                                       const long long* __restrict__ offsets,
                                                       uint16_t* __restrict__ codes, double* __restrict__ out) {
  __shared__ long long s_scan[kNW];
  long long running = COMPAT ? offsets[blockIdx.x] : 0;
  for (int it = 0; it < kIt; ++it) {
    const int64_t e0 = (int64_t)blockIdx.x * kChunk + ((int64_t)it * kT + threadIdx.x) * kE;
    if (!COMPAT && e0 >= n) break;  // (compat: every thread takes part in the block scans)
    double v[kE], u[kE];
    if (e0 < n) load4(x, e0, n, v);
    else
#pragma unroll
      for (int j = 0; j < kE; ++j) v[j] = 0.0;
    uniforms64<0, COMPAT>(v, e0, n, 0.0, seed, counter, compat_u, running, s_scan, u);
    if (e0 >= n) continue;
    double o[kE];
    uint32_t cd[kE];
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      cd[j] = natural64_code(v[j], u[j]);
      o[j] = natural64_value(cd[j]);
    }
    if (codes) {
      if (e0 + kE <= n) {
        *reinterpret_cast<uint2*>(codes + e0) = make_uint2(cd[0] | (cd[1] << 16), cd[2] | (cd[3] << 16));
      } else {
        for (int j = 0; j < kE && e0 + j < n; ++j) codes[e0 + j] = (uint16_t)cd[j];
      }
    }
    if (out) store4(out, e0, n, o);
  }
}

__global__ __launch_bounds__(kT) void natural64_decode_kernel(const uint16_t* __restrict__ codes, int64_t n,
                                                              double* __restrict__ out) {
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kT)
    out[e] = natural64_value(codes[e]);
}

// ------------------------------------------------------------------------------------------------
// dithering norm (compressors.py:332, 372 np.linalg.norm(x, p)): p = inf -> max |x| (NaN propagates: the
// largest |x| bit pattern), p = 2 -> sqrt of an fp64 sum of squares, partials per chunk folded in a fixed order
// ------------------------------------------------------------------------------------------------
template <int NORM>
__global__ __launch_bounds__(kT) void norm64_partial_kernel(const double* __restrict__ x, int64_t n,
                                                            unsigned long long* __restrict__ part) {
  __shared__ unsigned long long s_red[kNW];
  unsigned long long mx = 0;
  double ss = 0.0;
  for (int it = 0; it < kIt; ++it) {
    const int64_t e0 = (int64_t)blockIdx.x * kChunk + ((int64_t)it * kT + threadIdx.x) * kE;
    if (e0 >= n) break;
    double v[kE];
    load4(x, e0, n, v);
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      if (NORM == FLC_NORM_INF) {
        const unsigned long long b = (unsigned long long)__double_as_longlong(v[j]) & 0x7fffffffffffffffull;
        mx = b > mx ? b : mx;
      } else {
        ss = fma(v[j], v[j], ss);
      }
    }
  }
  unsigned long long r;
  if (NORM == FLC_NORM_INF) {
    unsigned long long w = mx;
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long t = __shfl_xor(w, o);
      w = t > w ? t : w;
    }
    if ((threadIdx.x & (kWave - 1)) == 0) s_red[threadIdx.x >> 6] = w;
    __syncthreads();
    r = 0;
    for (int i = 0; i < kNW; ++i) r = s_red[i] > r ? s_red[i] : r;
  } else {
    const double w = wave_sum(ss);
    if ((threadIdx.x & (kWave - 1)) == 0) s_red[threadIdx.x >> 6] = (unsigned long long)__double_as_longlong(w);
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < kNW; ++i) t += __longlong_as_double((long long)s_red[i]);
    r = (unsigned long long)__double_as_longlong(t);
  }
  if (threadIdx.x == 0) part[blockIdx.x] = r;
}

template <int NORM>
__global__ __launch_bounds__(kWave) void norm64_fold_kernel(const unsigned long long* __restrict__ part, int64_t nparts,
                                                            double* __restrict__ norm) {
  const int lane = threadIdx.x;
  if (NORM == FLC_NORM_INF) {
    unsigned long long m = 0;
    for (int64_t p = lane; p < nparts; p += kWave) m = part[p] > m ? part[p] : m;
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long t = __shfl_xor(m, o);
      m = t > m ? t : m;
    }
    if (lane == 0) *norm = __longlong_as_double((long long)m);
  } else {
    double acc = 0.0;
    for (int64_t p = lane; p < nparts; p += kWave) acc += __longlong_as_double((long long)part[p]);
    const double t = wave_sum(acc);
    if (lane == 0) *norm = sqrt(t);
  }
}

// ------------------------------------------------------------------------------------------------
// dithering (compressors.py:339-357 standard, 376-393 natural) on fp64
// ------------------------------------------------------------------------------------------------
// first index j in [0, s] with lv(j) >= y (y in [0, 1])
template <int KIND>
__device__ __forceinline__ int level_lb64(double y, int s, double step) {
  if (KIND == 0) {
    int j = (int)ceil(y * (double)s);
    j = j < 0 ? 0 : (j > s ? s : j);
    while (j > 0 && level_value<0>(j - 1, s, step) >= y) --j;
    while (j < s && level_value<0>(j, s, step) < y) ++j;
    return j;
  }
  if (y == 0.0) return 0;
  int E;
  const double m = frexp(y, &E);             // y = m * 2^E, m in [0.5, 1)
  const int j = s + ((m == 0.5) ? E - 1 : E);  // s + ceil(log2 y)
  return j < 1 ? 1 : (j > s ? s : j);
}

// code of x (sign << 7 | level); 0 for x == 0; a non-regular norm: 1 (decodes to NaN, as the float32 codec)
template <int KIND>
__device__ __forceinline__ uint32_t quant64_code(double xv, double nrm, int s, double step, double u) {
  if (xv == 0.0) return 0u;
  if (!norm_ok64(nrm)) return 1u;
  const double y = fabs(xv) / nrm;  // compressors.py:344 (fp64 / fp64)
  const int j = level_lb64<KIND>(y, s, step);
  const int sl = j > 0 ? j - 1 : 0;
  const double lo = level_value<KIND>(sl, s, step), hi = level_value<KIND>(sl + 1, s, step);
  const double p = (y - hi) / (lo - hi);  // compressors.py:348
  const int lvl = (u < p) ? sl : sl + 1;  // compressors.py:349-353
  return ((signbit(xv) ? 1u : 0u) << 7) | (uint32_t)lvl;
}

// lv * sign * norm (compressors.py:357: out[i] = levelsValues[s] * sign * pnorm, all fp64)
template <int KIND>
__device__ __forceinline__ double quant64_value(uint32_t code, double nrm, int s, double step) {
  if (!norm_ok64(nrm)) return code == 0u ? 0.0 : __longlong_as_double(0x7ff8000000000000ll);
  const double lv = level_value<KIND>((int)(code & 127u), s, step);
  return ((code >> 7) ? -lv : lv) * nrm;
}

template <int KIND, bool COMPAT>
__global__ __launch_bounds__(kT) void quant64_kernel(const double* __restrict__ x, int64_t n, int s, double step,
                                                     const double* __restrict__ norm, uint64_t seed, uint64_t counter,
                                                     const double* __restrict__ compat_u,
                                                     const long long* __restrict__ offsets,
                                                     uint8_t* __restrict__ codes, double* __restrict__ out,
                                                     unsigned long long* __restrict__ nnz) {
  __shared__ long long s_scan[kNW];
  __shared__ unsigned long long s_nnz;
  const double nrm = *norm;
  long long running = COMPAT ? offsets[blockIdx.x] : 0;
  if (threadIdx.x == 0) s_nnz = 0;
  __syncthreads();
  unsigned my_nnz = 0;
  for (int it = 0; it < kIt; ++it) {
    const int64_t e0 = (int64_t)blockIdx.x * kChunk + ((int64_t)it * kT + threadIdx.x) * kE;
    if (!COMPAT && e0 >= n) break;
    double v[kE], u[kE];
    if (e0 < n) load4(x, e0, n, v);
    else
#pragma unroll
      for (int j = 0; j < kE; ++j) v[j] = 0.0;
    uniforms64<1, COMPAT>(v, e0, n, nrm, seed, counter, compat_u, running, s_scan, u);
    if (e0 >= n) continue;
    uint32_t cd[kE];
    double o[kE];
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      cd[j] = quant64_code<KIND>(v[j], nrm, s, step, u[j]);
      o[j] = quant64_value<KIND>(cd[j], nrm, s, step);
      my_nnz += (e0 + j < n && v[j] != 0.0) ? 1u : 0u;
    }
    if (codes) {
      if (e0 + kE <= n) *reinterpret_cast<uint32_t*>(codes + e0) = cd[0] | (cd[1] << 8) | (cd[2] << 16) | (cd[3] << 24);
      else
        for (int j = 0; j < kE && e0 + j < n; ++j) codes[e0 + j] = (uint8_t)cd[j];
    }
    if (out) store4(out, e0, n, o);
  }
  if (nnz) {
    const unsigned w = wave_sum(my_nnz);
    if ((threadIdx.x & (kWave - 1)) == 0 && w) atomicAdd(&s_nnz, (unsigned long long)w);
    __syncthreads();
    if (threadIdx.x == 0 && s_nnz) atomicAdd(nnz, s_nnz);
  }
}

template <int KIND>
__global__ __launch_bounds__(kT) void quant64_decode_kernel(const uint8_t* __restrict__ codes, int64_t n, int s,
                                                            double step, const double* __restrict__ norm,
                                                            double* __restrict__ out) {
  const double nrm = *norm;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kT)
    out[e] = quant64_value<KIND>(codes[e], nrm, s, step);
}

// ------------------------------------------------------------------------------------------------
// top-k on fp64 (compressors.py:293-296: out = x.copy(); out[np.argsort(out)[:-K]] = 0): out = x on the K largest,
// +0 elsewhere; among the ties of the K-th largest, the highest indices are kept (the float32 encoder's rule).
//
// Three launches; on the common path x is read once and out written once (the HBM floor: 16 B per element):
//   prep      kSampleBlocks blocks: S strided sample keys (order-preserving 64-bit keys); block 0 resets the state
//   select    one block of 1024 threads per CU, grid-synchronised (block b takes chunks b, b + G, ...):
//             every block finds, identically, a band [t_lo, t_hi) from the sample's r_lo-th and r_hi-th largest keys
//             (the K-th largest lies inside it with ~4 sigma (+16) of the sample to spare on each side); then the
//             filter pass over its 8192-element chunks (8 elements per thread, the next chunk's loads in flight):
//             every key >= t_lo appended to the chunk's segment (the value's bits and its u16 position), keys
//             >= t_hi counted, band keys binned into a 2048-bin LDS histogram; the block's nonzero bins go to the
//             global histogram (memory-side atomics, one block per CU), then ONE grid barrier; every block finds
//             the bin holding the K-th largest and appends its keys in that bin to one list; block 0 waits for all
//             appends and selects the exact K-th key T among them (~100 keys: each key's rank by comparison), its
//             ties and, when only some are kept, the index threshold of the highest-index ones.  When the band
//             fails (the sample missed on either side, a segment overflowed, the bin held more keys than the
//             list) or is off (n < 64 Ki, k near n), the same blocks run the exact radix select over x instead:
//             8 digit passes of the key, up to 8 of the tie index, a grid barrier each
//   emit      one 64-lane wave per 256-element piece: a 2 KB LDS tile zeroed, the piece's kept candidates
//             scattered into it, the tile written out whole with non-temporal 16-B stores (after the fallback, or
//             with long segments: x read again, kept in place)
// ------------------------------------------------------------------------------------------------
// order-preserving key of a double: NaN largest, -0 == +0
__device__ __forceinline__ unsigned long long order_key64(double v) {
  unsigned long long b = (unsigned long long)__double_as_longlong(v);
  if ((b & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) return ~0ull;
  if (b == 0x8000000000000000ull) b = 0ull;
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
constexpr int kDigits = 8;          // 8-bit digits of a 64-bit key, most significant first
constexpr int kSample64 = 16384;    // sample keys
constexpr int kSampleDigits = 3;    // the band's ends keep the sample keys' top 24 bits
constexpr int kBand = 2048;         // band histogram bins
constexpr int kBandCopies = 8;      // copies of the band histogram: block b adds into copy b % 8 (fewer atomics per word)
constexpr int kBinCap = 16384;      // keys of the K-th largest's bin the gather's list holds
constexpr int kGT = 1024;           // threads of the sample, gather and fallback blocks
constexpr int kGNW = kGT / kWave;
constexpr int kMaxG64 = 1024;       // blocks of the grid-synchronised select (one flag each)
constexpr int kSampleBlocks = 64;   // blocks loading the sample
// the prep kernel writes the compact sample exactly when its grid covers the whole sample (gridDim.x * kT == kSample64)
// and the select reads it whenever S == kSample64: the two conditions agree only while this holds
static_assert(kSampleBlocks * kT == kSample64, "the compact sample's writer and reader disagree");
constexpr int kMaxCPB = 2048;       // chunks per select block (more: the band is off, the passes over x run)
constexpr unsigned long long kOvf = 1ull << 44;  // (n < 2^44)
static_assert(kBand == 2 * kGT, "gather: two band bins per thread");
static_assert(kSample64 % kGT == 0 && kBinCap % kGT == 0, "whole keys per thread");

struct Sel64 {
  unsigned long long stamps[32];      // diagnostic builds (FLC_SELECT_STAMPS): phase times, s_memrealtime
#ifdef FLC_SELECT_STAMPS
  unsigned long long bstamps[2][kMaxG64];  // per block: filter pass done, histogram flushed
#endif
  int fb;                             // 1 when T came from the passes over x (the emit reads x again)
  int err;                            // a grid barrier timed out (lost co-residency)
  unsigned nbin;                      // the bin's list: keys appended
  unsigned long long T;               // the K-th largest key
  long long need, ties;               // ties of T kept / present
  long long ithr;                     // the kept ties: index >= ithr
  unsigned long long flags[kMaxG64];  // grid barriers (zeroed by the prep kernel: targets 1, 2, ... in each call)
  unsigned long long pab[kMaxG64];    // per block: keys >= t_hi in its chunks + kOvf if a segment overflowed
  unsigned hist[kBandCopies][kBand];  // the band histogram, in copies (their sum is the histogram)
  unsigned fhist[2 * kDigits][256];   // the fallback's digit histograms: key digits, then tie-index digits
  unsigned long long bkey[kBinCap];   // the K-th largest's bin: keys (less the bin's base) and their indices
  long long bidx[kBinCap];
  unsigned sample[kSample64];         // the sample's keys, top 32 bits (the band needs no more; half the bytes)
  unsigned top[kSample64 / 64 * 8];   // the compact sample: each 64-key wave's 8 largest (top 32 bits), descending
};

#ifdef FLC_SELECT_STAMPS  // (tools/stamps64.py)
static_assert(offsetof(Sel64, bstamps) == 256, "tools/stamps64.py reads the per-block stamps at this offset");
#define STAMP64(cond, i)                                                                      \
  do {                                                                                        \
    if ((cond) && threadIdx.x == 0) const_cast<Sel64*>(st)->stamps[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define STAMP64(cond, i) \
  do {                   \
  } while (0)
#endif

// LDS histogram add of one key per lane.  Lanes adding to one address serialise (a wave of keys sharing their sign
// and exponent — the high digits of most data — is a 64-way conflict), so the wave's first two bins are added once
// each with their lane counts, and only the lanes left over add one by one
__device__ __forceinline__ void hist_add64(unsigned* h, unsigned bin, bool in) {
  unsigned long long m = __ballot(in);
  const int lane = (int)(threadIdx.x & (kWave - 1));
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (m == 0ull) return;
    const int first = __builtin_ctzll(m);
    const unsigned b0 = (unsigned)__builtin_amdgcn_readlane((int)bin, first);
    const unsigned long long same = __ballot(in && bin == b0) & m;
    if (lane == first) atomicAdd(&h[b0], (unsigned)__popcll(same));
    m &= ~same;
  }
  if ((m >> lane) & 1ull) atomicAdd(&h[bin], 1u);
}

// block-wide (NW waves): the bin of a 256-bin histogram (count of bin 255 - t in thread t < 256, 0 elsewhere)
// holding rank `rem` from the top.  Returns, in every thread, (digit, count above it, its count) in s_res.
template <int NW>
__device__ __forceinline__ void pick256(long long c, long long rem, long long* s_scan, long long* s_res) {
  long long tot;
  const long long ex = block_excl_scan<long long, NW>(c, s_scan, &tot);  // keys in the bins above this thread's
  if (threadIdx.x < 256 && c > 0 && ex < rem && ex + c >= rem) {
    s_res[0] = 255 - (long long)threadIdx.x;
    s_res[1] = ex;
    s_res[2] = c;
  }
  __syncthreads();
}

// a wave's slots for its lanes with `in` set, from an LDS (or global) counter: the lane's slot, or any value when !in
__device__ __forceinline__ unsigned wave_append(unsigned* counter, bool in, unsigned long long m) {
  unsigned base = 0u;
  if ((threadIdx.x & (kWave - 1)) == 0) base = atomicAdd(counter, (unsigned)__popcll(m));
  base = (unsigned)__builtin_amdgcn_readlane((int)base, 0);
  return base + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// the bin of a kBand-bin histogram holding rank r from the top (bin j's count in h(j)): every thread gets (bin, rank
// in it, its count) in s_out; bin -1 when the histogram holds fewer than r keys.  Thread t holds bins kBand - 1 - 2t
// and kBand - 2 - 2t (1024 threads).
template <class H>
__device__ __forceinline__ void pick_band(H h, long long r, long long* s_scan, long long* s_out) {
  const int tid = threadIdx.x;
  const long long ha = h(kBand - 1 - 2 * tid), hb = h(kBand - 2 - 2 * tid);
  if (tid == 0) s_out[0] = -1;
  long long tot;
  // (LDS-only barriers: global loads the caller has in flight stay in flight)
  const long long ex = block_excl_scan_lds<long long, kGNW>(ha + hb, s_scan, &tot);  // (barriers: s_out[0] set)
  if (r >= 1 && ex < r && ex + ha + hb >= r) {
    const bool first = ex + ha >= r;
    s_out[0] = first ? kBand - 1 - 2 * tid : kBand - 2 - 2 * tid;
    s_out[1] = first ? r - ex : r - ex - ha;
    s_out[2] = first ? ha : hb;
  }
  lds_barrier();
}

// pick_band for two ranks of one histogram (r < 1: none), one scan: results in s_out[0] and s_out[1]
template <class H>
__device__ __forceinline__ void pick_band2(H h, long long r0, long long r1, long long* s_scan, long long (*s_out)[3]) {
  const int tid = threadIdx.x;
  const long long ha = h(kBand - 1 - 2 * tid), hb = h(kBand - 2 - 2 * tid);
  if (tid == 0) s_out[0][0] = s_out[1][0] = -1;
  long long tot;
  const long long ex = block_excl_scan_lds<long long, kGNW>(ha + hb, s_scan, &tot);  // (barriers: s_out[.][0] set)
  auto put = [&](long long r, long long* o) {
    if (r >= 1 && ex < r && ex + ha + hb >= r) {
      const bool first = ex + ha >= r;
      o[0] = first ? kBand - 1 - 2 * tid : kBand - 2 - 2 * tid;
      o[1] = first ? r - ex : r - ex - ha;
      o[2] = first ? ha : hb;
    }
  };
  put(r0, s_out[0]);
  put(r1, s_out[1]);
  lds_barrier();
}

// the shift that maps key offsets 0 .. maxoff onto at most 2^bits bins
__device__ __forceinline__ int range_shift64(unsigned long long maxoff, int bits) {
  if (maxoff == 0ull) return 0;
  const int len = 64 - __clzll((long long)maxoff);
  return len > bits ? len - bits : 0;
}

// The sample's S keys, loaded by kSampleBlocks blocks (scattered loads from one CU wait on its address translation a
// page at a time); block 0 also resets the state the select kernel accumulates into
__global__ __launch_bounds__(kT) void sel64_prep_kernel(const double* __restrict__ x, int64_t n, int S,
                                                        Sel64* __restrict__ st) {
  const int tid = threadIdx.x;
  STAMP64(blockIdx.x == 0, 0);
  for (int i = (int)blockIdx.x * kT + tid; i < kBandCopies * kBand; i += (int)gridDim.x * kT) (&st->hist[0][0])[i] = 0u;
  if (blockIdx.x == 0) {
    for (int i = tid; i < 2 * kDigits * 256; i += kT) (&st->fhist[0][0])[i] = 0u;
    for (int i = tid; i < kMaxG64; i += kT) st->flags[i] = 0ull;
    if (tid == 0) {
      st->fb = 0;
      st->err = 0;
      st->nbin = 0u;
      st->T = 0ull;
      st->need = st->ties = st->ithr = 0;
    }
  }
  for (int j = blockIdx.x * kT + tid; j < S; j += gridDim.x * kT) {
    const int64_t pos = (int64_t)(((double)j + 0.5) * (double)n / (double)S);
    unsigned key = (unsigned)(order_key64(x[pos < n ? pos : n - 1]) >> 32);
    st->sample[j] = key;
    if (S == kSample64 && gridDim.x * kT == kSample64) {  // (one key per thread: every lane of the wave holds one)
      // the compact sample: the wave's 8 largest keys, descending (topk.hip's compact sample for float32)
      const int lane = tid & (kWave - 1);
      unsigned mine = 0u;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const unsigned m = wave_max_u32(key);
        if (lane == r) mine = m;
        const unsigned long long at = __ballot(key == m);
        if (lane == __ffsll((long long)at) - 1) key = 0u;
      }
      if (lane < 8) st->top[(j >> 6) * 8 + lane] = mine;
    }
  }
}

// the select kernel's LDS
struct SelLds {
  unsigned hb[2][kBand];  // the band's histograms (sample), then the band histogram of the block's chunks (hb[0])
  unsigned h[2][256];
  unsigned long long d[kGT];  // the K-th largest's bin list (block 0)
  long long i[kGT];
  unsigned long long mm[2][kGNW];
  long long scan[kGNW], res[3], out[2][3], sel[4];
  unsigned cn[kMaxCPB];  // the candidates of the block's chunks
  int ovf;
  int bad;  // the compact sample's band is not exact (a wave of the sample holds more keys above the floor)
};

// The band [t_lo, t_hi) from the sample's r_lo-th and r_hi-th largest keys (r_hi <= 0: no ceiling); every block of
// the select kernel computes the same one from the same keys.
//   r_lo <= 1024 (k up to ~6 % of n): B = the smallest thread maximum of the 16 keys each thread holds, so at least
//   1024 sample keys lie at or above it; one 2048-bin histogram of the keys in [B, max] locates both ranks (few
//   keys, spread over many bins: no LDS atomic contention), and a bin holding more than 8 keys is refined once inside
//   it.  The floor is the floor of rank r_lo's bin, the ceiling the end of rank r_hi's bin.
//   Otherwise: three 8-bit digit passes per rank (the keys' top 24 bits).
constexpr int kSPer = kSample64 / kGT;  // sample keys per thread
__device__ __forceinline__ void sample_keys(const Sel64* __restrict__ st, int S, unsigned long long (&key)[kSPer]) {
#pragma unroll
  for (int i = 0; i < kSPer; ++i) {
    const int j = i * kGT + (int)threadIdx.x;
    key[i] = j < S ? (unsigned long long)st->sample[j] << 32 : 0ull;  // (truncated: key' <= key)
  }
}
// (N = kSPer: the full sample; N = 2: the compact sample, 2048 keys, only for r_lo <= kGT)
template <int N>
__device__ __forceinline__ void sample_band(const Sel64* st, const unsigned long long (&key)[N], int S,
                                            long long r_lo, long long r_hi, SelLds& L, unsigned long long& t_lo,
                                            unsigned long long& t_hi) {
  constexpr int kPer = N;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid >> 6;
  const bool hi = r_hi > 0;
  if (r_lo <= kGT && S == kSample64) {
    unsigned long long m = 0ull;
#pragma unroll
    for (int i = 0; i < kPer; ++i) m = key[i] > m ? key[i] : m;
    unsigned long long mn = m, mx = m;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const unsigned long long a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
    }
    if (lane == 0) {
      L.mm[0][wid] = mn;
      L.mm[1][wid] = mx;
    }
    for (int i = tid; i < 2 * kBand; i += kGT) (&L.hb[0][0])[i] = 0u;
    lds_barrier();
    STAMP64(blockIdx.x == 0, 16);
    unsigned long long B = ~0ull, M = 0ull;
#pragma unroll
    for (int w = 0; w < kGNW; ++w) {
      B = L.mm[0][w] < B ? L.mm[0][w] : B;
      M = L.mm[1][w] > M ? L.mm[1][w] : M;
    }
    const int sh = range_shift64(M - B, 11);
#pragma unroll
    for (int i = 0; i < kPer; ++i)
      if (key[i] >= B) atomicAdd(&L.hb[0][(unsigned)((key[i] - B) >> sh)], 1u);
    lds_barrier();
    STAMP64(blockIdx.x == 0, 17);
    pick_band2([&](int j) { return (long long)L.hb[0][j]; }, r_lo, hi ? r_hi : 0ll, L.scan, L.out);
    unsigned long long lo0 = B + ((unsigned long long)L.out[0][0] << sh);
    unsigned long long lo1 = hi ? B + ((unsigned long long)L.out[1][0] << sh) : 0ull;
    int sh_hi = sh;
    STAMP64(blockIdx.x == 0, 18);
    const bool ref0 = sh > 0 && L.out[0][2] > 8, ref1 = hi && sh > 0 && L.out[1][2] > 8;  // (block-uniform)
    if (ref0 || ref1) {  // one finer pass inside the bins holding more than 8 keys
      const int sh2 = sh > 11 ? sh - 11 : 0;
      const unsigned long long bw = 1ull << sh;
      lds_barrier();
      for (int i = tid; i < 2 * kBand; i += kGT) (&L.hb[0][0])[i] = 0u;
      lds_barrier();
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        if (ref0 && key[i] >= lo0 && key[i] - lo0 < bw) atomicAdd(&L.hb[0][(unsigned)((key[i] - lo0) >> sh2)], 1u);
        if (ref1 && key[i] >= lo1 && key[i] - lo1 < bw) atomicAdd(&L.hb[1][(unsigned)((key[i] - lo1) >> sh2)], 1u);
      }
      lds_barrier();
      const long long q0 = L.out[0][1], q1 = L.out[1][1];
      lds_barrier();
      if (ref0) {
        pick_band([&](int j) { return (long long)L.hb[0][j]; }, q0, L.scan, L.out[0]);
        lo0 += (unsigned long long)L.out[0][0] << sh2;
      }
      if (ref1) {
        pick_band([&](int j) { return (long long)L.hb[1][j]; }, q1, L.scan, L.out[1]);
        lo1 += (unsigned long long)L.out[1][0] << sh2;
        sh_hi = sh2;
      }
    }
    t_lo = lo0;  // (from truncated keys: at least as many true keys lie at or above it)
    const unsigned long long e1 = lo1 + (1ull << sh_hi);
    // (rounded up to a multiple of 2^32, so that key >= t_hi exactly when the truncated key is: the ceiling's rank
    // holds for the true keys too)
    const unsigned long long e2 = (e1 + 0xffffffffull) & ~0xffffffffull;
    t_hi = !hi || e1 < lo1 || e2 < e1 ? ~0ull : e2;  // (saturated at the top of the key range)
  } else if constexpr (N == kSPer) {
    unsigned long long plo = 0ull, phi = 0ull;
    long long rlo = r_lo, rhi = r_hi;
    for (int pass = 0; pass < kSampleDigits; ++pass) {
      if (tid < 256) {
        L.h[0][tid] = 0u;
        L.h[1][tid] = 0u;
      }
      __syncthreads();
      const int sh = 56 - 8 * pass;
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const bool v = i * kGT + tid < S;
        const unsigned d = (unsigned)(key[i] >> sh) & 255u;
        hist_add64(L.h[0], d, v && (pass == 0 || (key[i] >> (sh + 8)) == plo));
        if (hi) hist_add64(L.h[1], d, v && (pass == 0 || (key[i] >> (sh + 8)) == phi));
      }
      __syncthreads();
      pick256<kGNW>(tid < 256 ? (long long)L.h[0][255 - tid] : 0ll, rlo, L.scan, L.res);
      plo = (plo << 8) | (unsigned long long)L.res[0];
      rlo -= L.res[1];
      __syncthreads();  // (res is rewritten next)
      if (hi) {
        pick256<kGNW>(tid < 256 ? (long long)L.h[1][255 - tid] : 0ll, rhi, L.scan, L.res);
        phi = (phi << 8) | (unsigned long long)L.res[0];
        rhi -= L.res[1];
        __syncthreads();
      }
    }
    constexpr int low = 64 - 8 * kSampleDigits;
    t_lo = plo << low;
    t_hi = (!hi || phi == (1ull << (8 * kSampleDigits)) - 1ull) ? ~0ull : (phi + 1ull) << low;
  }
  lds_barrier();  // (L is reused by the caller)
}

// block-wide radix select of the rem-th largest among the cnt values v[q] (slot q * kGT + tid, values < 2^bits;
// `eq` restricts the count to the lanes' flagged values): returns the value; rem becomes its rank among its equals,
// cnt their number
template <int PER>
__device__ __forceinline__ unsigned long long block_select(const unsigned long long (&v)[PER], const bool (&ok)[PER],
                                                           int bits, long long& rem, long long& cnt, unsigned* s_h,
                                                           long long* s_scan, long long* s_res) {
  const int tid = threadIdx.x;
  unsigned long long pre = 0ull;
  for (int hb = bits; hb > 0;) {
    const int w = hb >= 8 ? 8 : hb, lo = hb - w;
    if (tid < 256) s_h[tid] = 0u;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q)
      hist_add64(s_h, (unsigned)(v[q] >> lo) & ((1u << w) - 1u), ok[q] && (hb >= 64 || (v[q] >> hb) == pre));
    __syncthreads();
    pick256<kGNW>(tid < 256 ? (long long)s_h[255 - tid] : 0ll, rem, s_scan, s_res);
    pre = (pre << w) | (unsigned long long)s_res[0];
    rem -= s_res[1];
    cnt = s_res[2];
    __syncthreads();
    hb = lo;
  }
  return pre;
}

// The K-th largest among a short list of cnt <= blockDim.x keys (s_d: offsets in the bin, s_i: their indices, in
// LDS), rank rem0 from the top: each key's rank by comparing it with all others, P threads per key (P * cnt <= 1024,
// each comparing a P-th of the list; their counts summed across the P adjacent lanes).  Returns T's offset dt, its rank
// among its ties (rem), their number, and the index threshold of the kept ties.
__device__ __forceinline__ void rank_small(const unsigned long long* s_d, const long long* s_i, int cnt, long long rem0,
                                           long long* s_sel, unsigned long long& dt, long long& rem, long long& ties,
                                           long long& ithr) {
  const int tid = threadIdx.x;
  int P = 1;  // (uniform; a power of two <= 64, so a key's threads are adjacent lanes of one wave)
  while (P < kWave && 2 * P * cnt <= kGT) P *= 2;
  const int q = tid / P, part = tid & (P - 1);
  const unsigned long long my = q < cnt ? s_d[q] : 0ull;
  int gt = 0, eq = 0;
  if (q < cnt) {
    for (int j = part; j < cnt; j += P) {
      const unsigned long long o = s_d[j];
      gt += o > my ? 1 : 0;
      eq += o == my ? 1 : 0;
    }
  }
  for (int o = 1; o < P; o <<= 1) {
    gt += __shfl_xor(gt, o);
    eq += __shfl_xor(eq, o);
  }
  if (q < cnt && part == 0 && gt < rem0 && rem0 <= gt + eq) {  // (every copy of T writes the same values)
    s_sel[0] = (long long)my;
    s_sel[1] = rem0 - gt;
    s_sel[2] = eq;
  }
  __syncthreads();
  dt = (unsigned long long)s_sel[0];
  rem = s_sel[1];
  ties = s_sel[2];
  ithr = 0;
  if (rem < ties) {  // keep the rem ties with the highest indices: the one with rem - 1 tie indices above it
    const bool tie = q < cnt && my == dt;
    const long long ix = tie ? s_i[q] : 0ll;
    int gi = 0;
    if (tie) {
      for (int j = part; j < cnt; j += P) gi += (s_d[j] == dt && s_i[j] > ix) ? 1 : 0;
    }
    for (int o = 1; o < P; o <<= 1) gi += __shfl_xor(gi, o);
    if (tie && part == 0 && gi == rem - 1) s_sel[3] = ix;
    __syncthreads();
    ithr = s_sel[3];
  }
}

// the select's grid barrier: this block's stores and atomics drained, its flag raised to `target`, every flag polled
__device__ __forceinline__ void grid_arrive64(Sel64* st, unsigned long long target) {
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(st->flags + blockIdx.x, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void grid_sync64(Sel64* st, unsigned long long target, unsigned spin_lim) {
  grid_arrive64(st, target);
  const int tid = threadIdx.x;
  if (tid < kWave) {
    const int G = (int)gridDim.x;
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < kMaxG64 / kWave; ++i) {
        const int b = tid + i * kWave;
        if (i * kWave < G) {  // (uniform)
          const unsigned long long f =
              __hip_atomic_load(st->flags + (b < G ? b : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= b >= G || f >= target;
        }
      }
      if (__ballot(!ok) == 0ull) break;
      __builtin_amdgcn_s_sleep(1);
      // ~1 s (spin_lim = 2^22): a block never arrived (lost co-residency); flag it and let the launch drain.  (spin_lim 0,
      // a test knob: the first barrier reports a timeout whatever the flags say)
      if (spin_lim == 0u || ++spins > spin_lim) {
        if (tid == 0) atomicOr(&st->err, 1);
        break;
      }
    }
  }
  __syncthreads();
}

// The select, one block per CU (grid-synchronised; block b takes chunks b, b + G, ...):
//   1. the band from the sample (every block the same);
//   2. the filter pass: each chunk's 8192 elements (8 per thread, the next chunk's loads in flight while this one is
//      processed), every key >= t_lo appended to the chunk's segment, the keys above the band counted and the band
//      keys binned (LDS);
//   3. the block's nonzero bins added to the global histogram, its above / overflow count published; a grid barrier;
//   4. the bin of the K-th largest (every block the same), its keys appended to one list, block 0 waits for every
//      block's appends and selects T among them;
// else (the band off or failed) the exact radix select over x.
__global__ __launch_bounds__(kGT) void sel64_select_kernel(const double* __restrict__ x, int64_t n, long long k, int S,
                                                           long long r_lo, long long r_hi, int segcap,
                                                           Sel64* __restrict__ st, unsigned long long* __restrict__ seg,
                                                           unsigned short* __restrict__ segi, int* __restrict__ counts,
                                                           int64_t nch, unsigned spin_lim) {
  constexpr int kPer = kBinCap / kGT;
  constexpr int kR = kChunk / (2 * kGT);  // 16-B loads per thread per chunk (4)
  __shared__ SelLds L;
  unsigned* const s_h = L.h[0];
  long long* const s_scan = L.scan;
  long long* const s_res = L.res;
  long long* const s_bin = L.out[0];
  unsigned long long* const s_d = L.d;
  long long* const s_i = L.i;
  long long* const s_sel = L.sel;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int G = (int)gridDim.x;
  unsigned long long target = 0ull;
  STAMP64(blockIdx.x == 0, 5);
  bool band = S > 0;
  if (band) {
    // 1. the band (the block's first chunk already streaming: its loads do not depend on it)
    // Branch-free loads: every chunk is four 16-B loads per thread, the pairs past the end clamped onto the last
    // aligned pair (their elements are masked by index, an odd n's last element taken from xlast).  A load under a
    // branch leaves the compiler unsure how many loads follow an earlier one, and it then waits for all of them:
    // with the tail's branch, every chunk's processing waited for the loads of the next one too.
    // (The chunk's base is uniform and the lane's offset 32-bit: few registers, so the three sets fit unspilled.  The
    // loads are non-temporal, as in the float32 pass: on fresh inputs 98-99 us per 25 M call against 104 us with
    // cached loads; only an input still resident in the memory-side cache from the previous call reads faster cached.)
    const int64_t nl2 = (n & ~1ll) - 2;  // (n >= 64 Ki here)
    const double xlast = x[n - 1];
    auto load_chunk = [&](int64_t ch, double2 (&v)[kR]) {
      // (a chunk past the end loads chunk 0, never processed; the last chunk's pairs past nl2 load the pair at nl2)
      const int64_t cb = ch < nch ? min(ch * kChunk, nl2) : 0;
      const unsigned lim = (unsigned)min<int64_t>(kChunk - 2, nl2 - cb);
      const double* xb = x + cb;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const unsigned o = 2u * (unsigned)(r * kGT + tid);
        const u64x2 t = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(xb + (o <= lim ? o : lim)));
        v[r].x = __longlong_as_double((long long)t.x);
        v[r].y = __longlong_as_double((long long)t.y);
      }
    };
    double2 va[kR], vb[kR], vc[kR];
    const int64_t c0 = blockIdx.x;
    // (the sample's keys are loaded first: loads complete in order, so keys issued behind the chunk would wait for it)
    unsigned long long t_lo, t_hi;
    bool have_band = false;
    if (S == kSample64 && r_lo <= kGT) {
      // The compact sample (each 64-key wave's 8 largest, 2048 keys: one 8-B load per thread instead of 16): the band
      // from it when no wave of the sample has its 8th largest at or above the floor (then the floor's and the
      // ceiling's ranks among the compact keys are their ranks in the sample), else from the full sample below
      const uint2 c2 = *reinterpret_cast<const uint2*>(st->top + 2 * tid);
      load_chunk(c0, va);
      load_chunk(c0 + G, vb);  // (two chunks in flight across the compact band: 2 keys per thread, not 16)
      if (tid == 0) L.bad = 0;
      const unsigned long long ck[2] = {(unsigned long long)c2.x << 32, (unsigned long long)c2.y << 32};
      sample_band<2>(st, ck, S, r_lo, r_hi, L, t_lo, t_hi);
      if ((tid & 3) == 3 && ck[1] >= t_lo) L.bad = 1;  // (threads 4w .. 4w + 3 hold wave w's 8 keys: .y of the last, its 8th)
      lds_barrier();
      have_band = L.bad == 0;
      lds_barrier();  // (L is reused by the full-sample band)
    }
    if (!have_band) {
      unsigned long long skey[kSPer];
      sample_keys(st, S, skey);
      if (!(S == kSample64 && r_lo <= kGT)) load_chunk(c0, va);  // (a second chunk held across the band's keys would spill)
      sample_band<kSPer>(st, skey, S, r_lo, r_hi, L, t_lo, t_hi);
    }
    if (!(S == kSample64 && r_lo <= kGT)) load_chunk(c0 + G, vb);
    const int sh = range_shift64(t_hi - t_lo - 1ull, 11);  // (t_hi > t_lo)
    STAMP64(blockIdx.x == 0, 6);
    // 2. the filter pass over the block's chunks: chunk q of the block (ch = b + q G) appends through its own LDS
    //    counter, so the waves never wait for each other; three register sets rotate (the loop unrolled three
    //    times, no copies), two chunks' loads in flight while one is processed (a fourth set spills)
    for (int i = tid; i < kBand; i += kGT) L.hb[0][i] = 0u;
    for (int i = tid; i < kMaxCPB; i += kGT) L.cn[i] = 0u;
    if (tid == 0) L.ovf = 0;
    lds_barrier();
    unsigned above = 0u;  // (at most 8 per chunk)
    auto chunk_work = [&](int64_t ch, int q, const double2 (&cv)[kR]) {
      unsigned long long* my = seg + (size_t)ch * segcap;
      unsigned short* myi = segi + (size_t)ch * segcap;
      const int rem = (int)min<int64_t>(n - ch * kChunk, kChunk + 1);  // (the chunk's elements; uniform)
#pragma unroll
      for (int r = 0; r < kR; ++r) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int loc = 2 * (r * kGT + tid) + j;
          const double v = loc == rem - 1 ? xlast : j ? cv[r].y : cv[r].x;
          const unsigned long long key = order_key64(v);
          const bool in = loc < rem && key >= t_lo;
          const unsigned long long m = __ballot(in);
          if (m == 0ull) continue;
          const unsigned p = wave_append(&L.cn[q], in, m);
          if (in) {
            if (p < (unsigned)segcap) {
              my[p] = (unsigned long long)__double_as_longlong(v);
              myi[p] = (unsigned short)loc;
            }
            if (key >= t_hi) ++above;
            else atomicAdd(&L.hb[0][(unsigned)((key - t_lo) >> sh)], 1u);
          }
        }
      }
    };
    {
      for (int q = 0; c0 + (int64_t)q * G < nch; q += 3) {
        const int64_t ch = c0 + (int64_t)q * G;
        load_chunk(ch + 2 * G, vc);
        chunk_work(ch, q, va);
        if (ch + G >= nch) break;
        load_chunk(ch + 3 * G, va);
        chunk_work(ch + G, q + 1, vb);
        if (ch + 2 * G >= nch) break;
        load_chunk(ch + 4 * G, vb);
        chunk_work(ch + 2 * G, q + 2, vc);
      }
    }
    __syncthreads();
#ifdef FLC_SELECT_STAMPS
    if (tid == 0) const_cast<Sel64*>(st)->bstamps[0][blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
    for (int q = tid; blockIdx.x + (int64_t)q * G < nch; q += kGT) {
      counts[blockIdx.x + (int64_t)q * G] = (int)L.cn[q];
      if (L.cn[q] > (unsigned)segcap) L.ovf = 1;  // (benign race: every writer stores 1)
    }
    __syncthreads();
    // 3. the block's band histogram into the global one, its above / overflow count published; one grid barrier
    const unsigned long long ab_blk =
        block_sum<unsigned long long, kGNW>((unsigned long long)above, reinterpret_cast<unsigned long long*>(s_scan));
    for (int i = tid; i < kBand; i += kGT)
      if (L.hb[0][i]) atomicAdd(&st->hist[blockIdx.x % kBandCopies][i], L.hb[0][i]);
    if (tid == 0) st_sc1(&st->pab[blockIdx.x], ab_blk + (L.ovf ? kOvf : 0ull));
    STAMP64(blockIdx.x == 0, 7);
#ifdef FLC_SELECT_STAMPS
    if (tid == 0) const_cast<Sel64*>(st)->bstamps[1][blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
    grid_sync64(st, ++target, spin_lim);
    STAMP64(blockIdx.x == 0, 8);
    // 3. the bin of the K-th largest (every block the same); the thread's two bins of every copy are loaded together
    // with the above counts
    const int ja = kBand - 1 - 2 * tid, jb = kBand - 2 - 2 * tid;  // (pick_band's two bins of thread tid)
    unsigned hca[kBandCopies], hcb[kBandCopies];
#pragma unroll
    for (int c = 0; c < kBandCopies; ++c) {
      hca[c] = ld_sc1(&st->hist[c][ja]);
      hcb[c] = ld_sc1(&st->hist[c][jb]);
    }
    unsigned long long ab = 0ull;
    for (int s = tid; s < G; s += kGT) ab += ld_sc1(&st->pab[s]);
    long long ha = 0, hb = 0;
#pragma unroll
    for (int c = 0; c < kBandCopies; ++c) {
      ha += hca[c];
      hb += hcb[c];
    }
    ab = block_sum<unsigned long long, kGNW>(ab, reinterpret_cast<unsigned long long*>(s_scan));
    const bool ovf = ab >= kOvf;
    // (the K-th largest's rank among the band keys: k less the keys above the band)
    pick_band([&](int j) { return j == ja ? ha : hb; }, k - (long long)(ab & (kOvf - 1ull)), s_scan, s_bin);
    const long long bin = s_bin[0], rem0 = s_bin[1], cnt0 = s_bin[2];
    band = !ovf && bin >= 0 && cnt0 <= kBinCap;  // bin < 0: the sample's ceiling was too low or its floor too high
    STAMP64(blockIdx.x == 0, 10);
    if (band) {
      // 4. the bin's keys to the list; the last block selects T among them
      const unsigned long long lo_b = t_lo + ((unsigned long long)bin << sh), wb = 1ull << sh;
      for (int64_t ch = blockIdx.x + (int64_t)G * (tid >> 6); ch < nch; ch += (int64_t)G * kGNW) {
        const int c = counts[ch];  // (this block's own chunks: written by it above, in its XCD's L2)
        const unsigned long long* sc = seg + (size_t)ch * segcap;
        const unsigned short* si = segi + (size_t)ch * segcap;
        for (int i0 = 0; i0 < c; i0 += kWave) {  // (wave-uniform bounds)
          const int i = i0 + lane;
          const unsigned long long key = i < c ? order_key64(__longlong_as_double((long long)sc[i])) : 0ull;
          // (and below t_hi: the band's top bin may reach past the ceiling — its width need not be a multiple of the
          // bin width — and the keys above the ceiling were counted apart, in `above`, not in the bin)
          const bool in = i < c && key >= lo_b && key - lo_b < wb && key < t_hi;
          const unsigned long long m = __ballot(in);
          if (m == 0ull) continue;
          const unsigned p = wave_append(&st->nbin, in, m);
          if (in && p < (unsigned)kBinCap) {
            st_sc1(&st->bkey[p], key - lo_b);
            st_sc1(&st->bidx[p], (long long)(ch * kChunk + si[i]));
          }
        }
      }
      STAMP64(blockIdx.x == 0, 11);
      if (blockIdx.x != 0) {  // (block 0 alone waits for every block's appends, then selects T)
        grid_arrive64(st, ++target);
        return;
      }
      grid_sync64(st, ++target, spin_lim);
      STAMP64(true, 12);
      // (block 0: every list entry is in)
      const long long cnt = min((long long)ld_sc1(&st->nbin), cnt0);
      unsigned long long dt;
      long long rem, ties, ithr = 0;
      if (cnt <= kGT) {  // each key's rank by comparing it with all others
        if (tid < cnt) {
          s_d[tid] = ld_sc1(&st->bkey[tid]);
          s_i[tid] = ld_sc1(&st->bidx[tid]);
        }
        __syncthreads();
        STAMP64(true, 15);
        rank_small(s_d, s_i, (int)cnt, rem0, s_sel, dt, rem, ties, ithr);
      } else {  // a radix select over the list (up to kBinCap keys)
        unsigned long long d[kPer];
        bool ok[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
          const int p = q * kGT + tid;
          ok[q] = p < cnt;
          d[q] = ok[q] ? ld_sc1(&st->bkey[p]) : 0ull;
        }
        rem = rem0;
        ties = cnt;
        dt = block_select<kPer>(d, ok, sh, rem, ties, s_h, s_scan, s_res);
        if (rem < ties) {  // keep the rem ties with the highest indices: ithr = the rem-th largest index among them
          unsigned long long ix[kPer];
#pragma unroll
          for (int q = 0; q < kPer; ++q) {
            ok[q] = ok[q] && d[q] == dt;
            ix[q] = ok[q] ? (unsigned long long)ld_sc1(&st->bidx[q * kGT + tid]) : 0ull;
          }
          long long ir = rem, ic = ties;
          ithr = (long long)block_select<kPer>(ix, ok, 64 - __clzll((long long)(n - 1 > 0 ? n - 1 : 1)), ir, ic,
                                               s_h, s_scan, s_res);
        }
      }
      STAMP64(true, 13);
      if (tid == 0) {
        st->T = lo_b + dt;
        st->need = rem;
        st->ties = ties;
        st->ithr = ithr;
      }
      return;
    }
  }
  // the fallback: the exact radix select over x (every block reached this point with the same decision)
  // one digit pass: `digit(i, key)` returns the element's digit, or -1 when it is not counted
  auto pass = [&](int slot, long long rem, auto digit) {
    if (tid < 256) s_h[tid] = 0u;
    __syncthreads();
    for (int64_t i0 = (int64_t)blockIdx.x * kGT * 2; i0 < n; i0 += (int64_t)G * kGT * 2) {
      const int64_t i = i0 + 2 * tid;
      double v0 = 0.0, v1 = 0.0;
      if (i + 2 <= n) {
        const double2 a = *reinterpret_cast<const double2*>(x + i);
        v0 = a.x;
        v1 = a.y;
      } else if (i < n) {
        v0 = x[i];
      }
      const int d0 = i < n ? digit(i, order_key64(v0)) : -1;
      const int d1 = i + 1 < n ? digit(i + 1, order_key64(v1)) : -1;
      hist_add64(s_h, (unsigned)d0, d0 >= 0);
      hist_add64(s_h, (unsigned)d1, d1 >= 0);
    }
    __syncthreads();
    if (tid < 256 && s_h[tid]) atomicAdd(&st->fhist[slot][tid], s_h[tid]);
    grid_sync64(st, ++target, spin_lim);
    pick256<kGNW>(tid < 256 ? (long long)ld_sc1(&st->fhist[slot][255 - tid]) : 0ll, rem, s_scan, s_res);
  };
  unsigned long long T = 0ull;
  long long need = k, ties = 0;
  for (int q = 0; q < kDigits; ++q) {
    const int sh = 56 - 8 * q;
    pass(q, need, [&](int64_t, unsigned long long key) {
      return (q == 0 || (key >> (sh + 8)) == T) ? (int)((key >> sh) & 255u) : -1;
    });
    T = (T << 8) | (unsigned long long)s_res[0];
    need -= s_res[1];
    ties = s_res[2];
    __syncthreads();
  }
  long long ithr = 0;
  if (need < ties) {  // the need-th largest index among the ties of T
    const int bits = 64 - __clzll((long long)(n - 1 > 0 ? n - 1 : 1));
    unsigned long long ip = 0ull;
    long long ir = need;
    for (int hb = bits, q = 0; hb > 0; ++q) {
      const int w = hb >= 8 ? 8 : hb, lo = hb - w;
      pass(kDigits + q, ir, [&](int64_t i, unsigned long long key) {
        return (key == T && ((unsigned long long)i >> hb) == ip) ? (int)(((unsigned long long)i >> lo) & ((1u << w) - 1u))
                                                                 : -1;
      });
      ip = (ip << w) | (unsigned long long)s_res[0];
      ir -= s_res[1];
      __syncthreads();
      hb = lo;
    }
    ithr = (long long)ip;
  }
  if (blockIdx.x == 0 && tid == 0) {
    st->T = T;
    st->need = need;
    st->ties = ties;
    st->ithr = ithr;
    st->fb = 1;
  }
}

// dense write: keep key > T, and the ties of T at index >= ithr.  One 64-lane wave per 256-element piece (2 KB of
// output), 32 per chunk: a zeroed LDS tile, the chunk's candidates of this piece scattered into it (each wave scans
// the chunk's ~150-entry segment, its first 64 entries loaded with the state: one round trip before the stores), the
// tile written with non-temporal 16-B stores — the 200 MB of output are written through, not left in the
// memory-side cache for the next call's filter pass to evict (measured: 131 -> 107-109 us per 25 M call).  The wave
// is short so that many are in flight: pieces of 1024 / 512 / 256 / 128 elements took 41 / ~35 / 29.6 / ~47 us at
// 25 M, k = 1 % (the 128-element pieces rescan the segment 64 times).  Segments longer than kEmitSegMax (k above
// ~4.5 % of n) would be rescanned as often: x is read again instead (12 % of n: 165 us against 217 us).
#ifndef FLC_EMIT_PIECE
#define FLC_EMIT_PIECE 256
#endif
constexpr int kPiece = FLC_EMIT_PIECE;
#ifndef FLC_EMIT_SEG_MAX
#define FLC_EMIT_SEG_MAX 1024
#endif
constexpr int kEmitSegMax = FLC_EMIT_SEG_MAX;
constexpr int kPieces = kChunk / kPiece;
__global__ __launch_bounds__(kWave) void sel64_emit_kernel(const double* __restrict__ x, int64_t n, int segcap,
                                                           const Sel64* __restrict__ st,
                                                           const unsigned long long* __restrict__ seg,
                                                           const unsigned short* __restrict__ segi,
                                                           const int* __restrict__ counts, double* __restrict__ out,
                                                           unsigned long long* __restrict__ sticky) {
  __shared__ __attribute__((aligned(16))) unsigned long long s_tile[kPiece];  // 8 KB
  const int lane = threadIdx.x;
  // the select's barrier timeout (this call's output is invalid) into the workspace's sticky error word (bit 4, as the
  // float32 encoders report it), which flc_f64_status reads
  if (blockIdx.x == 0 && lane == 0 && st->err)
    __hip_atomic_fetch_or(sticky, 4ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long T = st->T;
  const long long ithr = st->ithr;
  const int64_t p = blockIdx.x, c = p / kPieces;
  const int sub = (int)(p - c * kPieces);
  const int64_t e0 = p * kPiece;
#ifdef FLC_SELECT_STAMPS
  if (lane == 0 && blockIdx.x == 0) const_cast<Sel64*>(st)->stamps[14] = __builtin_amdgcn_s_memrealtime();
#endif
  // (the chunk's count and first 64 segment entries are loaded with the state, not after it: one round trip)
  const unsigned long long* sc = seg + (size_t)c * segcap;
  const unsigned short* si = segi + (size_t)c * segcap;
  int cc = 0, loc0 = 0;
  unsigned long long b0 = 0ull;
  if (segcap > 0) {  // (the band on: every chunk's count written by the select, its segment allocated)
    cc = counts[c];
    b0 = sc[lane];
    loc0 = si[lane];
  }
  if (segcap > 0 && !st->fb) {  // the piece's candidates (all in its chunk's segment) scattered into a zeroed tile
    u64x2* t2 = reinterpret_cast<u64x2*>(s_tile);
#pragma unroll
    for (int u = 0; u < kPiece / 2 / kWave; ++u) t2[lane + u * kWave] = u64x2{0ull, 0ull};
    auto put = [&](int loc, unsigned long long b) {
      const unsigned long long key = order_key64(__longlong_as_double((long long)b));
      if ((loc / kPiece) == sub && (key > T || (key == T && c * kChunk + loc >= ithr))) s_tile[loc % kPiece] = b;
    };
    if (lane < cc) put(loc0, b0);
    for (int i = lane + kWave; i < cc; i += kWave) put(si[i], sc[i]);
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < kPiece / 2 / kWave; ++u) {
      const int q = lane + u * kWave;
      const int64_t e = e0 + 2 * q;
      if (e + 2 <= n) {
        __builtin_nontemporal_store(t2[q], reinterpret_cast<u64x2*>(out + e));  // (one 16-B store)
      } else if (e < n) {
        out[e] = __longlong_as_double((long long)s_tile[2 * q]);
      }
    }
    return;
  }
  // (after the fallback, or with long segments: x read again, kept in place)
  double2 v[kPiece / 2 / kWave];
#pragma unroll
  for (int u = 0; u < kPiece / 2 / kWave; ++u) {
    const int64_t e = e0 + 2 * (lane + u * kWave);
    const int64_t ec = e + 2 <= n ? e : (n & ~1ll) - 2;  // (branch-free loads: the pairs past the end re-read one)
    v[u] = n >= 2 ? *reinterpret_cast<const double2*>(x + ec) : double2{x[0], 0.0};
  }
#pragma unroll
  for (int u = 0; u < kPiece / 2 / kWave; ++u) {
    const int64_t e = e0 + 2 * (lane + u * kWave);
    auto keep = [&](double d, int64_t i) {
      const unsigned long long key = order_key64(d);
      return (key > T || (key == T && i >= ithr)) ? d : 0.0;
    };
    if (e + 2 <= n) {
      __builtin_nontemporal_store(u64x2{(unsigned long long)__double_as_longlong(keep(v[u].x, e)),
                                        (unsigned long long)__double_as_longlong(keep(v[u].y, e + 1))},
                                  reinterpret_cast<u64x2*>(out + e));
    } else if (e < n) {  // (the odd last element)
      out[e] = keep(x[e], e);
    }
  }
}

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

int flc_copy_f64(const double* x, int64_t n, double* out, void* stream) {
  if (!x || !out || n < 0) return fail(FLC_EINVAL, "flc_copy_f64: bad arguments");
  if (n == 0) return FLC_OK;
  if (!aligned16(x) || !aligned16(out)) return fail(FLC_EINVAL, "flc_copy_f64: 16-B aligned buffers required");
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(cdiv(cdiv(n, 2), kT), 1), 256 * 16);
  FLC_LAUNCH("copy_f64", ew_kernel<false>, dim3(grid), dim3(kT), 0, st, x, n, 1.0, out);
  return FLC_OK;
}

int flc_scale_div_f64(const double* x, int64_t n, double p, double* out, void* stream) {
  if (!x || !out || n < 0) return fail(FLC_EINVAL, "flc_scale_div_f64: bad arguments");
  if (n == 0) return FLC_OK;
  if (!aligned16(x) || !aligned16(out)) return fail(FLC_EINVAL, "flc_scale_div_f64: 16-B aligned buffers required");
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(cdiv(cdiv(n, 2), kT), 1), 256 * 16);
  FLC_LAUNCH("scale_div_f64", ew_kernel<true>, dim3(grid), dim3(kT), 0, st, x, n, p, out);
  return FLC_OK;
}

int flc_randk_apply_f64(const double* x, int64_t n, const int32_t* idx, int64_t k, double scale, double* out,
                        void* stream) {
  if (!x || !out || n <= 0 || k < 0 || (k > 0 && !idx)) return fail(FLC_EINVAL, "flc_randk_apply_f64: bad arguments");
  hipStream_t st = as_stream(stream);
  FLC_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)n * sizeof(double), st));
  if (k == 0) return FLC_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(k, kT), 256 * 16);
  FLC_LAUNCH("randk_scatter_f64", randk_scatter64_kernel, dim3(grid), dim3(kT), 0, st, x, idx, (long long)k, scale, out);
  return FLC_OK;
}

}  // extern "C"

namespace {
// the top-k band's geometry: sample size, the sample ranks of its floor and ceiling, and each chunk's candidate
// segment
struct Filt64 {
  int S;
  long long r_lo, r_hi;
  bool on;
  int segcap;
};
Filt64 filt64(int64_t n, int64_t k) {
  Filt64 f{};
  if (n < 65536 || k <= 0 || k >= n) return f;
  f.S = (int)std::min<int64_t>(n, kSample64);
  const double m = (double)f.S * (double)k / (double)n, sd = 4.0 * sqrt(m) + 16.0;
  f.r_lo = (long long)ceil(m + sd);
  if (f.r_lo >= f.S) return f;
  f.r_hi = std::max<long long>(0, (long long)floor(m - sd));
  const double frac = (double)f.r_lo / (double)f.S;
  f.segcap = (int)align_up((size_t)std::min<double>(kChunk, ceil(2.0 * frac * kChunk) + 256.0), 64);
  f.on = true;
  return f;
}

// FLC_F64_FORCE_TIMEOUT=1 (tests only): the select's first grid barrier reports a timeout, so that the error path
// (Sel64::err -> the sticky word -> flc_f64_status -> the caller's check) can be exercised
bool force_timeout64() {
  static const bool on = getenv("FLC_F64_FORCE_TIMEOUT") && atoi(getenv("FLC_F64_FORCE_TIMEOUT")) == 1;
  return on;
}

struct Ws64 {
  unsigned long long* sticky;  // the sticky error word (flc_f64_status): first in every float64 workspace
  int* counts;
  long long* offsets;
  unsigned long long* part;
  Sel64* sel;
  unsigned long long* seg;  // top-k candidate segments: [chunks][segcap] value bits
  unsigned short* segi;     //   ... and positions in the chunk
  size_t need;
};
Ws64 carve64(void* ws, size_t bytes, int64_t n, int64_t k = 0) {
  Carver c(ws, bytes);
  const int64_t nch = cdiv(n < 1 ? 1 : n, kChunk);
  Ws64 w;
  w.sticky = c.take<unsigned long long>(32);
  w.counts = c.take<int>((size_t)nch);
  w.offsets = c.take<long long>((size_t)nch + 1);
  w.part = c.take<unsigned long long>((size_t)nch);
  w.sel = c.take<Sel64>(k > 0 ? 1 : 0);
  const Filt64 f = filt64(n, k);
  w.seg = c.take<unsigned long long>(f.on ? (size_t)nch * f.segcap : 0);
  w.segi = c.take<unsigned short>(f.on ? (size_t)nch * f.segcap : 0);
  w.need = c.off;
  return w;
}
}  // namespace

extern "C" {

size_t flc_f64_workspace_size(int64_t n, int64_t k) { return carve64(nullptr, 0, n, k).need; }

int flc_count_consumers_f64(const double* x, int64_t n, const double* norm, int64_t* count, void* ws, size_t ws_bytes,
                            void* stream) {
  if (!x || !count || n <= 0) return fail(FLC_EINVAL, "flc_count_consumers_f64: bad arguments");
  if (!aligned16(x)) return fail(FLC_EINVAL, "flc_count_consumers_f64: x must be 16-B aligned");
  Ws64 w = carve64(ws, ws_bytes, n);
  if (!ws || w.need > ws_bytes) return fail(FLC_EWORKSPACE, "flc_count_consumers_f64: workspace %zu < %zu", ws_bytes, w.need);
  const int64_t nch = cdiv(n, kChunk);
  hipStream_t st = as_stream(stream);
  if (norm)
    FLC_LAUNCH("count64", count64_kernel<1>, dim3((unsigned)nch), dim3(kT), 0, st, x, n, norm, w.counts);
  else
    FLC_LAUNCH("count64", count64_kernel<0>, dim3((unsigned)nch), dim3(kT), 0, st, x, n, norm, w.counts);
  FLC_LAUNCH("scan64", scan64_kernel, dim3(1), dim3(1024), 0, st, w.counts, w.offsets, nch);
  FLC_CHECK_HIP(hipMemcpyAsync(count, w.offsets + nch, sizeof(int64_t), hipMemcpyDeviceToDevice, st));
  return FLC_OK;
}

int flc_natural_f64(const double* x, int64_t n, uint64_t seed, uint64_t counter, const double* compat_u,
                    uint16_t* codes, double* out, void* ws, size_t ws_bytes, void* stream) {
  if (!x || n <= 0 || (!codes && !out)) return fail(FLC_EINVAL, "flc_natural_f64: bad arguments");
  if (!aligned16(x) || (out && !aligned16(out)) || (codes && !aligned16(codes)))
    return fail(FLC_EINVAL, "flc_natural_f64: 16-B aligned buffers required");
  const int64_t nch = cdiv(n, kChunk);
  hipStream_t st = as_stream(stream);
  if (compat_u) {
    Ws64 w = carve64(ws, ws_bytes, n);
    if (!ws || w.need > ws_bytes) return fail(FLC_EWORKSPACE, "flc_natural_f64: workspace %zu < %zu", ws_bytes, w.need);
    FLC_LAUNCH("count64", count64_kernel<0>, dim3((unsigned)nch), dim3(kT), 0, st, x, n, (const double*)nullptr,
               w.counts);
    FLC_LAUNCH("scan64", scan64_kernel, dim3(1), dim3(1024), 0, st, w.counts, w.offsets, nch);
    FLC_LAUNCH("natural_f64", natural64_kernel<true>, dim3((unsigned)nch), dim3(kT), 0, st, x, n, seed, counter,
               compat_u, (const long long*)w.offsets, codes, out);
  } else {
    FLC_LAUNCH("natural_f64", natural64_kernel<false>, dim3((unsigned)nch), dim3(kT), 0, st, x, n, seed, counter,
               compat_u, (const long long*)nullptr, codes, out);
  }
  return FLC_OK;
}

int flc_natural_decode_f64(const uint16_t* codes, int64_t n, double* out, void* stream) {
  if (!codes || !out || n <= 0) return fail(FLC_EINVAL, "flc_natural_decode_f64: bad arguments");
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(n, kT), 256 * 32);
  FLC_LAUNCH("natural_decode_f64", natural64_decode_kernel, dim3(grid), dim3(kT), 0, st, codes, n, out);
  return FLC_OK;
}

int flc_quant_norm_f64(const double* x, int64_t n, int norm_p, double* norm, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !norm || n <= 0) return fail(FLC_EINVAL, "flc_quant_norm_f64: bad arguments");
  if (norm_p != FLC_NORM_INF && norm_p != FLC_NORM_L2) return fail(FLC_EUNSUPPORTED, "flc_quant_norm_f64: p = inf or 2");
  if (!aligned16(x)) return fail(FLC_EINVAL, "flc_quant_norm_f64: x must be 16-B aligned");
  Ws64 w = carve64(ws, ws_bytes, n);
  if (!ws || w.need > ws_bytes) return fail(FLC_EWORKSPACE, "flc_quant_norm_f64: workspace %zu < %zu", ws_bytes, w.need);
  const int64_t nch = cdiv(n, kChunk);
  hipStream_t st = as_stream(stream);
  if (norm_p == FLC_NORM_INF) {
    FLC_LAUNCH("norm64", norm64_partial_kernel<FLC_NORM_INF>, dim3((unsigned)nch), dim3(kT), 0, st, x, n, w.part);
    FLC_LAUNCH("norm64_fold", norm64_fold_kernel<FLC_NORM_INF>, dim3(1), dim3(kWave), 0, st, w.part, nch, norm);
  } else {
    FLC_LAUNCH("norm64", norm64_partial_kernel<FLC_NORM_L2>, dim3((unsigned)nch), dim3(kT), 0, st, x, n, w.part);
    FLC_LAUNCH("norm64_fold", norm64_fold_kernel<FLC_NORM_L2>, dim3(1), dim3(kWave), 0, st, w.part, nch, norm);
  }
  return FLC_OK;
}

int flc_quant_f64(const double* x, int64_t n, int kind, int levels, const double* norm, uint64_t seed,
                  uint64_t counter, const double* compat_u, uint8_t* codes, double* out, int64_t* nnz, void* ws,
                  size_t ws_bytes, void* stream) {
  if (!x || !norm || n <= 0 || (!codes && !out)) return fail(FLC_EINVAL, "flc_quant_f64: bad arguments");
  if (kind != FLC_Q_STANDARD_DITHER && kind != FLC_Q_NATURAL_DITHER) return fail(FLC_EINVAL, "flc_quant_f64: bad kind");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_quant_f64: levels must be in [1, 127]");
  if (!aligned16(x) || (out && !aligned16(out)) || (codes && !aligned16(codes)))
    return fail(FLC_EINVAL, "flc_quant_f64: 16-B aligned buffers required");
  const int64_t nch = cdiv(n, kChunk);
  hipStream_t st = as_stream(stream);
  unsigned long long* nz = reinterpret_cast<unsigned long long*>(nnz);
  if (nnz) FLC_CHECK_HIP(hipMemsetAsync(nnz, 0, sizeof(int64_t), st));
  const double step = 1.0 / (double)levels;
  const long long* offs = nullptr;
  if (compat_u) {
    Ws64 w = carve64(ws, ws_bytes, n);
    if (!ws || w.need > ws_bytes) return fail(FLC_EWORKSPACE, "flc_quant_f64: workspace %zu < %zu", ws_bytes, w.need);
    FLC_LAUNCH("count64", count64_kernel<1>, dim3((unsigned)nch), dim3(kT), 0, st, x, n, norm, w.counts);
    FLC_LAUNCH("scan64", scan64_kernel, dim3(1), dim3(1024), 0, st, w.counts, w.offsets, nch);
    offs = w.offsets;
  }
#define FLC_Q64(K, C)                                                                                              \
  FLC_LAUNCH("quant_f64", (quant64_kernel<K, C>), dim3((unsigned)nch), dim3(kT), 0, st, x, n, levels, step, norm, \
             seed, counter, compat_u, offs, codes, out, nz)
  if (kind == FLC_Q_STANDARD_DITHER) {
    if (compat_u) FLC_Q64(0, true);
    else FLC_Q64(0, false);
  } else {
    if (compat_u) FLC_Q64(1, true);
    else FLC_Q64(1, false);
  }
#undef FLC_Q64
  return FLC_OK;
}

int flc_quant_decode_f64(const uint8_t* codes, int64_t n, int kind, int levels, const double* norm, double* out,
                         void* stream) {
  if (!codes || !norm || !out || n <= 0) return fail(FLC_EINVAL, "flc_quant_decode_f64: bad arguments");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_quant_decode_f64: levels must be in [1, 127]");
  hipStream_t st = as_stream(stream);
  const double step = 1.0 / (double)levels;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(n, kT), 256 * 32);
  if (kind == FLC_Q_STANDARD_DITHER)
    FLC_LAUNCH("quant_decode_f64", quant64_decode_kernel<0>, dim3(grid), dim3(kT), 0, st, codes, n, levels, step, norm, out);
  else
    FLC_LAUNCH("quant_decode_f64", quant64_decode_kernel<1>, dim3(grid), dim3(kT), 0, st, codes, n, levels, step, norm, out);
  return FLC_OK;
}

int flc_topk_dense_f64(const double* x, int64_t n, int64_t k, double* out, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !out || n <= 0) return fail(FLC_EINVAL, "flc_topk_dense_f64: bad arguments");
  if (k <= 0 || k >= n) return fail(FLC_EINVAL, "flc_topk_dense_f64: need 0 < k < n (got k=%lld, n=%lld)",
                                    (long long)k, (long long)n);
  if (!aligned16(x) || !aligned16(out)) return fail(FLC_EINVAL, "flc_topk_dense_f64: 16-B aligned buffers required");
  Ws64 w = carve64(ws, ws_bytes, n, k);
  if (!ws || w.need > ws_bytes) return fail(FLC_EWORKSPACE, "flc_topk_dense_f64: workspace %zu < %zu", ws_bytes, w.need);
  hipStream_t st = as_stream(stream);
  const int64_t nch = cdiv(n, kChunk);
  Filt64 f = filt64(n, k);
  int dev = 0;
  const int cus = std::min(stream_cus(st, &dev), kMaxG64);
  if (cdiv(nch, cus) > kMaxCPB) f.on = false;  // (more chunks per block than its LDS counters: the exact passes)
  FLC_LAUNCH("sel64_prep", sel64_prep_kernel, dim3(f.on ? (unsigned)kSampleBlocks : 1u), dim3(kT), 0, st, x, n,
             f.on ? f.S : 0, w.sel);
  {  // (grid-synchronised: one block per CU, all resident)
    Coresident co(st, dev);
    if (co.status()) return co.status();
    FLC_LAUNCH_CO(co, "sel64_select", sel64_select_kernel, dim3((unsigned)cus), dim3(kGT), 0, st, x, n, (long long)k,
               f.on ? f.S : 0, f.r_lo, f.r_hi, f.on ? f.segcap : 0, w.sel, w.seg, w.segi, w.counts, f.on ? nch : 0,
               force_timeout64() ? 0u : (1u << 22));
    const int rc = co.finish();
    if (rc) return rc;
  }
  // (segments longer than kEmitSegMax: x is read again instead, every piece's wave would scan its chunk's segment)
  FLC_LAUNCH("sel64_emit", sel64_emit_kernel, dim3((unsigned)cdiv(n, kPiece)), dim3(kWave), 0, st, x, n,
             f.on && f.segcap <= kEmitSegMax ? f.segcap : 0,
             (const Sel64*)w.sel, (const unsigned long long*)w.seg, (const unsigned short*)w.segi,
             (const int*)w.counts, out, w.sticky);
  return FLC_OK;
}

int flc_f64_status(void* ws, uint64_t* err_out, int reset, void* stream) {
  if (!ws || !err_out) return fail(FLC_EINVAL, "flc_f64_status: null workspace or output");
  hipStream_t st = as_stream(stream);
  FLC_CHECK_HIP(hipMemcpyAsync(err_out, ws, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
  if (reset) FLC_CHECK_HIP(hipMemsetAsync(ws, 0, sizeof(uint64_t), st));
  return FLC_OK;
}

}  // extern "C"
