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
//                                    0 elsewhere (compressors.py:293-296): a radix select over 64-bit order keys,
//                                    eight 8-bit digit passes, then one counting pass and the dense write
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
// top-k on fp64 (compressors.py:293-296): out = x on the K largest, +0 elsewhere
// ------------------------------------------------------------------------------------------------
// order-preserving key of a double: NaN largest, -0 == +0
__device__ __forceinline__ unsigned long long order_key64(double v) {
  unsigned long long b = (unsigned long long)__double_as_longlong(v);
  if ((b & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) return ~0ull;
  if (b == 0x8000000000000000ull) b = 0ull;
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

constexpr int kDigits = 8;  // 8-bit digits, most significant first
constexpr int kSample64 = 8192;   // sample keys of the top-k floor
constexpr int kFloorDigits = 3;   // the floor keeps the sample's r-th key to its top 24 bits (a floor below it)
struct Sel64 {
  // after q digit passes: the resolved high digits of the K-th largest key, its rank among the keys sharing them
  // (from the top, 1-based), and the size of the last digit's bin (after all kDigits passes: the ties of T)
  unsigned long long pre[kDigits + 1];
  long long rem[kDigits + 1], cnt[kDigits + 1];
  unsigned long long t_lo;  // candidate floor key (from the sample)
  int mode;                 // 0: the digit passes run over the candidates, 1: over x itself
  int ovf;                  // a chunk had more candidates than its segment holds
  unsigned hist[kDigits][256];
  unsigned long long sample[kSample64];
};

// LDS histogram add of one key per lane; a wave whose counted keys all fall in one bin (the common case in the high
// digits, where the keys share their sign and exponent) adds once
__device__ __forceinline__ void hist_add64(unsigned* h, unsigned bin, bool in) {
  const unsigned long long m = __ballot(in);
  if (m == 0ull) return;
  const int first = __builtin_ctzll(m);
  const unsigned b0 = (unsigned)__builtin_amdgcn_readlane((int)bin, first);
  if (__ballot(in && bin != b0) == 0ull) {
    if ((int)(threadIdx.x & (kWave - 1)) == first) atomicAdd(&h[b0], (unsigned)__popcll(m));
  } else if (in) {
    atomicAdd(&h[bin], 1u);
  }
}

// block-wide (NW waves): the bin of a 256-bin histogram (count of bin 255 - t in thread t < 256, 0 elsewhere)
// holding rank `rem` from the top.  Returns, in every thread, (digit, count above it, its count).
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

// state q + 1 from state q and the q-th pass's histogram (every block of a kernel computes it the same way; the
// caller's block 0 stores it for the next kernel)
__device__ __forceinline__ void sel64_step(const Sel64* __restrict__ st, int q, long long* s_scan, long long* s_res,
                                           unsigned long long& pre, long long& rem, long long& cnt) {
  const long long c = threadIdx.x < 256 ? (long long)st->hist[q][255 - threadIdx.x] : 0ll;
  pre = st->pre[q];
  rem = st->rem[q];
  pick256<kNW>(c, rem, s_scan, s_res);
  pre = (pre << 8) | (unsigned long long)s_res[0];
  rem -= s_res[1];
  cnt = s_res[2];
}

// block 0 resets the state; with S > 0 the blocks also take S evenly strided keys (the float32 encoder's sample
// positions)
__global__ __launch_bounds__(kT) void sel64_init_kernel(const double* __restrict__ x, int64_t n, int S, long long k,
                                                        int mode, Sel64* __restrict__ st) {
  if (blockIdx.x == 0) {
    for (int i = threadIdx.x; i < kDigits * 256; i += kT) (&st->hist[0][0])[i] = 0u;
    if (threadIdx.x == 0) {
      st->pre[0] = 0ull;
      st->rem[0] = k;
      st->cnt[0] = 0;
      st->t_lo = 0ull;
      st->mode = mode;
      st->ovf = 0;
    }
  }
  const int j = blockIdx.x * kT + threadIdx.x;
  if (j >= S) return;
  const int64_t pos = (int64_t)(((double)j + 0.5) * (double)n / (double)S);
  st->sample[j] = order_key64(x[pos < n ? pos : n - 1]);
}

// one block: t_lo = the r-th largest sample key truncated to its top 24 bits (three digit passes over the sample
// held in registers), so that count(key >= t_lo) >= ~k + 4 sigma over the whole vector
__global__ __launch_bounds__(1024) void sel64_floor_kernel(int S, long long r, Sel64* __restrict__ st) {
  constexpr int kPer = kSample64 / 1024, kW = 1024 / kWave;
  __shared__ unsigned s_h[256];
  __shared__ long long s_scan[kW], s_res[3];
  unsigned long long key[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int j = i * 1024 + threadIdx.x;
    key[i] = j < S ? st->sample[j] : 0ull;
  }
  unsigned long long prefix = 0ull;
  long long rem = r;
  for (int pass = 0; pass < kFloorDigits; ++pass) {
    if (threadIdx.x < 256) s_h[threadIdx.x] = 0u;
    __syncthreads();
    const int sh = 56 - 8 * pass;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const bool in = i * 1024 + (int)threadIdx.x < S && (pass == 0 || (key[i] >> (sh + 8)) == prefix);
      hist_add64(s_h, (unsigned)(key[i] >> sh) & 255u, in);
    }
    __syncthreads();
    pick256<kW>(threadIdx.x < 256 ? (long long)s_h[255 - threadIdx.x] : 0ll, rem, s_scan, s_res);
    prefix = (prefix << 8) | (unsigned long long)s_res[0];
    rem -= s_res[1];
    __syncthreads();  // (s_res and s_h are rewritten by the next pass)
  }
  if (threadIdx.x == 0) st->t_lo = prefix << (64 - 8 * kFloorDigits);
}

// the candidates (key >= t_lo) of each 8192-element chunk appended to the chunk's own segment (no global atomics);
// counts[c] = the chunk's candidate count (a count beyond the segment flags st->ovf: the passes then run over x)
__global__ __launch_bounds__(kT) void sel64_filter_kernel(const double* __restrict__ x, int64_t n, int segcap,
                                                          Sel64* __restrict__ st, unsigned long long* __restrict__ seg,
                                                          int* __restrict__ counts) {
  // (the digit passes only histogram the candidates: their order inside a segment is free, so each wave appends
  // through one LDS counter, without block-wide barriers)
  __shared__ unsigned s_n;
  if (threadIdx.x == 0) s_n = 0u;
  __syncthreads();
  const unsigned long long t_lo = st->t_lo;
  unsigned long long* my = seg + (size_t)blockIdx.x * segcap;
  const int lane = threadIdx.x & (kWave - 1);
  for (int it = 0; it < kIt; ++it) {
    const int64_t e0 = (int64_t)blockIdx.x * kChunk + ((int64_t)it * kT + threadIdx.x) * kE;
    double v[kE] = {0.0, 0.0, 0.0, 0.0};
    if (e0 < n) load4(x, e0, n, v);
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      const unsigned long long key = order_key64(v[j]);
      const bool in = e0 + j < n && key >= t_lo;
      const unsigned long long m = __ballot(in);
      if (m == 0ull) continue;
      unsigned base = 0;
      if (lane == 0) base = atomicAdd(&s_n, (unsigned)__popcll(m));
      base = (unsigned)__builtin_amdgcn_readlane((int)base, 0);
      const unsigned p = base + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      if (in && p < (unsigned)segcap) my[p] = key;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    counts[blockIdx.x] = (int)s_n;
    if (s_n > (unsigned)segcap) atomicOr(&st->ovf, 1);
  }
}

// digit pass `pass`: the previous pass's digit resolved first (state pass from state pass - 1), then mode 0 over the
// chunk segments (block b takes chunks b, b + grid, ...: slots i < counts[c]), mode 1 over x
__global__ __launch_bounds__(kT) void sel64_hist_kernel(const double* __restrict__ x, int64_t n, int pass,
                                                        Sel64* __restrict__ st, const unsigned long long* __restrict__ seg,
                                                        const int* __restrict__ counts, int64_t nch, int segcap) {
  __shared__ unsigned s_h[256];
  __shared__ long long s_scan[kNW], s_res[3];
  __shared__ int s_mode;
  s_h[threadIdx.x] = 0u;
  unsigned long long prefix = 0ull;
  if (pass == 0) {
    // the candidates serve unless a segment overflowed or the floor admitted fewer than k elements (the sample
    // missed): every block sums the chunk counts itself (block 0 records the decision for the later passes)
    long long c = 0;
    if (st->mode == 0)
      for (int64_t i = threadIdx.x; i < nch; i += kT) c += counts[i];
    c = block_sum<long long, kNW>(c, s_scan);
    if (threadIdx.x == 0) {
      s_mode = (st->mode != 0 || st->ovf || c < st->rem[0]) ? 1 : 0;
      if (blockIdx.x == 0) st->mode = s_mode;
    }
  } else {
    if (threadIdx.x == 0) s_mode = st->mode;
  }
  if (pass > 0) {
    long long rem, cnt;
    sel64_step(st, pass - 1, s_scan, s_res, prefix, rem, cnt);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->pre[pass] = prefix;
      st->rem[pass] = rem;
      st->cnt[pass] = cnt;
    }
  }
  __syncthreads();
  const int sh = 56 - 8 * pass;
  auto add = [&](unsigned long long key, bool valid) {
    hist_add64(s_h, (unsigned)(key >> sh) & 255u, valid && (pass == 0 || (key >> (sh + 8)) == prefix));
  };
  if (s_mode == 0) {
    for (int64_t c = blockIdx.x; c < nch; c += gridDim.x) {
      const int cnt = counts[c];
      const unsigned long long* sc = seg + (size_t)c * segcap;
      for (int i0 = 0; i0 < cnt; i0 += kT) {  // (block-uniform bounds)
        const int i = i0 + (int)threadIdx.x;
        add(i < cnt ? sc[i] : 0ull, i < cnt);
      }
    }
  } else {
    for (int64_t i0 = (int64_t)blockIdx.x * kT * 2; i0 < n; i0 += (int64_t)gridDim.x * kT * 2) {
      const int64_t i = i0 + 2 * threadIdx.x;
      double v[2] = {0.0, 0.0};
      if (i + 2 <= n) {
        const double2 a = *reinterpret_cast<const double2*>(x + i);
        v[0] = a.x;
        v[1] = a.y;
      } else if (i < n) {
        v[0] = x[i];
      }
      add(order_key64(v[0]), i < n);
      add(order_key64(v[1]), i + 1 < n);
    }
  }
  __syncthreads();
  if (s_h[threadIdx.x]) atomicAdd(&st->hist[pass][threadIdx.x], s_h[threadIdx.x]);
}

// ties (keys == T) per chunk, for the highest-index rule; nothing to count when every tie is kept (need == ties)
__global__ __launch_bounds__(kT) void sel64_ties_kernel(const double* __restrict__ x, int64_t n, Sel64* __restrict__ st,
                                                        int* __restrict__ counts) {
  __shared__ int s_red[kNW];
  __shared__ long long s_scan[kNW], s_res[3];
  unsigned long long T;
  long long need, ties;
  sel64_step(st, kDigits - 1, s_scan, s_res, T, need, ties);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->pre[kDigits] = T;
    st->rem[kDigits] = need;
    st->cnt[kDigits] = ties;
  }
  if (need == ties) {
    if (threadIdx.x == 0) counts[blockIdx.x] = 0;
    return;
  }
  int cnt = 0;
  for (int it = 0; it < kIt; ++it) {
    const int64_t e0 = (int64_t)blockIdx.x * kChunk + ((int64_t)it * kT + threadIdx.x) * kE;
    if (e0 >= n) break;
    double v[kE];
    load4(x, e0, n, v);
#pragma unroll
    for (int j = 0; j < kE; ++j) cnt += (e0 + j < n && order_key64(v[j]) == T) ? 1 : 0;
  }
  const int tot = block_sum<int, kNW>(cnt, s_red);
  if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

// dense write: keep key > T, and the `rem` ties with the highest indices (tie rank from the top < rem)
__global__ __launch_bounds__(kT) void sel64_emit_kernel(const double* __restrict__ x, int64_t n,
                                                        const Sel64* __restrict__ st,
                                                        const long long* __restrict__ offsets, int64_t nchunks,
                                                        double* __restrict__ out) {
  __shared__ long long s_scan[kNW];
  const unsigned long long T = st->pre[kDigits];
  const long long need = st->rem[kDigits];
  // ties after this chunk = total - ties up to the end of this chunk (all 0 when every tie is kept: then
  // `higher` below is negative, hence < need, for every tie)
  if (need == st->cnt[kDigits]) {  // every tie kept (the common case): key >= T, no tie ranks
    for (int it = 0; it < kIt; ++it) {
      const int64_t e0 = (int64_t)blockIdx.x * kChunk + ((int64_t)it * kT + threadIdx.x) * kE;
      if (e0 >= n) break;
      double v[kE];
      load4(x, e0, n, v);
#pragma unroll
      for (int j = 0; j < kE; ++j) v[j] = order_key64(v[j]) >= T ? v[j] : 0.0;
      store4(out, e0, n, v);
    }
    return;
  }
  long long after = offsets[nchunks] - offsets[blockIdx.x];
  for (int it = 0; it < kIt; ++it) {
    const int64_t e0 = (int64_t)blockIdx.x * kChunk + ((int64_t)it * kT + threadIdx.x) * kE;
    double v[kE];
    if (e0 < n) load4(x, e0, n, v);
    else
#pragma unroll
      for (int j = 0; j < kE; ++j) v[j] = 0.0;
    int c[kE], cnt = 0;
    unsigned long long key[kE];
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      key[j] = order_key64(v[j]);
      c[j] = (e0 + j < n && key[j] == T) ? 1 : 0;
      cnt += c[j];
    }
    long long tot;
    const long long before = block_excl_scan<long long, kNW>((long long)cnt, s_scan, &tot);
    // ties with a higher index than element j: those after this iteration, and those after it inside it
    long long higher = after - before - cnt;  // (after counts this iteration's ties too)
    double o[kE];
#pragma unroll
    for (int j = kE - 1; j >= 0; --j) {
      const bool keep = key[j] > T || (c[j] && higher < need);
      higher += c[j];
      o[j] = keep ? v[j] : 0.0;
    }
    after -= tot;
    if (e0 < n) store4(out, e0, n, o);
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
// the top-k filter's geometry: sample size, the floor's rank in the sample, and each chunk's candidate segment
struct Filt64 {
  int S;
  long long r_lo;
  bool on;
  int segcap;
};
Filt64 filt64(int64_t n, int64_t k) {
  Filt64 f{};
  if (n < 65536 || k <= 0 || k >= n) return f;
  f.S = (int)std::min<int64_t>(n, kSample64);
  const double m = (double)f.S * (double)k / (double)n;
  f.r_lo = (long long)ceil(m + 4.0 * sqrt(m) + 16.0);
  if (f.r_lo >= f.S) return f;
  const double frac = (double)f.r_lo / (double)f.S;
  f.segcap = (int)align_up((size_t)std::min<double>(kChunk, ceil(2.0 * frac * kChunk) + 256.0), 64);
  f.on = true;
  return f;
}

struct Ws64 {
  int* counts;
  long long* offsets;
  unsigned long long* part;
  Sel64* sel;
  unsigned long long* seg;  // top-k candidate segments: [chunks][segcap]
  size_t need;
};
Ws64 carve64(void* ws, size_t bytes, int64_t n, int64_t k = 0) {
  Carver c(ws, bytes);
  const int64_t nch = cdiv(n < 1 ? 1 : n, kChunk);
  Ws64 w;
  w.counts = c.take<int>((size_t)nch);
  w.offsets = c.take<long long>((size_t)nch + 1);
  w.part = c.take<unsigned long long>((size_t)nch);
  w.sel = c.take<Sel64>(1);
  const Filt64 f = filt64(n, k);
  w.seg = c.take<unsigned long long>(f.on ? (size_t)nch * f.segcap : 0);
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
  const Filt64 f = filt64(n, k);
  // the candidates: a sample's floor t_lo (count(key >= t_lo) ~ k + 4 sigma), one filtering pass into per-chunk
  // segments; the digit passes then read the candidates (~1.3 k keys) instead of x, unless a segment overflowed or the
  // floor admitted fewer than k elements (then they read x: the same result)
  FLC_LAUNCH("sel64_init", sel64_init_kernel, dim3((unsigned)std::max<int64_t>(1, cdiv(f.S, kT))), dim3(kT), 0, st, x,
             n, f.on ? f.S : 0, (long long)k, f.on ? 0 : 1, w.sel);
  if (f.on) {
    FLC_LAUNCH("sel64_floor", sel64_floor_kernel, dim3(1), dim3(1024), 0, st, f.S, f.r_lo, w.sel);
    FLC_LAUNCH("sel64_filter", sel64_filter_kernel, dim3((unsigned)nch), dim3(kT), 0, st, x, n, f.segcap, w.sel, w.seg,
               w.counts);
  }
  // (the candidate passes need few blocks: each block flushes up to 256 bins with global atomics; the fallback over x
  // streams with them too)
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(cdiv(n, 2), kT), 512);
  // (each pass first resolves the previous pass's digit; the ties kernel resolves the last one)
  for (int pass = 0; pass < kDigits; ++pass)
    FLC_LAUNCH("sel64_hist", sel64_hist_kernel, dim3(grid), dim3(kT), 0, st, x, n, pass, w.sel,
               (const unsigned long long*)w.seg, (const int*)w.counts, nch, f.on ? f.segcap : 1);
  FLC_LAUNCH("sel64_ties", sel64_ties_kernel, dim3((unsigned)nch), dim3(kT), 0, st, x, n, w.sel, w.counts);
  FLC_LAUNCH("scan64", scan64_kernel, dim3(1), dim3(1024), 0, st, w.counts, w.offsets, nch);
  FLC_LAUNCH("sel64_emit", sel64_emit_kernel, dim3((unsigned)nch), dim3(kT), 0, st, x, n, (const Sel64*)w.sel,
             (const long long*)w.offsets, nch, out);
  return FLC_OK;
}

}  // extern "C"
