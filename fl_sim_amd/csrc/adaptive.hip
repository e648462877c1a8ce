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
// Every rounding above is reproduced.  The one sequential dependency, the fp64 running sum, is made
// parallel without giving up exactness by speculation with a translation argument: inside one binade
// [2^E, 2^(E+1)) fp64 values are the multiples of U = 2^(E-52), and round-to-nearest-even commutes with a
// shift by an EVEN multiple of U.  So a chunk's sequential run started from a guess g (close to its true
// start t, same binade) ends at exactly e + (t - g) whenever (t - g) / U is even and both runs stay in
// that binade.  Each chunk of kChunk elements is run twice, from g and from g + U (one of the two
// differences is even), in parallel (phase A); one thread then chains the chunks (phase B), shifting the
// speculated ends and re-running a chunk sequentially only when a binade boundary gets in the way
// (a few dozen chunks per call: the running sum crosses each binade once).  Then the chunk holding the
// crossing of u is re-run to find the index.  The guesses come from an fp64 prefix of the chunk sums of
// |x|; their accuracy only decides how often a re-run happens, never the result.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kBuf = 8192;    // numpy's reduction buffer (np.getbufsize() default)
constexpr int kLeaf = 128;    // numpy PW_BLOCKSIZE
constexpr int kChunk = 2048;  // elements per speculated cdf chunk (4 per reduction buffer)
constexpr int kQ = kBuf / kChunk;
constexpr int kPad = kBuf + kBuf / kLeaf;  // LDS copy of one buffer, one pad word per leaf
constexpr int kRec = 1024;                 // chunk records staged in LDS per step of phase B

// status word (device int32) written by ar_check
constexpr int kStNan = 1, kStSum = 2;
constexpr double kAtol = 3.4526698300124393e-04;  // sqrt(finfo(float32).eps)

struct ArWs {
  float* buf_sum;   // [nbuf] pairwise sum of |x| per reduction buffer
  double* q_abs;    // [nq]  approximate sum of |x| per cdf chunk (guesses only)
  double* guess;    // [nq]  speculated start of each chunk's running sum
  double* end_a;    // [nq]  end of the run started at guess
  double* end_b;    // [nq]  end of the run started at guess + U
  double* p_sum;    // [nq]  fp64 sum of p per chunk (the "sum to 1" check)
  double* start;    // [nq + 1] exact running sum before each chunk; start[nq] = cdf[-1]
  float* total;     // [1]   S
  int32_t* status;  // [1]
};

__device__ __forceinline__ int binade(double v) {  // exponent field: one grid spacing per value
  return (int)((uint64_t)__double_as_longlong(v) >> 52);  // v >= 0 here
}
__device__ __forceinline__ double spacing(int e) {  // grid spacing of binade e (e = 0: subnormals)
  return e == 0 ? 4.9406564584124654e-324 : ldexp(1.0, e - 1075);
}

// ---- numpy's pairwise_sum on fp32 (loops_utils.h.src), general n <= kBuf, one thread ------------------
__device__ float pw_leaf(const float* a, int n) {
  if (n < 8) {
    float r = 0.0f;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  }
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

template <int DEPTH>
__device__ __attribute__((noinline)) float pw_sum(const float* a, int n) {
  if (n <= kLeaf) return pw_leaf(a, n);
  if constexpr (DEPTH == 0) {
    return __builtin_nanf("");  // unreachable for n <= kBuf (depth <= 7)
  } else {
    int n2 = n / 2;
    n2 -= n2 % 8;
    const float l = pw_sum<DEPTH - 1>(a, n2);
    const float r = pw_sum<DEPTH - 1>(a + n2, n - n2);
    return l + r;
  }
}

// ---- K1: full reduction buffers (n2 splits of 8192 are a perfect tree of 64 leaves of 128) ----------
__global__ __launch_bounds__(256) void ar_buffer_sum_kernel(const float* __restrict__ x, int64_t n_full_bufs,
                                                            ArWs ws) {
  __shared__ float sh[kPad];
  const int64_t b = blockIdx.x;
  if (b >= n_full_bufs) return;
  const float* src = x + b * kBuf;
  // 256 threads x 8 float4: coalesced, |x| written with one pad word per 128-element leaf
  for (int v = threadIdx.x; v < kBuf / 4; v += 256) {
    const float4 q = *reinterpret_cast<const float4*>(src + 4 * v);
    const int i = 4 * v;
    const int o = i + (i >> 7);
    sh[o] = fabsf(q.x);
    sh[o + 1] = fabsf(q.y);
    sh[o + 2] = fabsf(q.z);
    sh[o + 3] = fabsf(q.w);
  }
  __syncthreads();
  if (threadIdx.x >= kWave) return;
  const int l = threadIdx.x;
  const float* a = sh + l * (kLeaf + 1);  // lane l's leaf: banks l + c, conflict-free
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
#pragma unroll
  for (int i = 8; i < kLeaf; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  }
  float s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  // the tree above the leaves is balanced: a butterfly over the lanes (fp32 + is commutative)
#pragma unroll
  for (int m = 1; m < kWave; m <<= 1) {
    s += __shfl_xor(s, m);
    if (m == kChunk / kLeaf / 2 && (l & (kChunk / kLeaf - 1)) == 0)
      ws.q_abs[b * kQ + l / (kChunk / kLeaf)] = (double)s;  // 16-leaf subtree = one cdf chunk
  }
  if (l == 0) ws.buf_sum[b] = s;
}

// ---- K1b: the last, partial buffer (irregular tree), one thread ------------------------------------
__global__ __launch_bounds__(64) void ar_tail_sum_kernel(const float* __restrict__ x, int64_t n, ArWs ws) {
  __shared__ float sh[kBuf];
  const int64_t b = n / kBuf;
  const int len = (int)(n - b * kBuf);
  for (int i = threadIdx.x; i < len; i += 64) sh[i] = fabsf(x[b * kBuf + i]);
  __syncthreads();
  if (threadIdx.x != 0) return;
  ws.buf_sum[b] = pw_sum<8>(sh, len);
  for (int q = 0; q * kChunk < len; ++q) {
    double s = 0.0;
    const int hi = std::min(len, (q + 1) * kChunk);
    for (int i = q * kChunk; i < hi; ++i) s += (double)sh[i];
    ws.q_abs[b * kQ + q] = s;
  }
}

// ---- K2: S (buffers folded in order, fp32) and the chunk guesses (fp64 prefix of |x| / S) -----------
__global__ __launch_bounds__(1024) void ar_total_kernel(int64_t nbuf, int64_t nq, ArWs ws) {
  __shared__ float tile[1024];
  __shared__ double scan_lds[1024 / kWave];
  __shared__ float s_total;
  float S = 0.0f;
  for (int64_t base = 0; base < nbuf; base += 1024) {
    const int64_t i = base + threadIdx.x;
    tile[threadIdx.x] = i < nbuf ? ws.buf_sum[i] : 0.0f;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int cnt = (int)std::min<int64_t>(1024, nbuf - base);
      for (int j = 0; j < cnt; ++j) S = S + tile[j];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    s_total = S;
    ws.total[0] = S;
  }
  __syncthreads();
  const double inv = 1.0 / (double)s_total;
  double carry = 0.0;
  for (int64_t base = 0; base < nq; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const double v = i < nq ? ws.q_abs[i] : 0.0;
    double tot;
    const double ex = block_excl_scan<double, 1024 / kWave>(v, scan_lds, &tot);
    if (i < nq) ws.guess[i] = (carry + ex) * inv;
    carry += tot;
    __syncthreads();
  }
}

// ---- K3 (phase A): two speculative sequential runs per chunk, plus the chunk's sum of p -------------
__global__ __launch_bounds__(256) void ar_phase_a_kernel(const float* __restrict__ x, int64_t n, int64_t nq,
                                                         ArWs ws) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= nq) return;
  const float S = ws.total[0];
  const int64_t lo = j * kChunk;
  const int len = (int)std::min<int64_t>(kChunk, n - lo);
  const double ga = ws.guess[j];
  const double gb = ga + spacing(binade(ga));
  double ca = ga, cb = gb, ps = 0.0;
  const float* src = x + lo;
  if (len == kChunk) {
    for (int i = 0; i < kChunk; i += 4) {
      const float4 v = *reinterpret_cast<const float4*>(src + i);
      const double q0 = (double)(fabsf(v.x) / S), q1 = (double)(fabsf(v.y) / S);
      const double q2 = (double)(fabsf(v.z) / S), q3 = (double)(fabsf(v.w) / S);
      ca = ca + q0; cb = cb + q0;
      ca = ca + q1; cb = cb + q1;
      ca = ca + q2; cb = cb + q2;
      ca = ca + q3; cb = cb + q3;
      ps += (q0 + q1) + (q2 + q3);
    }
  } else {
    for (int i = 0; i < len; ++i) {
      const double q = (double)(fabsf(src[i]) / S);
      ca = ca + q;
      cb = cb + q;
      ps += q;
    }
  }
  ws.end_a[j] = ca;
  ws.end_b[j] = cb;
  ws.p_sum[j] = ps;
}

// ---- K4: numpy's checks on p (before any uniform is drawn) -------------------------------------------
__global__ __launch_bounds__(1024) void ar_check_kernel(int64_t nq, ArWs ws) {
  __shared__ double lds[1024 / kWave];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < nq; i += 1024) s += ws.p_sum[i];
  s = block_sum<double, 1024 / kWave>(s, lds);
  if (threadIdx.x == 0) {
    int st = 0;
    if (isnan(s)) st = kStNan;
    else if (!(fabs(s - 1.0) <= kAtol)) st = kStSum;
    ws.status[0] = st;
  }
}

// Sequential run of chunk j from an exact start (one thread).  The loads of 64 elements are issued
// together ahead of their dependent adds; with `u` (> -1) the run stops at the first element whose
// normalised running sum exceeds u and returns its index through *hit.
constexpr int kRun = 64;
__device__ double run_chunk(const float* __restrict__ x, int64_t n, int64_t j, double c, float S, double cD = 1.0,
                            double u = -1.0, int64_t* hit = nullptr) {
  const int64_t lo = j * kChunk;
  const int64_t hi = std::min<int64_t>(n, lo + kChunk);
  int64_t i = lo;
  for (; i + kRun <= hi; i += kRun) {
    float4 v[kRun / 4];
#pragma unroll
    for (int k = 0; k < kRun / 4; ++k) v[k] = *reinterpret_cast<const float4*>(x + i + 4 * k);
#pragma unroll
    for (int k = 0; k < kRun / 4; ++k) {
      const float e[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        c = c + (double)(fabsf(e[m]) / S);
        if (u > -1.0 && c / cD > u) {
          *hit = i + 4 * k + m;
          return c;
        }
      }
    }
  }
  for (; i < hi; ++i) {
    c = c + (double)(fabsf(x[i]) / S);
    if (u > -1.0 && c / cD > u) {
      *hit = i;
      return c;
    }
  }
  return c;
}

// ---- K5 (phase B + search): chain the chunks exactly, then searchsorted(u, side='right') ------------
__global__ __launch_bounds__(1024) void ar_select_kernel(const float* __restrict__ x, int64_t n, int64_t nq, double u,
                                                         ArWs ws, int64_t* __restrict__ index, float* __restrict__ out) {
  __shared__ double g_s[kRec], ea_s[kRec], eb_s[kRec];
  if (ws.status[0] != 0) return;  // the host raises numpy's ValueError; nothing is drawn or written
  const float S = ws.total[0];
  double t = 0.0;  // cumsum starts from 0: c_0 = 0 + p_0
  for (int64_t base = 0; base < nq; base += kRec) {
    const int64_t i = base + threadIdx.x;
    if (i < nq) {
      g_s[threadIdx.x] = ws.guess[i];
      ea_s[threadIdx.x] = ws.end_a[i];
      eb_s[threadIdx.x] = ws.end_b[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const int cnt = (int)std::min<int64_t>(kRec, nq - base);
      for (int r = 0; r < cnt; ++r) {
        const int64_t j = base + r;
        ws.start[j] = t;
        const double ga = g_s[r];
        const double d = t - ga;
        if (d == 0.0) {  // the speculated run IS the run
          t = ea_s[r];
          continue;
        }
        const int e = binade(ga);
        bool ok = e > 64 && binade(t) == e;  // then d is exact and a multiple of U (and d / U fits)
        double cand = 0.0;
        if (ok) {
          const double k = d * ldexp(1.0, 1075 - e);  // d / U, an exact integer
          const bool even = (((long long)k) & 1LL) == 0;
          const double g = even ? ga : ga + spacing(e);
          const double end = even ? ea_s[r] : eb_s[r];
          cand = end + (t - g);
          ok = binade(g) == e && binade(end) == e && binade(cand) == e;
        }
        t = ok ? cand : run_chunk(x, n, j, t, S);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  ws.start[nq] = t;
  const double cD = t;
  // first chunk whose last normalised cdf value exceeds u (the normalised cdf is non-decreasing)
  int64_t lo = 0, hi = nq - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi) / 2;
    const double end = mid + 1 < nq ? ws.start[mid + 1] : cD;
    if (end / cD > u) hi = mid;
    else lo = mid + 1;
  }
  int64_t ind = std::min<int64_t>(n, (lo + 1) * kChunk) - 1;  // cdf[-1] / cdf[-1] == 1 > u always qualifies
  (void)run_chunk(x, n, lo, ws.start[lo], S, cD, u, &ind);
  index[0] = ind;
  out[ind] = x[ind];
}

ArWs carve(void* base, int64_t n, size_t* bytes) {
  const int64_t nbuf = cdiv(n, kBuf), nq = cdiv(n, kChunk);
  Carver c(base, base ? ~size_t(0) : 0);
  ArWs w;
  w.buf_sum = c.take<float>(nbuf);
  w.q_abs = c.take<double>(nbuf * kQ);
  w.guess = c.take<double>(nq);
  w.end_a = c.take<double>(nq);
  w.end_b = c.take<double>(nq);
  w.p_sum = c.take<double>(nq);
  w.start = c.take<double>(nq + 1);
  w.total = c.take<float>(1);
  w.status = c.take<int32_t>(1);
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

int flc_adaptive_prepare(const float* x, int64_t n, int32_t* status, void* ws, size_t ws_bytes, void* stream) {
  if (!x || n <= 0 || n >= (int64_t(1) << 31) || !ws) return fail(FLC_EINVAL, "flc_adaptive_prepare: bad arguments");
  if (ws_bytes < flc_adaptive_workspace_size(n)) return fail(FLC_EWORKSPACE, "flc_adaptive_prepare: workspace too small");
  if (!aligned16(x)) return fail(FLC_EINVAL, "flc_adaptive_prepare: x must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  ArWs w = carve(ws, n, nullptr);
  const int64_t nfull = n / kBuf, nbuf = cdiv(n, kBuf), nq = cdiv(n, kChunk);
  if (nfull > 0)
    FLC_LAUNCH("adaptive_buffer_sum", ar_buffer_sum_kernel, dim3((unsigned)nfull), dim3(256), 0, st, x, nfull, w);
  if (nbuf > nfull) FLC_LAUNCH("adaptive_tail_sum", ar_tail_sum_kernel, dim3(1), dim3(64), 0, st, x, n, w);
  FLC_LAUNCH("adaptive_total", ar_total_kernel, dim3(1), dim3(1024), 0, st, nbuf, nq, w);
  FLC_LAUNCH("adaptive_phase_a", ar_phase_a_kernel, dim3((unsigned)cdiv(nq, 256)), dim3(256), 0, st, x, n, nq, w);
  FLC_LAUNCH("adaptive_check", ar_check_kernel, dim3(1), dim3(1024), 0, st, nq, w);
  if (status) FLC_CHECK_HIP(hipMemcpyAsync(status, w.status, sizeof(int32_t), hipMemcpyDeviceToDevice, st));
  return FLC_OK;
}

int flc_adaptive_select(const float* x, int64_t n, double u, int64_t* index, float* out, void* ws, size_t ws_bytes,
                        void* stream) {
  if (!x || n <= 0 || n >= (int64_t(1) << 31) || !ws || !index || !out || !(u >= 0.0 && u < 1.0))
    return fail(FLC_EINVAL, "flc_adaptive_select: bad arguments");
  if (ws_bytes < flc_adaptive_workspace_size(n)) return fail(FLC_EWORKSPACE, "flc_adaptive_select: workspace too small");
  hipStream_t st = as_stream(stream);
  ArWs w = carve(ws, n, nullptr);
  const int64_t nq = cdiv(n, kChunk);
  FLC_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)n * sizeof(float), st));
  FLC_LAUNCH("adaptive_select", ar_select_kernel, dim3(1), dim3(1024), 0, st, x, n, nq, u, w, index, out);
  return FLC_OK;
}

}  // extern "C"
