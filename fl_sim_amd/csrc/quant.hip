// quant.hip — dense stochastic quantizer codec for gfx950: standard / natural dithering
// (reference: fl_sim/compressors/compressors.py:327-365 and 367-404).
//
// Data layout in HBM: x is a [rows, d] fp32 batch (one client delta per row).  The wire is
//   norms[rows] fp32 + a flat packed code stream, BITS (2/4/8) bits per element, element i of the
//   flattened batch at bit offset i*BITS (little-endian), code = sign << (BITS-1) | level.
// Kernels (all HBM-streaming, no MFMA):
//   quant_norm     per-row max|x| (exact) or fp64 sum of squares; one partial per block, folded per row in a
//                  fixed order (quant_norm_fold, or inside the encode: flc_quant_encode_auto) -> deterministic.
//                  algorithmic bytes: 4 per element read.
//   quant_count    compat mode only: consumers (x != 0) per encode chunk, then one-block scan.
//   quant_encode   per element: y = fp32(|x| / norm), bracket [lv(s), lv(s+1)] found in fp64,
//                  p_down = (y - lv(s+1)) / (lv(s) - lv(s+1)) in fp64, level = u < p_down ? s : s+1.
//                  algorithmic bytes: 4 read + BITS/8 written per element.
//   quant_decode   v = fp32(fp32(lv) * sign) * norm, optionally fmaf-accumulated with a row weight.
//                  algorithmic bytes: BITS/8 read + 4 written (+4 read when accumulating).
// Each thread owns GROUP = 8 consecutive elements (two 16-B loads, one 2..8-B code store): a wave
// touches 2 KiB of x per step, fully coalesced.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kThreads = 256;
constexpr int kNW = kThreads / kWave;
constexpr int kGroup = 8;                  // elements per thread per step
constexpr int kGroupsPerBlock = 1024;      // 8192 elements per block (4 steps of 256 groups)
constexpr int kNormMaxParts = 1024;         // partial blocks per row for the norm
constexpr int kNormChunk = 4096;            // elements per norm block (16 per thread: the whole batch in flight)
constexpr int kRowSlots = 16;              // per-block LDS nnz slots

struct QuantWs {
  unsigned long long* err;       // [1] sticky error word: 4 = a fused launch's exchange timed out (flc_quant_status)
  unsigned long long* stamps;    // [2 * kMaxFused] fused launch: each block's max |x| bits of its (<= 2) rows, tagged
                                 // with the call (tag << 31 | max bits)
  unsigned long long* partials;  // [rows * kNormMaxParts]
  int* chunk_counts;             // [nblocks]  (compat)
  long long* chunk_offsets;      // [nblocks]  (compat)
};

QuantWs carve(void* ws, size_t bytes, int64_t rows, int64_t nblocks, size_t* need) {
  Carver c(ws, bytes);
  QuantWs w;
  w.err = c.take<unsigned long long>(1);
  w.stamps = c.take<unsigned long long>(2 * 1024);
  w.partials = c.take<unsigned long long>((size_t)rows * kNormMaxParts);
  w.chunk_counts = c.take<int>((size_t)nblocks);
  w.chunk_offsets = c.take<long long>((size_t)nblocks);
  *need = c.off;
  return w;
}

// ------------------------------------------------------------------------------------------------
// norm
// ------------------------------------------------------------------------------------------------
// fold of the per-block partials of a row in a fixed order (deterministic), by one wave (every lane gets it)
template <int NORM>
__device__ __forceinline__ float fold_row(int parts, const QuantWs& ws, int64_t row) {
  const int lane = threadIdx.x & (kWave - 1);
  const unsigned long long* pr = ws.partials + row * kNormMaxParts;
  if (NORM == FLC_NORM_INF) {
    uint32_t m = 0;
    for (int p = lane; p < parts; p += kWave) {
      const uint32_t v = (uint32_t)pr[p];
      m = v > m ? v : m;
    }
    return __uint_as_float(wave_max_u32(m));
  }
  double acc = 0.0;
  for (int p = lane; p < parts; p += kWave) acc += __longlong_as_double(pr[p]);
  return (float)sqrt(wave_sum(acc));
}

template <int NORM>
__global__ __launch_bounds__(kThreads) void quant_norm_kernel(const float* __restrict__ x, int64_t d,
                                                              int parts, int64_t chunk, int vec_ok,
                                                              QuantWs ws) {
  __shared__ unsigned long long s_red[kNW];
  const int row = blockIdx.y, part = blockIdx.x;
  const float* xr = x + (int64_t)row * d;
  const int64_t lo = (int64_t)part * chunk;
  const int64_t hi = lo + chunk < d ? lo + chunk : d;

  uint32_t mx = 0;
  double ss = 0.0;
  auto take = [&](float v) {
    if (NORM == FLC_NORM_INF) {
      const uint32_t a = __float_as_uint(v) & 0x7fffffffu;  // |v| bits; NaN > inf > finite
      mx = a > mx ? a : mx;
    } else {
      const double dv = (double)v;
      ss = fma(dv, dv, ss);
    }
  };
  if (vec_ok) {
    // x is 16-B aligned: a scalar head up to the next 16-B boundary of the flat batch, float4 body, scalar tail
    const int64_t flat_lo = (int64_t)row * d + lo;
    const int64_t head = std::min<int64_t>((4 - (flat_lo & 3)) & 3, hi - lo);
    if (threadIdx.x < head) take(xr[lo + threadIdx.x]);
    const float4* x4 = reinterpret_cast<const float4*>(xr + lo + head);
    const int64_t n4 = (hi - lo - head) >> 2;
    for (int64_t i = threadIdx.x; i < n4; i += kThreads) {
      const float4 v = x4[i];
      take(v.x); take(v.y); take(v.z); take(v.w);
    }
    for (int64_t i = lo + head + (n4 << 2) + threadIdx.x; i < hi; i += kThreads) take(xr[i]);
  } else {
    for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) take(xr[i]);
  }

  unsigned long long part_bits;
  if (NORM == FLC_NORM_INF) {
    uint32_t m = wave_max_u32(mx);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t r = 0;
      for (int w = 0; w < kNW; ++w) r = (uint32_t)s_red[w] > r ? (uint32_t)s_red[w] : r;
      s_red[0] = r;
    }
    __syncthreads();
    part_bits = s_red[0];
  } else {
    double s = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = __double_as_longlong(s);
    __syncthreads();
    if (threadIdx.x == 0) {
      double r = 0.0;
      for (int w = 0; w < kNW; ++w) r += __longlong_as_double(s_red[w]);
      s_red[0] = __double_as_longlong(r);
    }
    __syncthreads();
    part_bits = s_red[0];
  }

  if (threadIdx.x == 0) ws.partials[(int64_t)row * kNormMaxParts + part] = part_bits;
}

// fold of the partials in a separate launch (flc_quant_norm), one wave per row
template <int NORM>
__global__ __launch_bounds__(kWave) void quant_norm_fold_kernel(int parts, QuantWs ws, float* __restrict__ norms) {
  const float v = fold_row<NORM>(parts, ws, blockIdx.x);
  if (threadIdx.x == 0) norms[blockIdx.x] = v;
}

// ------------------------------------------------------------------------------------------------
// per-element quantizer
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool norm_regular(float nrm) { return nrm > 0.0f && nrm <= 3.402823466e38f; }

// consumer = the reference draws random.random() for this element (compressors.py:339-354)
__device__ __forceinline__ bool consumes(float xv, float nrm) {
  if (xv == 0.0f) return false;
  if (norm_regular(nrm)) return true;
  return !isnan(fabsf(xv) / nrm);
}

template <int KIND, int BITS>
__device__ __forceinline__ uint32_t quant_code(float xv, float nrm, int s, double step, double u) {
  if (xv == 0.0f) return 0u;
  if (!norm_regular(nrm)) return 1u;
  const float y = fabsf(xv) / nrm;  // IEEE fp32 division (compressors.py:344)
  const int lvl = dither_level<KIND>(y, s, step, u);  // compressors.py:346-353 (fp64 rule, exact)
  return ((__float_as_uint(xv) >> 31) << (BITS - 1)) | (uint32_t)lvl;
}

template <int KIND, int BITS>
__device__ __forceinline__ float dequant(uint32_t code, float nrm, int s, double step) {
  if (!norm_regular(nrm)) return code == 0u ? 0.0f : __uint_as_float(0x7fc00000u);
  const uint32_t lvl = code & ((1u << (BITS - 1)) - 1u);
  const float lv = (float)level_value<KIND>((int)lvl, s, step);
  const float sv = (code >> (BITS - 1)) ? -lv : lv;  // fp32(lv) * sign, -0 kept
  return sv * nrm;                                   // compressors.py:357
}

struct RowCursor {
  int64_t d;
  int64_t row, row_end;
  __device__ __forceinline__ void seek(int64_t e) {
    row = e / d;
    row_end = (row + 1) * d;
  }
  __device__ __forceinline__ int64_t at(int64_t e) {
    if (e >= row_end) seek(e);
    return row;
  }
};

__device__ __forceinline__ void load_group(const float* __restrict__ x, int64_t e0, int valid, float v[kGroup]) {
  if (valid == kGroup) {
    const float4 a = *reinterpret_cast<const float4*>(x + e0);
    const float4 b = *reinterpret_cast<const float4*>(x + e0 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < kGroup; ++j) v[j] = j < valid ? x[e0 + j] : 0.0f;
  }
}

template <int BITS>
__device__ __forceinline__ void store_codes(uint8_t* __restrict__ codes, int64_t e0, int valid, uint64_t packed) {
  constexpr int kBytes = kGroup * BITS / 8;
  uint8_t* dst = codes + (e0 * BITS) / 8;
  if (valid == kGroup) {
    if (kBytes == 8) *reinterpret_cast<uint2*>(dst) = make_uint2((uint32_t)packed, (uint32_t)(packed >> 32));
    else if (kBytes == 4) *reinterpret_cast<uint32_t*>(dst) = (uint32_t)packed;
    else *reinterpret_cast<uint16_t*>(dst) = (uint16_t)packed;
  } else {
    const int nb = (valid * BITS + 7) / 8;
    for (int b = 0; b < nb; ++b) dst[b] = (uint8_t)(packed >> (8 * b));
  }
}

template <int BITS>
__device__ __forceinline__ uint64_t load_codes(const uint8_t* __restrict__ codes, int64_t e0, int valid) {
  constexpr int kBytes = kGroup * BITS / 8;
  const uint8_t* src = codes + (e0 * BITS) / 8;
  if (valid == kGroup) {
    if (kBytes == 8) {
      const uint2 v = *reinterpret_cast<const uint2*>(src);
      return (uint64_t)v.x | ((uint64_t)v.y << 32);
    }
    if (kBytes == 4) return *reinterpret_cast<const uint32_t*>(src);
    return *reinterpret_cast<const uint16_t*>(src);
  }
  uint64_t p = 0;
  const int nb = (valid * BITS + 7) / 8;
  for (int b = 0; b < nb; ++b) p |= (uint64_t)src[b] << (8 * b);
  return p;
}

// consumers per encode chunk (compat mode)
__global__ __launch_bounds__(kThreads) void quant_count_kernel(const float* __restrict__ x, int64_t n, int64_t d,
                                                               const float* __restrict__ norms, QuantWs ws) {
  __shared__ int s_red[kNW];
  const int64_t g_begin = (int64_t)blockIdx.x * kGroupsPerBlock;
  RowCursor rc{d, 0, 0};
  rc.seek(g_begin * kGroup < n ? g_begin * kGroup : 0);
  int cnt = 0;
  for (int it = 0; it < kGroupsPerBlock / kThreads; ++it) {
    const int64_t g = g_begin + it * kThreads + threadIdx.x;
    const int64_t e0 = g * kGroup;
    if (e0 >= n) break;
    const int valid = n - e0 < kGroup ? (int)(n - e0) : kGroup;
    float v[kGroup];
    load_group(x, e0, valid, v);
#pragma unroll
    for (int j = 0; j < kGroup; ++j)
      if (j < valid) cnt += consumes(v[j], norms[rc.at(e0 + j)]) ? 1 : 0;
  }
  const int tot = block_sum<int, kNW>(cnt, s_red);
  if (threadIdx.x == 0) ws.chunk_counts[blockIdx.x] = tot;
}

// total consumers of a batch (norms == nullptr: x != 0)
__global__ __launch_bounds__(kThreads) void count_consumers_kernel(const float* __restrict__ x, int64_t n, int64_t d,
                                                                   const float* __restrict__ norms,
                                                                   unsigned long long* __restrict__ out) {
  __shared__ unsigned long long s_red[kNW];
  unsigned long long cnt = 0;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const float v = x[i];
    cnt += norms ? (consumes(v, norms[i / d]) ? 1 : 0) : (v != 0.0f ? 1 : 0);
  }
  const unsigned long long tot = block_sum<unsigned long long, kNW>(cnt, s_red);
  if (threadIdx.x == 0 && tot) atomicAdd(out, tot);
}

// exclusive scan of chunk counts (one block)
__global__ __launch_bounds__(1024) void chunk_scan_kernel(const int* __restrict__ counts, long long* __restrict__ offsets,
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
}

template <int KIND, int BITS, bool COMPAT, int GPB, bool DEC>
__global__ __launch_bounds__(kThreads) void quant_encode_kernel(
    const float* __restrict__ x, int64_t n, int64_t d, int s, double step, const float* __restrict__ norms,
    uint64_t seed, uint64_t counter, const double* __restrict__ compat_u, uint8_t* __restrict__ codes,
    long long* __restrict__ nnz, QuantWs ws, float* __restrict__ out) {
  __shared__ long long s_scan[kNW];
  __shared__ unsigned long long s_nnz[kRowSlots];
  const int64_t g_begin = (int64_t)blockIdx.x * GPB;
  const int64_t e_first = g_begin * kGroup;
  RowCursor rc{d, 0, 0};
  rc.seek(e_first);
  const int64_t row_base = rc.row;
  if (threadIdx.x < kRowSlots) s_nnz[threadIdx.x] = 0;
  __syncthreads();
  long long running = COMPAT ? ws.chunk_offsets[blockIdx.x] : 0;

  for (int it = 0; it < GPB / kThreads; ++it) {
    const int64_t g = g_begin + it * kThreads + threadIdx.x;
    const int64_t e0 = g * kGroup;
    const int valid = e0 >= n ? 0 : (n - e0 < kGroup ? (int)(n - e0) : kGroup);
    float v[kGroup];
    float nr[kGroup];
    int rl[kGroup];  // row of each element relative to the block's first row
    if (valid > 0) load_group(x, e0, valid, v);
#pragma unroll
    for (int j = 0; j < kGroup; ++j) {
      const int64_t r = (j < valid) ? rc.at(e0 + j) : rc.row;
      rl[j] = (int)(r - row_base);
      nr[j] = (j < valid) ? norms[r] : 1.0f;
    }

    double u[kGroup];
    if (COMPAT) {
      int c[kGroup];
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < kGroup; ++j) {
        c[j] = (j < valid && consumes(v[j], nr[j])) ? 1 : 0;
        cnt += c[j];
      }
      long long tot;
      const long long ex = block_excl_scan<long long, kNW>((long long)cnt, s_scan, &tot);
      long long r = running + ex;
#pragma unroll
      for (int j = 0; j < kGroup; ++j) {
        u[j] = c[j] ? compat_u[r] : 0.0;
        r += c[j];
      }
      running += tot;
    } else if (valid > 0) {
      const U4 a = philox_group((uint64_t)e0 >> 2, seed, counter);
      const U4 b = philox_group(((uint64_t)e0 >> 2) + 1, seed, counter);
      u[0] = u01(a.x); u[1] = u01(a.y); u[2] = u01(a.z); u[3] = u01(a.w);
      u[4] = u01(b.x); u[5] = u01(b.y); u[6] = u01(b.z); u[7] = u01(b.w);
    }
    if (valid == 0) continue;

    uint64_t packed = 0;
    float o[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; ++j) {
      if (j < valid) {
        const uint32_t c = quant_code<KIND, BITS>(v[j], nr[j], s, step, u[j]);
        packed |= (uint64_t)c << (j * BITS);
        if (DEC) o[j] = dequant<KIND, BITS>(c, nr[j], s, step);  // the decoder's value of this code
      }
    }
    store_codes<BITS>(codes, e0, valid, packed);
    if (DEC) {
      if (valid == kGroup) {
        *reinterpret_cast<float4*>(out + e0) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(out + e0 + 4) = make_float4(o[4], o[5], o[6], o[7]);
      } else {
        for (int j = 0; j < valid; ++j) out[e0 + j] = o[j];
      }
    }

    if (nnz) {
      // rows of this group: at most a few; count nonzeros per row into LDS slots
#pragma unroll
      for (int j = 0; j < kGroup; ++j) {
        if (j < valid && v[j] != 0.0f) {
          const int r = rl[j];
          if (r < kRowSlots) atomicAdd(&s_nnz[r], 1ull);
          else atomicAdd(reinterpret_cast<unsigned long long*>(&nnz[r + row_base]), 1ull);
        }
      }
    }
  }
  if (nnz) {
    __syncthreads();
    if (threadIdx.x < kRowSlots && s_nnz[threadIdx.x] != 0)
      atomicAdd(reinterpret_cast<unsigned long long*>(&nnz[row_base + threadIdx.x]), s_nnz[threadIdx.x]);
  }
}

// One group of 8 elements (flat index e0, `valid` of them real) in Philox mode: the common case — a full group inside
// one row — takes one norm lookup and, for standard dithering, a branch-light fp32 level decision; groups straddling a
// row boundary or the end take the per-element path.  norm_of(r): row r's norm; nnz_add(r, count) when counting.
// DEC also writes the decoded values (flc_quant_encode_decode).
// the group's 8 Philox words (element e: word e & 3 of counter group e >> 2)
__device__ __forceinline__ void group_words(int64_t e0, uint64_t seed, uint64_t counter, uint32_t (&wd)[kGroup]) {
  const U4 a = philox_group((uint64_t)e0 >> 2, seed, counter);
  const U4 b = philox_group(((uint64_t)e0 >> 2) + 1, seed, counter);
  wd[0] = a.x; wd[1] = a.y; wd[2] = a.z; wd[3] = a.w;
  wd[4] = b.x; wd[5] = b.y; wd[6] = b.z; wd[7] = b.w;
}

template <int KIND, int BITS, bool DEC, class NormOf, class NnzAdd>
__device__ __forceinline__ void philox_group_encode(const float (&v)[kGroup], const uint32_t (&wd)[kGroup], int64_t e0,
                                                    int valid, int64_t d, int s, double step,
                                                    uint8_t* __restrict__ codes, float* __restrict__ out, bool count,
                                                    NormOf norm_of, NnzAdd nnz_add, bool nt = false,
                                                    const float* lvt = nullptr) {
  const int64_t r0 = e0 / d;
  const int64_t r_end = (r0 + 1) * d;
  uint64_t packed = 0;
  float o[kGroup];
  const bool whole = valid == kGroup && e0 + kGroup <= r_end;
  const float nr0 = whole ? norm_of(r0) : 0.0f;
  if (KIND == 0 && whole && norm_regular(nr0)) {
    // standard dithering, branch-light: an fp32 decision for all 8 elements, then the exact fp64 rule for the rare
    // elements its margins do not decide (whole-wave branch).  No division: t' = |x| * fp32(s / norm) is within
    // 2^-23 t <= 1.6e-5 of s|x|/norm, and the reference's t = fp32(|x| / norm) * s within 7.6e-6 of it, so
    // |t' - t| < 2.4e-5 and the same holds for p = ceil(t) - t (the subtraction is exact); u in fp32 straight
    // from the Philox word is within 6e-8 of u.  Margins 1e-4 (bracket) and 5e-5 (u vs p) cover that.
    const float rs = (float)s / nr0;
    uint32_t lvl[kGroup];
    uint32_t slow = 0;
#pragma unroll
    for (int j = 0; j < kGroup; ++j) {
      const float t = fabsf(v[j]) * rs;
      const float jf = ceilf(t);
      const float pf = jf - t;
      const float uf = (float)wd[j] * 2.3283064365386963e-10f;
      const bool ok = (pf > 1e-4f) & (t - (jf - 1.0f) > 1e-4f) & (fabsf(uf - pf) > 5e-5f);
      lvl[j] = (uint32_t)(int)jf - (uf < pf ? 1u : 0u);
      slow |= (uint32_t)(!ok && v[j] != 0.0f) << j;
    }
    if (slow) {
#pragma unroll
      for (int j = 0; j < kGroup; ++j)
        if ((slow >> j) & 1u) lvl[j] = (uint32_t)dither_level<0>(fabsf(v[j]) / nr0, s, step, u01(wd[j]));
    }
#pragma unroll
    for (int j = 0; j < kGroup; ++j) {
      const uint32_t c = v[j] == 0.0f ? 0u : (((__float_as_uint(v[j]) >> 31) << (BITS - 1)) | lvl[j]);
      packed |= (uint64_t)c << (j * BITS);
      if (DEC) {
        if (lvt) {  // fp32(level value) from the block's LDS table: dequant's (float)(i * step) without the fp64 work
          const float lv = lvt[c & ((1u << (BITS - 1)) - 1u)];
          o[j] = ((c >> (BITS - 1)) ? -lv : lv) * nr0;
        } else {
          o[j] = dequant<KIND, BITS>(c, nr0, s, step);
        }
      }
    }
  } else if (whole) {
#pragma unroll
    for (int j = 0; j < kGroup; ++j) {
      const uint32_t c = quant_code<KIND, BITS>(v[j], nr0, s, step, u01(wd[j]));
      packed |= (uint64_t)c << (j * BITS);
      if (DEC) o[j] = dequant<KIND, BITS>(c, nr0, s, step);
    }
  } else {
    for (int j = 0; j < valid; ++j) {
      const int64_t r = (e0 + j) / d;
      const float nr = norm_of(r);
      const uint32_t c = quant_code<KIND, BITS>(v[j], nr, s, step, u01(wd[j]));
      packed |= (uint64_t)c << (j * BITS);
      if (DEC) o[j] = dequant<KIND, BITS>(c, nr, s, step);
      if (count && v[j] != 0.0f) nnz_add(r, 1);
    }
  }
  if (count && whole) {
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < kGroup; ++j) cnt += v[j] != 0.0f;
    if (cnt) nnz_add(r0, cnt);
  }
  if (nt && BITS == 8 && valid == kGroup) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    u32x2 t = {(uint32_t)packed, (uint32_t)(packed >> 32)};
    __builtin_nontemporal_store(t, reinterpret_cast<u32x2*>(codes + e0));
  } else {
    store_codes<BITS>(codes, e0, valid, packed);
  }
  if (DEC) {
    if (valid == kGroup && nt) {
      st_stream(out + e0, make_float4(o[0], o[1], o[2], o[3]));
      st_stream(out + e0 + 4, make_float4(o[4], o[5], o[6], o[7]));
    } else if (valid == kGroup) {
      *reinterpret_cast<float4*>(out + e0) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(out + e0 + 4) = make_float4(o[4], o[5], o[6], o[7]);
    } else {
      for (int j = 0; j < valid; ++j) out[e0 + j] = o[j];
    }
  }
}

// Philox mode, one group of 8 elements per thread (every wave's loads in flight at once: a small batch fills the chip).
// FOLD (FLC_NORM_INF / FLC_NORM_L2 + 1; 0 = norms given): the block folds the norm partials of its rows itself
// (d >= the block's span, so at most two rows) and the block holding a row's first element writes norms[row].
template <int KIND, int BITS, bool DEC, int FOLD>
__global__ __launch_bounds__(kThreads) void quant_encode_philox_kernel(
    const float* __restrict__ x, int64_t n, int64_t d, int s, double step, float* __restrict__ norms, uint64_t seed,
    uint64_t counter, uint8_t* __restrict__ codes, long long* __restrict__ nnz, float* __restrict__ out, QuantWs ws,
    int parts) {
  __shared__ unsigned long long s_nnz[kRowSlots];
  __shared__ float s_norm[2];
  const int64_t b0 = (int64_t)blockIdx.x * kThreads * kGroup;
  const int64_t row_base = b0 / d;
  if (nnz && threadIdx.x < kRowSlots) s_nnz[threadIdx.x] = 0;
  if (FOLD && threadIdx.x < kWave) {
    const int64_t rows = (n + d - 1) / d;
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int64_t r = row_base + rr;
      if (r < rows && r * d < b0 + kThreads * kGroup) {
        const float v = fold_row<FOLD - 1>(parts, ws, r);
        if (threadIdx.x == 0) {
          s_norm[rr] = v;
          if (r * d >= b0) norms[r] = v;
        }
      }
    }
  }
  if (nnz || FOLD) __syncthreads();
  const int64_t e0 = b0 + (int64_t)threadIdx.x * kGroup;
  if (e0 < n) {
    const int valid = n - e0 < kGroup ? (int)(n - e0) : kGroup;
    float v[kGroup];
    load_group(x, e0, valid, v);
    uint32_t wd[kGroup];
    group_words(e0, seed, counter, wd);
    philox_group_encode<KIND, BITS, DEC>(
        v, wd, e0, valid, d, s, step, codes, out, nnz != nullptr,
        [&](int64_t r) { return FOLD ? s_norm[r - row_base] : norms[r]; },
        [&](int64_t r, int cnt) {
          const int rl = (int)(r - row_base);
          if (rl < kRowSlots) atomicAdd(&s_nnz[rl], (unsigned long long)cnt);
          else atomicAdd(reinterpret_cast<unsigned long long*>(&nnz[r]), (unsigned long long)cnt);
        });
  }
  if (nnz) {
    __syncthreads();
    if (threadIdx.x < kRowSlots && s_nnz[threadIdx.x] != 0)
      atomicAdd(reinterpret_cast<unsigned long long*>(&nnz[row_base + threadIdx.x]), s_nnz[threadIdx.x]);
  }
}

// ------------------------------------------------------------------------------------------------
// configs[1] in one launch (flc_quant_encode_auto with p = inf, Philox): one 1024-thread block per CU, block b owning
// the flat span [b SPAN, (b + 1) SPAN) of the batch (SPAN = 8192 GPT elements, d >= SPAN: at most two rows per block).
// Each thread loads its GPT groups of 8 (coalesced: group j of thread t at (j * 1024 + t) * 8) and keeps them in
// registers; the block's max |x| of each of its rows goes to its own two workspace slots, tagged with the call; then
// every block polls and folds its rows' maxima over the blocks that hold them (a contiguous range: one wave's coherent
// loads, repeated until every tag is this call's) and encodes (+ decodes) from the registers.  x is read once, the codes and the decoded batch written once: 9 B/element
// in one launch, bit-identical to the two-launch form (max is exact in any order; same Philox words, same rule).
// ------------------------------------------------------------------------------------------------
constexpr int kFT = 1024;
constexpr int kMaxFused = 1024;  // blocks (stamp words: 2 each)

// The exchange carries its payload in its flags: each block publishes the max |x| bits of its two row slots as two
// 64-bit words tagged with the call (tag << 31 | bits), one agent-scope atomic store each (write-through to the
// coherent level; no release / acquire fence, which on gfx950 writes back / invalidates the whole L2 — measured 6-8 us
// over 510 blocks, quant.hip's dropped ticket fold).  A reader polls only the words of the blocks that hold its rows,
// until every tag is this call's: one round trip for flag and payload, and a block waits for its row neighbours, not
// for the slowest block of the grid.  Tags are 33 bits, never 0 (a fresh workspace's words), equal to a stale word's
// only if that word was last written 2^33 - 1 calls earlier.
__device__ __forceinline__ unsigned long long stamp_word(unsigned long long tag, uint32_t bits) {
  return (tag << 31) | bits;
}

// wave-wide: the max of slot words [c0, c1] of row r (slot: the row is block c's first or second), polled until every
// word carries `tag`; every lane gets the result.  Spins are bounded: a block that never arrived (lost co-residency)
// sets the sticky error word and the launch drains.
__device__ __forceinline__ uint32_t row_max_polled(const QuantWs& ws, int64_t r, int64_t d, int64_t SPAN, int64_t c0,
                                                   int64_t c1, unsigned long long tag, bool poll) {
  const int lane = threadIdx.x & (kWave - 1);
  uint32_t m = 0;
  for (int64_t cb = c0; cb <= c1; cb += kWave) {  // (uniform)
    const int64_t c = cb + lane;
    const bool mine = c <= c1;
    const int slot = mine && (c * SPAN) / d != r ? 1 : 0;
    const unsigned long long* wp = ws.stamps + 2 * (mine ? c : c0) + slot;
    unsigned long long v = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (poll && __ballot(mine && (v >> 31) != tag) != 0ull) {
      __builtin_amdgcn_s_sleep(1);
      if (mine && (v >> 31) != tag) v = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (++spins > (1u << 22)) {  // ~1 s
        if (lane == 0) __hip_atomic_fetch_or(ws.err, 4ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    const uint32_t b = mine ? (uint32_t)(v & 0x7fffffffu) : 0u;
    m = b > m ? b : m;
  }
  return wave_max_u32(m);
}

template <int KIND, int BITS, bool DEC, int GPT>
__global__ __launch_bounds__(kFT) void quant_fused_kernel(const float* __restrict__ x, int64_t n, int64_t d, int s,
                                                          double step, float* __restrict__ norms, uint64_t seed,
                                                          uint64_t counter, uint8_t* __restrict__ codes,
                                                          long long* __restrict__ nnz, float* __restrict__ out,
                                                          QuantWs ws, unsigned long long tag, int cal) {
  constexpr int64_t SPAN = (int64_t)kFT * kGroup * GPT;
  __shared__ uint32_t s_m[2][kFT / kWave];
  __shared__ float s_norm[2];
  __shared__ unsigned long long s_nnz[2];
  __shared__ float s_lvt[128];  // standard dithering: fp32 level values (dequant's (float)level_value), s <= 127
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * SPAN;
  const int64_t r0 = base / d, rb = (r0 + 1) * d, rows = (n + d - 1) / d;
  float v[GPT][kGroup];
  uint32_t m0 = 0, m1 = 0;
#pragma unroll
  for (int g = 0; g < GPT; ++g) {
    const int64_t e0 = base + ((int64_t)g * kFT + tid) * kGroup;
    const int valid = e0 >= n ? 0 : (n - e0 < kGroup ? (int)(n - e0) : kGroup);
    if (valid == kGroup) {
      load_group(x, e0, kGroup, v[g]);
    } else {
#pragma unroll
      for (int j = 0; j < kGroup; ++j) v[g][j] = j < valid ? x[e0 + j] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < kGroup; ++j) {
      const uint32_t a = __float_as_uint(v[g][j]) & 0x7fffffffu;  // |v| bits; NaN > inf > finite
      if (e0 + j < rb) m0 = a > m0 ? a : m0;
      else m1 = a > m1 ? a : m1;
    }
  }
  m0 = wave_max_u32(m0);
  m1 = wave_max_u32(m1);
  if (lane == 0) {
    s_m[0][wid] = m0;
    s_m[1][wid] = m1;
  }
  if (tid < 2) s_nnz[tid] = 0ull;
  __syncthreads();
  if (tid < 2) {  // slot 0: row r0, slot 1: row r0 + 1 (0 when the block holds none of it)
    uint32_t m = 0;
    for (int w = 0; w < kFT / kWave; ++w) m = s_m[tid][w] > m ? s_m[tid][w] : m;
    __hip_atomic_store(ws.stamps + 2 * blockIdx.x + tid, stamp_word(tag, m), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  // The Philox words and the level table do not depend on the norm: computed after this block's words are out and
  // before its poll, so that they fill the wait for the row's slowest block instead of delaying this block's words
  // (GPT = 2; at 4 they would not fit the registers).  (Computed under the x loads instead: no faster.)
  constexpr bool kPre = GPT <= 2;
  uint32_t wd[kPre ? GPT : 1][kGroup];
  if constexpr (kPre) {
#pragma unroll
    for (int g = 0; g < GPT; ++g) group_words(base + ((int64_t)g * kFT + tid) * kGroup, seed, counter, wd[g]);
  }
  if (KIND == 0 && tid <= s) s_lvt[tid] = (float)level_value<0>(tid, s, step);
  // waves 0 and 1: the max of row r0 + wid over the blocks holding it (row r0 + 1 only when this block holds some of it)
  if (wid < 2 && r0 + wid < rows && (wid == 0 || rb < base + SPAN)) {
    {
      const int rr = wid;
      const int64_t r = r0 + rr;
      const int64_t c0 = r * d / SPAN, c1 = ((r + 1) * d - 1) / SPAN < (int64_t)gridDim.x - 1
                                               ? ((r + 1) * d - 1) / SPAN
                                               : (int64_t)gridDim.x - 1;
      const uint32_t m = row_max_polled(ws, r, d, SPAN, c0, c1, tag, !(cal & 2));
      if (lane == 0) {
        s_norm[rr] = __uint_as_float(m);
        if (r * d >= base && r * d < base + SPAN) norms[r] = __uint_as_float(m);  // the block holding its 1st element
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < GPT; ++g) {
    const int64_t e0 = base + ((int64_t)g * kFT + tid) * kGroup;
    if (e0 < n) {
      const int valid = n - e0 < kGroup ? (int)(n - e0) : kGroup;
      if (cal & 4) {  // calibration: the memory traffic alone (x copied to out, zero codes)
        if (valid == kGroup) {
          store_codes<BITS>(codes, e0, valid, 0ull);
          if (DEC) {
            *reinterpret_cast<float4*>(out + e0) = make_float4(v[g][0], v[g][1], v[g][2], v[g][3]);
            *reinterpret_cast<float4*>(out + e0 + 4) = make_float4(v[g][4], v[g][5], v[g][6], v[g][7]);
          }
        }
        continue;
      }
      if constexpr (!kPre) group_words(e0, seed, counter, wd[0]);
      philox_group_encode<KIND, BITS, DEC>(
          v[g], wd[kPre ? g : 0], e0, valid, d, s, step, codes, out, nnz != nullptr,
          [&](int64_t r) { return s_norm[r - r0]; },
          [&](int64_t r, int cnt) { atomicAdd(&s_nnz[r - r0], (unsigned long long)cnt); }, cal & 1,
          KIND == 0 ? s_lvt : nullptr);
    }
  }
  if (nnz) {
    __syncthreads();
    if (tid < 2 && s_nnz[tid] != 0)
      atomicAdd(reinterpret_cast<unsigned long long*>(&nnz[r0 + tid]), s_nnz[tid]);
  }
}

template <int KIND, int BITS, bool ACC>
__global__ __launch_bounds__(kThreads) void quant_decode_kernel(const uint8_t* __restrict__ codes, int64_t n, int64_t d,
                                                                int s, double step, const float* __restrict__ norms,
                                                                const float* __restrict__ row_w, float* __restrict__ out) {
  const int64_t ngroups = (n + kGroup - 1) / kGroup;
  for (int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x; g < ngroups; g += (int64_t)gridDim.x * kThreads) {
    const int64_t e0 = g * kGroup;
    const int valid = n - e0 < kGroup ? (int)(n - e0) : kGroup;
    RowCursor rc{d, 0, 0};
    rc.seek(e0);
    const uint64_t packed = load_codes<BITS>(codes, e0, valid);
    float o[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; ++j) {
      const int64_t r = rc.at(e0 + j < n ? e0 + j : e0);
      const float val = dequant<KIND, BITS>((uint32_t)(packed >> (j * BITS)) & ((1u << BITS) - 1u), norms[r], s, step);
      o[j] = (!ACC && row_w) ? row_w[r] * val : val;
    }
    if (ACC) {
      float prev[kGroup];
      load_group(out, e0, valid, prev);
      rc.seek(e0);
#pragma unroll
      for (int j = 0; j < kGroup; ++j) {
        const int64_t r = rc.at(e0 + j < n ? e0 + j : e0);
        o[j] = fmaf(row_w ? row_w[r] : 1.0f, o[j], prev[j]);
      }
    }
    if (valid == kGroup) {
      *reinterpret_cast<float4*>(out + e0) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(out + e0 + 4) = make_float4(o[4], o[5], o[6], o[7]);
    } else {
      for (int j = 0; j < valid; ++j) out[e0 + j] = o[j];
    }
  }
}

int check_quant_args(int kind, int levels, int bits) {
  if (kind != FLC_Q_STANDARD_DITHER && kind != FLC_Q_NATURAL_DITHER)
    return fail(FLC_EINVAL, "quant: unknown kind %d", kind);
  if (bits != 2 && bits != 4 && bits != 8) return fail(FLC_EINVAL, "quant: bits must be 2, 4 or 8 (got %d)", bits);
  if (levels < 1 || levels > (1 << (bits - 1)) - 1)
    return fail(FLC_EINVAL, "quant: levels %d does not fit %d-bit codes", levels, bits);
  return FLC_OK;
}

double level_step(int levels) { return 1.0 / (double)levels; }

// the one-launch encode's exchange tags: process-wide, 33 bits, never 0 (a fresh workspace's words); a word left by an
// earlier call (of any shape, on any workspace) carries another tag unless it is 2^33 - 1 calls old
unsigned long long next_tag() {
  static std::atomic<unsigned long long> calls{0};
  return (calls++ % ((1ull << 33) - 1)) + 1;
}

template <int KIND, int BITS, bool DEC>
int launch_encode(const float* x, int64_t n, int64_t d, int levels, const float* norms, uint64_t seed, uint64_t counter,
                  const double* compat_u, uint8_t* codes, int64_t* nnz, const QuantWs& w, int64_t nblocks,
                  float* out, hipStream_t st) {
  const char* name = DEC ? "quant_encode_decode" : "quant_encode";
  const double step = level_step(levels);
  long long* nz = reinterpret_cast<long long*>(nnz);
  if (compat_u) {
    FLC_LAUNCH(DEC ? "quant_count" : "quant_count", quant_count_kernel, dim3((unsigned)nblocks), dim3(kThreads), 0, st, x, n, d, norms, w);
    FLC_LAUNCH("quant_chunk_scan", chunk_scan_kernel, dim3(1), dim3(1024), 0, st, w.chunk_counts, w.chunk_offsets,
               nblocks);
    FLC_LAUNCH(name, (quant_encode_kernel<KIND, BITS, true, kGroupsPerBlock, DEC>), dim3((unsigned)nblocks),
               dim3(kThreads), 0, st, x, n, d, levels, step, norms, seed, counter, compat_u, codes, nz, w, out);
  } else {
    // philox: one group per thread, so every wave's loads are in flight at once (a small batch fills the chip)
    const int64_t nb1 = cdiv(n, (int64_t)kGroup * kThreads);
    FLC_LAUNCH(name, (quant_encode_philox_kernel<KIND, BITS, DEC, 0>), dim3((unsigned)nb1), dim3(kThreads), 0, st, x,
               n, d, levels, step, const_cast<float*>(norms), seed, counter, codes, nz, out, w, 0);
  }
  return FLC_OK;
}

template <int KIND, int BITS>
int launch_decode(const uint8_t* codes, int64_t n, int64_t d, int levels, const float* norms, const float* row_w,
                  int acc, float* out, hipStream_t st) {
  const double step = level_step(levels);
  const int64_t ngroups = cdiv(n, kGroup);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(ngroups, kThreads), 256 * 32);
  if (acc)
    FLC_LAUNCH("quant_decode", (quant_decode_kernel<KIND, BITS, true>), dim3(grid), dim3(kThreads), 0, st, codes, n, d,
               levels, step, norms, row_w, out);
  else
    FLC_LAUNCH("quant_decode", (quant_decode_kernel<KIND, BITS, false>), dim3(grid), dim3(kThreads), 0, st, codes, n,
               d, levels, step, norms, row_w, out);
  return FLC_OK;
}

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

int flc_quant_status(void* ws, uint64_t* err_out, int reset, void* stream) {
  if (!ws || !err_out) return fail(FLC_EINVAL, "flc_quant_status: null workspace or output");
  hipStream_t st = as_stream(stream);
  FLC_CHECK_HIP(hipMemcpyAsync(err_out, ws, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));  // QuantWs::err
  if (reset) FLC_CHECK_HIP(hipMemsetAsync(ws, 0, sizeof(uint64_t), st));
  return FLC_OK;
}

size_t flc_quant_workspace_size(int64_t rows, int64_t d) {
  size_t need = 0;
  const int64_t nblocks = cdiv(rows * d, (int64_t)kGroup * kGroupsPerBlock);
  (void)carve(nullptr, 0, rows, nblocks < 1 ? 1 : nblocks, &need);
  return need;
}

int flc_quant_norm(const float* x, int64_t rows, int64_t d, int norm_p, float* norms, void* ws, size_t ws_bytes,
                   void* stream) {
  if (rows <= 0 || d <= 0 || !x || !norms) return fail(FLC_EINVAL, "flc_quant_norm: bad arguments");
  if (rows > 65535) return fail(FLC_EINVAL, "flc_quant_norm: at most 65535 rows per call");
  if (norm_p != FLC_NORM_INF && norm_p != FLC_NORM_L2) return fail(FLC_EINVAL, "flc_quant_norm: p must be inf(0) or 2");
  size_t need = 0;
  const int64_t nblocks = cdiv(rows * d, (int64_t)kGroup * kGroupsPerBlock);
  QuantWs w = carve(ws, ws_bytes, rows, nblocks < 1 ? 1 : nblocks, &need);
  if (need > ws_bytes || !ws) return fail(FLC_EWORKSPACE, "flc_quant_norm: workspace %zu < %zu", ws_bytes, need);
  int64_t parts = cdiv(d, kNormChunk);
  if (parts > kNormMaxParts) parts = kNormMaxParts;
  int64_t chunk = align_up((size_t)cdiv(d, parts), 4);
  parts = cdiv(d, chunk);
  const int vec_ok = aligned16(x);
  hipStream_t st = as_stream(stream);
  if (norm_p == FLC_NORM_INF) {
    FLC_LAUNCH("quant_norm", quant_norm_kernel<FLC_NORM_INF>, dim3((unsigned)parts, (unsigned)rows), dim3(kThreads), 0,
               st, x, d, (int)parts, chunk, vec_ok, w);
    FLC_LAUNCH("quant_norm_fold", quant_norm_fold_kernel<FLC_NORM_INF>, dim3((unsigned)rows), dim3(kWave), 0, st,
               (int)parts, w, norms);
  } else {
    FLC_LAUNCH("quant_norm", quant_norm_kernel<FLC_NORM_L2>, dim3((unsigned)parts, (unsigned)rows), dim3(kThreads), 0,
               st, x, d, (int)parts, chunk, vec_ok, w);
    FLC_LAUNCH("quant_norm_fold", quant_norm_fold_kernel<FLC_NORM_L2>, dim3((unsigned)rows), dim3(kWave), 0, st,
               (int)parts, w, norms);
  }
  return FLC_OK;
}

}  // extern "C"

namespace flc {
namespace {
int quant_encode_entry(const float* x, int64_t rows, int64_t d, int kind, int levels, int bits, const float* norms,
                       uint64_t seed, uint64_t counter, const double* compat_u, uint8_t* codes, int64_t* nnz,
                       float* out, void* ws, size_t ws_bytes, void* stream, const char* who) {
  if (rows <= 0 || d <= 0 || !x || !norms || !codes) return fail(FLC_EINVAL, "%s: bad arguments", who);
  if (int rc = check_quant_args(kind, levels, bits)) return rc;
  if (!aligned16(x) || !aligned16(codes) || (out && !aligned16(out)))
    return fail(FLC_EINVAL, "%s: x, codes and out must be 16-B aligned", who);
  const int64_t n = rows * d;
  const int64_t nblocks = cdiv(n, (int64_t)kGroup * kGroupsPerBlock);
  size_t need = 0;
  QuantWs w = carve(ws, ws_bytes, rows, nblocks, &need);
  if (need > ws_bytes || !ws) return fail(FLC_EWORKSPACE, "%s: workspace %zu < %zu", who, ws_bytes, need);
  hipStream_t st = as_stream(stream);
  if (nnz) FLC_CHECK_HIP(hipMemsetAsync(nnz, 0, (size_t)rows * sizeof(int64_t), st));
#define FLC_ENC(K, B)                                                                                              \
  return out ? launch_encode<K, B, true>(x, n, d, levels, norms, seed, counter, compat_u, codes, nnz, w, nblocks, out, st) \
             : launch_encode<K, B, false>(x, n, d, levels, norms, seed, counter, compat_u, codes, nnz, w, nblocks, out, st)
  if (kind == FLC_Q_STANDARD_DITHER) {
    if (bits == 8) FLC_ENC(0, 8);
    if (bits == 4) FLC_ENC(0, 4);
    FLC_ENC(0, 2);
  } else {
    if (bits == 8) FLC_ENC(1, 8);
    if (bits == 4) FLC_ENC(1, 4);
    FLC_ENC(1, 2);
  }
#undef FLC_ENC
}
// norm partials -> (fold) -> philox encode (+ decode), norms written by the encode
template <int KIND, int BITS, bool DEC>
int launch_auto(const float* x, int64_t rows, int64_t d, int levels, int norm_p, uint64_t seed, uint64_t counter,
                uint8_t* codes, float* norms, int64_t* nnz, float* out, const QuantWs& w, hipStream_t st) {
  const int64_t n = rows * d;
  int64_t parts = std::min<int64_t>(cdiv(d, kNormChunk), kNormMaxParts);
  const int64_t chunk = align_up((size_t)cdiv(d, parts), 4);
  parts = cdiv(d, chunk);
  const int vec_ok = aligned16(x);
  const bool fold_in = d >= (int64_t)kThreads * kGroup;  // a block spans at most two rows
  const double step = level_step(levels);
  const int64_t nb1 = cdiv(n, (int64_t)kGroup * kThreads);
  long long* nz = reinterpret_cast<long long*>(nnz);
  const char* name = DEC ? "quant_encode_decode" : "quant_encode";
  // Under stream capture the two-launch path: the one-launch encode's exchange tag is made on the host per call, and
  // a captured graph replays the same tag, so a word left by the previous replay (right tag, stale row maximum) would
  // pass the check; the co-residency gate is off under capture as well.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  FLC_CHECK_HIP(hipStreamIsCapturing(st, &cap));
  if (norm_p == FLC_NORM_INF && cap == hipStreamCaptureStatusNone && !getenv("FLC_QUANT_TWO_LAUNCH")) {
    // one launch when the batch fits one 1024-thread block per CU with at most two rows per block (configs[1])
    int dev = 0;
    const int cus = std::min(stream_cus(st, &dev), kMaxFused);
    const int gpt = (d >= 2 * kFT * kGroup && n <= (int64_t)cus * 2 * kFT * kGroup)   ? 2
                    : (d >= 4 * kFT * kGroup && n <= (int64_t)cus * 4 * kFT * kGroup) ? 4
                                                                                        : 0;
    if (gpt) {
      const unsigned long long ep = next_tag();
      const unsigned grid = (unsigned)cdiv(n, (int64_t)gpt * kFT * kGroup);
      const char* fname = DEC ? "quant_fused_encode_decode" : "quant_fused_encode";
#ifdef FLC_CALIB  // calibration builds (tools/quant_cal_probe.py): 1 non-temporal stores, 2 no exchange, 4 traffic only
      const int cal = getenv("FLC_QUANT_CAL") ? atoi(getenv("FLC_QUANT_CAL")) : 0;
#else
      constexpr int cal = 0;
#endif
      Coresident co(st, dev);
      if (co.status()) return co.status();
      if (gpt == 2)
        FLC_LAUNCH_CO(co, fname, (quant_fused_kernel<KIND, BITS, DEC, 2>), dim3(grid), dim3(kFT), 0, st, x, n, d, levels, step,
                   norms, seed, counter, codes, nz, out, w, ep, cal);
      else
        FLC_LAUNCH_CO(co, fname, (quant_fused_kernel<KIND, BITS, DEC, 4>), dim3(grid), dim3(kFT), 0, st, x, n, d, levels, step,
                   norms, seed, counter, codes, nz, out, w, ep, cal);
      return co.finish();
    }
  }
  if (norm_p == FLC_NORM_INF) {
    FLC_LAUNCH("quant_norm", quant_norm_kernel<FLC_NORM_INF>, dim3((unsigned)parts, (unsigned)rows), dim3(kThreads), 0,
               st, x, d, (int)parts, chunk, vec_ok, w);
    if (fold_in) {
      FLC_LAUNCH(name, (quant_encode_philox_kernel<KIND, BITS, DEC, FLC_NORM_INF + 1>), dim3((unsigned)nb1),
                 dim3(kThreads), 0, st, x, n, d, levels, step, norms, seed, counter, codes, nz, out, w, (int)parts);
      return FLC_OK;
    }
    FLC_LAUNCH("quant_norm_fold", quant_norm_fold_kernel<FLC_NORM_INF>, dim3((unsigned)rows), dim3(kWave), 0, st,
               (int)parts, w, norms);
  } else {
    FLC_LAUNCH("quant_norm", quant_norm_kernel<FLC_NORM_L2>, dim3((unsigned)parts, (unsigned)rows), dim3(kThreads), 0,
               st, x, d, (int)parts, chunk, vec_ok, w);
    if (fold_in) {
      FLC_LAUNCH(name, (quant_encode_philox_kernel<KIND, BITS, DEC, FLC_NORM_L2 + 1>), dim3((unsigned)nb1),
                 dim3(kThreads), 0, st, x, n, d, levels, step, norms, seed, counter, codes, nz, out, w, (int)parts);
      return FLC_OK;
    }
    FLC_LAUNCH("quant_norm_fold", quant_norm_fold_kernel<FLC_NORM_L2>, dim3((unsigned)rows), dim3(kWave), 0, st,
               (int)parts, w, norms);
  }
  FLC_LAUNCH(name, (quant_encode_philox_kernel<KIND, BITS, DEC, 0>), dim3((unsigned)nb1), dim3(kThreads), 0, st, x, n,
             d, levels, step, norms, seed, counter, codes, nz, out, w, 0);
  return FLC_OK;
}

}  // namespace
}  // namespace flc

extern "C" {

int flc_quant_encode_auto(const float* x, int64_t rows, int64_t d, int kind, int levels, int bits, int norm_p,
                          uint64_t seed, uint64_t counter, uint8_t* codes, float* norms, int64_t* nnz, float* out,
                          void* ws, size_t ws_bytes, void* stream) {
  if (rows <= 0 || d <= 0 || !x || !norms || !codes) return fail(FLC_EINVAL, "flc_quant_encode_auto: bad arguments");
  if (rows > 65535) return fail(FLC_EINVAL, "flc_quant_encode_auto: at most 65535 rows per call");
  if (norm_p != FLC_NORM_INF && norm_p != FLC_NORM_L2) return fail(FLC_EINVAL, "flc_quant_encode_auto: p must be inf(0) or 2");
  if (int rc = check_quant_args(kind, levels, bits)) return rc;
  if (!aligned16(x) || !aligned16(codes) || (out && !aligned16(out)))
    return fail(FLC_EINVAL, "flc_quant_encode_auto: x, codes and out must be 16-B aligned");
  size_t need = 0;
  QuantWs w = carve(ws, ws_bytes, rows, cdiv(rows * d, (int64_t)kGroup * kGroupsPerBlock), &need);
  if (need > ws_bytes || !ws) return fail(FLC_EWORKSPACE, "flc_quant_encode_auto: workspace %zu < %zu", ws_bytes, need);
  hipStream_t st = as_stream(stream);
  if (nnz) FLC_CHECK_HIP(hipMemsetAsync(nnz, 0, (size_t)rows * sizeof(int64_t), st));
#define FLC_AUTO(K, B)                                                                                            \
  return out ? launch_auto<K, B, true>(x, rows, d, levels, norm_p, seed, counter, codes, norms, nnz, out, w, st)   \
             : launch_auto<K, B, false>(x, rows, d, levels, norm_p, seed, counter, codes, norms, nnz, out, w, st)
  if (kind == FLC_Q_STANDARD_DITHER) {
    if (bits == 8) FLC_AUTO(0, 8);
    if (bits == 4) FLC_AUTO(0, 4);
    FLC_AUTO(0, 2);
  } else {
    if (bits == 8) FLC_AUTO(1, 8);
    if (bits == 4) FLC_AUTO(1, 4);
    FLC_AUTO(1, 2);
  }
#undef FLC_AUTO
}

int flc_quant_encode(const float* x, int64_t rows, int64_t d, int kind, int levels, int bits, const float* norms,
                     uint64_t seed, uint64_t counter, const double* compat_u, uint8_t* codes, int64_t* nnz, void* ws,
                     size_t ws_bytes, void* stream) {
  return quant_encode_entry(x, rows, d, kind, levels, bits, norms, seed, counter, compat_u, codes, nnz, nullptr, ws,
                            ws_bytes, stream, "flc_quant_encode");
}

int flc_quant_encode_decode(const float* x, int64_t rows, int64_t d, int kind, int levels, int bits, const float* norms,
                            uint64_t seed, uint64_t counter, const double* compat_u, uint8_t* codes, int64_t* nnz,
                            float* out, void* ws, size_t ws_bytes, void* stream) {
  if (!out) return fail(FLC_EINVAL, "flc_quant_encode_decode: null out");
  return quant_encode_entry(x, rows, d, kind, levels, bits, norms, seed, counter, compat_u, codes, nnz, out, ws,
                            ws_bytes, stream, "flc_quant_encode_decode");
}

int flc_count_consumers(const float* x, int64_t rows, int64_t d, const float* norms, int64_t* count, void* stream) {
  if (!x || !count || rows <= 0 || d <= 0) return fail(FLC_EINVAL, "flc_count_consumers: bad arguments");
  hipStream_t st = as_stream(stream);
  FLC_CHECK_HIP(hipMemsetAsync(count, 0, sizeof(int64_t), st));
  const int64_t n = rows * d;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(n, kThreads), 256 * 8);
  FLC_LAUNCH("count_consumers", count_consumers_kernel, dim3(grid), dim3(kThreads), 0, st, x, n, d, norms,
             reinterpret_cast<unsigned long long*>(count));
  return FLC_OK;
}

int flc_quant_decode(const uint8_t* codes, int64_t rows, int64_t d, int kind, int levels, int bits, const float* norms,
                     const float* row_weights, int accumulate, float* out, void* stream) {
  if (rows <= 0 || d <= 0 || !codes || !norms || !out) return fail(FLC_EINVAL, "flc_quant_decode: bad arguments");
  if (int rc = check_quant_args(kind, levels, bits)) return rc;
  if (!aligned16(out) || !aligned16(codes)) return fail(FLC_EINVAL, "flc_quant_decode: out and codes must be 16-B aligned");
  const int64_t n = rows * d;
  hipStream_t st = as_stream(stream);
#define FLC_DEC(K, B) return launch_decode<K, B>(codes, n, d, levels, norms, row_weights, accumulate, out, st)
  if (kind == FLC_Q_STANDARD_DITHER) {
    if (bits == 8) FLC_DEC(0, 8);
    if (bits == 4) FLC_DEC(0, 4);
    FLC_DEC(0, 2);
  } else {
    if (bits == 8) FLC_DEC(1, 8);
    if (bits == 4) FLC_DEC(1, 4);
    FLC_DEC(1, 2);
  }
#undef FLC_DEC
}

}  // extern "C"
