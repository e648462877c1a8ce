// flc_device.hpp — device-side building blocks shared by the codec kernels (gfx950 / CDNA4 only).
//
// Everything here is written for 64-lane wavefronts: integer scans and reductions are DPP sequences over
// 64 lanes (floating-point sums keep a fixed __shfl_xor butterfly), ballots are 64-bit, and block-level
// scans go through LDS one value per wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/flcodec.h"

namespace flc {

constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));

// streaming (non-temporal) 16-B load/store: data touched once should not displace L2 lines
__device__ __forceinline__ float4 ld_stream(const float* p) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_stream(float* p, float4 v) {
  f32x4 t = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(t, reinterpret_cast<f32x4*>(p));
}

// 16-B store written through past the XCD's L2 (sc1: the line is not left dirty in L2 for the kernel's end to write
// back).  No builtin sets sc1 on a 16-B store, so it is inline asm — and the compiler cannot see that the asm is a VMEM
// store of more than 8 bytes, after which gfx940+ needs 2 wait states before a VALU may overwrite the store's data
// VGPRs.  It schedules nothing for that, so the asm carries them itself (s_nop 1).  Without them the round-5 quantizer
// variant stored two data dwords already overwritten by the next store's address (profiles/r06/r06c_asm_store_hazard.txt).
// Waits the compiler counts (vmcnt) stay correct: an extra outstanding store only makes a counted wait for earlier
// loads, which return in order, wait as long or longer.
__device__ __forceinline__ void st_wt(float* p, float4 v) {
  const f32x4 w = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
}

// ------------------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11).  Counter = (group_lo, group_hi, ctr_lo, ctr_hi), key = seed.
// One call yields four 32-bit words; element e of a vector uses word (e & 3) of group e >> 2, so the
// stream is a pure function of (seed, counter, element index) — independent of launch geometry.
// ------------------------------------------------------------------------------------------------
struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // 64-bit products: one v_mad_u64_u32 each instead of a mul_hi + mul_lo pair
    const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

__device__ __forceinline__ U4 philox_group(uint64_t group, uint64_t seed, uint64_t counter) {
  return philox4x32_10(U4{(uint32_t)group, (uint32_t)(group >> 32), (uint32_t)counter,
                          (uint32_t)(counter >> 32)},
                       (uint32_t)seed, (uint32_t)(seed >> 32));
}

// 32-bit word -> uniform double in [0, 1), exact (r * 2^-32).
__device__ __forceinline__ double u01(uint32_t r) { return (double)r * 2.3283064365386963e-10; }

__device__ __forceinline__ uint32_t pick(const U4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

// ------------------------------------------------------------------------------------------------
// wave / block reductions (64-lane butterflies)
// ------------------------------------------------------------------------------------------------
// Cross-lane steps are DPP moves (VALU, a few cycles) rather than __shfl (ds_bpermute through the LDS
// pipe, ~100+ cycles each): row_shr:1/2/4/8 inside each 16-lane row, then row_bcast:15 / row_bcast:31
// across rows (gfx9 DPP; gfx950 has no permlane16).  Lanes whose DPP source falls outside the row take
// no part (the step's condition), so the bound / mask controls do not matter.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL, typename T>
__device__ __forceinline__ T dpp_mov(T v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit lanes");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, dpp_u32<CTRL>(__builtin_bit_cast(uint32_t, v)));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint64_t r = ((uint64_t)dpp_u32<CTRL>((uint32_t)(u >> 32)) << 32) | dpp_u32<CTRL>((uint32_t)u);
    return __builtin_bit_cast(T, r);
  }
}
template <typename T>
__device__ __forceinline__ T lane_bcast(T v, int l) {  // v of lane l (uniform l), as a scalar
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, (uint32_t)__builtin_amdgcn_readlane((int)__builtin_bit_cast(uint32_t, v), l));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint64_t r = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(u >> 32), l) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    return __builtin_bit_cast(T, r);
  }
}

// inclusive prefix combine across the 64 lanes of a wave
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan_op(T v, Op op) {
  const int lane = threadIdx.x & (kWave - 1), rl = lane & 15;
  T t;
  t = dpp_mov<0x111>(v);  // row_shr:1
  if (rl >= 1) v = op(t, v);
  t = dpp_mov<0x112>(v);  // row_shr:2
  if (rl >= 2) v = op(t, v);
  t = dpp_mov<0x114>(v);  // row_shr:4
  if (rl >= 4) v = op(t, v);
  t = dpp_mov<0x118>(v);  // row_shr:8
  if (rl >= 8) v = op(t, v);
  t = dpp_mov<0x142>(v);  // row_bcast:15
  if ((lane & 31) >= 16) v = op(t, v);
  t = dpp_mov<0x143>(v);  // row_bcast:31
  if (lane >= 32) v = op(t, v);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  return wave_incl_scan_op(v, [](T a, T b) { return a + b; });
}
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {  // (every lane gets the total)
  if constexpr (__is_floating_point(T)) {
    // floating point keeps the fixed butterfly order its results were pinned with
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
  } else {
    return lane_bcast(wave_incl_scan(v), kWave - 1);
  }
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  return lane_bcast(wave_incl_scan_op(v, [](uint32_t a, uint32_t b) { return a > b ? a : b; }), kWave - 1);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  return lane_bcast(wave_incl_scan_op(v, [](uint32_t a, uint32_t b) { return a < b ? a : b; }), kWave - 1);
}

// Block-wide exclusive scan of one value per thread; returns the exclusive prefix, *total gets the
// block sum.  `lds` must hold NW = blockDim/64 entries.  Contains two __syncthreads().
// inclusive prefix sum inside each 16-lane row (the first four steps of wave_incl_scan)
template <typename T>
__device__ __forceinline__ T row_incl_scan(T v) {
  const int rl = threadIdx.x & 15;
  T t;
  t = dpp_mov<0x111>(v);
  if (rl >= 1) v += t;
  t = dpp_mov<0x112>(v);
  if (rl >= 2) v += t;
  t = dpp_mov<0x114>(v);
  if (rl >= 4) v += t;
  t = dpp_mov<0x118>(v);
  if (rl >= 8) v += t;
  return v;
}

// the cross-wave step of the block scans: lane w of every wave reads wave w's total (one LDS read per
// lane instead of NW), a row scan over them, and the wave's base / the block total by readlane
template <typename T, int NW>
__device__ __forceinline__ void block_scan_fold(const T* lds, T* base, T* tot) {
  static_assert(NW >= 1 && NW <= 16, "one DPP row of wave totals");
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x >> 6;
  const T sc = row_incl_scan(lane < NW ? lds[lane] : T(0));
  *tot = lane_bcast(sc, NW - 1);
  *base = wid > 0 ? lane_bcast(sc, wid > 0 ? wid - 1 : 0) : T(0);
}

template <typename T, int NW>
__device__ __forceinline__ T block_excl_scan(T v, T* lds, T* total) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x >> 6;
  const T incl = wave_incl_scan(v);
  if (lane == kWave - 1) lds[wid] = incl;
  __syncthreads();
  T base, tot;
  block_scan_fold<T, NW>(lds, &base, &tot);
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

// The same with LDS-only barriers (s_waitcnt lgkmcnt(0); s_barrier): outstanding global stores and loads
// stay in flight across it.  Only for values exchanged through LDS (defined after lds_barrier below).
__device__ __forceinline__ void lds_barrier();
template <typename T, int NW>
__device__ __forceinline__ T block_excl_scan_lds(T v, T* lds, T* total) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x >> 6;
  const T incl = wave_incl_scan(v);
  if (lane == kWave - 1) lds[wid] = incl;
  lds_barrier();
  T base, tot;
  block_scan_fold<T, NW>(lds, &base, &tot);
  lds_barrier();
  *total = tot;
  return base + incl - v;
}

template <typename T, int NW>
__device__ __forceinline__ T block_sum(T v, T* lds) {
  T tot;
  (void)block_excl_scan<T, NW>(v, lds, &tot);
  return tot;
}

// ------------------------------------------------------------------------------------------------
// inter-workgroup hand-off (MI355X_MICROARCH.md §Workgroup dispatch / Guideline 16):
// payload words are stored write-through (sc1) by ONE lane, drained with s_waitcnt vmcnt(0), then an
// agent-scope release + relaxed ticket add; the last arriver does an agent acquire and reads the
// payload with sc1 (L1-bypassing) loads or memory-side atomics.
// ------------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_sc1(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// returns the ticket (0-based arrival order); call from ONE lane after every storing wave drained
__device__ __forceinline__ unsigned arrive(unsigned* counter) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void acquire_agent() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The entry of a kernel-argument pack that holds block b, from the entries' first blocks blk0[0..N] (non-decreasing,
// blk0[0] = 0; entries past nt ignored): every compare reads blk0 at a static offset, so its scalar loads issue together
// (one round trip), where a `while (blk0[t + 1] <= b) ++t` walk waits for one dependent load per entry it passes.
#ifndef FLC_PACK_SEARCH_STATIC
#define FLC_PACK_SEARCH_STATIC 1
#endif
template <int N>
__device__ __forceinline__ int pack_entry(const int (&blk0)[N + 1], int nt, int b) {
  int t = 0;
#if FLC_PACK_SEARCH_STATIC
#pragma unroll
  for (int i = 1; i < N; ++i) t += (i < nt && blk0[i] <= b) ? 1 : 0;
#else
  while (t + 1 < nt && blk0[t + 1] <= b) ++t;
#endif
  return t;
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup-scope fence + s_barrier, and
// on gfx950 that fence waits for vmcnt(0): every global load and store the wave has in flight.  Kernels
// that keep prefetched loads (or fire-and-forget stores) in flight across a barrier use this instead:
// LDS operations drained, no wait on the vector-memory counter.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ------------------------------------------------------------------------------------------------
// order-preserving key of a float for "largest signed value" selection (np.argsort order,
// compressors.py:295): -0 == +0, every NaN is the single largest key.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t order_key(uint32_t b) {
  if ((b & 0x7fffffffu) > 0x7f800000u) return 0xffffffffu;  // NaN
  if (b == 0x80000000u) b = 0u;                             // -0 -> +0
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
// value of a key (canonical NaN / +0 for the collapsed classes)
__device__ __forceinline__ float key_value(uint32_t k) {
  if (k == 0xffffffffu) return __uint_as_float(0x7fc00000u);
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// ------------------------------------------------------------------------------------------------
// dithering levels (compressors.py:157, 194-197): standard lv(i) = i * (1/s) in fp64 (bit-equal to
// np.arange(0, 1.1, 1/s)), lv(s) pinned to 1.0; natural lv(0) = 0, lv(i) = 2^(i-s).
// ------------------------------------------------------------------------------------------------
template <int KIND>
__device__ __forceinline__ double level_value(int i, int s, double step) {
  if (KIND == 0) return (i == s) ? 1.0 : (double)i * step;
  return (i == 0) ? 0.0 : ldexp(1.0, i - s);
}

template <int KIND>
__device__ __forceinline__ int level_lower_bound(float yf, int s, double step);

// Level index chosen for y = fp32(|x| / norm) in [0, 1] and uniform u — the rule of
// compressors.py:346-353: bracket [lv(sl), lv(sl+1)] = the first with lv(sl) <= y <= lv(sl+1) (fp64),
// p = (y - lv(sl+1)) / (lv(sl) - lv(sl+1)) in fp64, lower level iff u < p.  Bit-exact with that rule:
//  * standard: an fp32 fast path decides whenever t = y*s is >= 1e-4 from an integer and |u - p| > 3e-5
//    (its error is < 1e-5), otherwise the fp64 rule runs (probability ~1e-4 per element);
//  * natural: levels are powers of two, so the division is an exact power-of-two scaling.
template <int KIND>
__device__ __forceinline__ int dither_level(float y, int s, double step, double u) {
  if (KIND == 0) {
    const float t = y * (float)s;
    const float jf = ceilf(t);
    if (jf - t > 1e-4f && t - (jf - 1.0f) > 1e-4f) {
      const float pf = jf - t;
      const float uf = (float)u;
      if (fabsf(uf - pf) > 3e-5f) return (uf < pf) ? (int)jf - 1 : (int)jf;
    }
  }
  const int j = level_lower_bound<KIND>(y, s, step);
  const int sl = j > 0 ? j - 1 : 0;
  const double lo = level_value<KIND>(sl, s, step), hi = level_value<KIND>(sl + 1, s, step);
  double p;
  if (KIND == 0) {
    p = ((double)y - hi) / (lo - hi);
  } else {
    // lo - hi = -2^(sl+1-s) (sl >= 1) or -hi (sl == 0): multiply by the exact power-of-two inverse
    p = ((double)y - hi) * -ldexp(1.0, (sl == 0 ? s - 1 : s - sl));
  }
  return (u < p) ? sl : sl + 1;
}

// first index j in [0, s] with lv(j) >= y (y in [0, 1], not NaN)
template <int KIND>
__device__ __forceinline__ int level_lower_bound(float yf, int s, double step) {
  const double y = (double)yf;
  if (KIND == 0) {
    int j = (int)ceil(y * (double)s);
    j = j < 0 ? 0 : (j > s ? s : j);
    while (j > 0 && level_value<0>(j - 1, s, step) >= y) --j;
    while (j < s && level_value<0>(j, s, step) < y) ++j;
    return j;
  } else {
    if (yf == 0.0f) return 0;
    int E;
    const float m = frexpf(yf, &E);      // yf = m * 2^E, m in [0.5, 1)
    const int e = (m == 0.5f) ? E - 1 : E;  // ceil(log2 y)
    int j = s + e;
    return j < 1 ? 1 : (j > s ? s : j);
  }
}

// decoded value of a stacked-codec code byte (sign << 7 | level) with the kept set's norm (compressors.py:357:
// fp32(fp32(lv) * sign) * norm); a non-regular norm decodes every nonzero code to NaN
__device__ __forceinline__ float stacked_dequant(uint32_t code, int levels, double step, float nrm) {
  if (!(nrm > 0.0f && nrm <= 3.402823466e38f)) return code == 0u ? 0.0f : __uint_as_float(0x7fc00000u);
  const float lv = (float)level_value<0>((int)(code & 127u), levels, step);
  return ((code >> 7) ? -lv : lv) * nrm;
}

// The element-wise tail of FedOptServer.update (_fedopt.py:213-237) on one folded delta value d: the v update of the
// server optimiser, then the model step, each rounded where the reference's torch CPU ops round (add_(alpha) is one
// fma; mul_, pow(2), sqrt and the additions one rounding each; nothing else contracted: -ffp-contract=off).
// omb = fp32(1 - beta2), nomb = fp32(-(1 - beta2)) as torch casts the Python scalars.
template <int OPT>
__device__ __forceinline__ void opt_step(float& th, float d, float* vp, float lr, float beta2, float omb, float nomb,
                                         float tau) {
  if (OPT == FLC_OPT_AVG) {
    th = fmaf(lr, d, th);
    return;
  }
  const float d2 = d * d;
  float vi = *vp;
  if (OPT == FLC_OPT_ADAGRAD) {
    vi = vi + d2;
  } else if (OPT == FLC_OPT_YOGI) {
    const float diff = vi - d2;
    const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : (diff == 0.f ? 0.f : diff));
    vi = vi + (nomb * d2) * sg;
  } else {
    vi = fmaf(omb, d2, vi * beta2);
  }
  *vp = vi;
  th = th + (lr * d) / (sqrtf(vi) + tau);
}

}  // namespace flc
