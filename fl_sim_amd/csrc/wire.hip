// wire.hip — the stacked codec's packed wire and the server-side fold of many clients' wires in one pass (gfx950).
//
// Packed wire (one contiguous, 256-B-aligned record per client; the layout is a function of (n, k) only, so a
// [clients, stride] byte tensor can be all-gathered over RCCL or copied over PCIe as one piece):
//   [0, 4)                     norm       fp32, the kept set's max |value| (compressors.py:344's pnorm at p = inf)
//   [16, 16 + 4k)              idx        int32, ascending
//   [codes, codes + max(k,16)) codes      u8, sign << 7 | level
//   [tiles, tiles + 4(T+1))    tiles      u32 CSR pointers over FLC_TILE-output tiles (T = ceil(n / FLC_TILE))
// The encoder writes it directly (flc_stacked_encode_tiled with the four pointers inside the record).
//
// Fold (flc_stacked_fold_wires): out = fmaf(w_c, decode(wire_c), out) for c = 0 .. m-1 in order, every element,
// every client — the server's sequential fold (nodes.py:1165-1180, _fedopt.py:202-208) in ONE
// pass over `out` instead of one decode-accumulate pass (read + write of 4n bytes) per client.  One 64-lane wave
// per 1024-output tile keeps its slice of the accumulator in registers; per client the tile's kept entries are
// scattered into a 4 KB LDS tile, read back densely (zeros included: fmaf(w, +0, acc) is applied exactly as the
// dense per-client fold applies it), and the scattered slots are cleared again.  All clients' entries of the tile
// are loaded in one batch (a wave prefix over the clients' counts) before the ordered fold; tiles holding more than
// 128 entries over all clients take a per-client loop.  Sparse variant (a fold from +0 with finite weights, the
// aggregation round's case): the accumulator lives in the LDS tile and only the kept entries are fma'd, in client
// order.  fmaf(w, +0, acc) == acc for every element no entry touches, with one exception: an accumulator that is -0
// (a negative fma result below half the smallest subnormal rounds to -0, fmaf(w, v, -0) keeps it when w * v is a
// zero of either sign, and a chained launch carries it in) becomes +0 at the next client whose w has a clear sign bit (w * +0 = +0, and
// +0 + -0 = +0).  So the sparse fold records, per element, the last client that wrote it (a byte in LDS) and, before
// each entry's fma and at the end, replays the skipped clients on a -0 (skip_clients) — the dense chain bit for bit.  Bytes: 4n written (+ 4n read when
// accumulating) + the wires' 5 B per kept entry and tile pointers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kMaxWires = 64;  // clients per launch (more: chained launches, accumulating)

struct WireLayout {
  long long norm, idx, codes, tiles;
};
struct FoldArgs {
  const uint8_t* rec[kMaxWires];  // the c-th client's record in fold order
  float w[kMaxWires];
};

WireLayout wire_layout(int64_t n, int64_t k, size_t* total) {
  WireLayout L;
  L.norm = 0;
  L.idx = 16;
  L.codes = (long long)align_up((size_t)(16 + 4 * k), 16);
  L.tiles = (long long)align_up((size_t)L.codes + (size_t)std::max<int64_t>(k, 16), 16);
  const int64_t ntiles = cdiv(n < 1 ? 1 : n, (int64_t)FLC_TILE);
  *total = align_up((size_t)L.tiles + 4 * (size_t)(ntiles + 1), 256);
  return L;
}

__device__ __forceinline__ unsigned long long lowmask(unsigned j) { return j >= 64u ? ~0ull : ((1ull << j) - 1ull); }

// the dense chain's clients [from, to) with no entry at an element, applied to its accumulator: fmaf(w, +0, a) only
// ever changes a -0, to +0, and only for a w with a clear sign bit (`pos`: one bit per such client of the launch)
__device__ __forceinline__ float skip_clients(float a, unsigned from, unsigned to, unsigned long long pos) {
  return (__float_as_uint(a) == 0x80000000u && (pos & lowmask(to) & ~lowmask(from)) != 0ull) ? 0.0f : a;
}

// Where a tile's accumulator comes from and where it goes.  Lane `lane` owns float4 groups q = lane + 64 u (u < 4)
// of the tile starting at flat element t0.
struct FlatIO {  // one flat vector: out = fold (from +0, or from out itself)
  float* out;
  int64_t n;
  int acc_in;
  __device__ __forceinline__ void load(int64_t t0, int lane, float4 acc[4]) const {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = t0 + 4 * (int64_t)(lane + u * kWave);
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (acc_in) {
        if (e + 4 <= n) {
          v = *reinterpret_cast<const float4*>(out + e);
        } else {
          if (e < n) v.x = out[e];
          if (e + 1 < n) v.y = out[e + 1];
          if (e + 2 < n) v.z = out[e + 2];
        }
      }
      acc[u] = v;
    }
  }
  __device__ __forceinline__ void store(int64_t t0, int lane, const float4 acc[4]) const {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = t0 + 4 * (int64_t)(lane + u * kWave);
      if (e + 4 <= n) {
        *reinterpret_cast<float4*>(out + e) = acc[u];
      } else {
        if (e < n) out[e] = acc[u].x;
        if (e + 1 < n) out[e + 1] = acc[u].y;
        if (e + 2 < n) out[e + 2] = acc[u].z;
      }
    }
  }
};

__device__ __forceinline__ float& comp(float4& v, int j) { return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w; }

// A server's model as the fold's accumulator (flc_fedopt_fold_records): the flat element e of the records is
// element e - start[t] of tensor t (the concatenation order of the client's flattened delta).  load: a = δ (· β0
// when `scale`: FedOptServer.update's mul_(betas[0]) first); store: δ = a, then, with OPT >= 0, the server
// optimiser's step on θ (and v) from a — _fedopt.py:202-237 in one pass.  The tile's tensors are walked with a
// uniform index (a tile usually lies inside one tensor); a float4 group inside one 16-B aligned tensor moves as one.
constexpr int kRoundT = 16;  // tensors per launch (kernel-argument budget)
struct ModelTab {
  float* delta[kRoundT];
  float* theta[kRoundT];
  float* v[kRoundT];
  int64_t start[kRoundT + 1];  // flat offsets; start[nt] = end of the launch's range
  int nt;
  unsigned vec;  // bit t: tensor t's operands 16-B aligned and start[t] % 4 == 0
  int scale;
  float beta0, lr, beta2, omb, nomb, tau;
};
template <int OPT>  // OPT < 0: the fold only (δ written, no step)
struct ModelIO {
  ModelTab m;
  __device__ __forceinline__ int first_tensor(int64_t t0) const {
    int t = 0;
#if FLC_PACK_SEARCH_STATIC  // (static offsets: the scalar loads of start issue together, flc_device.hpp pack_entry)
#pragma unroll
    for (int i = 1; i < kRoundT; ++i) t += (i < m.nt && m.start[i] <= t0) ? 1 : 0;
#else
    while (t + 1 < m.nt && m.start[t + 1] <= t0) ++t;
#endif
    return t;
  }
  __device__ __forceinline__ void load(int64_t t0, int lane, float4 acc[4]) const {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int t = first_tensor(t0); t < m.nt && m.start[t] < t0 + FLC_TILE; ++t) {
      const int64_t s0 = m.start[t], s1 = m.start[t + 1];
      const float* __restrict__ d = m.delta[t];
      const bool vec = (m.vec >> t) & 1u;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t e = t0 + 4 * (int64_t)(lane + u * kWave);
        if (vec && e >= s0 && e + 4 <= s1) {
          float4 x = *reinterpret_cast<const float4*>(d + (e - s0));
          if (m.scale) x = make_float4(x.x * m.beta0, x.y * m.beta0, x.z * m.beta0, x.w * m.beta0);
          acc[u] = x;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (e + j >= s0 && e + j < s1) {
              const float x = d[e + j - s0];
              comp(acc[u], j) = m.scale ? x * m.beta0 : x;
            }
        }
      }
    }
  }
  __device__ __forceinline__ void store(int64_t t0, int lane, float4 acc[4]) const {
    for (int t = first_tensor(t0); t < m.nt && m.start[t] < t0 + FLC_TILE; ++t) {
      const int64_t s0 = m.start[t], s1 = m.start[t + 1];
      float* __restrict__ d = m.delta[t];
      float* __restrict__ th = m.theta[t];
      float* __restrict__ vv = m.v[t];
      const bool vec = (m.vec >> t) & 1u;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t e = t0 + 4 * (int64_t)(lane + u * kWave);
        if (vec && e >= s0 && e + 4 <= s1) {
          const int64_t o = e - s0;
          *reinterpret_cast<float4*>(d + o) = acc[u];
          if (OPT >= 0) {
            float4 tv = *reinterpret_cast<const float4*>(th + o);
            float4 vq = OPT > 0 ? *reinterpret_cast<const float4*>(vv + o) : make_float4(0.f, 0.f, 0.f, 0.f);
            opt_step<OPT < 0 ? 0 : OPT>(tv.x, acc[u].x, &vq.x, m.lr, m.beta2, m.omb, m.nomb, m.tau);
            opt_step<OPT < 0 ? 0 : OPT>(tv.y, acc[u].y, &vq.y, m.lr, m.beta2, m.omb, m.nomb, m.tau);
            opt_step<OPT < 0 ? 0 : OPT>(tv.z, acc[u].z, &vq.z, m.lr, m.beta2, m.omb, m.nomb, m.tau);
            opt_step<OPT < 0 ? 0 : OPT>(tv.w, acc[u].w, &vq.w, m.lr, m.beta2, m.omb, m.nomb, m.tau);
            *reinterpret_cast<float4*>(th + o) = tv;
            if (OPT > 0) *reinterpret_cast<float4*>(vv + o) = vq;
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (e + j >= s0 && e + j < s1) {
              const int64_t o = e + j - s0;
              const float a = comp(acc[u], j);
              d[o] = a;
              if (OPT >= 0) {
                float vi = OPT > 0 ? vv[o] : 0.f;
                opt_step<OPT < 0 ? 0 : OPT>(th[o], a, &vi, m.lr, m.beta2, m.omb, m.nomb, m.tau);
                if (OPT > 0) vv[o] = vi;
              }
            }
          }
        }
      }
    }
  }
};

template <bool SPARSE, class IO>
__global__ __launch_bounds__(kWave) void stacked_fold_wires_kernel(FoldArgs a, WireLayout L, int nw, int levels,
                                                                   double step, int64_t tile0, IO io, unsigned k) {
  __shared__ __attribute__((aligned(16))) float s_tile[FLC_TILE];
  __shared__ __attribute__((aligned(16))) uint8_t s_last[SPARSE ? FLC_TILE : 4];  // sparse: last writer + 1 (0: none)
  float4* tile4 = reinterpret_cast<float4*>(s_tile);
  const int lane = threadIdx.x;
  const int64_t t = tile0 + blockIdx.x;
  const int64_t t0 = t * FLC_TILE;
  // the tile's slice of the accumulator: lane owns float4 q = lane + 64 u
  float4 acc[4];
  io.load(t0, lane, acc);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    // dense: a zero tile per client; sparse: the accumulator itself lives in the LDS tile
    tile4[lane + u * kWave] = SPARSE ? acc[u] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (SPARSE) reinterpret_cast<unsigned*>(s_last)[lane + u * kWave] = 0u;
  }
  // client `lane`'s record, entry range in this tile and norm (lanes >= nw: empty)
  const uint8_t* rec = nullptr;
  unsigned lo = 0, cnt = 0;
  float nrm = 0.0f, wl = 0.0f;
  if (lane < nw) {
    rec = a.rec[lane];
    wl = a.w[lane];
    const unsigned* tiles = reinterpret_cast<const unsigned*>(rec + L.tiles);
    // (clamped to the record's k entries: a malformed or unwritten tile pointer never reads past the record)
    lo = min(tiles[t], k);
    const unsigned hi = min(tiles[t + 1], k);
    cnt = hi > lo ? hi - lo : 0u;
    nrm = *reinterpret_cast<const float*>(rec + L.norm);
  }
  const unsigned long long pos = __ballot(lane < nw && !std::signbit(wl));  // sign-clear weights (sparse: -0 rule)
  const unsigned incl = wave_incl_scan(cnt);
  const unsigned excl = incl - cnt;
  const unsigned total = (unsigned)__builtin_amdgcn_readlane((int)incl, kWave - 1);

  if (total <= 2u * kWave) {
    // fast path: every entry of the tile over all clients in registers (g = lane, lane + 64), one load batch
    int cg[2] = {-1, -1};
    unsigned off[2] = {0u, 0u};
    float val[2] = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const unsigned g = (unsigned)lane + (unsigned)(r * kWave);
      int c = -1;
      for (int cc = 0; cc < nw; ++cc) {  // (uniform loop; the client whose range holds g)
        const unsigned ec = (unsigned)__builtin_amdgcn_readlane((int)excl, cc);
        const unsigned nc = (unsigned)__builtin_amdgcn_readlane((int)cnt, cc);
        if (g >= ec && g < ec + nc) c = cc;
      }
      cg[r] = g < total ? c : -1;
    }
    // the owning client's record / range / norm by lane shuffles, then the loads (one batch)
    unsigned idx_raw[2] = {0u, 0u}, code[2] = {0u, 0u};
    float nr[2] = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int src = cg[r] < 0 ? 0 : cg[r];
      const unsigned lo_c = (unsigned)__shfl((int)lo, src, kWave);
      const unsigned ex_c = (unsigned)__shfl((int)excl, src, kWave);
      const unsigned long long rp = (unsigned long long)(uintptr_t)rec;
      const unsigned rlo = (unsigned)__shfl((int)(unsigned)rp, src, kWave);
      const unsigned rhi = (unsigned)__shfl((int)(unsigned)(rp >> 32), src, kWave);
      nr[r] = __shfl(nrm, src, kWave);
      if (cg[r] >= 0) {
        const uint8_t* rc = reinterpret_cast<const uint8_t*>((uintptr_t)(((unsigned long long)rhi << 32) | rlo));
        const unsigned j = lo_c + ((unsigned)lane + (unsigned)(r * kWave) - ex_c);
        idx_raw[r] = reinterpret_cast<const unsigned*>(rc + L.idx)[j];
        code[r] = rc[L.codes + j];
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int64_t o = (int64_t)idx_raw[r] - t0;
      if (cg[r] >= 0 && (o < 0 || o >= FLC_TILE)) cg[r] = -1;  // (a malformed wire: ignored, never out of the tile)
      off[r] = (unsigned)(o < 0 ? 0 : (o >= FLC_TILE ? 0 : o));
      val[r] = stacked_dequant(code[r], levels, step, nr[r]);
    }
    if (SPARSE) {
      // the accumulator in LDS, updated at the kept entries only (see the launch: +0 start, finite weights, so
      // fmaf(w, +0, acc) == acc for every element no entry touches)
      for (int c = 0; c < nw; ++c) {
        const float wc = __shfl(wl, c, kWave);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          if (cg[r] == c) {
            s_tile[off[r]] = fmaf(wc, val[r], skip_clients(s_tile[off[r]], s_last[off[r]], (unsigned)c, pos));
            s_last[off[r]] = (uint8_t)(c + 1);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = tile4[lane + u * kWave];
    }
    for (int c = 0; c < (SPARSE ? 0 : nw); ++c) {  // the ordered fold
      const float wc = __shfl(wl, c, kWave);
      const bool any = __builtin_amdgcn_readlane((int)cnt, c) != 0;
      if (any) {
        if (cg[0] == c) s_tile[off[0]] = val[0];
        if (cg[1] == c) s_tile[off[1]] = val[1];
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float4 v = tile4[lane + u * kWave];
          acc[u] = make_float4(fmaf(wc, v.x, acc[u].x), fmaf(wc, v.y, acc[u].y), fmaf(wc, v.z, acc[u].z),
                               fmaf(wc, v.w, acc[u].w));
        }
        __builtin_amdgcn_wave_barrier();
        if (cg[0] == c) s_tile[off[0]] = 0.0f;
        if (cg[1] == c) s_tile[off[1]] = 0.0f;
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          acc[u] = make_float4(fmaf(wc, 0.0f, acc[u].x), fmaf(wc, 0.0f, acc[u].y), fmaf(wc, 0.0f, acc[u].z),
                               fmaf(wc, 0.0f, acc[u].w));
      }
    }
  } else {
    // dense tiles (skewed inputs): per client, its entries in rounds of 64, scattered, folded, cleared
    for (int c = 0; c < nw; ++c) {
      const float wc = __shfl(wl, c, kWave);
      const unsigned lo_c = (unsigned)__builtin_amdgcn_readlane((int)lo, c);
      const unsigned n_c = (unsigned)__builtin_amdgcn_readlane((int)cnt, c);
      const float nr_c = __shfl(nrm, c, kWave);
      const unsigned long long rp = (unsigned long long)(uintptr_t)rec;
      const unsigned rlo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)rp, c);
      const unsigned rhi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(rp >> 32), c);
      const uint8_t* rc = reinterpret_cast<const uint8_t*>((uintptr_t)(((unsigned long long)rhi << 32) | rlo));
      const unsigned* ix = reinterpret_cast<const unsigned*>(rc + L.idx);
      const uint8_t* cd = rc + L.codes;
      if (SPARSE) {
        for (unsigned j = lo_c + lane; j < lo_c + n_c; j += kWave) {
          const int64_t o = (int64_t)ix[j] - t0;
          if (o >= 0 && o < FLC_TILE) {
            s_tile[o] = fmaf(wc, stacked_dequant(cd[j], levels, step, nr_c),
                             skip_clients(s_tile[o], s_last[o], (unsigned)c, pos));
            s_last[o] = (uint8_t)(c + 1);
          }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        continue;
      }
      for (unsigned j = lo_c + lane; j < lo_c + n_c; j += kWave) {
        const int64_t o = (int64_t)ix[j] - t0;
        if (o >= 0 && o < FLC_TILE) s_tile[o] = stacked_dequant(cd[j], levels, step, nr_c);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 v = tile4[lane + u * kWave];
        acc[u] = make_float4(fmaf(wc, v.x, acc[u].x), fmaf(wc, v.y, acc[u].y), fmaf(wc, v.z, acc[u].z),
                             fmaf(wc, v.w, acc[u].w));
      }
      __builtin_amdgcn_wave_barrier();
      for (unsigned j = lo_c + lane; j < lo_c + n_c; j += kWave) {
        const int64_t o = (int64_t)ix[j] - t0;
        if (o >= 0 && o < FLC_TILE) s_tile[o] = 0.0f;
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (SPARSE) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = tile4[lane + u * kWave];
    }
  }
  if (SPARSE) {  // the clients after each element's last writer
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned lb = reinterpret_cast<const unsigned*>(s_last)[lane + u * kWave];
      acc[u].x = skip_clients(acc[u].x, lb & 0xFFu, 64u, pos);
      acc[u].y = skip_clients(acc[u].y, (lb >> 8) & 0xFFu, 64u, pos);
      acc[u].z = skip_clients(acc[u].z, (lb >> 16) & 0xFFu, 64u, pos);
      acc[u].w = skip_clients(acc[u].w, lb >> 24, 64u, pos);
    }
  }
  io.store(t0, lane, acc);
}

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

size_t flc_stacked_wire_layout(int64_t n, int64_t k, int64_t* offsets) {
  if (n <= 0 || k < 0) return 0;
  size_t total = 0;
  const WireLayout L = wire_layout(n, k, &total);
  if (offsets) {
    offsets[0] = L.norm;
    offsets[1] = L.idx;
    offsets[2] = L.codes;
    offsets[3] = L.tiles;
  }
  return total;
}

int flc_stacked_fold_wires(const void* wires, int64_t stride, const int32_t* slots, const float* weights, int n_wires,
                           int64_t n, int64_t k, int levels, int accumulate, float* out, void* stream) {
  if (!wires || !slots || !weights || !out || n_wires < 1 || n <= 0 || k < 0)
    return fail(FLC_EINVAL, "flc_stacked_fold_wires: bad arguments");
  if (n >= (1ll << 31) || k >= (1ll << 31)) return fail(FLC_EINVAL, "flc_stacked_fold_wires: n and k must be < 2^31");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_stacked_fold_wires: levels must be in [1, 127]");
  size_t need = 0;
  const WireLayout L = wire_layout(n, k, &need);
  if (stride < (int64_t)need || stride % 16 != 0)
    return fail(FLC_EINVAL, "flc_stacked_fold_wires: stride %lld < record size %zu (or not 16-B aligned)",
                (long long)stride, need);
  if (!aligned16(wires) || !aligned16(out)) return fail(FLC_EINVAL, "flc_stacked_fold_wires: 16-B aligned buffers required");
  for (int c = 0; c < n_wires; ++c)
    if (slots[c] < 0) return fail(FLC_EINVAL, "flc_stacked_fold_wires: slot %d is negative", c);
  hipStream_t st = as_stream(stream);
  const int64_t ntiles = cdiv(n, (int64_t)FLC_TILE);
  const double step = 1.0 / (double)levels;
  // Sparse fold (from +0, finite weights): only the kept entries are fma'd, and a final -0 is resolved as the dense
  // chain would (kernel header).  Otherwise (accumulating into a given vector, or a non-finite weight) every element
  // takes every client's fma.
  bool sparse = !accumulate;
  for (int c = 0; c < n_wires; ++c) sparse = sparse && std::isfinite(weights[c]);
  for (int c0 = 0; c0 < n_wires; c0 += kMaxWires) {
    const int nw = std::min(kMaxWires, n_wires - c0);
    FoldArgs a;
    for (int c = 0; c < kMaxWires; ++c) {
      a.w[c] = c < nw ? weights[c0 + c] : 0.0f;
      a.rec[c] = static_cast<const uint8_t*>(wires) + (c < nw ? (int64_t)slots[c0 + c] * stride : 0);
    }
    const FlatIO io{out, n, (c0 > 0 || accumulate) ? 1 : 0};
    if (sparse)
      FLC_LAUNCH("stacked_fold_wires", (stacked_fold_wires_kernel<true, FlatIO>), dim3((unsigned)ntiles), dim3(kWave), 0,
                 st, a, L, nw, levels, step, (int64_t)0, io, (unsigned)k);
    else
      FLC_LAUNCH("stacked_fold_wires", (stacked_fold_wires_kernel<false, FlatIO>), dim3((unsigned)ntiles), dim3(kWave),
                 0, st, a, L, nw, levels, step, (int64_t)0, io, (unsigned)k);
  }
  return FLC_OK;
}

int flc_fedopt_fold_records(const void* const* records, const float* weights, int n_records, int64_t n, int64_t k,
                            int levels, float* const* delta, float* const* theta, float* const* v,
                            const int64_t* sizes, int n_tensors, float beta0, int opt, double lr, double beta2,
                            double tau, void* stream) {
  if (n_records < 0 || (n_records > 0 && (!records || !weights)) || n <= 0 || k < 0 || n_tensors < 1 || !delta ||
      !sizes)
    return fail(FLC_EINVAL, "flc_fedopt_fold_records: bad arguments");
  if (n >= (1ll << 31) || k >= (1ll << 31)) return fail(FLC_EINVAL, "flc_fedopt_fold_records: n and k must be < 2^31");
  if (levels < 1 || levels > 127) return fail(FLC_EINVAL, "flc_fedopt_fold_records: levels must be in [1, 127]");
  const bool step_on = theta != nullptr;
  if (step_on && opt != FLC_OPT_AVG && opt != FLC_OPT_ADAGRAD && opt != FLC_OPT_YOGI && opt != FLC_OPT_ADAM)
    return fail(FLC_EINVAL, "flc_fedopt_fold_records: unknown optimiser %d", opt);
  if (step_on && opt != FLC_OPT_AVG && !v)
    return fail(FLC_EINVAL, "flc_fedopt_fold_records: v required for adaptive optimisers");
  int64_t total = 0;
  for (int t = 0; t < n_tensors; ++t) {
    if (sizes[t] < 0) return fail(FLC_EINVAL, "flc_fedopt_fold_records: negative size for tensor %d", t);
    if (sizes[t] > 0 && (!delta[t] || (step_on && !theta[t]) || (step_on && opt != FLC_OPT_AVG && !v[t])))
      return fail(FLC_EINVAL, "flc_fedopt_fold_records: null pointer for tensor %d", t);
    total += sizes[t];
  }
  if (total != n)
    return fail(FLC_EINVAL, "flc_fedopt_fold_records: the tensors hold %lld elements, the records %lld",
                (long long)total, (long long)n);
  for (int c = 0; c < n_records; ++c)
    if (!records[c] || !aligned16(records[c]))
      return fail(FLC_EINVAL, "flc_fedopt_fold_records: record %d is null or not 16-B aligned", c);
  size_t need = 0;
  const WireLayout L = wire_layout(n, k, &need);
  hipStream_t st = as_stream(stream);
  const double step = 1.0 / (double)levels;
  const float omb = (float)(1.0 - beta2), nomb = (float)(-(1.0 - beta2));
  // record chunks in order (the chain continues from the stored δ, the step after the last chunk only); within a
  // chunk, one launch per group of <= kRoundT tensors over the tiles their flat range touches
  int c0 = 0;
  do {
    const int nw = std::min(kMaxWires, n_records - c0);
    const bool last = c0 + nw >= n_records;
    FoldArgs a;
    for (int c = 0; c < kMaxWires; ++c) {
      a.w[c] = c < nw ? weights[c0 + c] : 0.0f;
      a.rec[c] = static_cast<const uint8_t*>(c < nw ? records[c0 + c] : nullptr);
    }
    int64_t off = 0;
    int t = 0;
    while (t < n_tensors) {
      ModelTab m{};
      m.scale = c0 == 0;
      m.beta0 = beta0;
      m.lr = (float)lr;
      m.beta2 = (float)beta2;
      m.omb = omb;
      m.nomb = nomb;
      m.tau = (float)tau;
      for (; t < n_tensors && m.nt < kRoundT; ++t) {
        if (sizes[t] == 0) continue;
        const int i = m.nt++;
        m.delta[i] = delta[t];
        m.theta[i] = step_on ? theta[t] : nullptr;
        m.v[i] = (step_on && opt != FLC_OPT_AVG) ? v[t] : nullptr;
        m.start[i] = off;
        const bool vec = off % 4 == 0 && aligned16(m.delta[i]) && (!m.theta[i] || aligned16(m.theta[i])) &&
                         (!m.v[i] || aligned16(m.v[i]));
        if (vec) m.vec |= 1u << i;
        off += sizes[t];
      }
      if (m.nt == 0) break;
      m.start[m.nt] = off;
      const int64_t tile_lo = m.start[0] / FLC_TILE, tile_hi = cdiv(off, (int64_t)FLC_TILE);
      const dim3 grid((unsigned)(tile_hi - tile_lo));
#define FLC_FR(O) \
  FLC_LAUNCH("fedopt_fold_records", (stacked_fold_wires_kernel<false, ModelIO<O>>), grid, dim3(kWave), 0, st, a, L, nw, \
             levels, step, tile_lo, ModelIO<O>{m}, (unsigned)k)
      if (!step_on || !last) FLC_FR(-1);
      else if (opt == FLC_OPT_AVG) FLC_FR(FLC_OPT_AVG);
      else if (opt == FLC_OPT_ADAGRAD) FLC_FR(FLC_OPT_ADAGRAD);
      else if (opt == FLC_OPT_YOGI) FLC_FR(FLC_OPT_YOGI);
      else FLC_FR(FLC_OPT_ADAM);
#undef FLC_FR
    }
    c0 += nw;
  } while (c0 < n_records);
  return FLC_OK;
}

}  // extern "C"
