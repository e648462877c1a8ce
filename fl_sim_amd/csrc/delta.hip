// delta.hip — client delta formation + flatten for gfx950 (the delta/flatten half).
//
// Reference: FedOptClient.communicate (fl_sim/algorithms/fedopt/_fedopt.py:294-297) forms the delta per parameter
// tensor as `dp = p.detach().clone()` (nodes.py:300-302) then `dp.add_(rp, alpha=-1)` — one fp32 fmaf(-1, rp, dp),
// which equals the single-rounded difference dp - rp — and the codec then needs the tensors as ONE flat vector
// (Compressor.compressVector takes a 1-D array).  delta_flatten does both in one pass: for tensor t,
//   out[off_t + i] = local_t[i] - global_t[i],   off_t = n_0 + ... + n_{t-1}
// HBM bytes per element: 8 read + 4 written (clone + add_ + cat move 28).  Each 256-thread block streams one
// 4096-element chunk of one tensor with 16-B non-temporal loads/stores where the tensor's operands and its slot in
// `out` are 16-B aligned (scalar accesses otherwise); a launch carries up to kMaxT tensors and their block offsets.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kThreads = 256;
constexpr int kUnroll = 4;
constexpr int64_t kChunk = (int64_t)kThreads * 4 * kUnroll;  // elements per block
constexpr int kMaxT = 48;                                     // tensors per launch (kernel-argument budget)

struct TensorPack {
  const float* l[kMaxT];
  const float* g[kMaxT];
  int64_t off[kMaxT];
  int64_t n[kMaxT];
  int blk0[kMaxT + 1];  // first block of tensor t; blk0[nt] = grid size
  unsigned long long vec;  // bit t: 16-B path for tensor t
  int nt;
};

__global__ __launch_bounds__(kThreads) void delta_flatten_kernel(TensorPack p, float* __restrict__ out) {
  const int b = blockIdx.x;
  const int t = pack_entry<kMaxT>(p.blk0, p.nt, b);  // (uniform)
  const float* __restrict__ l = p.l[t];
  const float* __restrict__ g = p.g[t];
  float* __restrict__ o = out + p.off[t];
  const int64_t n = p.n[t];
  const int64_t c0 = (int64_t)(b - p.blk0[t]) * kChunk;
  if ((p.vec >> t) & 1ull) {
    const int64_t n4 = n >> 2;
    float4 d[kUnroll];
    bool ok[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t i4 = (c0 >> 2) + u * kThreads + threadIdx.x;
      ok[u] = i4 < n4;
      const int64_t j = ok[u] ? 4 * i4 : 0;
      const float4 a = ld_stream(l + j), c = ld_stream(g + j);
      d[u] = make_float4(a.x - c.x, a.y - c.y, a.z - c.z, a.w - c.w);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      if (ok[u]) st_stream(o + 4 * ((c0 >> 2) + u * kThreads + threadIdx.x), d[u]);
    // the n % 4 tail, by the tensor's last block
    const int64_t tail = n & 3;
    if (c0 + kChunk >= n && (int64_t)threadIdx.x < tail) {
      const int64_t i = (n4 << 2) + threadIdx.x;
      o[i] = l[i] - g[i];
    }
    return;
  }
  for (int u = 0; u < 4 * kUnroll; ++u) {
    const int64_t i = c0 + u * kThreads + threadIdx.x;
    if (i < n) o[i] = l[i] - g[i];
  }
}

// The send statistics of the standard dithering stage of a compressed client delta (compressors.py:339-365 count
// one entry per nonzero element of their input; here: the delta at the top-k's kept indices): thread j looks up the
// tensor of idx[j] (a uniform walk over the pack's offsets) and forms the delta as delta_flatten does; one 64-bit
// atomic add per wave of the ballot's population count.
__global__ __launch_bounds__(kThreads) void delta_count_nonzero_kernel(TensorPack p, const int32_t* __restrict__ idx,
                                                                      int64_t k, unsigned long long* __restrict__ count) {
  const int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  bool nz = false;
  if (j < k) {
    const int64_t i = idx[j];
    for (int t = 0; t < p.nt; ++t) {
      if (i >= p.off[t] && i < p.off[t] + p.n[t]) {
        const int64_t o = i - p.off[t];
        nz = !(p.l[t][o] - p.g[t][o] == 0.0f);  // (a NaN delta counts, as `x[i] == 0.0` is false for it)
      }
    }
  }
  const unsigned long long b = __ballot(nz);
  if ((threadIdx.x & (kWave - 1)) == 0 && b != 0ull) atomicAdd(count, (unsigned long long)__popcll(b));
}

// The same count for a round's clients at once (flc_count_nonzero_at_batch: the deferred compressed messages of
// compressed.py, whose deltas were flattened when the messages were made): client c = blockIdx.y counts the nonzero
// x_c[idx_c[j]]; the counts are zeroed by a one-wave launch ahead of it (stream-ordered).
constexpr int kMaxCount = 32;  // clients per launch (kernel-argument budget)
struct CountPack {
  const float* x[kMaxCount];
  const int32_t* idx[kMaxCount];
  unsigned long long* out[kMaxCount];
  int nc;
};

__global__ __launch_bounds__(kWave) void zero_counts_kernel(CountPack p) {
  if ((int)threadIdx.x < p.nc) *p.out[threadIdx.x] = 0ull;
}

__global__ __launch_bounds__(kThreads) void count_nonzero_at_batch_kernel(CountPack p, int64_t k) {
  const int c = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool nz = j < k && !(p.x[c][p.idx[c][j]] == 0.0f);  // (a NaN counts, as for the fused form)
  const unsigned long long b = __ballot(nz);
  if ((threadIdx.x & (kWave - 1)) == 0 && b != 0ull) atomicAdd(p.out[c], (unsigned long long)__popcll(b));
}

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

int flc_count_nonzero_at_batch(const float* const* xs, const int32_t* const* idx, int n_clients, int64_t n,
                               int64_t k, int64_t* const* counts, void* stream) {
  if (n_clients < 0 || (n_clients > 0 && (!xs || !idx || !counts)) || n <= 0 || k < 0 || k > n)
    return fail(FLC_EINVAL, "flc_count_nonzero_at_batch: bad arguments");
  hipStream_t st = as_stream(stream);
  for (int c0 = 0; c0 < n_clients; c0 += kMaxCount) {
    CountPack p{};
    p.nc = std::min(n_clients - c0, kMaxCount);
    for (int c = 0; c < p.nc; ++c) {
      if (!xs[c0 + c] || !counts[c0 + c] || (k > 0 && !idx[c0 + c]))
        return fail(FLC_EINVAL, "flc_count_nonzero_at_batch: null pointer for client %d", c0 + c);
      p.x[c] = xs[c0 + c];
      p.idx[c] = idx[c0 + c];
      p.out[c] = reinterpret_cast<unsigned long long*>(counts[c0 + c]);
    }
    FLC_LAUNCH("zero_counts", zero_counts_kernel, dim3(1), dim3(kWave), 0, st, p);
    if (k > 0)
      FLC_LAUNCH("count_nonzero_at_batch", count_nonzero_at_batch_kernel,
                 dim3((unsigned)cdiv(k, kThreads), (unsigned)p.nc), dim3(kThreads), 0, st, p, k);
  }
  return FLC_OK;
}

int flc_delta_flatten(const float* const* local, const float* const* global, const int64_t* sizes, int n_tensors,
                      float* out, void* stream) {
  if (n_tensors < 0 || (n_tensors > 0 && (!local || !global || !sizes)))
    return fail(FLC_EINVAL, "flc_delta_flatten: bad arguments");
  hipStream_t st = as_stream(stream);
  int64_t off = 0;
  for (int t0 = 0; t0 < n_tensors; t0 += kMaxT) {
    TensorPack p{};
    int blocks = 0;
    p.nt = 0;
    for (int t = t0; t < std::min(n_tensors, t0 + kMaxT); ++t) {
      if (sizes[t] < 0) return fail(FLC_EINVAL, "flc_delta_flatten: negative size for tensor %d", t);
      if (sizes[t] > 0 && (!local[t] || !global[t] || !out))
        return fail(FLC_EINVAL, "flc_delta_flatten: null pointer for tensor %d", t);
      if (sizes[t] == 0) continue;
      const int i = p.nt++;
      p.l[i] = local[t];
      p.g[i] = global[t];
      p.off[i] = off;
      p.n[i] = sizes[t];
      p.blk0[i] = blocks;
      // (the 16-B path clamps idle lanes to element 0..3, so it needs n >= 4)
      if (sizes[t] >= 4 && aligned16(local[t]) && aligned16(global[t]) && aligned16(out + off)) p.vec |= 1ull << i;
      const int64_t nb = cdiv(sizes[t], kChunk);
      if (blocks + nb > 0x7fffffff) return fail(FLC_EINVAL, "flc_delta_flatten: too many elements");
      blocks += (int)nb;
      off += sizes[t];
    }
    p.blk0[p.nt] = blocks;
    if (blocks > 0) FLC_LAUNCH("delta_flatten", delta_flatten_kernel, dim3(blocks), dim3(kThreads), 0, st, p, out);
  }
  return FLC_OK;
}

int flc_delta_count_nonzero_at(const float* const* local, const float* const* global, const int64_t* sizes,
                               int n_tensors, const int32_t* idx, int64_t k, int64_t* count, void* stream) {
  if (n_tensors < 0 || (n_tensors > 0 && (!local || !global || !sizes)) || k < 0 || !count || (k > 0 && !idx))
    return fail(FLC_EINVAL, "flc_delta_count_nonzero_at: bad arguments");
  hipStream_t st = as_stream(stream);
  FLC_CHECK_HIP(hipMemsetAsync(count, 0, sizeof(int64_t), st));
  if (k == 0) return FLC_OK;
  int64_t off = 0;
  for (int t0 = 0; t0 < n_tensors; t0 += kMaxT) {
    TensorPack p{};
    for (int t = t0; t < std::min(n_tensors, t0 + kMaxT); ++t) {
      if (sizes[t] < 0) return fail(FLC_EINVAL, "flc_delta_count_nonzero_at: negative size for tensor %d", t);
      if (sizes[t] > 0 && (!local[t] || !global[t]))
        return fail(FLC_EINVAL, "flc_delta_count_nonzero_at: null pointer for tensor %d", t);
      if (sizes[t] == 0) continue;
      const int i = p.nt++;
      p.l[i] = local[t];
      p.g[i] = global[t];
      p.off[i] = off;
      p.n[i] = sizes[t];
      off += sizes[t];
    }
    if (p.nt > 0)
      FLC_LAUNCH("delta_count_nonzero", delta_count_nonzero_kernel, dim3((unsigned)cdiv(k, kThreads)), dim3(kThreads), 0,
                 st, p, idx, k, reinterpret_cast<unsigned long long*>(count));
  }
  return FLC_OK;
}

}  // extern "C"
