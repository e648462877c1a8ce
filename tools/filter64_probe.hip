// filter64_probe.hip — where does the float64 top-k filter pass (f64.hip sel64_filter_kernel) lose against a plain
// 200 MB read?  One block of 256 threads per 8192-element chunk of 25 M doubles, the chunk's 32 elements per thread
// loaded at once, then per mode:
//   0: sum only (the read alone)
//   1: + the order key and the candidate test, counted per thread (no LDS, no stores)
//   2: + the wave append through an LDS counter (ds_add_rtn per element slot with a candidate)
//   3: + the value's 8-B store into the chunk's segment
//   4: + the position's 2-B store (the full filter)
//   5: as 4, with the position stored as 4 B
// The candidate floor t_lo is the key of 2.326 (k = 1 % of a standard normal vector).
// Build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/filter64_probe tools/filter64_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kT = 256, kE = 4, kIt = 8, kChunk = kT * kE * kIt;

__device__ __forceinline__ unsigned long long order_key64(double v) {
  unsigned long long b = (unsigned long long)__double_as_longlong(v);
  if ((b & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) return ~0ull;
  if (b == 0x8000000000000000ull) b = 0ull;
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

template <int MODE>
__global__ __launch_bounds__(kT) void filt(const double* __restrict__ x, long n, unsigned long long t_lo, int segcap,
                                           unsigned long long* __restrict__ seg, unsigned short* __restrict__ segi,
                                           unsigned* __restrict__ segi4, int* __restrict__ counts) {
  __shared__ unsigned s_n;
  const int tid = threadIdx.x;
  if (tid == 0) s_n = 0u;
  const long c0 = (long)blockIdx.x * kChunk;
  double v[kIt][kE];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const long e0 = c0 + ((long)it * kT + tid) * kE;
    if (e0 + kE <= n) {
      const double2 a = *reinterpret_cast<const double2*>(x + e0);
      const double2 b = *reinterpret_cast<const double2*>(x + e0 + 2);
      v[it][0] = a.x; v[it][1] = a.y; v[it][2] = b.x; v[it][3] = b.y;
    } else {
#pragma unroll
      for (int j = 0; j < kE; ++j) v[it][j] = e0 + j < n ? x[e0 + j] : 0.0;
    }
  }
  __syncthreads();
  double acc = 0.0;
  int cnt = 0;
  unsigned long long* my = seg + (size_t)blockIdx.x * segcap;
#pragma unroll
  for (int it = 0; it < kIt; ++it)
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      const int loc = (it * kT + tid) * kE + j;
      if (MODE == 0) {
        acc += v[it][j];
        continue;
      }
      const unsigned long long key = order_key64(v[it][j]);
      const bool in = c0 + loc < n && key >= t_lo;
      if (MODE == 1) {
        cnt += in;
        continue;
      }
      const unsigned long long m = __ballot(in);
      if (m == 0ull) continue;
      unsigned base = 0u;
      if ((tid & 63) == 0) base = atomicAdd(&s_n, (unsigned)__popcll(m));
      base = (unsigned)__builtin_amdgcn_readlane((int)base, 0);
      const unsigned p = base + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      if (MODE >= 3 && in && p < (unsigned)segcap) {
        my[p] = (unsigned long long)__double_as_longlong(v[it][j]);
        if (MODE == 4) segi[(size_t)blockIdx.x * segcap + p] = (unsigned short)loc;
        if (MODE == 5) segi4[(size_t)blockIdx.x * segcap + p] = (unsigned)loc;
      }
    }
  __syncthreads();
  if (tid == 0) counts[blockIdx.x] = (int)s_n;
  if (acc == 1234.5 || cnt == 12345) counts[0] = -1;
}

int main() {
  const long n = 25000000;
  const int nch = (int)((n + kChunk - 1) / kChunk), segcap = 576;
  std::vector<double> h(n);
  std::mt19937_64 g(5);
  std::normal_distribution<double> nd;
  for (long i = 0; i < n; ++i) h[i] = nd(g);
  double* x;
  unsigned long long* seg;
  unsigned short* segi;
  unsigned* segi4;
  int* counts;
  CK(hipMalloc(&x, n * 8));
  CK(hipMalloc(&seg, (size_t)nch * segcap * 8));
  CK(hipMalloc(&segi, (size_t)nch * segcap * 2));
  CK(hipMalloc(&segi4, (size_t)nch * segcap * 4));
  CK(hipMalloc(&counts, nch * 4));
  CK(hipMemcpy(x, h.data(), n * 8, hipMemcpyHostToDevice));
  const unsigned long long t_lo = ((unsigned long long)__builtin_bit_cast(unsigned long long, 2.326)) | (1ull << 63);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](int mode) {
    auto launch = [&]() {
      switch (mode) {
        case 0: filt<0><<<nch, kT>>>(x, n, t_lo, segcap, seg, segi, segi4, counts); break;
        case 1: filt<1><<<nch, kT>>>(x, n, t_lo, segcap, seg, segi, segi4, counts); break;
        case 2: filt<2><<<nch, kT>>>(x, n, t_lo, segcap, seg, segi, segi4, counts); break;
        case 3: filt<3><<<nch, kT>>>(x, n, t_lo, segcap, seg, segi, segi4, counts); break;
        case 4: filt<4><<<nch, kT>>>(x, n, t_lo, segcap, seg, segi, segi4, counts); break;
        default: filt<5><<<nch, kT>>>(x, n, t_lo, segcap, seg, segi, segi4, counts); break;
      }
    };
    for (int w = 0; w < 3; ++w) launch();
    CK(hipEventRecord(e0));
    for (int it = 0; it < 20; ++it) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("mode %d: %.1f us per pass (%.2f TB/s of x)\n", mode, ms * 1000 / 20, n * 8.0 / (ms / 20 * 1e-3) / 1e12);
  };
  for (int round = 0; round < 2; ++round)
    for (int mode = 0; mode < 6; ++mode) run(mode);
  int c0;
  CK(hipMemcpy(&c0, counts + 1, 4, hipMemcpyDeviceToHost));
  printf("chunk 1 candidates: %d\n", c0);
  return 0;
}
