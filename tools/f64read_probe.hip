// f64read_probe.hip — the float64 top-k's filter pass (f64.hip sel64_select_kernel) streams 200 MB at ~5 TB/s inside
// the select, against 7.4 TB/s for the float32 encoder's pass.  Is it the access shape?  Read-only passes over
// 25 M doubles (200 MB) in rotation over 3 vectors (600 MB: HBM), one 1024-thread block per CU, non-temporal
// 16-B loads, two chunks in flight, shapes:
//   inter8:  8192-element chunks dealt round-robin to the blocks (ch = b + q G: the select's shape), 4 loads/thread;
//   inter16: 16384-element chunks round-robin, 8 loads/thread;
//   contig8: each block's contiguous range in 8192-element chunks;
//   contig16: the same in 16384-element chunks.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/f64read_probe tools/f64read_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int R, bool CONTIG>
__global__ __launch_bounds__(1024) void rd(const double* __restrict__ x, long nch, double* sink) {
  constexpr long C = 2048L * R;  // elements per chunk
  const int tid = threadIdx.x, G = gridDim.x;
  const long per = (nch + G - 1) / G;
  auto chunk = [&](long q) -> long {  // the block's q-th chunk, or -1
    const long c = CONTIG ? blockIdx.x * per + q : blockIdx.x + q * G;
    return (CONTIG ? q < per && c < nch : c < nch) ? c : -1;
  };
  double acc = 0.0;
  f64x2 a[R], b[R];
  auto ld = [&](long q, f64x2 (&v)[R]) {
    long c = chunk(q);
    if (c < 0) c = 0;
#pragma unroll
    for (int r = 0; r < R; ++r)
      v[r] = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(x + c * C + 2 * (r * 1024 + tid)));
  };
  ld(0, a);
  ld(1, b);
  for (long q = 0; chunk(q) >= 0; q += 2) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc += a[r].x + a[r].y;
    ld(q + 2, a);
    if (chunk(q + 1) < 0) break;
#pragma unroll
    for (int r = 0; r < R; ++r) acc += b[r].x + b[r].y;
    ld(q + 3, b);
  }
  if (acc == 1234.5) sink[tid] = acc;
}

int main() {
  const long n = 25165824;  // 3072 chunks of 8192 (25.2 M doubles, 201 MB)
  double* xs[3];
  double* sink;
  CK(hipMalloc(&sink, 8192));
  for (auto& p : xs) {
    CK(hipMalloc(&p, n * 8));
    CK(hipMemset(p, 0, n * 8));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto t = [&](auto launch) {
    for (int w = 0; w < 6; ++w) launch(w % 3);
    CK(hipEventRecord(e0));
    for (int it = 0; it < 30; ++it) launch(it % 3);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.0f / 30;
  };
  for (int round = 0; round < 2; ++round) {
    const float a = t([&](int v) { rd<4, false><<<256, 1024>>>(xs[v], n / 8192, sink); });
    const float b = t([&](int v) { rd<8, false><<<256, 1024>>>(xs[v], n / 16384, sink); });
    const float c = t([&](int v) { rd<4, true><<<256, 1024>>>(xs[v], n / 8192, sink); });
    const float d = t([&](int v) { rd<8, true><<<256, 1024>>>(xs[v], n / 16384, sink); });
    printf("round %d: inter8 %.1f us (%.2f TB/s) | inter16 %.1f (%.2f) | contig8 %.1f (%.2f) | contig16 %.1f (%.2f)\n",
           round, a, n * 8 / (a * 1e-6) / 1e12, b, n * 8 / (b * 1e-6) / 1e12, c, n * 8 / (c * 1e-6) / 1e12, d,
           n * 8 / (d * 1e-6) / 1e12);
  }
  return 0;
}
