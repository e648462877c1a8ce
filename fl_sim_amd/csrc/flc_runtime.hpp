// flc_runtime.hpp — host-side plumbing shared by the C-ABI entry points: error reporting, launch
// checking, and the kernel-duration probe bench.py reads for its live roofline figure.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/flcodec.h"

namespace flc {

int fail(int code, const char* fmt, ...);          // sets flc_last_error, returns code
int hip_fail(hipError_t e, const char* where);     // FLC_EHIP with the HIP error string

// probe: events recorded around launches of one named kernel (flc_probe_set)
void probe_before(const char* name, hipStream_t s);
void probe_after(const char* name, hipStream_t s);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// ---- persistent launches (runtime.cpp) --------------------------------------------------------------------------
// The top-k encoders and the fused quantizer run one block per CU and hand data between blocks inside the launch, so
// every block must be resident at once: one such launch per device at a time.  While every call comes on one stream,
// stream order is the guarantee and nothing is added (an event record after the launch costs the next kernel ~4 us
// of dispatch gap).  The first call on a second stream drains the device once (the earlier stream may be gone by
// now, so nothing is recorded on it), and from then on persistent launches are chained with an event recorded after
// each one (stream-ordered, no host blocking).  Not under stream capture (a captured graph replays in its own order).
int device_cus(int dev);                         // compute units of a device (cached)
int current_cus(int* dev_out);                   // ... of the calling thread's current device
int stream_cus(hipStream_t st, int* dev_out);    // ... of the stream's device (the current one for the null stream)

// The chaining event is bound to the persistent kernel's own dispatch (hipExtLaunchKernel's stop event, FLC_LAUNCH_CO)
// instead of a separate hipEventRecord after it: a marker packet behind each persistent launch had cost the next
// kernel ~4 us of dispatch gap (profiles/r05/r05zo_gate_ab.txt).
class Coresident {  // scoped: construct before the persistent launch(es) on `st`, finish() after them
 public:
  Coresident(hipStream_t st, int dev);
  ~Coresident();
  int status() const { return rc_; }
  hipEvent_t stop_event() const;  // the event a persistent launch carries as its stop event (null: none needed)
  void bound() { bound_ = stop_event() != nullptr; }
  int finish();  // records the chaining event when several streams are in use; returns FLC_OK or the error
 private:
  hipStream_t st_;
  int dev_, rc_ = 0;
  bool gated_ = false, locked_ = false, bound_ = false;
};

// workspace carving: every region 256-byte aligned
struct Carver {
  char* base;
  size_t off = 0, cap;
  Carver(void* b, size_t c) : base(static_cast<char*>(b)), cap(c) {}
  template <typename T>
  T* take(size_t count) {
    off = align_up(off, 256);
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += count * sizeof(T);
    return p;
  }
  bool ok() const { return off <= cap; }
};

}  // namespace flc

#define FLC_LAUNCH(name, kernel, grid, block, shmem, stream, ...)                  \
  do {                                                                            \
    flc::probe_before(name, stream);                                              \
    hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);          \
    flc::probe_after(name, stream);                                               \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) return flc::hip_fail(e_, name);                         \
  } while (0)

// a persistent launch inside a Coresident scope `co`: the gate's chaining event (if any) is the kernel's stop event
#define FLC_LAUNCH_CO(co, name, kernel, grid, block, shmem, stream, ...)                                  \
  do {                                                                                                \
    flc::probe_before(name, stream);                                                                  \
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, nullptr, (co).stop_event(), 0, __VA_ARGS__); \
    flc::probe_after(name, stream);                                                                   \
    hipError_t e_ = hipGetLastError();                                                                \
    if (e_ != hipSuccess) return flc::hip_fail(e_, name);                                             \
    (co).bound();                                                                                     \
  } while (0)

#define FLC_CHECK_HIP(expr)                                                       \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) return flc::hip_fail(e_, #expr);                        \
  } while (0)
