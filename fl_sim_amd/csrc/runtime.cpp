// runtime.cpp — error state, workspace init and the launch probe of the C ABI (include/flcodec.h).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "flc_runtime.hpp"

namespace flc {

static thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  return fail(FLC_EHIP, "%s: %s", where, hipGetErrorString(e));
}

// ---- probe ---------------------------------------------------------------------------------------
namespace {
struct ProbeState {
  std::mutex mu;
  std::string name;  // empty = disabled
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
  hipEvent_t cur_start = nullptr;
};
ProbeState& probe() {
  static ProbeState p;
  return p;
}
hipEvent_t new_event(ProbeState& p) {
  (void)p;
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

void probe_before(const char* name, hipStream_t s) {
  ProbeState& p = probe();
  if (p.name.empty() || p.name != name) return;
  std::lock_guard<std::mutex> lk(p.mu);
  hipEvent_t a;
  if (!p.pool.empty()) {
    a = p.pool.back().first;
    hipEvent_t b = p.pool.back().second;
    p.pool.pop_back();
    p.pending.push_back({a, b});
  } else {
    a = new_event(p);
    p.pending.push_back({a, new_event(p)});
  }
  (void)hipEventRecord(p.pending.back().first, s);
}

void probe_after(const char* name, hipStream_t s) {
  ProbeState& p = probe();
  if (p.name.empty() || p.name != name) return;
  std::lock_guard<std::mutex> lk(p.mu);
  if (!p.pending.empty()) (void)hipEventRecord(p.pending.back().second, s);
}

// ---- persistent launches: one at a time per device (flc_runtime.hpp) ----------------------------------------------
namespace {
struct Gate {
  std::mutex mu;
  hipEvent_t last[64] = {};
  hipStream_t first[64] = {};
  bool used[64] = {};
  bool multi[64] = {};
  bool recorded[64] = {};
  int cus[64] = {};
};
Gate& gate() {
  static Gate g;
  return g;
}
std::mutex& cus_mu() {
  static std::mutex m;
  return m;
}
}  // namespace

int device_cus(int dev) {
  Gate& g = gate();
  std::lock_guard<std::mutex> lk(cus_mu());
  if (g.cus[dev] == 0) {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cu <= 0) cu = 256;
    g.cus[dev] = cu;
  }
  return g.cus[dev];
}

int current_cus(int* dev_out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (dev < 0 || dev >= 64) dev = 0;
  if (dev_out) *dev_out = dev;
  return device_cus(dev);
}

int stream_cus(hipStream_t st, int* dev_out) {
  int dev = -1;
  if (st == nullptr || hipStreamGetDevice(st, &dev) != hipSuccess || dev < 0 || dev >= 64) return current_cus(dev_out);
  if (dev_out) *dev_out = dev;
  return device_cus(dev);
}

Coresident::Coresident(hipStream_t st, int dev) : st_(st), dev_(dev < 0 || dev >= 64 ? 0 : dev) {
  Gate& gt = gate();
  gt.mu.lock();
  locked_ = true;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipError_t e = hipStreamIsCapturing(st_, &cs);
  if (e != hipSuccess) {
    rc_ = hip_fail(e, "hipStreamIsCapturing");
    return;
  }
  gated_ = cs == hipStreamCaptureStatusNone;
  if (!gated_) return;
  if (!gt.used[dev_]) {
    gt.used[dev_] = true;
    gt.first[dev_] = st_;
  } else if (!gt.multi[dev_] && st_ != gt.first[dev_]) {
    // drain dev_ (the device of the earlier persistent launches, not necessarily the calling thread's current
    // device) and make its gate event there: dev_ is made current for these two calls only
    int cur = -1;
    if ((e = hipGetDevice(&cur)) != hipSuccess) {
      rc_ = hip_fail(e, "hipGetDevice");
      return;
    }
    if (cur != dev_ && (e = hipSetDevice(dev_)) != hipSuccess) {
      rc_ = hip_fail(e, "hipSetDevice");
      return;
    }
    e = hipDeviceSynchronize();
    if (e == hipSuccess && !gt.last[dev_]) e = hipEventCreate(&gt.last[dev_]);  // (a kernel's stop event)
    const hipError_t e2 = cur != dev_ ? hipSetDevice(cur) : hipSuccess;
    if (e != hipSuccess || e2 != hipSuccess) {
      rc_ = hip_fail(e != hipSuccess ? e : e2, "draining the gate's device");
      return;
    }
    gt.multi[dev_] = true;
  }
  if (gt.multi[dev_] && gt.recorded[dev_] && (e = hipStreamWaitEvent(st_, gt.last[dev_], 0)) != hipSuccess)
    rc_ = hip_fail(e, "hipStreamWaitEvent");
}

hipEvent_t Coresident::stop_event() const {
  return (rc_ == 0 && gated_ && gate().multi[dev_]) ? gate().last[dev_] : nullptr;
}

int Coresident::finish() {
  Gate& gt = gate();
  if (rc_ == 0 && gated_ && gt.multi[dev_]) {
    if (bound_) {  // the last persistent launch carried the event (FLC_LAUNCH_CO)
      gt.recorded[dev_] = true;
    } else {
      hipError_t e = hipEventRecord(gt.last[dev_], st_);
      if (e != hipSuccess) rc_ = hip_fail(e, "hipEventRecord");
      else gt.recorded[dev_] = true;
    }
  }
  if (locked_) {
    locked_ = false;
    gt.mu.unlock();
  }
  return rc_;
}

Coresident::~Coresident() {
  if (locked_) gate().mu.unlock();
}

}  // namespace flc

extern "C" {

int flc_abi_version(void) { return FLC_ABI_VERSION; }

const char* flc_last_error(void) { return flc::g_err; }

int flc_workspace_init(void* ws, size_t ws_bytes, void* stream) {
  if (ws_bytes == 0) return FLC_OK;
  if (!ws) return flc::fail(FLC_EINVAL, "flc_workspace_init: null workspace");
  FLC_CHECK_HIP(hipMemsetAsync(ws, 0, ws_bytes, flc::as_stream(stream)));
  return FLC_OK;
}

int flc_probe_set(const char* kernel_name) {
  flc::ProbeState& p = flc::probe();
  std::lock_guard<std::mutex> lk(p.mu);
  p.name = kernel_name ? kernel_name : "";
  return FLC_OK;
}

int flc_probe_read(double* total_ms, int64_t* launches) {
  flc::ProbeState& p = flc::probe();
  std::lock_guard<std::mutex> lk(p.mu);
  double tot = 0.0;
  int64_t n = 0;
  for (auto& ev : p.pending) {
    FLC_CHECK_HIP(hipEventSynchronize(ev.second));
    float ms = 0.f;
    FLC_CHECK_HIP(hipEventElapsedTime(&ms, ev.first, ev.second));
    tot += ms;
    ++n;
    p.pool.push_back(ev);
  }
  p.pending.clear();
  if (total_ms) *total_ms = tot;
  if (launches) *launches = n;
  return FLC_OK;
}

}  // extern "C"
