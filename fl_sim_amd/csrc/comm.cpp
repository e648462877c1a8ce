// comm.cpp — the multi-GPU exchange of the aggregation round for callers outside torch (SURVEY §8(b) item 3,
// §8(e)): RCCL (the NCCL API on ROCm; collectives over xGMI) behind the C ABI.
//
// One process per GPU.  The reference runs its clients one after another and places client i on device
// i mod N (nodes.py:706-713); the server folds every client's delta in message order (nodes.py:1165-1180).  Here a
// rank folds its own clients, then either
//   * flc_rccl_reduce sums the ranks' partial sums to the root (fp32; RCCL's summation order across ranks), or
//   * flc_rccl_allgather moves every rank's packed wire records (flc_stacked_wire_layout) to every rank, which then
//     folds all clients in client order (flc_stacked_fold_wires): bit-identical to one device at any N.
// RCCL is looked up on first use, so the library itself has no link-time dependency on it: FLC_RCCL_LIB (an explicit
// path) if set; else an RCCL already in the process — found by its symbols, or among the loaded objects by name
// (inside a torch process that is torch's own RCCL, whatever its soname, the one its process groups use); else
// dlopen("librccl.so.1").
#include <dlfcn.h>
#include <link.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

#include "flc_runtime.hpp"
#include "flcodec.h"

namespace flc {
namespace {

struct Rccl {
  bool ok = false;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclReduce) reduce = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommCount) count = nullptr;
  decltype(&ncclCommUserRank) user_rank = nullptr;
};

// the path of a loaded object whose file name starts with "librccl" (dl_iterate_phdr callback)
int find_loaded_rccl(struct dl_phdr_info* info, size_t, void* out) {
  const char* name = info->dlpi_name;
  if (!name || !*name) return 0;
  const char* base = strrchr(name, '/');
  base = base ? base + 1 : name;
  if (strncmp(base, "librccl", 7) != 0) return 0;
  *static_cast<const char**>(out) = name;
  return 1;
}

// where the symbols came from (flc_comm_rccl_origin): "env", "global", "loaded", "dlopen" or "none"
const char* g_origin = "none";

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    const char* origin = "none";
    if (const char* path = getenv("FLC_RCCL_LIB")) {
      h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
      if (h) origin = "env";
    }
    // in the global namespace already: every symbol is then resolved there.  glibc's RTLD_DEFAULT is a null handle,
    // so this case is tracked by its own flag, never by testing the handle
    bool global = false;
    if (!h && dlsym(RTLD_DEFAULT, "ncclCommInitRank")) {
      global = true;
      origin = "global";
    }
    if (!h && !global) {
      const char* loaded = nullptr;  // loaded privately (e.g. as a dependency of torch's HIP library)
      dl_iterate_phdr(find_loaded_rccl, &loaded);
      if (loaded) h = dlopen(loaded, RTLD_NOW | RTLD_NOLOAD);
      if (h) origin = "loaded";
    }
    if (!h && !global) {
      h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
      if (h) origin = "dlopen";
    }
    if (!h && !global) return;
    void* const src = global ? RTLD_DEFAULT : h;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(src, "ncclGetUniqueId"));
    r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(src, "ncclCommInitRank"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(src, "ncclCommDestroy"));
    r.reduce = reinterpret_cast<decltype(r.reduce)>(dlsym(src, "ncclReduce"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(src, "ncclAllReduce"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(src, "ncclAllGather"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(src, "ncclGetErrorString"));
    r.count = reinterpret_cast<decltype(r.count)>(dlsym(src, "ncclCommCount"));
    r.user_rank = reinterpret_cast<decltype(r.user_rank)>(dlsym(src, "ncclCommUserRank"));
    r.ok = r.get_unique_id && r.init_rank && r.destroy && r.reduce && r.all_reduce && r.all_gather &&
           r.error_string && r.count && r.user_rank;
    g_origin = r.ok ? origin : "none";
  });
  return r;
}

int need_rccl(const char* who) {
  if (!rccl().ok) return fail(FLC_ECOMM, "%s: RCCL (librccl.so.1) could not be loaded", who);
  return FLC_OK;
}

int nccl_fail(ncclResult_t e, const char* who) {
  return fail(FLC_ECOMM, "%s: %s", who, rccl().error_string ? rccl().error_string(e) : "RCCL error");
}

#define FLC_NCCL(expr, who)                                  \
  do {                                                       \
    const ncclResult_t r_ = (expr);                          \
    if (r_ != ncclSuccess) return nccl_fail(r_, who);        \
  } while (0)

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

size_t flc_comm_id_bytes(void) { return sizeof(ncclUniqueId); }

const char* flc_comm_rccl_origin(void) {
  rccl();
  return g_origin;
}

int flc_comm_unique_id(void* id_out) {
  if (!id_out) return fail(FLC_EINVAL, "flc_comm_unique_id: null output");
  if (int rc = need_rccl("flc_comm_unique_id")) return rc;
  ncclUniqueId id;
  FLC_NCCL(rccl().get_unique_id(&id), "flc_comm_unique_id");
  memcpy(id_out, &id, sizeof(id));
  return FLC_OK;
}

int flc_comm_init(const void* id, int nranks, int rank, int device, void** comm_out) {
  if (!id || !comm_out || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(FLC_EINVAL, "flc_comm_init: bad arguments (rank %d of %d)", rank, nranks);
  if (int rc = need_rccl("flc_comm_init")) return rc;
  // ncclCommInitRank binds the communicator to the current device: switch to `device` for the call only, and give
  // the calling thread (which torch shares) its own current device back
  int prev = -1;
  FLC_CHECK_HIP(hipGetDevice(&prev));
  if (device >= 0) FLC_CHECK_HIP(hipSetDevice(device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  const ncclResult_t r = rccl().init_rank(&c, nranks, uid, rank);
  if (device >= 0 && prev >= 0 && prev != device) FLC_CHECK_HIP(hipSetDevice(prev));
  if (r != ncclSuccess) return nccl_fail(r, "flc_comm_init");
  *comm_out = c;
  return FLC_OK;
}

int flc_comm_size(void* comm, int* nranks, int* rank) {
  if (!comm || !nranks || !rank) return fail(FLC_EINVAL, "flc_comm_size: bad arguments");
  if (int rc = need_rccl("flc_comm_size")) return rc;
  FLC_NCCL(rccl().count(static_cast<ncclComm_t>(comm), nranks), "flc_comm_size");
  FLC_NCCL(rccl().user_rank(static_cast<ncclComm_t>(comm), rank), "flc_comm_size");
  return FLC_OK;
}

int flc_comm_destroy(void* comm) {
  if (!comm) return FLC_OK;
  if (int rc = need_rccl("flc_comm_destroy")) return rc;
  FLC_NCCL(rccl().destroy(static_cast<ncclComm_t>(comm)), "flc_comm_destroy");
  return FLC_OK;
}

int flc_rccl_reduce(const float* send, float* recv, int64_t n, int root, void* comm, void* stream) {
  if (!send || !comm || n < 0) return fail(FLC_EINVAL, "flc_rccl_reduce: bad arguments");
  if (int rc = need_rccl("flc_rccl_reduce")) return rc;
  FLC_NCCL(rccl().reduce(send, recv, (size_t)n, ncclFloat32, ncclSum, root, static_cast<ncclComm_t>(comm),
                         as_stream(stream)),
           "flc_rccl_reduce");
  return FLC_OK;
}

int flc_rccl_allreduce(const float* send, float* recv, int64_t n, void* comm, void* stream) {
  if (!send || !recv || !comm || n < 0) return fail(FLC_EINVAL, "flc_rccl_allreduce: bad arguments");
  if (int rc = need_rccl("flc_rccl_allreduce")) return rc;
  FLC_NCCL(rccl().all_reduce(send, recv, (size_t)n, ncclFloat32, ncclSum, static_cast<ncclComm_t>(comm),
                             as_stream(stream)),
           "flc_rccl_allreduce");
  return FLC_OK;
}

int flc_rccl_allgather(const void* send, void* recv, int64_t bytes_per_rank, void* comm, void* stream) {
  if (!send || !recv || !comm || bytes_per_rank < 0) return fail(FLC_EINVAL, "flc_rccl_allgather: bad arguments");
  if (int rc = need_rccl("flc_rccl_allgather")) return rc;
  FLC_NCCL(rccl().all_gather(send, recv, (size_t)bytes_per_rank, ncclUint8, static_cast<ncclComm_t>(comm),
                             as_stream(stream)),
           "flc_rccl_allgather");
  return FLC_OK;
}

}  // extern "C"
