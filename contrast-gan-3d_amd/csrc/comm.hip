// Data-parallel gradient averaging issued from C++: RCCL all-reduces over
// xGMI as recordable plan entries, so a data-parallel step stays ONE launch plan (the generator's
// bucket all-reduces on the communication stream while its backward continues, the critic's on the
// critical path before its Adam step) instead of Python host callables splitting it.
//
// RCCL is the process's own: PyTorch-ROCm already loaded its librccl for torch.distributed, so the
// entry points are resolved from the loaded library (dlopen RTLD_NOLOAD) and only fall back to
// loading ROCm's librccl.so.1 — one RCCL per process.  The communicator a caller passes is, by
// default, the torch process group's own (ops.NativeComm: ProcessGroupNCCL's ncclComm_t, one
// communicator per process; a second one slowed every kernel of a one-GPU step ~2.4x); with
// cgan3d_comm_init the library builds its own from a unique id the caller broadcasts
// (CGAN3D_COMM=own).  On a shared communicator every rank must issue the same collectives in the
// same order, each ordered after the previous one by stream dependencies.
#include <dlfcn.h>

#include <cstring>

#include <rccl/rccl.h>

#include "common.h"

namespace cg {

struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
  bool shared = false;  // resolved from the RCCL the process had already loaded (torch.distributed's)
};

static Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = nullptr;
    for (const char* name : {"librccl.so", "librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);  // the one torch.distributed already uses
      if (h) break;
    }
    x.shared = h != nullptr;
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    x.init_rank = reinterpret_cast<decltype(x.init_rank)>(dlsym(h, "ncclCommInitRank"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(h, "ncclCommDestroy"));
    x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(dlsym(h, "ncclAllReduce"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(h, "ncclGetErrorString"));
    x.ok = x.get_unique_id && x.init_rank && x.destroy && x.all_reduce && x.error_string;
    return x;
  }();
  return r;
}

}  // namespace cg

using namespace cg;

#define CG_RCCL_READY(who) CG_CHECK_ARG(rccl().ok, "%s: RCCL (librccl) could not be loaded", who)

extern "C" int32_t cgan3d_comm_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

extern "C" int cgan3d_comm_unique_id(void* out) {
  CG_RCCL_READY("cgan3d_comm_unique_id");
  CG_CHECK_ARG(out != nullptr, "cgan3d_comm_unique_id: null output");
  ncclUniqueId id;
  const ncclResult_t r = rccl().get_unique_id(&id);
  if (r != ncclSuccess) {
    set_error("cgan3d_comm_unique_id: %s", rccl().error_string(r));
    return CGAN3D_EHIP;
  }
  std::memcpy(out, &id, sizeof(id));
  return CGAN3D_OK;
}

extern "C" int32_t cgan3d_comm_shared_library(void) { return rccl().ok && rccl().shared ? 1 : 0; }

extern "C" int cgan3d_comm_init(const void* unique_id, int32_t nranks, int32_t rank, void** comm) {
  CG_RCCL_READY("cgan3d_comm_init");
  CG_CHECK_ARG(unique_id && comm && nranks > 0 && rank >= 0 && rank < nranks, "cgan3d_comm_init: bad args");
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  ncclComm_t c = nullptr;
  const ncclResult_t r = rccl().init_rank(&c, nranks, id, rank);
  if (r != ncclSuccess) {
    set_error("cgan3d_comm_init: %s", rccl().error_string(r));
    return CGAN3D_EHIP;
  }
  *comm = c;
  return CGAN3D_OK;
}

extern "C" int cgan3d_comm_destroy(void* comm) {
  if (!comm) return CGAN3D_OK;
  CG_RCCL_READY("cgan3d_comm_destroy");
  const ncclResult_t r = rccl().destroy(static_cast<ncclComm_t>(comm));
  if (r != ncclSuccess) {
    set_error("cgan3d_comm_destroy: %s", rccl().error_string(r));
    return CGAN3D_EHIP;
  }
  return CGAN3D_OK;
}

// In place: buf = mean over the communicator's ranks of buf (n fp32), enqueued on `stream`.  While a
// plan is being recorded the all-reduce is recorded (re-issued by cgan3d_plan_run) instead.
extern "C" int cgan3d_allreduce_mean(void* comm, float* buf, int64_t n, void* stream) {
  CG_RCCL_READY("cgan3d_allreduce_mean");
  CG_CHECK_ARG(comm && buf && n > 0, "cgan3d_allreduce_mean: bad args");
  const ncclComm_t c = static_cast<ncclComm_t>(comm);
  const hipStream_t st = static_cast<hipStream_t>(stream);
  auto issue = [c, buf, n, st]() -> hipError_t {
    const ncclResult_t r = rccl().all_reduce(buf, buf, (size_t)n, ncclFloat32, ncclAvg, c, st);
    if (r != ncclSuccess) {
      set_error("ncclAllReduce: %s", rccl().error_string(r));
      return hipErrorUnknown;
    }
    return hipSuccess;
  };
  if (g_rec != nullptr) {
    g_rec->add(issue, st);
    return CGAN3D_OK;
  }
  if (issue() != hipSuccess) return CGAN3D_EHIP;
  return CGAN3D_OK;
}
