// Native RCCL all-reduce for hpe_fit_steps_dp (host code only).
//
// hpe_fit_steps_dp calls an hpe_allreduce_fn once per optimizer step on [gradient | sse, sae, 0, 0].
// With a gloo process group that hook is a Python callback into torch.distributed (one interpreter
// re-entry per step, tens of µs at the P = 1 steps).  On GPU ranks the hook can
// instead be hpe_rccl_allreduce below with `user` = an RCCL communicator of the same ranks: the sum
// is enqueued on the step's own stream, ordered before the optimizer launch that follows it, and the
// step loop never leaves C.  The communicator is this library's own (not torch's): rank 0 makes the
// id (hpe_rccl_unique_id), the caller broadcasts its 128 bytes over its process group, and every rank
// joins with hpe_rccl_comm_init on its current device (hpe/engine.py).
//
// librccl is opened at run time (dlopen), so libhpe.so has no link dependency on it; the symbols are
// the public NCCL API that rccl.h declares (types only are taken from the header).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/hpe.h"
#include "hpe_common.h"

namespace {

struct RcclApi {
  bool tried = false, ok = false;
  char why[256] = {0};
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

RcclApi load_api() {
  RcclApi a;
  a.tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    snprintf(a.why, sizeof a.why, "dlopen(librccl): %s", dlerror());
    return a;
  }
  a.get_unique_id = (decltype(a.get_unique_id))dlsym(h, "ncclGetUniqueId");
  a.comm_init_rank = (decltype(a.comm_init_rank))dlsym(h, "ncclCommInitRank");
  a.comm_destroy = (decltype(a.comm_destroy))dlsym(h, "ncclCommDestroy");
  a.all_reduce = (decltype(a.all_reduce))dlsym(h, "ncclAllReduce");
  a.error_string = (decltype(a.error_string))dlsym(h, "ncclGetErrorString");
  a.ok = a.get_unique_id && a.comm_init_rank && a.comm_destroy && a.all_reduce && a.error_string;
  if (!a.ok) snprintf(a.why, sizeof a.why, "librccl lacks the NCCL entry points");
  return a;
}

RcclApi& api() {
  static RcclApi a = load_api();  // once, thread-safe
  return a;
}

int rccl_fail(const char* what, ncclResult_t r) {
  char msg[320];
  snprintf(msg, sizeof msg, "%s: %s", what, api().error_string ? api().error_string(r) : "RCCL error");
  return hpe_fail(HPE_ERUNTIME, "%s", msg);
}

}  // namespace

extern "C" int hpe_rccl_available(void) { return api().ok ? 1 : 0; }

extern "C" int hpe_rccl_unique_id(void* id_out) {
  if (!id_out) return hpe_fail(HPE_EINVAL, "hpe_rccl_unique_id: null argument");
  RcclApi& a = api();
  if (!a.ok) return hpe_fail(HPE_ERUNTIME, "%s", a.why);
  ncclUniqueId id;
  const ncclResult_t r = a.get_unique_id(&id);
  if (r != ncclSuccess) return rccl_fail("ncclGetUniqueId", r);
  memcpy(id_out, id.internal, HPE_RCCL_ID_BYTES);
  return HPE_OK;
}

extern "C" int hpe_rccl_comm_init(const void* id, int32_t nranks, int32_t rank, void** comm_out) {
  if (!id || !comm_out) return hpe_fail(HPE_EINVAL, "hpe_rccl_comm_init: null argument");
  *comm_out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks) return hpe_fail(HPE_EINVAL, "hpe_rccl_comm_init: bad rank / size");
  RcclApi& a = api();
  if (!a.ok) return hpe_fail(HPE_ERUNTIME, "%s", a.why);
  ncclUniqueId uid;
  memcpy(uid.internal, id, HPE_RCCL_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t r = a.comm_init_rank(&c, nranks, uid, rank);  // on the current HIP device
  if (r != ncclSuccess) return rccl_fail("ncclCommInitRank", r);
  *comm_out = (void*)c;
  return HPE_OK;
}

extern "C" int hpe_rccl_comm_destroy(void* comm) {
  if (!comm) return HPE_OK;
  RcclApi& a = api();
  if (!a.ok) return hpe_fail(HPE_ERUNTIME, "%s", a.why);
  const ncclResult_t r = a.comm_destroy((ncclComm_t)comm);
  return r == ncclSuccess ? HPE_OK : rccl_fail("ncclCommDestroy", r);
}

// an hpe_allreduce_fn: in-place sum of buf[0, n) over the communicator's ranks, enqueued on `stream`
extern "C" int hpe_rccl_allreduce(float* buf, int64_t n, void* stream, void* comm) {
  if (!buf || !comm || n < 0) return hpe_fail(HPE_EINVAL, "hpe_rccl_allreduce: bad argument");
  RcclApi& a = api();
  if (!a.ok) return hpe_fail(HPE_ERUNTIME, "%s", a.why);
  const ncclResult_t r = a.all_reduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, (ncclComm_t)comm, (hipStream_t)stream);
  return r == ncclSuccess ? HPE_OK : rccl_fail("ncclAllReduce", r);
}
