// Data-parallel gradient exchange over RCCL (xGMI) for callers of the C ABI
// that do not run torch.distributed.  The reference has no collective at all
// (single process, lib/graph_model.py:296-298); the build inserts ONE fused
// all-reduce(sum) of the flat gradient bucket between compute_gradients and
// apply_gradients.  Buckets on this path are a few KB, so
// this is latency-bound: one call per step, no bucketing.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "../../include/cheb_mi355.h"

struct cg_comm {
  ncclComm_t comm = nullptr;
  int device = 0;
};

// cg_last_error's thread-local storage lives in cheb_abi.cpp.
extern "C" int cg_internal_set_error(int code, const char* msg);

namespace {
int comm_fail(const char* what, ncclResult_t r) {
  char buf[256];
  snprintf(buf, sizeof(buf), "%s: %s", what, ncclGetErrorString(r));
  return cg_internal_set_error(CG_ERR_COMM, buf);
}
}  // namespace

extern "C" {

int cg_comm_unique_id(unsigned char id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId must be 128 bytes");
  if (!id) return cg_internal_set_error(CG_ERR_ARG, "null id");
  ncclUniqueId uid;
  ncclResult_t r = ncclGetUniqueId(&uid);
  if (r != ncclSuccess) return comm_fail("ncclGetUniqueId", r);
  std::memcpy(id, &uid, sizeof(uid));
  return cg_internal_set_error(CG_OK, "");
}

int cg_comm_init(cg_comm** comm, int nranks, int rank, const unsigned char id[128], int device) {
  if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks)
    return cg_internal_set_error(CG_ERR_ARG, "comm_init: bad arguments");
  *comm = nullptr;
  if (hipSetDevice(device) != hipSuccess)
    return cg_internal_set_error(CG_ERR_HIP, "comm_init: hipSetDevice failed");
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  cg_comm* c = new (std::nothrow) cg_comm();
  if (!c) return cg_internal_set_error(CG_ERR_ALLOC, "comm_init: out of memory");
  c->device = device;
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return comm_fail("ncclCommInitRank", r);
  }
  *comm = c;
  return cg_internal_set_error(CG_OK, "");
}

int cg_allreduce_sum_f32(cg_comm* comm, float* buf, size_t count, void* stream) {
  if (!comm || (!buf && count)) return cg_internal_set_error(CG_ERR_ARG, "allreduce: bad arguments");
  if (count == 0) return cg_internal_set_error(CG_OK, "");
  ncclResult_t r = ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, comm->comm,
                                 reinterpret_cast<hipStream_t>(stream));
  if (r != ncclSuccess) return comm_fail("ncclAllReduce", r);
  return cg_internal_set_error(CG_OK, "");
}

int cg_comm_count(const cg_comm* comm, int* nranks) {
  if (!comm || !comm->comm || !nranks) return cg_internal_set_error(CG_ERR_ARG, "comm_count: bad arguments");
  ncclResult_t r = ncclCommCount(comm->comm, nranks);
  if (r != ncclSuccess) return comm_fail("ncclCommCount", r);
  return cg_internal_set_error(CG_OK, "");
}

int cg_comm_async_error(cg_comm* comm, int* async_status, int abort_on_error) {
  if (!comm || !comm->comm || !async_status)
    return cg_internal_set_error(CG_ERR_ARG, "comm_async_error: bad arguments");
  ncclResult_t async = ncclSuccess;
  ncclResult_t r = ncclCommGetAsyncError(comm->comm, &async);
  if (r != ncclSuccess) return comm_fail("ncclCommGetAsyncError", r);
  *async_status = int(async);
  if (async == ncclSuccess || async == ncclInProgress) {
    *async_status = 0;
    return cg_internal_set_error(CG_OK, "");
  }
  if (abort_on_error) {
    ncclCommAbort(comm->comm);
    comm->comm = nullptr;
  }
  return comm_fail("communicator async error", async);
}

int cg_comm_destroy(cg_comm* comm) {
  if (!comm) return cg_internal_set_error(CG_OK, "");
  ncclResult_t r = comm->comm ? ncclCommDestroy(comm->comm) : ncclSuccess;
  delete comm;
  if (r != ncclSuccess) return comm_fail("ncclCommDestroy", r);
  return cg_internal_set_error(CG_OK, "");
}

}  // extern "C"
