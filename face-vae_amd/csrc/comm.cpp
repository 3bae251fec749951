// RCCL communicator for the data-parallel step (replaces distributed.py:24-31's
// init_process_group("nccl") + DDP's gradient all-reduce, logger.py:55,58, and the SyncBN
// collectives).  One communicator per process (one process per GPU); the unique id is
// exchanged by the caller (torch.distributed TCPStore); collectives are stream-ordered
// on the caller's stream, so no host synchronisation is ever needed.
#include <rccl/rccl.h>
#include <string.h>

#include "common.h"

namespace {
int map_dtype(int dt, ncclDataType_t* out) {
  switch (dt) {
    case FV_F32: *out = ncclFloat32; return FV_OK;
    case FV_BF16: *out = ncclBfloat16; return FV_OK;
    case FV_F64: *out = ncclFloat64; return FV_OK;
  }
  fv_set_error("comm: unsupported dtype %d", dt);
  return FV_E_BADARG;
}
int nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    fv_set_error("%s: %s", what, ncclGetErrorString(r));
    return FV_E_COMM;
  }
  return FV_OK;
}
}  // namespace

extern "C" {

int fv_comm_unique_id(uint8_t out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "unique id size");
  ncclUniqueId id;
  int st = nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  if (st) return st;
  memcpy(out, &id, sizeof(id));
  return FV_OK;
}

int fv_comm_init(const uint8_t id[128], int nranks, int rank, int device, fv_comm_t* comm) {
  FV_REQUIRE(id && comm && nranks > 0 && rank >= 0 && rank < nranks, "comm init: bad args");
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    fv_set_error("hipSetDevice(%d): %s", device, hipGetErrorString(e));
    return (int)e;
  }
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c;
  int st = nccl_check(ncclCommInitRank(&c, nranks, uid, rank), "ncclCommInitRank");
  if (st) return st;
  *comm = (fv_comm_t)c;
  return FV_OK;
}

int fv_comm_allreduce(fv_comm_t comm, void* buf, size_t count, int dtype, int op, void* stream) {
  FV_REQUIRE(op >= 0 && op <= 2, "allreduce: unknown op %d (0 = sum, 1 = average, 2 = max)", op);
  FV_REQUIRE(comm && buf, "allreduce: bad args");
  ncclDataType_t dt;
  int st = map_dtype(dtype, &dt);
  if (st) return st;
  const ncclRedOp_t rop = op == 1 ? ncclAvg : op == 2 ? ncclMax : ncclSum;
  return nccl_check(ncclAllReduce(buf, buf, count, dt, rop, (ncclComm_t)comm, (hipStream_t)stream),
                    "ncclAllReduce");
}

int fv_comm_allgather(fv_comm_t comm, const void* send, void* recv, size_t count_per_rank, int dtype,
                      void* stream) {
  FV_REQUIRE(comm && send && recv, "allgather: bad args");
  ncclDataType_t dt;
  int st = map_dtype(dtype, &dt);
  if (st) return st;
  return nccl_check(ncclAllGather(send, recv, count_per_rank, dt, (ncclComm_t)comm, (hipStream_t)stream),
                    "ncclAllGather");
}

int fv_comm_broadcast(fv_comm_t comm, void* buf, size_t count, int dtype, int root, void* stream) {
  FV_REQUIRE(comm && buf, "broadcast: bad args");
  ncclDataType_t dt;
  int st = map_dtype(dtype, &dt);
  if (st) return st;
  return nccl_check(ncclBroadcast(buf, buf, count, dt, root, (ncclComm_t)comm, (hipStream_t)stream),
                    "ncclBroadcast");
}

// Failure detection (the reference's mp.spawn tears every rank down on an exception,
// train.py:54; a dead or stuck peer otherwise hangs every rank inside its next collective).
// *result = the communicator's asynchronous error (ncclResult_t; 0 = ncclSuccess, 7 =
// ncclInProgress).  Host-only query, safe from a watchdog thread while collectives are queued.
int fv_comm_async_error(fv_comm_t comm, int* result) {
  FV_REQUIRE(comm && result, "async_error: bad args");
  ncclResult_t r = ncclSuccess;
  int st = nccl_check(ncclCommGetAsyncError((ncclComm_t)comm, &r), "ncclCommGetAsyncError");
  if (st) return st;
  *result = (int)r;
  if (r != ncclSuccess && r != ncclInProgress) fv_set_error("RCCL async error: %s", ncclGetErrorString(r));
  return FV_OK;
}

// number of ranks the communicator spans (ncclCommCount)
int fv_comm_count(fv_comm_t comm, int* nranks) {
  FV_REQUIRE(comm && nranks, "comm_count: bad args");
  return nccl_check(ncclCommCount((ncclComm_t)comm, nranks), "ncclCommCount");
}

// abort every outstanding operation of the communicator and free it (ncclCommAbort); the
// handle is invalid afterwards
int fv_comm_abort(fv_comm_t comm) {
  if (!comm) return FV_OK;
  return nccl_check(ncclCommAbort((ncclComm_t)comm), "ncclCommAbort");
}

int fv_comm_destroy(fv_comm_t comm) {
  if (!comm) return FV_OK;
  return nccl_check(ncclCommDestroy((ncclComm_t)comm), "ncclCommDestroy");
}

}  // extern "C"
