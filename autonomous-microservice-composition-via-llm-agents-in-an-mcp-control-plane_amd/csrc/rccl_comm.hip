// K13: thin C++ wrapper over rccl.h (collective sites C1-C6).
//
// One communicator per tensor-parallel group, created from an ncclUniqueId the
// caller broadcasts over its bootstrap store (C5).  Collectives run on the
// caller's HIP stream, so they order with the engine's kernels and can be
// captured in a hipGraph.  No torch / c10 dependency: the Python side passes
// raw pointers, element counts and the stream.
#include <rccl/rccl.h>
#include <string.h>

#include "kernels.h"

namespace {

ncclDataType_t dtype_of(int code) {
  switch (code) {
    case 0: return ncclBfloat16;
    case 1: return ncclFloat32;
    case 2: return ncclInt32;
    case 3: return ncclFloat16;
    default: return ncclInt8;
  }
}

ncclRedOp_t op_of(int code) {
  switch (code) {
    case 1: return ncclMax;
    case 2: return ncclMin;
    default: return ncclSum;
  }
}

}  // namespace

size_t rccl_unique_id_bytes() { return sizeof(ncclUniqueId); }

int rccl_get_unique_id(void* out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
  memcpy(out, &id, sizeof(id));
  return 0;
}

void* rccl_init(int world, int rank, const void* unique_id) {
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  ncclComm_t comm = nullptr;
  if (ncclCommInitRank(&comm, world, id, rank) != ncclSuccess) return nullptr;
  return comm;
}

int rccl_all_reduce(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                    hipStream_t s) {
  return ncclAllReduce(send, recv, count, dtype_of(dtype), op_of(op), (ncclComm_t)comm, s) ==
                 ncclSuccess ? 0 : -1;
}

int rccl_all_gather(void* comm, const void* send, void* recv, size_t count, int dtype,
                    hipStream_t s) {
  return ncclAllGather(send, recv, count, dtype_of(dtype), (ncclComm_t)comm, s) == ncclSuccess
             ? 0 : -1;
}

int rccl_reduce_scatter(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                        hipStream_t s) {
  return ncclReduceScatter(send, recv, count, dtype_of(dtype), op_of(op), (ncclComm_t)comm, s) ==
                 ncclSuccess ? 0 : -1;
}

int rccl_broadcast(void* comm, void* buf, size_t count, int dtype, int root, hipStream_t s) {
  return ncclBroadcast(buf, buf, count, dtype_of(dtype), root, (ncclComm_t)comm, s) ==
                 ncclSuccess ? 0 : -1;
}

const char* rccl_last_error(void* comm) {
  ncclResult_t r;
  if (ncclCommGetAsyncError((ncclComm_t)comm, &r) != ncclSuccess) return "unknown";
  return ncclGetErrorString(r);
}

void rccl_destroy(void* comm) {
  if (comm) (void)ncclCommDestroy((ncclComm_t)comm);
}
