// qe_comm.cpp — multi-GPU aggregation of the engine's statistics over RCCL
// (xGMI within a node).  Groups shard across GPUs with no data-path
// exchange; the only collective is a sum of the 16-counter
// statistics vector (128 B), the batch counterpart of etcd's per-member
// Prometheus counters (server/etcdserver/metrics.go:29-85), which an
// operator otherwise sums across members outside the process.
//
// The communicator is RCCL's own: rank 0 creates a unique id
// (qe_comm_unique_id), the host ships those bytes to the other ranks over
// whatever transport it already has (torch.distributed in bench.py, the
// cluster's RPC layer in a Go host), and every rank calls qe_comm_init.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#include "../../include/etcd_quorum.h"

namespace qe {
int hip_status(hipError_t e);
void set_error(const char *msg);
}  // namespace qe

static int comm_status(ncclResult_t r) {
  if (r == ncclSuccess) return QE_OK;
  qe::set_error(ncclGetErrorString(r));
  return QE_ECOMM;
}

extern "C" {

size_t qe_comm_id_bytes(void) { return sizeof(ncclUniqueId); }

int qe_comm_unique_id(void *id) {
  if (!id) return QE_EINVAL;
  ncclUniqueId u;
  const int rc = comm_status(ncclGetUniqueId(&u));
  if (rc) return rc;
  memcpy(id, &u, sizeof(u));
  return QE_OK;
}

int qe_comm_init(void **comm, uint32_t nranks, uint32_t rank, const void *id, int device) {
  if (!comm || !id || nranks == 0 || rank >= nranks || device < 0) return QE_EINVAL;
  *comm = nullptr;
  int rc = qe::hip_status(hipSetDevice(device));
  if (rc) return rc;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  rc = comm_status(ncclCommInitRank(&c, static_cast<int>(nranks), u, static_cast<int>(rank)));
  if (rc) return rc;
  *comm = c;
  return QE_OK;
}

int qe_comm_destroy(void *comm) {
  if (!comm) return QE_EINVAL;
  return comm_status(ncclCommDestroy(static_cast<ncclComm_t>(comm)));
}

int qe_allreduce_stats(uint64_t *stats, uint32_t n, void *comm, void *stream) {
  if (!stats || !comm || n == 0 || n > QE_STATS_WORDS) return QE_EINVAL;
  return comm_status(ncclAllReduce(stats, stats, n, ncclUint64, ncclSum,
                                   static_cast<ncclComm_t>(comm),
                                   static_cast<hipStream_t>(stream)));
}

}  // extern "C"
