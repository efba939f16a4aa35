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

#include <chrono>
#include <thread>

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

// Bound on waiting for a non-blocking communicator's pending operation (an
// enqueue, a finalize) to leave ncclInProgress.  The wait sleeps between
// polls, so a stuck peer costs a thread sleeping, not a spinning core.
constexpr long long kCommWaitMs = 30000;

// Polls ncclCommGetAsyncError until `r` is no longer ncclInProgress or
// kCommWaitMs passed (then ncclInProgress is returned: the caller aborts).
static ncclResult_t comm_wait(ncclComm_t c, ncclResult_t r) {
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclInProgress) {
    const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                        std::chrono::steady_clock::now() - t0).count();
    if (ms >= kCommWaitMs) return ncclInProgress;
    std::this_thread::sleep_for(std::chrono::microseconds(100));
    if (ncclCommGetAsyncError(c, &r) != ncclSuccess) return ncclInternalError;
  }
  return r;
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

int qe_comm_init_timeout(void **comm, uint32_t nranks, uint32_t rank, const void *id,
                         int device, uint32_t timeout_ms) {
  if (!comm || !id || nranks == 0 || rank >= nranks || device < 0) return QE_EINVAL;
  *comm = nullptr;
  int rc = qe::hip_status(hipSetDevice(device));
  if (rc) return rc;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  if (timeout_ms == 0) {  // blocking: ncclCommInitRank returns once every rank joined
    rc = comm_status(ncclCommInitRank(&c, static_cast<int>(nranks), u, static_cast<int>(rank)));
    if (rc) return rc;
    *comm = c;
    return QE_OK;
  }
  // non-blocking communicator: the init returns at once and is polled, so a
  // rank whose peers never join (one of them failed before calling init)
  // gives up after timeout_ms instead of waiting forever; the caller then
  // agrees with its peers over its own transport which path to take
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = ncclCommInitRankConfig(&c, static_cast<int>(nranks), u, static_cast<int>(rank), &cfg);
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclInProgress && c != nullptr) {
    const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                        std::chrono::steady_clock::now() - t0).count();
    if (ms >= static_cast<long long>(timeout_ms)) {
      ncclCommAbort(c);
      qe::set_error("qe_comm_init_timeout: the other ranks did not join in time");
      return QE_ECOMM;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
    if (ncclCommGetAsyncError(c, &r) != ncclSuccess) break;
  }
  if (r != ncclSuccess) {
    if (c) ncclCommAbort(c);
    return comm_status(r == ncclInProgress ? ncclInternalError : r);
  }
  *comm = c;
  return QE_OK;
}

int qe_comm_init(void **comm, uint32_t nranks, uint32_t rank, const void *id, int device) {
  return qe_comm_init_timeout(comm, nranks, rank, id, device, 0);
}

int qe_comm_abort(void *comm) {
  if (!comm) return QE_EINVAL;
  return comm_status(ncclCommAbort(static_cast<ncclComm_t>(comm)));
}

int qe_comm_destroy(void *comm) {
  if (!comm) return QE_EINVAL;
  const ncclComm_t c = static_cast<ncclComm_t>(comm);
  // flush the communicator's operations first: on a non-blocking one
  // (qe_comm_init_timeout) the finalize returns ncclInProgress and is
  // polled, bounded; one that does not complete is aborted instead
  const ncclResult_t r = comm_wait(c, ncclCommFinalize(c));
  if (r != ncclSuccess) {
    ncclCommAbort(c);
    if (r == ncclInProgress) {
      qe::set_error("qe_comm_destroy: the communicator did not finalize in time (aborted)");
      return QE_ECOMM;
    }
    return comm_status(r);
  }
  return comm_status(ncclCommDestroy(c));
}

int qe_allreduce_stats(uint64_t *stats, uint32_t n, void *comm, void *stream) {
  if (!stats || !comm || n == 0 || n > QE_STATS_WORDS) return QE_EINVAL;
  const ncclComm_t c = static_cast<ncclComm_t>(comm);
  ncclResult_t r = ncclAllReduce(stats, stats, n, ncclUint64, ncclSum, c,
                                 static_cast<hipStream_t>(stream));
  // a non-blocking communicator (qe_comm_init_timeout) may return before the
  // collective is enqueued: wait for the enqueue (not for the sum itself),
  // bounded -- an enqueue still pending after kCommWaitMs is an error the
  // caller answers with qe_comm_abort
  r = comm_wait(c, r);
  if (r == ncclInProgress) {
    qe::set_error("qe_allreduce_stats: the collective was not enqueued in time");
    return QE_ECOMM;
  }
  return comm_status(r);
}

}  // extern "C"
