"""qe_allreduce_stats through the C ABI on the GPU (RCCL, world size 1):
the communicator set-up path a Go host uses (unique id -> qe_comm_init),
the in-place uint64 sum, and the folded-stats vector of a real launch.
World sizes > 1 run in the driver's 8-GPU bench; gloo rehearses the
sharding logic on CPU (tests/test_dist.py)."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from etcd_amd import engine
    return engine


def test_allreduce_stats_world_size_one(eng):
    L = eng._lib.lib()
    idb = (C.c_uint8 * L.qe_comm_id_bytes())()
    eng.check("qe_comm_unique_id", L.qe_comm_unique_id(idb))
    comm = C.c_void_p()
    eng.check("qe_comm_init", L.qe_comm_init(C.byref(comm), 1, 0, idb, 0))
    try:
        # the folded statistics of a real qe_commit_vote launch
        b = eng.SlotBatch(100_000, 5, DEV, masks=())
        eng.gen_groups(b, 0x5EED)
        stats = eng.stats_buffer(DEV)
        eng.commit_vote(b, stats=stats)
        folded = eng.stats_reduce(stats)
        want = folded.clone()
        eng.check("qe_allreduce_stats", L.qe_allreduce_stats(
            eng._ptr(folded), folded.numel(), comm, eng._stream(folded.device)))
        torch.cuda.synchronize()
        assert torch.equal(folded, want)  # sum over one rank
        # the wraparound of uint64 counters near 2^64 (int64 view)
        x = torch.tensor([-1, -(1 << 62), 7] + [0] * 13, dtype=torch.int64, device=DEV)
        y = x.clone()
        eng.check("qe_allreduce_stats", L.qe_allreduce_stats(eng._ptr(y), 16, comm,
                                                              eng._stream(y.device)))
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        assert int(eng.stats_dict(folded)["groups"]) == 100_000
    finally:
        eng.check("qe_comm_destroy", L.qe_comm_destroy(comm))


def test_bounded_init_world_size_one(eng):
    """qe_comm_init_timeout (non-blocking communicator, polled): world size 1
    joins at once; the all-reduce on that communicator waits for its enqueue
    (ncclInProgress) and sums like the blocking one; qe_comm_abort frees it."""
    L = eng._lib.lib()
    idb = (C.c_uint8 * L.qe_comm_id_bytes())()
    eng.check("qe_comm_unique_id", L.qe_comm_unique_id(idb))
    comm = C.c_void_p()
    eng.check("qe_comm_init_timeout", L.qe_comm_init_timeout(C.byref(comm), 1, 0, idb, 0, 60_000))
    try:
        x = torch.tensor([5, -3] + [0] * 14, dtype=torch.int64, device=DEV)
        y = x.clone()
        eng.check("qe_allreduce_stats", L.qe_allreduce_stats(eng._ptr(y), 16, comm,
                                                              eng._stream(y.device)))
        torch.cuda.synchronize()
        assert torch.equal(x, y)
    finally:
        eng.check("qe_comm_abort", L.qe_comm_abort(comm))


def test_bounded_init_times_out_when_peers_never_join(eng):
    """A 2-rank communicator whose second rank never calls init: the bound
    ends the wait with QE_ECOMM instead of hanging (the case bench.py's
    agreement step exists for)."""
    L = eng._lib.lib()
    idb = (C.c_uint8 * L.qe_comm_id_bytes())()
    eng.check("qe_comm_unique_id", L.qe_comm_unique_id(idb))
    comm = C.c_void_p()
    rc = L.qe_comm_init_timeout(C.byref(comm), 2, 0, idb, 0, 3000)
    assert rc == eng._lib.QE_ECOMM
    assert not comm.value


def test_bounded_init_then_destroy_world_size_one(eng):
    """A non-blocking communicator (qe_comm_init_timeout) freed through
    qe_comm_destroy: the finalize is polled (ncclInProgress) and bounded, then
    the communicator is destroyed -- after an all-reduce on it, and with the
    engine all-reduce on a stream of its own as bench.py runs it."""
    L = eng._lib.lib()
    idb = (C.c_uint8 * L.qe_comm_id_bytes())()
    eng.check("qe_comm_unique_id", L.qe_comm_unique_id(idb))
    comm = C.c_void_p()
    eng.check("qe_comm_init_timeout", L.qe_comm_init_timeout(C.byref(comm), 1, 0, idb, 0, 60_000))
    side = torch.cuda.Stream(DEV)
    x = torch.tensor([11, -2] + [0] * 14, dtype=torch.int64, device=DEV)
    y = x.clone()
    side.wait_stream(torch.cuda.current_stream(DEV))
    eng.check("qe_allreduce_stats", L.qe_allreduce_stats(eng._ptr(y), 16, comm,
                                                          C.c_void_p(side.cuda_stream)))
    ev = torch.cuda.Event()
    ev.record(side)
    ev.synchronize()
    assert torch.equal(x, y)
    eng.check("qe_comm_destroy", L.qe_comm_destroy(comm))
