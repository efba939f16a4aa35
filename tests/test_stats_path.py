"""bench.py's multi-rank statistics path (CPU, gloo, world_size 2).

The ranks decide TOGETHER whether the 16-counter statistics vector goes
through the engine's qe_allreduce_stats or through torch's all_reduce
(bench.Dist._select_stats_path / sum_stats): a failure on one rank only must
move every rank to the same fallback -- one rank in torch's all_reduce while
another waits in RCCL is a hang -- and the sums must still be right.  The
engine's C calls are replaced by fakes here (no GPU, no RCCL); the gloo
group carries the agreement exactly as on the GPU box, where bench.Dist
runs every agreement on a host-side gloo group beside the nccl one.
"""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeLib:
    def __init__(self, rank, fail_allreduce_on):
        self.rank = rank
        self.fail_allreduce_on = fail_allreduce_on
        self.aborted = 0

    def qe_allreduce_stats(self, ptr, n, comm, stream):
        return -1001 if self.rank in self.fail_allreduce_on else 0

    def qe_comm_abort(self, comm):
        self.aborted += 1
        return 0

    def qe_comm_destroy(self, comm):
        return 0


def _fake_engine(lib):
    def check(fn, status):
        if status != 0:
            raise RuntimeError(f"{fn} failed: {status}")
    return types.SimpleNamespace(check=check, _lib=types.SimpleNamespace(lib=lambda: lib),
                                 _ptr=lambda t: 0, _stream=lambda d: None)


def _worker(rank, world, port, fail_init_on, fail_allreduce_on, q, hang_on=()):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import bench
    lib = _FakeLib(rank, fail_allreduce_on)
    bench.engine = _fake_engine(lib)
    d = bench.Dist(backend="gloo")

    def try_comm():  # stands in for qe_comm_unique_id + qe_comm_init_timeout
        if rank in fail_init_on:
            return None, "qe_comm_init_timeout failed: -1001 (injected)"
        return object(), ""

    d._try_engine_comm = try_comm
    if rank in hang_on:  # the collective never completes on this rank
        d._engine_wait = lambda: "qe_allreduce_stats did not complete in 60 s (injected)"
    d._select_stats_path()
    folded = torch.arange(16, dtype=torch.int64) + 100 * (rank + 1)
    out = d.sum_stats(folded.clone())
    q.put((rank, out.tolist(), d.stats_path, d.stats_fallback, lib.aborted,
           d.comm is not None))
    d.close()


def _run(fail_init_on, fail_allreduce_on, hang_on=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, fail_init_on, fail_allreduce_on, q,
                                               tuple(hang_on)))
             for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r = q.get(timeout=90)  # a hang would end here, not in the driver's timeout
        got[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    return got


WANT = (2 * np.arange(16) + 300).tolist()  # rank 0 + rank 1 vectors


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_failed_init_on_one_rank_moves_every_rank_to_the_fallback(fail_rank):
    got = _run(fail_init_on={fail_rank}, fail_allreduce_on=set())
    for r in (0, 1):
        out, path, fallback, aborted, has_comm = got[r]
        assert out == WANT
        assert fallback and f"rank {fail_rank}" in fallback and "injected" in fallback
        assert path.startswith("torch.distributed all_reduce (FALLBACK")
        assert not has_comm
        # the rank whose init succeeded aborts its communicator: nobody uses it
        assert aborted == (0 if r == fail_rank else 1)


def test_engine_path_when_every_rank_succeeds():
    got = _run(fail_init_on=set(), fail_allreduce_on=set())
    for r in (0, 1):
        out, path, fallback, aborted, has_comm = got[r]
        # the fake qe_allreduce_stats leaves the vector as it was (sum of one)
        assert out == (np.arange(16) + 100 * (r + 1)).tolist()
        assert path == "qe_allreduce_stats (RCCL)" and fallback is None and aborted == 0


def test_failed_allreduce_on_one_rank_aborts_and_sums_through_torch():
    got = _run(fail_init_on=set(), fail_allreduce_on={1})
    for r in (0, 1):
        out, path, fallback, aborted, has_comm = got[r]
        assert out == WANT  # the saved copy, summed through torch
        assert "rank 1: qe_allreduce_stats" in fallback
        assert aborted == 1 and not has_comm


def test_allreduce_not_completing_on_one_rank_aborts_everywhere():
    """Enqueued on every rank but not complete in time on one (a peer lost
    mid-collective): the second agreement, on the host group, moves every
    rank to the abort and the host-side sum -- nothing waits on the device."""
    got = _run(fail_init_on=set(), fail_allreduce_on=set(), hang_on={0})
    for r in (0, 1):
        out, path, fallback, aborted, has_comm = got[r]
        assert out == WANT
        assert "rank 0: qe_allreduce_stats did not complete" in fallback
        assert path.startswith("torch.distributed gloo all_reduce (FALLBACK")
        assert aborted == 1 and not has_comm


def test_bench_exits_nonzero_on_fallback_unless_allowed():
    import bench
    assert bench.exit_status(None, False) == 0
    assert bench.exit_status("rank 1: injected", False) == 3
    assert bench.exit_status("rank 1: injected", True) == 0
