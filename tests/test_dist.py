"""Multi-rank path on CPU (gloo, world_size 2): group sharding by
group_offset plus the all-reduce of the 16-counter statistics vector gives
the same totals -- including the order-free checksum -- as one process over
the union of the shards.  This is the aggregation bench.py performs over RCCL
(SURVEY.md §8(e))."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

G_PER_RANK = 50_003
S = 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_stats(orc, rank, G, S, kind):
    goff = rank * G
    if kind == "commit_vote":
        b = orc.Batch(G, S, masks=())
        orc.gen_batch(b, 0x5EED, goff=goff)
        return orc.commit_vote(b, goff=goff)[4]
    # election simulation: shard keyed by group_offset as well
    b = orc.Batch(G, S)
    orc.gen_batch(b, 0xE1EC, goff=goff)
    term = np.zeros(G, np.uint64)
    state = np.zeros(G, np.uint8)
    voted = np.zeros(G, np.uint8)
    granted = np.zeros(G, np.uint8)
    self_slot = np.zeros(G, np.uint8)
    for s in reversed(range(S)):
        self_slot[(b.inc >> s) & 1 == 1] = s
    return orc.election_steps(G, goff, S, term, state, voted, granted, self_slot, b.inc, b.out,
                              b.learner, 77, 0, 16, 13107, 32768)


def _worker(rank, world, port, kind, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import orc
    st = _shard_stats(orc, rank, G_PER_RANK, S, kind)
    t = torch.from_numpy(st.view(np.int64).copy())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    if rank == 0:
        q.put(t.numpy().view(np.uint64).tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["commit_vote", "election"])
def test_sharded_stats_equal_single_process(orc, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process over the union [0, 2G): same generator keys
    if kind == "commit_vote":
        b = orc.Batch(2 * G_PER_RANK, S, masks=())
        orc.gen_batch(b, 0x5EED, goff=0)
        want = orc.commit_vote(b, goff=0)[4]
    else:
        want = _shard_stats(orc, 0, 2 * G_PER_RANK, S, kind)
    assert got == want.tolist()
    assert want[0] > 0 and want[14] == 0  # groups counted, no invariant violations


def test_bench_dist_defaults_single_rank(monkeypatch):
    """bench.Dist is world 1 without torchrun env (no process group)."""
    import importlib
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    bench = importlib.import_module("bench")
    assert bench.WORKLOADS["config2_n5"][1] == 1 << 26
    assert bench.WORKLOADS["config3_joint"][1] == 1 << 27
