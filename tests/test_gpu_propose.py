"""qe_propose (ABI 6): stepLeader's MsgProp arm, appendEntry and the
bcastAppend after it (raft/raft.go:1019-1076, :621-642, :515-522) on the
GPU, bit-for-bit against the oracle (orc_propose_batch) on random states and
proposals, and through the reference tests restated in
tests/propose_scenarios.py."""
import numpy as np
import pytest
import torch

from oracle import orc
from tests.propose_scenarios import SCENARIOS
from tests.test_gpu_progress import (DEV, EXTRAS, GpuBackend, assert_same, random_state,
                                     to_dev_mask, to_device)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from etcd_amd import engine
    return engine


@pytest.mark.parametrize("sc", SCENARIOS, ids=lambda f: f.__name__)
def test_propose_scenarios_on_gpu(eng, sc):
    """TestSingleNodeCommit, TestUncommittedEntryLimit, TestStepIgnoreConfig,
    TestNewLeaderPendingConfig, TestLeaderTransferIgnoreProposal,
    TestCannotCommitWithoutNewTermEntry, TestProposal and the conf-change
    gates, through qe_propose / qe_progress_step on one group."""
    sc(GpuBackend(eng))


def random_proposals(rng, pb, max_cc):
    G = pb.G
    ne = np.where(rng.random(G) < 0.15, 0, rng.integers(1, 4, G)).astype(np.uint32)
    payload = np.where(rng.random(G) < 0.3, 0, rng.integers(1, 40, G)).astype(np.uint64)
    cnt = (rng.integers(0, max_cc + 1, G) * (rng.random(G) < 0.5)).astype(np.uint8)
    cnt = np.minimum(cnt, ne).astype(np.uint8)
    m = max(1, max_cc)
    pos = np.zeros((m, G), np.uint32)
    for g in range(G):
        if cnt[g]:
            pos[: cnt[g], g] = np.sort(rng.choice(int(ne[g]), int(cnt[g]), replace=False))
    if max_cc:  # more conf-change entries than max_cc: QE_PROP_BAD_CC, refused whole
        cnt[(rng.random(G) < 0.05) & (ne > 0)] = max_cc + 1
    leave = (rng.random((m, G)) < 0.4).astype(np.uint8)
    size = rng.integers(0, 30, (m, G)).astype(np.uint32)
    li = pb.last_index.astype(np.int64)
    applied = (rng.random(G) * (li + 1)).astype(np.uint64)
    pci = np.where(rng.random(G) < 0.5, applied,
                   applied + rng.integers(0, 3, G).astype(np.uint64)).astype(np.uint64)
    unc = np.where(rng.random(G) < 0.3, 0, rng.integers(0, 80, G)).astype(np.uint64)
    return ne, payload, (max_cc, cnt, pos.reshape(-1), leave.reshape(-1), size.reshape(-1)), \
        applied, pci, unc


def load_props(eng, ps, ne, payload, cc, applied, pci, unc, max_unc, flags=0):
    max_cc, cnt, pos, leave, size = cc
    pr = eng.Proposals(ps, max_cc=max_cc, max_uncommitted=max_unc, flags=flags)
    put = lambda dst, a: dst[: a.size].copy_(torch.from_numpy(  # noqa: E731
        a.view(np.int64) if a.dtype == np.uint64 else (a.view(np.int32) if a.dtype == np.uint32
                                                       else a)).to(DEV))
    put(pr.num_entries, ne)
    put(pr.payload, payload)
    if max_cc:
        put(pr.cc_count, cnt)
        put(pr.cc_pos, pos)
        put(pr.cc_leave, leave)
        put(pr.cc_size, size)
    put(pr.applied, applied)
    put(pr.pending_conf_index, pci)
    put(pr.uncommitted_size, unc)
    return pr


@pytest.mark.parametrize("S,F,masks,extras,max_cc,max_ents,ring16", [
    (1, 8, (), EXTRAS, 0, 0, False), (3, 3, ("inc",), EXTRAS, 2, 1, False),
    (5, 8, (), ("self_slot",), 0, 0, False), (5, 8, ("inc", "out"), EXTRAS, 3, 2, False),
    (7, 32, (), EXTRAS, 1, 0, False), (10, 8, ("inc", "out"), EXTRAS, 2, 3, False),
    (16, 5, ("inc",), EXTRAS, 8, 0, False),
    (3, 8, ("inc",), EXTRAS, 2, 1, True), (5, 5, (), ("self_slot",), 0, 0, True),
    (9, 8, ("inc", "out"), EXTRAS, 3, 2, True)])
@pytest.mark.parametrize("flags", [0, 1])
def test_propose_matches_oracle(eng, S, F, masks, extras, max_cc, max_ents, flags, ring16):
    """Random leader states (every Progress state, compacted Next, full and
    empty rings, voters without a Progress, leaders without one, transfers
    in progress) and random proposals (none, several entries, conf-change
    entries refused or accepted, uncommitted tails at and over the limit):
    state, last_index, pendingConfIndex, uncommittedSize, every output, the
    statistics and the algorithmic byte count equal the oracle's, over two
    launches in a row (flags 1: appendEntry alone); ring16: the rings in
    the 16-bit form (ABI 8)."""
    from tests.test_gpu_progress import ring16_state
    rng = np.random.default_rng(7000 + 31 * S + F + flags + 500 * ring16)
    G = 4099
    pb = random_state(rng, G, S, F, 3, masks, extras, max_ents=max_ents)
    if ring16:
        ring16_state(rng, pb)
    ps = to_device(eng, pb, masks, extras)
    for rnd in range(2):
        ne, payload, cc, applied, pci, unc = random_proposals(rng, pb, max_cc)
        max_unc = 60 if rnd == 0 else 0
        pr = load_props(eng, ps, ne, payload, cc, applied, pci, unc, max_unc, flags)
        st = eng.stats_buffer(DEV)
        acct = rnd == 1
        if acct:
            got_bytes = eng.propose_bytes_requested(ps, pr)
        else:
            eng.propose(ps, pr, stats=st)
        o_pci, o_unc = pci.copy(), unc.copy()
        o = orc.propose(pb, ne, payload, cc=cc, applied=applied, pending_conf_index=o_pci,
                        uncommitted_size=o_unc, max_uncommitted=max_unc, flags=flags)
        md = orc.mask_dtype(S)
        np.testing.assert_array_equal(pr.result.cpu().numpy(), o.result, err_msg="result")
        np.testing.assert_array_equal(pr.cc_refused.cpu().numpy(), o.cc_refused, err_msg="cc")
        np.testing.assert_array_equal(pr.sent.cpu().numpy().view(md), o.sent, err_msg="sent")
        np.testing.assert_array_equal(pr.snap.cpu().numpy().view(md), o.snap, err_msg="snap")
        np.testing.assert_array_equal(pr.pending_conf_index.cpu().numpy().view(np.uint64), o_pci,
                                      err_msg="pendingConfIndex")
        np.testing.assert_array_equal(pr.uncommitted_size.cpu().numpy().view(np.uint64), o_unc,
                                      err_msg="uncommittedSize")
        np.testing.assert_array_equal(ps.last_index.cpu().numpy().view(np.uint64),
                                      pb.last_index, err_msg="last_index")
        assert_same(ps, pb)
        if acct:
            assert got_bytes == int(o.bytes[0]), (got_bytes, int(o.bytes[0]))
        else:
            got = eng.stats_reduce(st).cpu().numpy().view(np.uint64)
            np.testing.assert_array_equal(got, o.stats, err_msg="stats")
        res = o.result
        assert (res == 1).any() and (res == 0).any()
        if flags == 0 and "self_slot" in extras and S > 1:
            assert (res == 2).any() and o.sent.any()
        if flags == 0 and max_cc:
            assert (res == 5).any()  # QE_PROP_BAD_CC


def test_propose_argument_errors(eng):
    import ctypes as C
    L = eng._lib.lib()
    ps = eng.ProgressState(64, 3, 8, 2, DEV, extras=("self_slot",))
    p = ps.struct()
    pr = eng.Proposals(ps)
    q = pr.struct()
    assert L.qe_propose(C.byref(p), None, None, None) == eng._lib.QE_EINVAL
    q.flags = 2
    assert L.qe_propose(C.byref(p), C.byref(q), None, None) == eng._lib.QE_EINVAL
    q = pr.struct()
    q.max_cc = eng._lib.QE_PROP_MAX_CC + 1
    assert L.qe_propose(C.byref(p), C.byref(q), None, None) == eng._lib.QE_ERANGE
    q = pr.struct()
    q.uncommitted_size = None
    q.max_uncommitted = 5
    assert L.qe_propose(C.byref(p), C.byref(q), None, None) == eng._lib.QE_EINVAL
    q = pr.struct()
    q.result = None
    assert L.qe_propose(C.byref(p), C.byref(q), None, None) == eng._lib.QE_EINVAL
    q = pr.struct()
    p.self_slot = None  # MsgProp needs the leader's slot
    assert L.qe_propose(C.byref(p), C.byref(q), None, None) == eng._lib.QE_EINVAL
    p = ps.struct()
    assert L.qe_propose(C.byref(p), C.byref(q), None, None) == eng._lib.QE_OK


def test_propose_full_size_bench_state(eng):
    """The bench's propose workload state (16M groups would be the bench;
    here 1M): every group appends 3 entries and bcasts to its 4 followers;
    the checksum and counters equal a second, identical launch sequence's
    expectations computed from first principles (last_index + 3, every
    follower's Next = lastIndex + 1, one more Inflights entry)."""
    import bench
    bench.engine = eng
    G, S, F = 1 << 20, 5, 8
    ps = eng.ProgressState(G, S, F, 2, DEV, extras=("self_slot",), max_ents=0)
    bench.psend_state(ps)
    ps.self_slot.fill_(0)
    li0 = ps.last_index.clone()
    cnt0 = (ps.peer.view(S, -1)[1:, :G].to(torch.int64) >> 16) & 0xFF
    pr = eng.Proposals(ps)
    pr.num_entries.fill_(3)
    pr.payload.fill_(24)
    eng.propose(ps, pr)
    torch.cuda.synchronize()
    assert bool((pr.result == 1).all())
    assert bool((ps.last_index == li0 + 3).all())
    nx = ps.next.view(S, -1)[1:, :G]
    assert bool((nx == (li0 + 4).view(1, G)).all())
    cnt1 = (ps.peer.view(S, -1)[1:, :G].to(torch.int64) >> 16) & 0xFF
    assert bool((cnt1 == cnt0 + 1).all())
    assert bool((pr.sent.to(torch.int32) == 0b11110).all())


@pytest.mark.parametrize("S,masks,extras,reads", [(3, (), (), False), (5, ("inc",), EXTRAS, True),
                                                   (12, (), EXTRAS, True)])
@pytest.mark.parametrize("tpw", [-1, 3])
def test_heartbeat_matches_oracle(eng, S, masks, extras, reads, tpw):
    """qe_heartbeat (MsgBeat -> bcastHeartbeat, raft.go:524-541, sendHeartbeat
    :494-510) against the oracle: the slots sent to (tracked, not the
    leader), Commit = min(Match, committed) per slot, and the context of the
    newest pending ReadIndex request."""
    from tests.test_gpu_progress import random_queue
    rng = np.random.default_rng(4100 + S)
    G = 3001
    pb = random_state(rng, G, S, 8, 2, masks, extras)
    ext = extras
    if reads:
        random_queue(rng, pb)
        ext = extras + ("reads",)
    ps = to_device(eng, pb, masks, ext)
    # the default grid, and waves walking 3 tiles each (a ragged last walk)
    eng.tune("tiles_per_wave", tpw)
    try:
        commit, ctx, sent = eng.heartbeat(ps)
        torch.cuda.synchronize()
    finally:
        eng.tune("tiles_per_wave", -1)
    o_commit, o_ctx, o_sent = orc.heartbeat(pb)
    md = orc.mask_dtype(S)
    np.testing.assert_array_equal(sent.cpu().numpy().view(md), o_sent)
    np.testing.assert_array_equal(ctx.cpu().numpy().view(np.uint32), o_ctx)
    got = commit.cpu().numpy().view(np.uint64).reshape(S, -1)[:, :G]
    want = o_commit.reshape(S, -1)[:, :G]
    to = (o_sent.astype(np.int64)[None, :] >> np.arange(S)[:, None]) & 1
    np.testing.assert_array_equal(got[to == 1], want[to == 1])
    assert to.any() and (not reads or o_ctx.any())
