"""The leader's transitions (ABI 7) on the GPU, bit-for-bit against the oracle
on random states: qe_switch_config (raft.switchToConfig's leader side,
raft/raft.go:1651-1700; orc_switch_config_batch) under random configurations,
and qe_become_leader (raft.becomeLeader with reset, :724-759, :590-613;
orc_become_leader_batch).  The reference tests that pin switchToConfig
(TestCommitAfterRemoveNode, TestLeaderTransferRemoveNode,
TestLeaderTransferDemoteNode) run in test_gpu_progress.py's scenario list;
both entry points run in every interaction-trace replay
(tests/trace_replay.py)."""
import numpy as np
import pytest
import torch

from oracle import orc
from tests.test_gpu_progress import DEV, EXTRAS, assert_same, random_state, to_device

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from etcd_amd import engine
    return engine


def new_config(rng, pb, masks):
    """A configuration after a change: voters mostly tracked (some groups
    with a voter lacking a Progress, some leaders removed or demoted), a
    lead transferee in some groups."""
    G, S = pb.G, pb.S
    md = orc.mask_dtype(S)
    full = (1 << S) - 1
    inc = rng.integers(0, 1 << S, G)
    inc[rng.random(G) < 0.05] = 0  # Voters[0] empty
    out = rng.integers(0, 1 << S, G) * (rng.random(G) < 0.4) if "out" in masks else 0
    lrn = rng.integers(0, 1 << S, G) & ~(inc | out) & full
    trk = inc | out | lrn
    drop = rng.random(G) < 0.1  # a voter without a Progress (not a reachable config)
    trk = np.where(drop, trk & ~(1 << rng.integers(0, S, G)), trk)
    if "inc" in masks:
        pb.inc = inc.astype(md)
    if "out" in masks:
        pb.out = np.asarray(out).astype(md)
    pb.tracked = (trk & full).astype(md)
    # the leader: usually a voter, sometimes removed (untracked) or a learner
    vm = (inc | out) if "inc" in masks else np.full(G, full)
    self_slot = np.array([int(rng.choice(np.flatnonzero((int(v) >> np.arange(S)) & 1)))
                          if v else 0 for v in vm], np.uint8)
    odd = rng.random(G)
    self_slot = np.where(odd < 0.06, rng.integers(0, S + 2, G), self_slot).astype(np.uint8)
    pb.self_slot = self_slot
    pb.lead_transferee = np.where(rng.random(G) < 0.5, 0xFF, rng.integers(0, S, G)).astype(np.uint8)


@pytest.mark.parametrize("S,F,masks,max_ents,ring16", [
    (1, 8, ("inc",), 0, False), (3, 3, ("inc",), 1, False), (5, 8, ("inc",), 0, False),
    (5, 8, ("inc", "out"), 2, False), (7, 32, ("inc",), 0, False),
    (10, 8, ("inc", "out"), 3, False), (16, 5, ("inc", "out"), 0, False),
    (5, 8, ("inc",), 0, True), (9, 5, ("inc", "out"), 2, True)])
@pytest.mark.parametrize("all_groups", [False, True])
def test_switch_config_matches_oracle(eng, S, F, masks, max_ents, all_groups, ring16):
    """Random leader states (every Progress state, compacted Next, full and
    empty rings) under random new configurations: result (outcome and the
    transfer-abort bit), sent / snap masks, committed, lead_transferee, every
    Progress field and ring, the statistics and the algorithmic byte count
    equal the oracle's, over two launches in a row (the second sees the
    first's sends: probes paused, commits already made)."""
    from tests.test_gpu_progress import ring16_state
    rng = np.random.default_rng(8100 + 37 * S + F + all_groups + 500 * ring16)
    G = 4099
    pb = random_state(rng, G, S, F, 3, masks, EXTRAS, max_ents=max_ents)
    if ring16:  # ABI 8: the 16-bit Inflights form
        ring16_state(rng, pb)
    new_config(rng, pb, masks)
    ps = to_device(eng, pb, masks, EXTRAS)
    md = orc.mask_dtype(S)
    outcomes = set()
    for rnd in range(2):
        sw_h = None if all_groups else (rng.random(G) < 0.8).astype(np.uint8)
        sw_d = None if sw_h is None else torch.from_numpy(sw_h).to(DEV)
        sw = eng.Switch(ps, sw_d)
        st = eng.stats_buffer(DEV)
        acct = rnd == 1
        if acct:
            got_bytes = eng.switch_bytes_requested(ps, sw)
        else:
            eng.switch_config(ps, sw, stats=st)
        o = orc.switch_config(pb, sw_h)
        np.testing.assert_array_equal(sw.result.cpu().numpy(), o.result, err_msg="result")
        np.testing.assert_array_equal(sw.sent.cpu().numpy().view(md), o.sent, err_msg="sent")
        np.testing.assert_array_equal(sw.snap.cpu().numpy().view(md), o.snap, err_msg="snap")
        np.testing.assert_array_equal(ps.lead_transferee.cpu().numpy(), pb.lead_transferee,
                                      err_msg="lead_transferee")
        assert_same(ps, pb)
        if acct:
            assert got_bytes == int(o.bytes[0]), (got_bytes, int(o.bytes[0]))
        else:
            got = eng.stats_reduce(st).cpu().numpy().view(np.uint64)
            np.testing.assert_array_equal(got, o.stats, err_msg="stats")
        outcomes |= set(int(r) for r in np.unique(o.result))
    want = {1, 3, 4} | ({0} if not all_groups else set())
    assert want <= {r & 0xF for r in outcomes}, outcomes
    if S > 1:
        assert any(r & 0x10 for r in outcomes), outcomes
        assert o.sent.any() or rnd == 0


def test_switch_config_argument_errors(eng):
    import ctypes as C
    L = eng._lib.lib()
    ps = eng.ProgressState(64, 3, 8, 2, DEV, extras=("self_slot",))
    p = ps.struct()
    sw = eng.Switch(ps)
    q = sw.struct()
    assert L.qe_switch_config(C.byref(p), None, None, None) == eng._lib.QE_EINVAL
    q.result = None
    assert L.qe_switch_config(C.byref(p), C.byref(q), None, None) == eng._lib.QE_EINVAL
    q = sw.struct()
    p.inflight_cap = 0
    assert L.qe_switch_config(C.byref(p), C.byref(q), None, None) == eng._lib.QE_ERANGE
    p = ps.struct()
    assert L.qe_switch_config(C.byref(p), C.byref(q), None, None) == eng._lib.QE_OK


@pytest.mark.parametrize("S,F,masks,max_ents,reads,ring16", [
    (1, 8, (), 0, False, False), (3, 8, ("inc",), 1, True, False), (5, 8, (), 0, True, False),
    (5, 32, ("inc", "out"), 2, False, False), (9, 8, ("inc",), 0, True, False),
    (16, 5, ("inc", "out"), 0, False, False), (5, 8, ("inc",), 1, True, True)])
def test_become_leader_matches_oracle(eng, S, F, masks, max_ents, reads, ring16):
    """qe_become_leader (raft.becomeLeader + reset, raft.go:724-759,
    :590-613) against the oracle on random states: elected and not, leaders
    without a Progress, full run tables, a new term equal to the last run's
    (the bootstrap case), ReadIndex queues dropped, bcastAppend's probes
    (compacted logs: nothing to an inactive peer); every Progress field, the
    log model (runs, term start, lastIndex, committed), the outputs and the
    statistics equal the oracle's."""
    from tests.test_gpu_progress import random_queue, ring16_state
    rng = np.random.default_rng(8300 + 11 * S + F + 500 * ring16)
    G = 4099
    R = 4
    pb = random_state(rng, G, S, F, R, masks, EXTRAS, max_ents=max_ents)
    if ring16:  # ABI 8: the 16-bit Inflights form (reset empties every ring)
        ring16_state(rng, pb)
    pb.run_count[rng.random(G) < 0.3] -= 1  # room for the new term's run in most groups
    pb.run_count[:] = np.maximum(pb.run_count, 1)
    if reads:
        random_queue(rng, pb)
    ps = to_device(eng, pb, masks, EXTRAS + (("reads",) if reads else ()))
    el = (rng.random(G) < 0.8).astype(np.uint8)
    last_term = pb.run_term.reshape(R, G)[pb.run_count.astype(np.int64) - 1, np.arange(G)]
    term = (last_term + rng.integers(0, 3, G).astype(np.uint64)).astype(np.uint64)
    for bcast in (True, False):
        ld = eng.Leader(ps, torch.from_numpy(el).to(DEV), bcast=bcast)
        ld.term.copy_(torch.from_numpy(term.view(np.int64)).to(DEV))
        st = eng.stats_buffer(DEV)
        eng.become_leader(ps, ld, stats=st)
        o = orc.become_leader(pb, term, elected=el, bcast=bcast)
        md = orc.mask_dtype(S)
        np.testing.assert_array_equal(ld.result.cpu().numpy(), o.result, err_msg="result")
        np.testing.assert_array_equal(ld.sent.cpu().numpy().view(md), o.sent, err_msg="sent")
        np.testing.assert_array_equal(ld.snap.cpu().numpy().view(md), o.snap, err_msg="snap")
        lv = o.result == 1
        np.testing.assert_array_equal(ld.pending_conf_index.cpu().numpy().view(np.uint64)[lv],
                                      o.pending_conf_index[lv], err_msg="pendingConfIndex")
        h = ps.host()
        for k in ("term_start", "last_index", "run_count", "run_first", "run_term"):
            np.testing.assert_array_equal(h[k], getattr(pb, k), err_msg=k)
        assert_same(ps, pb)
        got = eng.stats_reduce(st).cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(got, o.stats, err_msg="stats")
        assert {0, 1, 2, 3} <= set(np.unique(o.result).tolist()) or S == 1
        assert not bcast or S == 1 or o.sent.any()
        term = term + np.uint64(1)  # a second election on the new state
