"""GPU parity of the Progress state machine (qe_progress_step /
qe_progress_send) against the oracle, which
tests/test_progress_oracle.py pins to the reference's tables."""
import numpy as np
import pytest
import torch

from oracle import orc
from tests.golden_util import raft_tables
from tests.test_progress_oracle import log_runs

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from etcd_amd import engine
    return engine


def random_state(rng, G, S, F, R, masks):
    pb = orc.ProgressBatch(G, S, F, R)
    # leader log: runs over [dummy, last]
    for g in range(G):
        nr = int(rng.integers(1, R + 1))
        dummy = int(rng.integers(0, 20))
        firsts = np.sort(rng.choice(np.arange(dummy + 1, dummy + 60), nr - 1, replace=False))
        first = np.concatenate([[dummy], firsts]).astype(np.uint64)
        terms = np.sort(rng.integers(0, 9, nr)).astype(np.uint64)
        last = int(first[-1] + rng.integers(0, 8))
        pb.run_first[np.arange(nr) * G + g] = first
        pb.run_term[np.arange(nr) * G + g] = terms
        pb.run_count[g] = nr
        pb.first_index[g] = dummy + 1
        pb.last_index[g] = last
        pb.term_start[g] = int(rng.integers(dummy, last + 2))
        pb.committed[g] = int(rng.integers(0, last + 1))
    n = S * G
    li = np.tile(pb.last_index, S)
    pb.match[:] = (rng.random(n) * (li + 1)).astype(np.uint64)
    pb.next[:] = pb.match + rng.integers(1, 4, n).astype(np.uint64)
    pb.next[rng.random(n) < 0.05] = 0  # edge: Next = 0 (MaybeDecrTo wrap)
    pb.pending[:] = rng.integers(0, 70, n).astype(np.uint64)
    pb.flags[:] = (rng.integers(0, 3, n) | (rng.integers(0, 2, n) * 4) |
                   (rng.integers(0, 2, n) * 8)).astype(np.uint8)
    pb.icount[:] = rng.integers(0, F + 1, n).astype(np.uint8)
    pb.istart[:] = rng.integers(0, F, n).astype(np.uint8)
    base = pb.match.copy()
    for k in range(F):
        pb.ibuf[(np.arange(S)[:, None] * G + np.arange(G)[None, :]) * F + k] = \
            (base.reshape(S, G) + 1 + 2 * ((k - pb.istart.reshape(S, G).astype(int)) % F)).astype(np.uint64)
    md = orc.mask_dtype(S)
    if "inc" in masks:
        pb.inc = rng.integers(0, 1 << S, G).astype(md)
    if "out" in masks:
        pb.out = rng.integers(0, 1 << S, G).astype(md)
    return pb


def random_msgs(rng, pb):
    n = pb.S * pb.G
    mtype = rng.integers(0, 5, n).astype(np.uint8)  # 4 = unknown kind -> ignored
    li = np.tile(pb.last_index, pb.S)
    mindex = np.where(rng.random(n) < 0.5, pb.next - 1,
                      (rng.random(n) * (li + 3)).astype(np.uint64)).astype(np.uint64)
    mhint = (rng.random(n) * (li + 2)).astype(np.uint64)
    mlogterm = np.where(rng.random(n) < 0.3, 0, rng.integers(1, 10, n)).astype(np.uint64)
    return mtype, mindex, mhint, mlogterm


def to_device(eng, pb, masks):
    ps = eng.ProgressState(pb.G, pb.S, pb.F, pb.R, DEV, masks=masks, stride=pb.stride)
    ps.load_host(match=pb.match, next=pb.next, pending=pb.pending, flags=pb.flags,
                 istart=pb.istart, icount=pb.icount, ibuf=pb.ibuf, committed=pb.committed,
                 term_start=pb.term_start, first_index=pb.first_index, last_index=pb.last_index,
                 run_first=pb.run_first, run_term=pb.run_term, run_count=pb.run_count,
                 inc=pb.inc, out=pb.out)
    return ps


def assert_same(ps, pb):
    h = ps.host()
    for k in ("match", "next", "pending", "flags", "istart", "icount", "committed"):
        np.testing.assert_array_equal(h[k], getattr(pb, k), err_msg=k)
    # inflight buffers: compare the live ring entries only (freed slots keep
    # stale values in both, but compare everything anyway: identical ops)
    np.testing.assert_array_equal(h["ibuf"], pb.ibuf, err_msg="ibuf")


@pytest.mark.parametrize("S,masks", [(1, ()), (3, ()), (5, ()), (5, ("inc",)),
                                     (7, ("inc", "out")), (10, ("inc", "out")), (16, ("inc",))])
def test_progress_rounds_match_oracle(eng, S, masks):
    rng = np.random.default_rng(100 + S)
    G, F, R = 3001, 8, 6
    pb = random_state(rng, G, S, F, R, masks)
    ps = to_device(eng, pb, masks)
    for rnd in range(6):
        mtype, mindex, mhint, mlogterm = random_msgs(rng, pb)
        msgs = eng.PeerMsgs(ps)
        for name, a in (("type", mtype), ("index", mindex), ("reject_hint", mhint),
                        ("log_term", mlogterm)):
            t = torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(DEV)
            getattr(msgs, name).copy_(t)
        stats = eng.stats_buffer(DEV)
        eng.progress_step(ps, msgs, stats)
        got = eng.stats_reduce(stats).cpu().numpy().view(np.uint64)
        send, bcast, ostats = orc.progress_step(pb, mtype, mindex, mhint, mlogterm)
        assert_same(ps, pb)
        md = orc.mask_dtype(S)
        np.testing.assert_array_equal(msgs.send_mask.cpu().numpy().view(md), send)
        np.testing.assert_array_equal(msgs.bcast.cpu().numpy(), bcast)
        np.testing.assert_array_equal(got, ostats)
        # send appends to the peers the step asked for (plus random others)
        want = (send | rng.integers(0, 1 << S, G).astype(md)).astype(md)
        tw = torch.from_numpy(want.view(np.int16) if S > 8 else want).to(DEV)
        sei, me = int(rnd % 2), int(rng.integers(1, 5))
        sent, snap = eng.progress_send(ps, tw, sei, me)
        o_sent, o_snap = orc.progress_send(pb, want, sei, me)
        np.testing.assert_array_equal(sent.cpu().numpy().view(md), o_sent)
        np.testing.assert_array_equal(snap.cpu().numpy().view(md), o_snap)
        assert_same(ps, pb)


def test_fast_log_rejection_on_gpu(eng):
    L = orc.lib()
    for r in raft_tables()["TestFastLogRejection"]["rows"]:
        lead = [tuple(e) for e in r["leader_log"]]
        l_last = max(i for i, _ in lead)
        rf, rt, last = log_runs(lead, (l_last + 1, 1))
        ps = eng.ProgressState(1, 1, 16, 16, DEV)
        R = len(rf)
        run_first = np.zeros(16 * ps.stride, np.uint64)
        run_term = np.zeros(16 * ps.stride, np.uint64)
        run_first[np.arange(R) * ps.stride] = rf
        run_term[np.arange(R) * ps.stride] = rt
        ps.load_host(run_first=run_first, run_term=run_term, run_count=np.array([R], np.uint8),
                     first_index=np.array([1], np.uint64), last_index=np.array([last], np.uint64),
                     term_start=np.array([l_last + 1], np.uint64),
                     next=np.array([l_last + 1], np.uint64), match=np.array([0], np.uint64))
        msgs = eng.PeerMsgs(ps)
        msgs.type.fill_(3)  # MsgHeartbeatResp
        eng.progress_step(ps, msgs)
        assert int(msgs.send_mask[0]) == 1
        sent, _ = eng.progress_send(ps, msgs.send_mask, False, 1 << 20)
        assert int(sent[0]) == 1
        msgs = eng.PeerMsgs(ps)
        msgs.type.fill_(2)  # MsgAppResp reject of the probe at Index = l_last
        msgs.index.fill_(l_last)
        msgs.reject_hint.fill_(r["reject_hint_index"])
        msgs.log_term.fill_(r["reject_hint_term"])
        eng.progress_step(ps, msgs)
        idx = int(ps.next[0]) - 1
        term = L.orc_log_term(R, orc.P(rf), orc.P(rt), last, idx)
        assert (idx, term) == (r["next_append_index"], r["next_append_term"]), r


def test_maybe_decr_table_on_gpu(eng):
    """TestProgressMaybeDecr through the reject path (log_term 0 -> the hint
    goes straight to MaybeDecrTo)."""
    rows = raft_tables()["TestProgressMaybeDecr"]["rows"]
    G = len(rows)
    ps = eng.ProgressState(G, 1, 4, 1, DEV)
    u = lambda k: np.array([r[k] for r in rows], np.uint64)
    ps.load_host(match=u("match"), next=u("next"),
                 flags=np.array([r["state"] for r in rows], np.uint8),
                 last_index=np.full(G, 100, np.uint64), run_count=np.ones(G, np.uint8))
    msgs = eng.PeerMsgs(ps)
    msgs.type[:G].fill_(2)
    msgs.index[:G].copy_(torch.from_numpy(u("rejected").view(np.int64)))
    msgs.reject_hint[:G].copy_(torch.from_numpy(u("last").view(np.int64)))
    eng.progress_step(ps, msgs)
    h = ps.host()
    for i, r in enumerate(rows):
        assert int(h["next"][i]) == r["want_next"], r
        assert int(h["match"][i]) == r["match"], r
        assert bool(int(msgs.send_mask[i]) & 1) == r["want"], r
