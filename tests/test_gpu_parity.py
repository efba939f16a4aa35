"""GPU parity: every entry point of the C ABI against the CPU oracle, bit
for bit, on the golden fixtures and on seeded synthetic batches (all slot
counts 1..16, majority / masked / joint configs, tie-heavy and uniform value
distributions, ragged G, learners, invariant violations)."""
import numpy as np
import pytest
import torch

from oracle import quorum_ref as Q
from tests.golden_util import INF, case_acked, case_votes, datadriven_cases, raft_tables

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from etcd_amd import engine
    return engine


def gpu_batch(eng, G, S, seed, goff=0, masks=("inc", "out", "learner"), votes=True, **gen):
    b = eng.SlotBatch(G, S, DEV, masks=masks, votes=votes, group_offset=goff)
    eng.gen_groups(b, seed, **gen)
    return b


def host_batch(orc, b):
    h = b.host()
    hb = orc.Batch(b.G, b.S, masks=tuple(n for n in ("inc", "out", "learner") if h[n] is not None),
                   votes=h["voted"] is not None)
    hb.match[:] = h["match"].reshape(-1)
    for n in ("inc", "out", "learner", "voted", "granted"):
        if h[n] is not None:
            getattr(hb, n)[:] = h[n]
    return hb


CV_KERNELS = (0, 1)  # qe_tune("cv_kernel"): pair kernel, stream kernel


def check_commit_vote(eng, orc, b, goff=0):
    """Both qe_commit_vote kernels against the oracle, bit for bit."""
    hb = host_batch(orc, b)
    commit, vote, gc, rc, ostats = orc.commit_vote(hb, goff=goff)
    try:
        for k in CV_KERNELS:
            eng.tune("cv_kernel", k)
            stats = eng.stats_buffer(DEV)
            out = eng.commit_vote(b, stats=stats)
            folded = eng.stats_reduce(stats)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.commit.cpu().numpy().view(np.uint64), commit,
                                          err_msg=f"cv_kernel {k}")
            np.testing.assert_array_equal(out.vote.cpu().numpy(), vote, err_msg=f"cv_kernel {k}")
            np.testing.assert_array_equal(out.granted.cpu().numpy(), gc, err_msg=f"cv_kernel {k}")
            np.testing.assert_array_equal(out.rejected.cpu().numpy(), rc, err_msg=f"cv_kernel {k}")
            got = folded.cpu().numpy().view(np.uint64)
            np.testing.assert_array_equal(got, ostats, err_msg=f"cv_kernel {k}")
    finally:
        eng.tune("cv_kernel", -1)
    return commit, vote


# --------------------------------------------------------------------------
# golden fixtures through the reference-API mirror
# --------------------------------------------------------------------------
def test_golden_datadriven_through_mirror(eng):
    import etcd_amd as E
    cases = datadriven_cases()
    com = [c for c in cases if c["cmd"] == "committed"]
    vot = [c for c in cases if c["cmd"] == "vote"]
    got = E.CommittedIndexBatch([E.JointConfig(c["cfg"], c["cfgj"]) for c in com],
                                [E.MapAckIndexer(case_acked(c)) for c in com], DEV)
    assert [int(x) for x in got] == [c["expect"] for c in com]
    # symmetry (datadriven_test.go:218-221)
    got2 = E.CommittedIndexBatch([E.JointConfig(c["cfgj"], c["cfg"]) for c in com],
                                 [E.MapAckIndexer(case_acked(c)) for c in com], DEV)
    assert got2 == got
    gotv = E.VoteResultBatch([E.JointConfig(c["cfg"], c["cfgj"]) for c in vot],
                             [case_votes(c) for c in vot], DEV)
    assert [int(x) for x in gotv] == [c["expect"] for c in vot]
    assert str(gotv[0]) in ("VotePending", "VoteLost", "VoteWon")
    # per-group methods (batch of one) on a few cases
    for c in com[:6]:
        mc = E.MajorityConfig(c["cfg"])
        if not c["joint"]:
            assert int(mc.CommittedIndex(E.MapAckIndexer(case_acked(c)), DEV)) == c["expect"]
    assert str(E.Index(INF)) == "∞"


def test_golden_through_fixed_majority_kernel(eng, orc):
    """Non-joint golden cases through MODE 0 (no masks): voters occupy all S
    slots, so each distinct voter count is its own batch."""
    by_n = {}
    for c in datadriven_cases():
        if c["joint"] or not c["cfg"]:
            continue
        by_n.setdefault(len(c["cfg"]), []).append(c)
    for n, cs in by_n.items():
        b = eng.SlotBatch(len(cs), n, DEV, masks=(), votes=True)
        match = np.zeros((n, len(cs)), np.uint64)
        vd = np.zeros(len(cs), np.uint64)
        gr = np.zeros(len(cs), np.uint64)
        for i, c in enumerate(cs):
            ids = sorted(c["cfg"])
            l, v = case_acked(c), case_votes(c)
            for s, vid in enumerate(ids):
                match[s, i] = l.get(vid, 0)
                if vid in v:
                    vd[i] |= 1 << s
                    gr[i] |= (1 << s) if v[vid] else 0
        b.load_host(match, voted=vd, granted=gr)
        out = eng.commit_vote(b)
        commit = out.commit.cpu().numpy().view(np.uint64)
        vote = out.vote.cpu().numpy()
        for i, c in enumerate(cs):
            want = c["expect"]
            assert (int(commit[i]) if c["cmd"] == "committed" else int(vote[i])) == want, c["source"]


def test_tracker_mirror(eng):
    import etcd_amd as E
    pt = E.MakeProgressTracker(256)
    pt.Voters = E.JointConfig({1, 2, 3}, {3, 4, 5})
    pt.Learners = {6}
    for vid, m in [(1, 10), (2, 7), (3, 9), (4, 3), (5, 8), (6, 100)]:
        pt.Progress[vid] = E.Progress(Match=m, Next=m + 1, IsLearner=(vid == 6),
                                      RecentActive=vid in (1, 2, 6))
    # c0 {10,7,9} -> 9 ; c1 {9,3,8} -> 8 ; joint -> 8
    assert pt.Committed(DEV) == 8
    pt.RecordVote(1, True)
    pt.RecordVote(1, False)   # first vote sticks
    pt.RecordVote(6, True)    # learner vote: not counted
    pt.RecordVote(4, False)
    g, r, res = pt.TallyVotes(DEV)
    assert (g, r) == (1, 1) and res == E.VotePending
    # recent: 1,2 active in c0 (won), c1 {3,4,5} none active -> lost
    assert pt.QuorumActive(DEV) is False
    pt.Progress[5].RecentActive = True
    pt.Progress[3].RecentActive = True
    assert pt.QuorumActive(DEV) is True


# --------------------------------------------------------------------------
# generator parity
# --------------------------------------------------------------------------
@pytest.mark.parametrize("S,n_inc,n_out,mask_mode,dist", [
    (3, 0, 0, 0, 0), (5, 0, 0, 0, 1), (7, 0, 0, 0, 2), (10, 5, 5, 0, 0), (16, 7, 9, 0, 2),
    (8, 0, 0, 1, 0), (13, 0, 0, 1, 1), (10, 5, 5, 2, 0), (7, 4, 0, 2, 2)])
def test_generator_bit_identical(eng, orc, S, n_inc, n_out, mask_mode, dist):
    G = 4099
    b = gpu_batch(eng, G, S, 0xABCD + S, goff=77, dist=dist, n_inc=n_inc, n_out=n_out,
                  mask_mode=mask_mode)
    h = b.host()
    hb = orc.Batch(G, S)
    orc.gen_batch(hb, 0xABCD + S, goff=77, dist=dist, n_inc=n_inc, n_out=n_out,
                  mask_mode=mask_mode)
    np.testing.assert_array_equal(h["match"], hb.match.reshape(S, G))
    for n in ("inc", "out", "learner", "voted", "granted"):
        np.testing.assert_array_equal(h[n], getattr(hb, n), err_msg=n)


# --------------------------------------------------------------------------
# qe_commit_vote parity
# --------------------------------------------------------------------------
@pytest.mark.parametrize("S", list(range(1, 17)))
def test_commit_vote_fixed_majority_all_slots(eng, orc, S):
    for dist in (0, 1, 2):
        b = gpu_batch(eng, 30001, S, 1000 + S * 7 + dist, masks=(), dist=dist)
        check_commit_vote(eng, orc, b)


@pytest.mark.parametrize("S", list(range(1, 17)))
def test_commit_vote_masked_and_joint(eng, orc, S):
    for mask_mode in (0, 1, 2):
        for dist in (0, 2):
            n_inc = max(1, S // 2)
            n_out = max(1, S - n_inc) if S > 1 else 1
            b = gpu_batch(eng, 20011, S, 77 * S + mask_mode * 3 + dist, goff=S * 1000,
                          dist=dist, n_inc=n_inc, n_out=n_out, mask_mode=mask_mode)
            check_commit_vote(eng, orc, b, goff=S * 1000)
            # masked majority only (inc mask, no out mask)
            b2 = gpu_batch(eng, 5003, S, 5 + S, masks=("inc", "learner"), dist=dist,
                           n_inc=n_inc, mask_mode=mask_mode)
            check_commit_vote(eng, orc, b2)


@pytest.mark.parametrize("G", [1, 2, 3, 63, 64, 65, 127, 128, 129, 255, 257, 1000])
def test_commit_vote_ragged_sizes(eng, orc, G):
    for S, masks in ((5, ()), (10, ("inc", "out", "learner"))):
        b = gpu_batch(eng, G, S, G * 31 + S, masks=masks, n_inc=5, n_out=5, dist=2)
        check_commit_vote(eng, orc, b)


@pytest.mark.parametrize("S", [2, 5, 10, 16])
def test_joint_key_window_boundary(eng, orc, S):
    """joint_committed's 32-bit key fast path vs the 64-bit fallback on
    random spans around 2^30, with zeros, non-members at extreme values, ties, values near
    2^64, and both kinds of group interleaved inside every wave."""
    G = 64 * 40
    rng = np.random.default_rng(4242 + S)
    W = (1 << 30) - 1
    md = eng.mask_np_dtype(S)
    full = (1 << S) - 1
    inc = rng.integers(0, 1 << S, G).astype(md)
    out = np.where(rng.random(G) < 0.7, rng.integers(0, 1 << S, G), 0).astype(md)
    learner = (rng.integers(0, 1 << S, G) & ~(inc.astype(np.int64) | out.astype(np.int64))
               & full).astype(md)
    base = rng.integers(1, 1 << 62, G, dtype=np.uint64)
    base[rng.random(G) < 0.1] = np.uint64((1 << 64) - (1 << 31))  # near the top of u64
    span = np.array([W - 1, W, W + 1, 0, 1, 1 << 40], np.uint64)[rng.integers(0, 6, G)]
    m = base[None, :] + (rng.random((S, G)) * span.astype(np.float64)).astype(np.uint64)
    # pin the extremes so the span is exact: slot 0 = min, slot S-1 = max
    m[0] = base
    m[S - 1] = base + span
    m[rng.random((S, G)) < 0.15] = 0  # absent voters
    tie = rng.random((S, G)) < 0.1
    m[tie] = base[np.nonzero(tie)[1]]
    m[:, rng.random(G) < 0.05] = np.uint64((1 << 64) - 1)  # all-max groups
    voted = rng.integers(0, 1 << S, G).astype(md)
    granted = (rng.integers(0, 1 << S, G) & voted.astype(np.int64)).astype(md)
    b = eng.SlotBatch(G, S, DEV, masks=("inc", "out", "learner"))
    b.load_host(m.reshape(-1), inc=inc, out=out, learner=learner, voted=voted, granted=granted)
    check_commit_vote(eng, orc, b)


@pytest.mark.parametrize("S", [2, 5, 10, 16])
def test_joint_key_prefix_boundary(eng, orc, S):
    """joint_committed's fast path needs every nonzero value to share bits
    29..63.  Groups sit just below, on and across a 2^29 block edge, across
    a 2^32 edge (same bits 29..60, different high word) and across a 2^61
    edge, so both paths and every kind of prefix mismatch occur inside each
    wave; values inside one block exercise offset 0 (the block's first
    value) next to absent (0) voters."""
    G = 64 * 48
    rng = np.random.default_rng(9191 + S)
    md = eng.mask_np_dtype(S)
    full = (1 << S) - 1
    inc = rng.integers(0, 1 << S, G).astype(md)
    out = np.where(rng.random(G) < 0.7, rng.integers(0, 1 << S, G), 0).astype(md)
    B = np.uint64(1 << 29)
    blk = rng.integers(0, 1 << 34, G, dtype=np.uint64) * B  # a 2^29-aligned block start
    edge = np.array([1 << 29, 1 << 32, 1 << 61, 1 << 63], np.uint64)[rng.integers(0, 4, G)]
    blk = np.where(rng.random(G) < 0.5, blk, (blk // edge) * edge)  # on a larger edge
    kind = rng.integers(0, 4, G)
    lo = np.where(kind == 0, blk, np.where(kind == 1, blk + B - np.uint64(1),
                                            blk - np.uint64(3)))  # kind 2/3 straddle
    lo = np.where(lo == 0, np.uint64(1), lo)
    width = np.where(kind == 1, 1, np.where(kind == 0, (1 << 29) - 1, 7)).astype(np.uint64)
    m = lo[None, :] + (rng.random((S, G)) * width.astype(np.float64)).astype(np.uint64)
    m[0] = lo
    m[rng.random((S, G)) < 0.15] = 0
    voted = rng.integers(0, 1 << S, G).astype(md)
    granted = (rng.integers(0, 1 << S, G) & voted.astype(np.int64)).astype(md)
    learner = (rng.integers(0, 1 << S, G) & ~(inc.astype(np.int64) | out.astype(np.int64))
               & full).astype(md)
    b = eng.SlotBatch(G, S, DEV, masks=("inc", "out", "learner"))
    b.load_host(m.reshape(-1), inc=inc, out=out, learner=learner, voted=voted, granted=granted)
    check_commit_vote(eng, orc, b)


def test_commit_vote_scalar_path_odd_stride(eng, orc):
    """stride odd -> slot rows not 16-B aligned -> scalar (non-vector) path."""
    G, S = 1001, 7
    b = eng.SlotBatch(G, S, DEV, masks=("inc", "out"), stride=1003)
    eng.gen_groups(b, 99, n_inc=4, n_out=3)
    check_commit_vote(eng, orc, b)


def test_commit_vote_extremes(eng, orc):
    """Values at the top of the uint64 range (inf-1, 2^63), all-absent and
    empty configs (CommittedIndex = inf, VoteResult = VoteWon)."""
    G, S = 512, 6
    rng = np.random.default_rng(3)
    match = rng.choice(np.array([0, 1, (1 << 63), INF - 1, INF, 12345], dtype=np.uint64),
                       size=(S, G))
    inc = rng.integers(0, 1 << S, G)
    inc[:8] = 0
    out = rng.integers(0, 1 << S, G)
    out[8:16] = 0
    b = eng.SlotBatch(G, S, DEV, masks=("inc", "out", "learner"))
    b.load_host(match, inc=inc, out=out, learner=np.zeros(G), voted=rng.integers(0, 64, G),
                granted=rng.integers(0, 64, G))
    commit, vote = check_commit_vote(eng, orc, b)
    assert all(int(c) == INF for c in commit[:8][(out[:8] == 0)])


def test_committed_index_and_vote_result_entry_points(eng, orc):
    b = gpu_batch(eng, 7777, 9, 4242, n_inc=5, n_out=4, dist=0)
    commit = eng.committed_index(b)
    vote = eng.vote_result(b)
    hb = host_batch(orc, b)
    c_ref, v_ref, _, _, _ = orc.commit_vote(hb)
    np.testing.assert_array_equal(commit.cpu().numpy().view(np.uint64), c_ref)
    np.testing.assert_array_equal(vote.cpu().numpy(), v_ref)


def test_full_size_config2_bit_exact(eng, orc):
    """BASELINE config 2 at full size: 64M groups x 5 voters, every group
    compared with the OpenMP oracle, plus the stats vector."""
    G, S = 1 << 26, 5
    b = gpu_batch(eng, G, S, 0x5EED, masks=())
    check_commit_vote(eng, orc, b)


def test_commit_vote_bucketed_across_buckets(eng, orc):
    """Shape-bucketed layout (mask_mode 2) over several 2^20-group buckets:
    whole waves skip learner slot rows; results stay bit-exact."""
    G, S = (1 << 22) + 12345, 10
    for goff in (0, (1 << 20) - 777):
        b = gpu_batch(eng, G, S, 0xB0C, goff=goff, n_inc=5, n_out=5, mask_mode=2)
        check_commit_vote(eng, orc, b, goff=goff)


@pytest.mark.parametrize("S", [6, 10, 16])
@pytest.mark.parametrize("joint", [False, True])
def test_commit_vote_low_slot_chunks(eng, orc, S, joint):
    """Chunk-uniform "top" specialisation (joint_committed_top): every run of
    256..1024 groups keeps its voters below a random top slot (1..S), so each
    smaller selection network runs, chunks straddle runs, and learners sit
    both above and below top."""
    G = 64 * 8 * 37 + 29
    rng = np.random.default_rng(31 * S + joint)
    md = eng.mask_np_dtype(S)
    tops = np.empty(G, np.int64)
    i = 0
    while i < G:
        n = int(rng.integers(256, 1025))
        tops[i:i + n] = rng.integers(1, S + 1)
        i += n
    lim = (np.int64(1) << tops) - 1
    inc = rng.integers(0, 1 << S, G) & lim
    out = (rng.integers(0, 1 << S, G) & lim) if joint else np.zeros(G, np.int64)
    out[rng.random(G) < 0.2] = 0
    learner = rng.integers(0, 1 << S, G) & ~(inc | out) & ((1 << S) - 1)
    base = rng.integers(1, 1 << 50, G, dtype=np.uint64)
    m = base[None, :] + rng.integers(0, 1 << 20, (S, G), dtype=np.uint64)
    m[rng.random((S, G)) < 0.15] = 0
    voted = rng.integers(0, 1 << S, G)
    granted = rng.integers(0, 1 << S, G) & voted
    masks = ("inc", "out", "learner") if joint else ("inc", "learner")
    b = eng.SlotBatch(G, S, DEV, masks=masks)
    kw = dict(inc=inc.astype(md), learner=learner.astype(md), voted=voted.astype(md),
              granted=granted.astype(md))
    if joint:
        kw["out"] = out.astype(md)
    b.load_host(m.reshape(-1), **kw)
    check_commit_vote(eng, orc, b)


@pytest.mark.parametrize("layout", ["rotated", "bucketed"])
def test_full_size_config3_properties(eng, orc, layout):
    """BASELINE config 3 at full size (128M joint 5+5 groups), in both bench
    layouts (per-group rotated slots; shape-bucketed): every group's commit
    and vote compared with the OpenMP oracle, the order-free stats vector
    (incl. checksum) matches, and the result is symmetric in the halves
    (swap inc/out)."""
    G, S = 1 << 27, 10
    gen = {"mask_mode": 2} if layout == "bucketed" else {}
    b = gpu_batch(eng, G, S, 0xC0FFEE, n_inc=5, n_out=5, **gen)
    out = eng.Outputs(G, DEV, tally=False)
    got, per_group = {}, {}
    try:
        for k in CV_KERNELS:
            eng.tune("cv_kernel", k)
            stats = eng.stats_buffer(DEV)
            eng.commit_vote(b, out, stats=stats)
            got[k] = eng.stats_reduce(stats).cpu().numpy().view(np.uint64)
            if not per_group:
                per_group["commit"] = out.commit.cpu().numpy().view(np.uint64)
                per_group["vote"] = out.vote.cpu().numpy()
            else:
                assert torch.equal(torch.from_numpy(per_group["commit"].view(np.int64)).to(DEV),
                                   out.commit), f"cv_kernel {k}"
            c1 = out.commit.clone()
            b.inc, b.out = b.out, b.inc
            eng.commit_vote(b, out)
            assert torch.equal(c1, out.commit), f"cv_kernel {k}"
            b.inc, b.out = b.out, b.inc
            del c1
    finally:
        eng.tune("cv_kernel", -1)
    del out
    hb = host_batch(orc, b)
    del b
    torch.cuda.empty_cache()
    c_ref, v_ref, _, _, ostats = orc.commit_vote(hb)
    np.testing.assert_array_equal(per_group["commit"], c_ref)
    np.testing.assert_array_equal(per_group["vote"], v_ref)
    for k in CV_KERNELS:
        np.testing.assert_array_equal(got[k], ostats, err_msg=f"cv_kernel {k}")


# --------------------------------------------------------------------------
# QuorumActive / RecordVote
# --------------------------------------------------------------------------
@pytest.mark.parametrize("S", [1, 3, 5, 8, 9, 12, 16])
def test_quorum_active_and_record_votes(eng, orc, S):
    G = 10007
    b = gpu_batch(eng, G, S, 55 + S, mask_mode=1)
    rng = np.random.default_rng(S)
    md = eng.mask_torch_dtype(S)
    npd = eng.mask_np_dtype(S)
    recent = rng.integers(0, 1 << S, G).astype(npd)
    rec_t = torch.from_numpy(recent.view(np.int16) if S > 8 else recent).to(DEV, dtype=md)
    act = eng.quorum_active(b, rec_t).cpu().numpy()
    h = b.host()
    want = orc.quorum_active(G, S, h["inc"], h["out"], h["learner"], recent)
    np.testing.assert_array_equal(act, want)
    # RecordVote twice: the first vote sticks
    voted, granted = h["voted"].copy(), h["granted"].copy()
    for rnd in range(2):
        resp = rng.integers(0, 1 << S, G).astype(npd)
        val = rng.integers(0, 1 << S, G).astype(npd)
        tr = torch.from_numpy(resp.view(np.int16) if S > 8 else resp).to(DEV, dtype=md)
        tv = torch.from_numpy(val.view(np.int16) if S > 8 else val).to(DEV, dtype=md)
        eng.record_votes(b, tr, tv)
        orc.record_votes(G, S, voted, granted, resp, val)
    h2 = b.host()
    np.testing.assert_array_equal(h2["voted"], voted)
    np.testing.assert_array_equal(h2["granted"], granted)


# --------------------------------------------------------------------------
# Replication round (config 4)
# --------------------------------------------------------------------------
def _repl_setup(eng, G, S, seed, joint):
    """joint: False (fixed MajorityConfig), True (JointConfig), "masked"
    (MajorityConfig over a per-group voter subset: inc_mask only)."""
    masks = ("inc", "out") if joint is True else ("inc",) if joint else ()
    b = eng.SlotBatch(G, S, DEV, masks=masks, votes=False)
    eng.gen_groups(b, seed, dist=0, p_absent=0, n_inc=(S + 1) // 2 if joint else 0,
                   n_out=S // 2 + 1 if joint is True else 0)
    base = b.match_rows().clone()
    lo = base.min(dim=0).values
    hi = base.max(dim=0).values
    committed = lo.clone()
    last_index = hi + 64
    term_start = lo + (hi - lo) // 2
    st = eng.ReplicationState(b, committed, term_start, last_index)
    return b, st


@pytest.mark.parametrize("rk", [0, 1])  # qe_tune("repl_kernel"): pair kernel, stream kernel
@pytest.mark.parametrize("S,joint,G", [(3, False, 20011), (5, False, 20011), (7, False, 20011),
                                       (5, True, 20011), (10, True, 20011), (16, True, 20011),
                                       (6, "masked", 20011), (5, False, 1), (5, False, 63),
                                       (5, False, 65), (9, True, 1000), (5, False, 640)])
def test_replication_rounds(eng, orc, S, joint, G, rk):
    eng.tune("repl_kernel", rk)
    try:
        _replication_rounds(eng, orc, S, joint, G)
    finally:
        eng.tune("repl_kernel", -1)


def _replication_rounds(eng, orc, S, joint, G):
    b, st = _repl_setup(eng, G, S, 0x1234 + S, joint)
    rng = np.random.default_rng(S)
    h = {k: v.cpu().numpy().view(np.uint64).copy() for k, v in
         (("match", b.match), ("next", st.next), ("committed", st.committed),
          ("term_start", st.term_start), ("last_index", st.last_index))}
    hm = b.host()
    md = eng.mask_torch_dtype(S)
    npd = eng.mask_np_dtype(S)
    for rnd in range(4):
        resp = (h["match"].reshape(S, -1)[:, :G] + rng.integers(0, 40, (S, G)).astype(np.uint64))
        resp_full = np.zeros((S, b.stride), np.uint64)
        resp_full[:, :G] = resp
        rmask = rng.integers(0, 1 << S, G).astype(npd)
        acks = rng.integers(0, 1 << S, G).astype(npd)
        t_resp = torch.from_numpy(resp_full.reshape(-1).view(np.int64)).to(DEV)
        t_rm = torch.from_numpy(rmask.view(np.int16) if S > 8 else rmask).to(DEV, dtype=md)
        t_ack = torch.from_numpy(acks.view(np.int16) if S > 8 else acks).to(DEV, dtype=md)
        read_ok = torch.zeros(G, dtype=torch.uint8, device=DEV)
        adv = torch.zeros(G, dtype=torch.uint8, device=DEV)
        stats = eng.stats_buffer(DEV)
        eng.replication_round(st, t_resp, t_rm, t_ack, read_ok, adv, stats)
        folded = eng.stats_reduce(stats).cpu().numpy().view(np.uint64)
        o_ro, o_adv, o_stats = orc.replication_round(
            G, 0, S, b.stride, h["match"], h["next"], h["committed"], h["term_start"],
            h["last_index"], hm["inc"], hm["out"], resp_full.reshape(-1), rmask, acks)
        np.testing.assert_array_equal(b.match.cpu().numpy().view(np.uint64), h["match"])
        np.testing.assert_array_equal(st.next.cpu().numpy().view(np.uint64), h["next"])
        np.testing.assert_array_equal(st.committed.cpu().numpy().view(np.uint64), h["committed"])
        np.testing.assert_array_equal(read_ok.cpu().numpy(), o_ro)
        np.testing.assert_array_equal(adv.cpu().numpy(), o_adv)
        np.testing.assert_array_equal(folded, o_stats)
        if G > 1000:
            assert o_adv.sum() > 0


def test_test_commit_table_on_gpu(eng):
    """TestCommit (raft/raft_test.go:1127-1174) through qe_replication_round:
    matches arrive as MsgAppResp on a fresh Progress, then maybeCommit."""
    rows = raft_tables()["TestCommit"]["rows"]
    by_n = {}
    for r in rows:
        by_n.setdefault(len(r["matches"]), []).append(r)
    for n, rs in by_n.items():
        G = len(rs)
        b = eng.SlotBatch(G, n, DEV, masks=(), votes=False)
        resp = np.zeros((n, b.stride), np.uint64)
        ts = np.zeros(G, np.uint64)
        li = np.zeros(G, np.uint64)
        for i, r in enumerate(rs):
            resp[:, i] = r["matches"]
            ts[i], li[i] = Q.log_term_range(r["logs"], r["sm_term"])
        st = eng.ReplicationState(
            b, torch.zeros(G, dtype=torch.int64, device=DEV),
            torch.from_numpy(ts.view(np.int64)).to(DEV), torch.from_numpy(li.view(np.int64)).to(DEV),
            nxt=torch.ones(n * b.stride, dtype=torch.int64, device=DEV))
        full = (1 << n) - 1
        rm = torch.full((G,), full, dtype=torch.uint8, device=DEV)
        eng.replication_round(st, torch.from_numpy(resp.reshape(-1).view(np.int64)).to(DEV), rm)
        got = st.committed.cpu().numpy()
        assert [int(x) for x in got] == [r["want"] for r in rs]


# --------------------------------------------------------------------------
# Election simulation (config 5)
# --------------------------------------------------------------------------
@pytest.mark.parametrize("S,joint,flags", [(1, False, 0), (3, False, 0), (5, False, 0),
                                           (7, False, 0), (10, True, 0), (16, True, 0),
                                           (1, False, 3), (3, False, 1), (5, False, 2),
                                           (5, False, 3), (10, True, 3), (16, True, 1)])
def test_election_steps(eng, orc, S, joint, flags):
    """Random election steps (RNG drops/grants), optionally with PreVote (1)
    and CheckQuorum (2), bit-exact against the oracle."""
    G = 30011
    masks = ("inc", "out", "learner")
    b = eng.SlotBatch(G, S, DEV, masks=masks, votes=False, group_offset=999)
    eng.gen_groups(b, 0xE1EC + S, n_inc=(S + 1) // 2 if joint else 0,
                   n_out=(S // 2 if joint else 0))
    self_slot = eng.first_voter_slot(b)
    est = eng.ElectionState(b, self_slot)
    h = b.host()
    term = np.zeros(G, np.uint64)
    state = np.zeros(G, np.uint8)
    voted = np.zeros(G, eng.mask_np_dtype(S))
    granted = np.zeros(G, eng.mask_np_dtype(S))
    ss = self_slot.cpu().numpy()
    step0 = 0
    leaders = 0
    for launch, steps in enumerate((1, 7, 32)):
        stats = eng.stats_buffer(DEV)
        eng.election_steps(est, 77, step0, steps, p_drop=13107, p_grant=32768, stats=stats,
                           flags=flags, p_active=45875)
        got = eng.stats_reduce(stats).cpu().numpy().view(np.uint64)
        want = orc.election_steps(G, 999, S, term, state, voted, granted, ss, h["inc"], h["out"],
                                  h["learner"], 77, step0, steps, 13107, 32768, flags=flags,
                                  p_active=45875)
        step0 += steps
        np.testing.assert_array_equal(est.term.cpu().numpy().view(np.uint64), term)
        np.testing.assert_array_equal(est.state.cpu().numpy(), state)
        np.testing.assert_array_equal(est.voted.cpu().numpy().view(voted.dtype), voted)
        np.testing.assert_array_equal(est.granted.cpu().numpy().view(granted.dtype), granted)
        np.testing.assert_array_equal(got, want)
        assert want[14] == 0  # invariant violations
        leaders += int(want[12])
    assert leaders > 0  # some leaders elected


def test_election_scenarios_on_gpu(eng):
    """The scripted election scenarios (TestLeaderElectionInOneRoundRPC,
    TestLeaderStepdownWhenQuorumLost, TestPreVoteWithSplitVote node views)
    through k_election on the GPU."""
    from tests.election_scenarios import run_scenario, scenarios, script_arrays
    for sc in scenarios():
        S = sc["S"]
        b = eng.SlotBatch(1, S, DEV, masks=("inc", "learner"), votes=False)
        b.inc.fill_((1 << S) - 1)
        est = eng.ElectionState(b, torch.tensor([sc["self"]], dtype=torch.uint8, device=DEV))
        est.term.fill_(sc["term"])
        est.state.fill_(sc["state"])
        resp, grant, hup = (torch.from_numpy(x).to(DEV) for x in script_arrays(sc))
        if S > 8:
            resp, grant = resp.view(torch.int16), grant.view(torch.int16)

        def step(k, est=est, resp=resp, grant=grant, hup=hup, sc=sc):
            eng.election_steps(est, 0, k, 1, p_drop=0, p_grant=0, flags=sc["flags"],
                               script=(resp[k:], grant[k:], hup[k:], 1))
            return int(est.term[0]), int(est.state[0])
        run_scenario(sc, step)


def test_leader_election_table_on_gpu(eng):
    """TestLeaderElectionInOneRoundRPC through the GPU primitives:
    campaign self-vote (qe_record_votes) then one response round
    (qe_record_votes) and TallyVotes (qe_commit_vote)."""
    rows = raft_tables()["TestLeaderElectionInOneRoundRPC"]["rows"]
    for r in rows:
        n = r["size"]
        b = eng.SlotBatch(1, n, DEV, masks=(), votes=True)
        b.load_host(np.zeros((n, 1), np.uint64))
        one = torch.ones(1, dtype=torch.uint8, device=DEV)
        eng.record_votes(b, one, one)  # self (slot 0 = id 1) votes yes
        out = eng.commit_vote(b)
        state = "StateLeader" if int(out.vote[0]) == 3 else "StateCandidate"
        for vid, v in r["votes"]:
            if state != "StateCandidate":
                break
            bit = torch.tensor([1 << (vid - 1)], dtype=torch.uint8, device=DEV)
            eng.record_votes(b, bit, bit if v else torch.zeros_like(bit))
            res = int(eng.commit_vote(b).vote[0])
            state = {3: "StateLeader", 2: "StateFollower"}.get(res, "StateCandidate")
        assert state == r["state"], r


def test_tuning_knobs_do_not_change_results(eng, orc):
    b = gpu_batch(eng, 100003, 7, 31337, masks=())
    try:
        for bpc in (1, 2, 0):
            for nt in (0, 1, 2, 3):
                for tpw in (0, 1, 3):
                    eng.tune("blocks_per_cu", bpc)
                    eng.tune("nontemporal", nt)
                    eng.tune("tiles_per_wave", tpw)
                    check_commit_vote(eng, orc, b)
    finally:
        eng.tune("blocks_per_cu", 0)
        eng.tune("nontemporal", 3)
        eng.tune("tiles_per_wave", -1)


# --------------------------------------------------------------------------
# Sparse MsgAppResp deltas + wire-format packing end to end
# --------------------------------------------------------------------------
def test_apply_append_resps_matches_sequential_maybe_update(eng):
    """qe_apply_append_resps (atomic max) == Progress.MaybeUpdate applied
    one ack at a time in arrival order (progress.go:144-153), incl.
    duplicates, stale acks, skipped (-1) slots and out-of-range groups."""
    import ctypes as C
    rng = np.random.default_rng(11)
    G, S, n = 10007, 7, 200000
    b = eng.SlotBatch(G, S, DEV, masks=(), votes=False)
    eng.gen_groups(b, 5, dist=2)
    match0 = b.match.cpu().numpy().view(np.uint64).reshape(S, b.stride).copy()
    nxt = b.match.clone() + 1
    next0 = nxt.cpu().numpy().view(np.uint64).reshape(S, b.stride).copy()
    group = rng.integers(0, G + 3, n).astype(np.uint64)
    slot = rng.integers(-1, S, n).astype(np.int8)
    index = rng.integers(0, 8, n).astype(np.uint64)
    touched = torch.zeros(G, dtype=torch.uint8, device=DEV)
    dg = torch.from_numpy(group.view(np.int64)).to(DEV)
    ds = torch.from_numpy(slot).to(DEV)
    di = torch.from_numpy(index.view(np.int64)).to(DEV)
    eng.check("qe_apply_append_resps", eng._lib.lib().qe_apply_append_resps(
        G, S, b.stride, eng._ptr(b.match), eng._ptr(nxt), n, eng._ptr(dg), eng._ptr(ds),
        eng._ptr(di), eng._ptr(touched), eng._stream(b.device)))
    m, nx = match0.copy(), next0.copy()
    want_touched = np.zeros(G, np.uint8)
    for g, s, x in zip(group.tolist(), slot.tolist(), index.tolist()):
        if g >= G or s < 0:
            continue
        _, m[s, g], nx[s, g] = Q.maybe_update(int(m[s, g]), int(nx[s, g]), x)
        want_touched[g] = 1
    np.testing.assert_array_equal(b.match.cpu().numpy().view(np.uint64).reshape(S, -1), m)
    np.testing.assert_array_equal(nxt.cpu().numpy().view(np.uint64).reshape(S, -1), nx)
    np.testing.assert_array_equal(touched.cpu().numpy(), want_touched)


def test_wire_format_to_gpu_decisions(eng):
    """ConfState CSR -> native packer -> device -> qe_commit_vote equals the
    map-based restatement on the same ConfStates / Progress / Votes."""
    import random
    from etcd_amd.packing import ConfStates, pack_confstates, pack_progress, pack_votes
    rng = random.Random(99)
    confs, progress, votes = [], [], []
    for _ in range(5000):
        pool = rng.sample(range(1, 1 << 30), 10)
        c0 = pool[:rng.randint(0, 5)]
        c1 = (rng.sample(c0, rng.randint(0, len(c0))) + pool[5:5 + rng.randint(0, 3)]
              if rng.random() < 0.5 else [])
        lrn = pool[8:8 + rng.randint(0, 2)]
        confs.append((c0, c1, lrn))
        peers = list(dict.fromkeys(c0 + c1 + lrn))
        progress.append({i: rng.randrange(100) for i in peers if rng.random() < 0.9})
        votes.append([(i, rng.random() < 0.5) for i in peers if rng.random() < 0.8])
    cs = ConfStates([c[0] for c in confs], [c[1] for c in confs], [c[2] for c in confs])
    p = pack_confstates(cs, 12)
    pack_progress(p, progress)
    pack_votes(p, votes)
    b = eng.SlotBatch(p.G, p.S, DEV)
    b.load_host(p.match, inc=p.inc, out=p.out, learner=p.learner, voted=p.voted,
                granted=p.granted)
    out = eng.commit_vote(b)
    commit = out.commit.cpu().numpy().view(np.uint64)
    vote, gc, rc = (x.cpu().numpy() for x in (out.vote, out.granted, out.rejected))
    for g, (c0, c1, lrn) in enumerate(confs):
        vmap = {}
        for i, v in votes[g]:
            Q.record_vote(vmap, i, v)
        assert int(commit[g]) == Q.joint_committed(c0, c1, progress[g])
        assert (int(gc[g]), int(rc[g]), int(vote[g])) == Q.tally_votes(c0, c1, set(lrn), vmap)


def test_wire_format_bucketed_to_gpu_decisions(eng):
    """The same wire-format path in the shape-bucketed order (qe_pack_order,
    ABI 3): packed position i holds the caller's group perm[i]; its commit /
    vote / tally equal the map-based restatement of that caller group, and
    qe_collect with the perm reports caller group ids."""
    import random
    from etcd_amd.packing import ConfStates, pack_confstates, pack_progress, pack_votes
    rng = random.Random(199)
    confs, progress, votes = [], [], []
    for _ in range(20000):
        pool = rng.sample(range(1, 1 << 30), 10)
        c0 = pool[:rng.randint(0, 5)]
        c1 = (rng.sample(c0, rng.randint(0, len(c0))) + pool[5:5 + rng.randint(0, 3)]
              if rng.random() < 0.5 else [])
        lrn = pool[8:8 + rng.randint(0, 2)]
        confs.append((c0, c1, lrn))
        peers = list(dict.fromkeys(c0 + c1 + lrn))
        progress.append({i: rng.randrange(1000) for i in peers if rng.random() < 0.9})
        votes.append([(i, rng.random() < 0.5) for i in peers if rng.random() < 0.8])
    cs = ConfStates([c[0] for c in confs], [c[1] for c in confs], [c[2] for c in confs])
    p = pack_confstates(cs, 12, bucketed=True)
    perm = p.perm.astype(np.int64)
    assert sorted(perm.tolist()) == list(range(len(confs)))
    pack_progress(p, progress)
    pack_votes(p, votes)
    b = eng.SlotBatch(p.G, p.S, DEV)
    b.load_host(p.match, inc=p.inc, out=p.out, learner=p.learner, voted=p.voted,
                granted=p.granted)
    out = eng.commit_vote(b)
    commit = out.commit.cpu().numpy().view(np.uint64)
    vote, gc, rc = (x.cpu().numpy() for x in (out.vote, out.granted, out.rejected))
    for i in range(p.G):
        g = int(perm[i])
        c0, c1, lrn = confs[g]
        vmap = {}
        for k, v in votes[g]:
            Q.record_vote(vmap, k, v)
        assert int(commit[i]) == Q.joint_committed(c0, c1, progress[g]), (i, g)
        assert (int(gc[i]), int(rc[i]), int(vote[i])) == Q.tally_votes(c0, c1, set(lrn), vmap)
    # Ready deltas in caller ids: the won groups and their commit index
    flags = (out.vote == 3).to(torch.uint8)
    perm_d = torch.from_numpy(perm).to(DEV)
    groups, vals = eng.collect(flags, out.commit, group_offset=1000, perm=perm_d)
    torch.cuda.synchronize()
    sel = np.nonzero(vote == 3)[0]
    np.testing.assert_array_equal(groups.cpu().numpy(), perm[sel] + 1000)
    np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint64), commit[sel])


def test_config3_packed_workload_matches_oracle(eng, orc):
    """bench.py config3_joint_packed at 2M groups: ConfStates of per-group
    uniform overlap built by bench.joint_confstates, packed through
    qe_pack_order + qe_pack_confstate in 1M-group batches; every packed
    group's commit / vote equals the oracle, the layout is bucketed (each
    wave's voters sit in the same low slots), and per caller group the
    packed masks equal an identity packing of the same ConfState."""
    import bench
    from etcd_amd.packing import pack_confstates
    bench.engine = eng
    G, S, goff = 1 << 21, 10, 12345
    b = eng.SlotBatch(G, S, DEV, group_offset=goff)
    perm = bench.pack_joint_batches(b, goff, chunk=1 << 20).cpu().numpy()
    eng.gen_groups(b, 0x5EED, values_only=True)
    check_commit_vote(eng, orc, b, goff=goff)
    h = b.host()
    uni = (h["inc"] | h["out"]).astype(np.int64)
    # voters first: the union is the low slots of every group
    u = np.array([bin(x).count("1") for x in range(1 << S)])[uni]
    np.testing.assert_array_equal(uni, (1 << u) - 1)
    # tiles whose 64 groups share one union size: all but the bucket edges
    tiles = u[: G // 64 * 64].reshape(-1, 64)
    mixed = int((tiles.min(1) != tiles.max(1)).sum())
    assert mixed <= 2 * 6 * 2, mixed  # <= 2 edges per shape per 1M batch
    # per caller group: identity packing of its own ConfState
    cs, o = bench.joint_confstates(goff, 1 << 20, DEV)
    ident = pack_confstates(cs, S)
    first = perm[: 1 << 20]
    np.testing.assert_array_equal(h["inc"][: 1 << 20], ident.inc[first])
    np.testing.assert_array_equal(h["out"][: 1 << 20], ident.out[first])
    np.testing.assert_array_equal(10 - u[: 1 << 20], o[first])
