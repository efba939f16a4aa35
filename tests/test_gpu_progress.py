"""GPU parity of the Progress state machine (qe_progress_step /
qe_progress_send / qe_check_quorum, SURVEY.md §8(f) rows 3-4 and the
ReadIndex / CheckQuorum decisions) against the oracle, which
tests/test_progress_oracle.py pins to the reference's tables, the
leader-side scenarios of tests/golden/progress_scenarios.json and the
ReadIndex / CheckQuorum transcriptions of tests/leader_round_scenarios.py.
The same scenarios run here through the HIP kernels, and the instrumented
kernel's byte count must equal the oracle's restatement of the accounting
rules exactly."""
import numpy as np
import pytest
import torch

from oracle import orc
from tests.golden_util import raft_tables
from tests.progress_scenarios import cap, peer_view, run_scenario, scenarios
from tests.test_progress_oracle import log_runs

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
EXTRAS = ("tracked", "self_slot", "lead_transferee", "snap_index")
READS = EXTRAS + ("reads",)


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from etcd_amd import engine
    return engine


def random_state(rng, G, S, F, R, masks, extras=(), max_ents=0, base=0):
    """A random leader-side state.  `base` shifts every log index (ABI 4:
    near a 2^32 boundary the Inflights rings straddle two epochs, past 2^43
    every ring is wide)."""
    pb = orc.ProgressBatch(G, S, F, R, max_ents=max_ents)
    pb.base = base
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
    fi = np.tile(pb.first_index, S)
    low = rng.random(n) < 0.08  # compacted: Next < firstIndex (snapshot path)
    pb.next[low] = (rng.random(int(low.sum())) * fi[low]).astype(np.uint64)
    flags = (rng.integers(0, 3, n) | (rng.integers(0, 2, n) * 4) |
             (rng.integers(0, 2, n) * 8)).astype(np.uint8)
    # PendingSnapshot only in StateSnapshot (reachable states; the ABI's
    # precondition: ResetState clears it on every state change)
    pb.pending[:] = np.where((flags & 3) == 2, rng.integers(0, 70, n), 0).astype(np.uint64)
    pb.set_peer(flags=flags, istart=rng.integers(0, F, n).astype(np.uint8),
                icount=rng.integers(0, F + 1, n).astype(np.uint8))
    m0 = pb.match.copy()
    for k in range(F):  # entry-major rings: entry k of slot s at (s*F + k)*stride + g
        pb.ibuf[(np.arange(S)[:, None] * F + k) * pb.stride + np.arange(G)[None, :]] = \
            (m0.reshape(S, G) + 1 + 2 * ((k - pb.istart.reshape(S, G).astype(int)) % F)).astype(np.uint64)
    md = orc.mask_dtype(S)
    if "inc" in masks:
        pb.inc = rng.integers(0, 1 << S, G).astype(md)
    if "out" in masks:
        pb.out = rng.integers(0, 1 << S, G).astype(md)
    if "tracked" in extras:
        t = rng.integers(0, 1 << S, G)
        t[rng.random(G) < 0.5] = (1 << S) - 1
        pb.tracked = t.astype(md)
    if "self_slot" in extras:
        pb.self_slot = rng.integers(0, S + 2, G).astype(np.uint8)  # >= S: no self
    if "lead_transferee" in extras:
        pb.lead_transferee = np.where(rng.random(G) < 0.5, 0xFF,
                                      rng.integers(0, S, G)).astype(np.uint8)
    if "snap_index" in extras:
        pb.snap_index = (pb.first_index - 1 + rng.integers(0, 3, G)).astype(np.uint64)
    if base:
        b = np.uint64(base)
        for k in ("match", "next", "ibuf", "committed", "term_start", "first_index",
                  "last_index", "run_first"):
            setattr(pb, k, (getattr(pb, k) + b).astype(np.uint64))
        # (a StateSnapshot peer's PendingSnapshot shifts; every other stays 0)
        pb.pending = np.where(pb.pending != 0, pb.pending + b, pb.pending).astype(np.uint64)
        if pb.snap_index is not None:
            pb.snap_index = (pb.snap_index + b).astype(np.uint64)
    return pb


def random_msgs(rng, pb):
    n = pb.S * pb.G
    mtype = rng.integers(0, 9, n).astype(np.uint8)  # 8 = unknown kind -> ignored
    li = np.tile(pb.last_index, pb.S)
    lo = np.uint64(getattr(pb, "base", 0))
    mindex = np.where(rng.random(n) < 0.5, pb.next - 1,
                      lo + (rng.random(n) * (li - lo + 3)).astype(np.uint64)).astype(np.uint64)
    mhint = (lo + (rng.random(n) * (li - lo + 2)).astype(np.uint64)).astype(np.uint64)
    mlogterm = np.where(rng.random(n) < 0.3, 0, rng.integers(1, 10, n)).astype(np.uint64)
    return mtype, mindex, mhint, mlogterm


def to_device(eng, pb, masks, extras=()):
    if pb.read_keys is not None:
        extras = tuple(extras) + ("read_keys",)
    ps = eng.ProgressState(pb.G, pb.S, pb.F, pb.R, DEV, masks=masks, stride=pb.stride,
                           extras=extras, max_ents=pb.max_ents, read_cap=pb.read_cap,
                           ring16=pb.ring16)
    md = orc.mask_dtype(pb.S)
    ps.load_host(match=pb.match, next=pb.next, pending=pb.pending, peer=pb.pw,
                 ibuf=pb.ibuf, committed=pb.committed,
                 term_start=pb.term_start, first_index=pb.first_index, last_index=pb.last_index,
                 run_first=pb.run_first, run_term=pb.run_term, run_count=pb.run_count,
                 inc=pb.inc, out=pb.out, tracked=pb.tracked, self_slot=pb.self_slot,
                 lead_transferee=pb.lead_transferee, snap_index=pb.snap_index,
                 read_acks=None if pb.read_acks is None else pb.read_acks.view(md),
                 read_head=pb.read_head, read_count=pb.read_count,
                 read_ovf=None if pb.read_ovf is None else pb.read_ovf.view(md),
                 read_keys=pb.read_keys)
    return ps


RING_MASK = np.uint32(0xFF0000F0)  # QE_PW_RING_MASK: representation bits (ABI 4)


def live_entries(pw, S, F, stride):
    """Entry-major [S][F][stride] mask of the live Inflights positions
    (start .. start+count-1 mod F, raft/tracker/inflights.go:25-37)."""
    w = pw.reshape(S, 1, stride).astype(np.int64)
    start, count = (w >> 8) & 0xFF, (w >> 16) & 0xFF
    k = np.arange(F).reshape(1, F, 1)
    return (((k - start) % F) < count).reshape(-1)


def assert_same(ps, pb):
    """Progress state equal to the oracle's: every field, the peer words
    without their ring representation bits, and every live ring entry
    (decoded from the 32-bit form; dead positions are unobservable)."""
    h = ps.host()
    for k in ("match", "next", "pending", "committed"):
        np.testing.assert_array_equal(h[k], getattr(pb, k), err_msg=k)
    if pb.lead_transferee is not None:
        np.testing.assert_array_equal(h["lead_transferee"], pb.lead_transferee,
                                      err_msg="lead_transferee")
    if pb.read_acks is not None:  # the ReadIndex queue (ABI 5), raw words
        np.testing.assert_array_equal(h["read_acks"], pb.read_acks.view(orc.mask_dtype(pb.S)),
                                      err_msg="read_acks")
        np.testing.assert_array_equal(h["read_head"], pb.read_head, err_msg="read_head")
        np.testing.assert_array_equal(h["read_count"], pb.read_count, err_msg="read_count")
        if pb.read_ovf is not None:  # ABI 7: the overflow ring, raw (dead slots untouched)
            np.testing.assert_array_equal(h["read_ovf"], pb.read_ovf, err_msg="read_ovf")
        if pb.read_keys is not None:
            np.testing.assert_array_equal(h["read_keys"], pb.read_keys, err_msg="read_keys")
    np.testing.assert_array_equal(h["peer"] & ~RING_MASK, pb.pw, err_msg="packed peer words")
    live = live_entries(pb.pw, pb.S, pb.F, pb.stride)
    np.testing.assert_array_equal(h["ibuf"][live], pb.ibuf[live], err_msg="live ring entries")


def to_dev_mask(a, S):
    return torch.from_numpy(a.view(np.int16) if S > 8 else a).to(DEV)


def load_msgs(eng, ps, mtype, mindex, mhint, mlogterm):
    msgs = eng.PeerMsgs(ps)
    for name, a in (("type", mtype), ("index", mindex), ("reject_hint", mhint),
                    ("log_term", mlogterm)):
        t = torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(DEV)
        getattr(msgs, name)[: t.numel()].copy_(t)
    return msgs


def assert_outputs(msgs, o, S):
    md = orc.mask_dtype(S)
    for k in ("sent", "snap", "timeout_now"):
        np.testing.assert_array_equal(getattr(msgs, k).cpu().numpy().view(md), getattr(o, k),
                                      err_msg=k)
    np.testing.assert_array_equal(msgs.bcast.cpu().numpy(), o.bcast, err_msg="bcast")
    cnt = msgs.msg_count.cpu().numpy()
    np.testing.assert_array_equal(cnt, o.msg_count, err_msg="msg_count")
    got_ix = msgs.msg_index.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got_ix[cnt > 0], o.msg_index[cnt > 0], err_msg="msg_index")
    np.testing.assert_array_equal(msgs.read_released.cpu().numpy(), o.read_released,
                                  err_msg="read_released")
    tc = msgs.term_commit.cpu().numpy()
    np.testing.assert_array_equal(tc, o.term_commit, err_msg="term_commit")
    tci = msgs.term_commit_index.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(tci[tc > 0], o.term_commit_index[tc > 0],
                                  err_msg="term_commit_index")


def ring16_state(rng, pb):
    """ABI 8: the batch in the 16-bit Inflights form (pb.ring16: the oracle
    counts 2-byte entries).  Next moved just above the live entries of most
    peers with a ring (the form holds them), 65536+ above some (wide) and
    left below others (an inconsistent input: wide); every entry stays
    exact either way."""
    pb.ring16 = True
    S, F, st = pb.S, pb.F, pb.stride
    live = live_entries(pb.pw, S, F, st).reshape(S, F, st)
    ent = pb.ibuf.reshape(S, F, st)
    mx = np.where(live, ent, np.uint64(0)).max(1)
    has = live.any(1)
    pick = rng.random((S, st))
    nxt = pb.next.reshape(S, st)
    new = np.where(pick < 0.75, mx + np.uint64(1) + rng.integers(0, 3, (S, st)).astype(np.uint64),
                   np.where(pick < 0.85, mx + np.uint64(65536) + rng.integers(0, 3, (S, st)).astype(np.uint64),
                            nxt))
    pb.next[:] = np.where(has, new, nxt).reshape(-1)


def random_queue(rng, pb):
    """A random ReadIndex queue per group (ABI 5): 0..4 pending requests with
    random acks (dead entries hold garbage), context numbers from near 1 to
    near 2^32."""
    pb.track_reads()
    G = pb.G
    pb.read_count[:] = rng.integers(0, 5, G)
    pb.read_head[:] = np.where(rng.random(G) < 0.8, rng.integers(1, 50, G),
                               rng.integers(1, 1 << 32, G, dtype=np.uint64)).astype(np.uint32)
    wbits = 32 if pb.S <= 8 else 64
    pb.read_acks[:] = rng.integers(0, 1 << 62, G, dtype=np.uint64).astype(
        np.uint32 if wbits == 32 else np.uint64)


def random_read_ctx(rng, pb):
    """The context numbers heartbeat responses carry: none, a pending
    request's (any), a released or not-yet-assigned one, or garbage."""
    n = pb.S * pb.G
    head = np.tile(pb.read_head, pb.S).astype(np.int64)
    cnt = np.tile(pb.read_count, pb.S).astype(np.int64)
    pick = rng.integers(0, 4, n)
    off = rng.integers(-2, 6, n)
    ctx = np.where(pick == 0, 0, np.where(pick == 3, rng.integers(0, 1 << 32, n),
                                           head + np.where(pick == 1, rng.integers(0, 4, n) % np.maximum(cnt, 1), off)))
    return (ctx & 0xFFFFFFFF).astype(np.uint32)


CASES = [(1, (), ()), (3, (), EXTRAS), (5, (), ()), (5, (), EXTRAS), (5, ("inc",), EXTRAS),
         (7, ("inc", "out"), EXTRAS), (10, ("inc", "out"), ()), (16, ("inc",), EXTRAS)]


@pytest.mark.parametrize("F", [3, 5, 8, 32])
@pytest.mark.parametrize("R", [3, 6])
@pytest.mark.parametrize("S,masks,extras", CASES)
def test_progress_rounds_match_oracle(eng, S, masks, extras, R, F):
    """Random states and the full message mix (rejects with LogTerm > 0,
    snapshots, heartbeats carrying ReadIndex contexts against a random
    queue, MsgTransferLeader, ...) through the 4-run (R = 3, the production
    kernel) and 8-run (R = 6) kernels; row-resident rings of one 16-byte
    access (F = 3), padded pitch (F = 5) and two accesses (F = 8), and
    memory rings (F = 32).  Odd rounds run the instrumented variant, whose
    byte count must equal the oracle's exactly."""
    rounds_vs_oracle(eng, S, masks, extras, R, F, ring16=False)


@pytest.mark.parametrize("F", [3, 5, 8])
@pytest.mark.parametrize("S,masks,extras", [(1, (), ()), (3, (), EXTRAS), (5, (), ()),
                                            (5, ("inc",), EXTRAS), (7, ("inc", "out"), EXTRAS),
                                            (9, (), EXTRAS)])
def test_progress_rounds_ring16_match_oracle(eng, S, masks, extras, F):
    """The same rounds with the rings in the 16-bit form (ABI 8): the
    pipelined step, the send, CheckQuorum and ReadIndex on states whose rings
    mostly fit below Next, some wide; the instrumented variant counts 2-byte
    entries, as the oracle does."""
    rounds_vs_oracle(eng, S, masks, extras, 3, F, ring16=True)


def rounds_vs_oracle(eng, S, masks, extras, R, F, ring16):
    rng = np.random.default_rng(100 + S + 7 * len(extras) + 31 * R + F + 1000 * ring16)
    G = 3001
    pb = random_state(rng, G, S, F, R, masks, extras, max_ents=int(rng.integers(0, 4)))
    if ring16:
        ring16_state(rng, pb)
    reads = "lead_transferee" in extras  # the ReadIndex queue with the full extras
    if reads:
        random_queue(rng, pb)
    ps = to_device(eng, pb, masks, extras + (("reads",) if reads else ()))
    md = orc.mask_dtype(S)
    for rnd in range(6):
        mtype, mindex, mhint, mlogterm = random_msgs(rng, pb)
        msgs = load_msgs(eng, ps, mtype, mindex, mhint, mlogterm)
        ctx = None
        if reads and rnd % 3 != 2:  # every third round: the newest-context default
            ctx = random_read_ctx(rng, pb)
            msgs.set_read_ctx(ps, ctx)
        if reads and rnd == 3:  # new requests (qe_read_index) between rounds
            req = (rng.random(G) < 0.6).astype(np.uint8)
            lease = bool(rng.integers(0, 2))
            r_g, c_g, i_g = eng.read_index(ps, torch.from_numpy(req).to(DEV), lease)
            r_o, c_o, i_o = orc.read_index(pb, req, lease)
            np.testing.assert_array_equal(r_g.cpu().numpy(), r_o)
            q = r_o == 3
            np.testing.assert_array_equal(c_g.cpu().numpy().view(np.uint32)[q], c_o[q])
            w = (r_o == 1) | q
            np.testing.assert_array_equal(i_g.cpu().numpy().view(np.uint64)[w], i_o[w])
            assert_same(ps, pb)
        stats = eng.stats_buffer(DEV)
        if rnd % 2:
            msgs.bytes_requested = torch.zeros(1, dtype=torch.int64, device=DEV)
        eng.progress_step(ps, msgs, stats)
        got = eng.stats_reduce(stats).cpu().numpy().view(np.uint64)
        o = orc.progress_step(pb, mtype, mindex, mhint, mlogterm, read_ctx=ctx, count_bytes=True)
        assert_same(ps, pb)
        assert_outputs(msgs, o, S)
        np.testing.assert_array_equal(got, o.stats)
        if rnd % 2:
            assert int(msgs.bytes_requested.item()) == int(o.bytes[0]), (rnd, S)
        # a sendAppend / bcastAppend round to random peers
        want = rng.integers(0, 1 << S, G).astype(md)
        sei, me = int(rnd % 2), int(rng.integers(0, 5))
        ps.max_ents = pb.max_ents = me
        sent, snap = eng.progress_send(ps, to_dev_mask(want, S), sei)
        o_sent, o_snap = orc.progress_send(pb, want, sei)
        np.testing.assert_array_equal(sent.cpu().numpy().view(md), o_sent)
        np.testing.assert_array_equal(snap.cpu().numpy().view(md), o_snap)
        assert_same(ps, pb)
        # CheckQuorum every third round (RecentActive set by the step above)
        if rnd % 3 == 1:
            st2 = eng.stats_buffer(DEV)
            qa = eng.check_quorum(ps, stats=st2)
            got2 = eng.stats_reduce(st2).cpu().numpy().view(np.uint64)
            o_qa, o_st = orc.check_quorum(pb)
            np.testing.assert_array_equal(qa.cpu().numpy(), o_qa)
            np.testing.assert_array_equal(got2, o_st)
            assert_same(ps, pb)


@pytest.mark.parametrize("F", [3, 5, 8])
@pytest.mark.parametrize("S,masks", [(2, ()), (3, ()), (4, ("inc",)), (5, ()), (5, ("inc",)),
                                     (6, ("inc", "out")), (7, ("inc",)), (8, ()), (9, ())])
def test_progress_quiet_slot_tiles(eng, S, masks, F):
    """Tiles (64 groups) in which one slot is quiet in every group -- no
    message, and the leader's own slot or an untracked one -- as the
    leader's slot is in a steady round: the pipelined loop (rings in row
    form, up to 9 slots) walks the other slots only and writes MsgCount = 0
    for that one.  Tile t's quiet slot is t % (S + 1) (S: none); in every
    fourth tile one group breaks it (a message from a tracked follower in
    that slot: every slot walked), and the last tile is partial."""
    rng = np.random.default_rng(700 + 13 * S + F + len(masks))
    G = 64 * 23 + 17
    pb = random_state(rng, G, S, F, 3, masks, EXTRAS)
    random_queue(rng, pb)
    tile = np.arange(G) // 64
    q = tile % (S + 1)
    quiet = q < S
    own = quiet & (rng.random(G) < 0.6)  # the leader's slot; otherwise untracked
    pb.self_slot[own] = q[own]
    md = orc.mask_dtype(S)
    unt = quiet & ~own
    pb.tracked[unt] &= np.array(~(1 << q[unt]) & ((1 << S) - 1)).astype(md)
    pb.self_slot[unt & (pb.self_slot == q)] = 0xFF
    brk = np.zeros(G, bool)
    for t in range(0, tile[-1] + 1, 4):  # one group per fourth tile breaks the quiet slot
        g = t * 64 + int(rng.integers(0, min(64, G - t * 64)))
        if quiet[g]:
            brk[g] = True
            pb.tracked[g] |= np.array(1 << q[g]).astype(md)
            pb.self_slot[g] = (q[g] + 1) % S
    ps = to_device(eng, pb, masks, EXTRAS + ("reads",))
    gq = np.flatnonzero(quiet)
    for rnd in range(4):
        mtype, mindex, mhint, mlogterm = random_msgs(rng, pb)
        mt = mtype.reshape(S, G)
        mt[q[gq], gq] = 0
        b = np.flatnonzero(brk)
        mt[q[b], b] = rng.choice([1, 2, 3], b.size)  # (accept / reject / heartbeat response)
        msgs = load_msgs(eng, ps, mtype, mindex, mhint, mlogterm)
        ctx = random_read_ctx(rng, pb)
        msgs.set_read_ctx(ps, ctx)
        eng.progress_step(ps, msgs, eng.stats_buffer(DEV))
        o = orc.progress_step(pb, mtype, mindex, mhint, mlogterm, read_ctx=ctx)
        assert_same(ps, pb)
        assert_outputs(msgs, o, S)
        gk = np.flatnonzero(quiet & ~brk)
        assert not msgs.msg_count.cpu().numpy().reshape(S, -1)[q[gk], gk].any()


@pytest.mark.parametrize("F", [3, 5, 8, 32])
@pytest.mark.parametrize("base", [(1 << 32) - 37, (1 << 43) - 29, 3 * (1 << 44) + 11])
def test_progress_rings_across_epochs(eng, base, F):
    """ABI 4's 32-bit ring words with every log index shifted by `base`:
    rings straddling a 2^32 boundary (wide conversions on append, on the
    whole-ring rewrite and in the memory form), and indices past the 11-bit
    epoch (every ring wide), through the step, the send and CheckQuorum,
    against the oracle's plain uint64 rings."""
    rng = np.random.default_rng(base % 1000 + F)
    G, S, R = 3001, 5, 3
    pb = random_state(rng, G, S, F, R, (), EXTRAS, max_ents=int(rng.integers(0, 4)), base=base)
    ps = to_device(eng, pb, (), EXTRAS)
    md = orc.mask_dtype(S)
    wide_seen = 0
    for rnd in range(5):
        mtype, mindex, mhint, mlogterm = random_msgs(rng, pb)
        msgs = load_msgs(eng, ps, mtype, mindex, mhint, mlogterm)
        if rnd % 2:
            msgs.bytes_requested = torch.zeros(1, dtype=torch.int64, device=DEV)
        eng.progress_step(ps, msgs)
        o = orc.progress_step(pb, mtype, mindex, mhint, mlogterm, count_bytes=True)
        assert_same(ps, pb)
        assert_outputs(msgs, o, S)
        if rnd % 2:
            assert int(msgs.bytes_requested.item()) == int(o.bytes[0])
        want = rng.integers(0, 1 << S, G).astype(md)
        sei, me = int(rnd % 2), int(rng.integers(0, 5))
        ps.max_ents = pb.max_ents = me
        sent, snap = eng.progress_send(ps, to_dev_mask(want, S), sei)
        o_sent, o_snap = orc.progress_send(pb, want, sei)
        np.testing.assert_array_equal(sent.cpu().numpy().view(md), o_sent)
        np.testing.assert_array_equal(snap.cpu().numpy().view(md), o_snap)
        assert_same(ps, pb)
        wide_seen += int(((ps.peer & 16) != 0).sum())
    assert wide_seen > 0


@pytest.mark.parametrize("R", [8, 9, 16])
def test_progress_run_table_sizes(eng, R):
    """Leader logs of up to QE_MAX_LOG_RUNS term runs: R = 8 is the largest
    for the 8-run kernel, 9 and 16 take the 16-run one."""
    rng = np.random.default_rng(500 + R)
    G, S, F = 2500, 5, 8
    pb = random_state(rng, G, S, F, R, (), EXTRAS, max_ents=int(rng.integers(0, 4)))
    ps = to_device(eng, pb, (), EXTRAS)
    for _ in range(3):
        mtype, mindex, mhint, mlogterm = random_msgs(rng, pb)
        msgs = load_msgs(eng, ps, mtype, mindex, mhint, mlogterm)
        stats = eng.stats_buffer(DEV)
        eng.progress_step(ps, msgs, stats)
        got = eng.stats_reduce(stats).cpu().numpy().view(np.uint64)
        o = orc.progress_step(pb, mtype, mindex, mhint, mlogterm)
        assert_same(ps, pb)
        assert_outputs(msgs, o, S)
        np.testing.assert_array_equal(got, o.stats)


def test_progress_long_rings_and_bcasts(eng):
    """F = 32 > the 8-entry prefetch (FreeLE continues from memory), small
    max_ents so the send loop fills rings, and every accept advancing the
    commit (bcasts to every peer from several slots)."""
    rng = np.random.default_rng(77)
    G, S, F, R = 2000, 5, 32, 4
    pb = random_state(rng, G, S, F, R, (), EXTRAS, max_ents=1)
    pb.term_start[:] = 0
    pb.set_peer(flags=1 | 8)  # Replicate, RecentActive
    pb.pending[:] = 0  # (no StateSnapshot peer: PendingSnapshot 0)
    ps = to_device(eng, pb, (), EXTRAS)
    for _ in range(4):
        n = S * G
        mtype = np.where(rng.random(n) < 0.8, 1, 3).astype(np.uint8)
        li = np.tile(pb.last_index, S)
        mindex = np.minimum(pb.match + rng.integers(0, 30, n).astype(np.uint64), li)
        z = np.zeros(n, np.uint64)
        msgs = load_msgs(eng, ps, mtype, mindex, z, z)
        eng.progress_step(ps, msgs)
        o = orc.progress_step(pb, mtype, mindex, z, z)
        assert_same(ps, pb)
        assert_outputs(msgs, o, S)
        assert int(o.bcast.sum()) > G // 2  # bcasts in most groups
        pb.last_index[:] += 40  # the leader appends
        ps.last_index.copy_(torch.from_numpy(pb.last_index.view(np.int64)).to(DEV))


def gpu_propose(be, n, payload=0, append_only=False, cc=None):
    from tests.progress_scenarios import cc_arrays
    for k, v in (("pci", 0), ("unc", 0), ("applied", 0), ("max_unc", 0)):
        if not hasattr(be, k):
            setattr(be, k, v)
    m, cnt, pos, lv, sz = cc_arrays(cc)
    pr = be.eng.Proposals(be.ps, max_cc=m, max_uncommitted=be.max_unc,
                          flags=be.eng._lib.QE_PROP_APPEND_ONLY if append_only else 0)
    pr.num_entries.fill_(n)
    pr.payload.fill_(payload)
    pr.cc_count.copy_(torch.from_numpy(cnt).to(DEV))
    pr.cc_pos.copy_(torch.from_numpy(pos.view(np.int32)).to(DEV))
    pr.cc_leave.copy_(torch.from_numpy(lv).to(DEV))
    pr.cc_size.copy_(torch.from_numpy(sz.view(np.int32)).to(DEV))
    pr.applied.fill_(be.applied)
    pr.pending_conf_index.fill_(be.pci)
    pr.uncommitted_size.fill_(be.unc)
    be.eng.propose(be.ps, pr)
    be.pci = int(pr.pending_conf_index[0])
    be.unc = int(pr.uncommitted_size[0])
    return {"result": int(pr.result[0]), "sent": int(pr.sent[0]), "snap": int(pr.snap[0]),
            "cc_refused": int(pr.cc_refused[0])}


class GpuBackend:
    """tests/progress_scenarios.py / leader_round_scenarios.py backend over
    the HIP engine (one group)."""

    def __init__(self, eng):
        self.eng = eng

    def load(self, sc, a, inc=None, tracked=None, out=None, read_cap=0):
        # stride 1: the scenario arrays are [S] (the kernels need no row alignment)
        masks = (("inc",) if inc is not None else ()) + (("out",) if out is not None else ())
        ps = self.eng.ProgressState(1, sc["S"], cap(sc), sc.get("log_runs", len(sc["log"]["runs"])),
                                    DEV, stride=1,
                                    extras=READS + ("read_keys",), max_ents=sc["max_ents"],
                                    masks=masks, read_cap=read_cap)
        if tracked is None:
            ps.tracked = None  # every slot holds a Progress (as the oracle backend)
        else:
            ps.tracked.fill_(tracked)
        if "snap_index" not in a:
            ps.snap_index = None
        ps.load_host(**a)
        if inc is not None:
            ps.inc.fill_(inc)
        if out is not None:
            ps.out.fill_(out)
        self.ps, self.sc = ps, sc
        self.pci = self.unc = self.applied = self.max_unc = 0  # MsgProp state (qe_propose)

    def step(self, t, idx, hint, lt, ctx=None):
        msgs = load_msgs(self.eng, self.ps, t, idx, hint, lt)
        msgs.set_read_ctx(self.ps, ctx)
        self.eng.progress_step(self.ps, msgs)
        st = self.ps.stride
        return {"sent": int(msgs.sent[0]), "snap": int(msgs.snap[0]),
                "timeout_now": int(msgs.timeout_now[0]),
                "msg_count": msgs.msg_count.cpu().numpy()[: self.sc["S"] * st: st],
                "msg_index": msgs.msg_index.cpu().numpy().view(np.uint64)[: self.sc["S"] * st: st],
                "bcast": int(msgs.bcast[0]), "read_released": int(msgs.read_released[0]),
                "term_commit": int(msgs.term_commit[0]),
                "term_commit_index": int(msgs.term_commit_index[0])}

    def heartbeat(self):
        """qe_heartbeat -> (commit per slot, ctx, sent mask)."""
        commit, ctx, sent = self.eng.heartbeat(self.ps)
        st = self.ps.stride
        c = commit.cpu().numpy().view(np.uint64)[: self.sc["S"] * st: st]
        return [int(x) for x in c], int(ctx[0]) & 0xFFFFFFFF, int(sent[0])

    def read_index(self, lease_based=False, key=None):
        req = torch.ones(1, dtype=torch.uint8, device=DEV)
        k = None if key is None else torch.tensor([key], dtype=torch.int64, device=DEV)
        r, c, i = self.eng.read_index(self.ps, req, lease_based, key=k)
        return int(r[0]), int(c[0]) & 0xFFFFFFFF, int(i[0])

    def queue(self):
        ps = self.ps
        n, head = int(ps.read_count[0]), int(ps.read_head[0]) & 0xFFFFFFFF
        cap = max(4, ps.read_cap)
        m = 0xFFFF if self.sc["S"] > 8 else 0xFF
        return n, head, [(int(ps.read_acks[j]) if j < 4 else int(ps.read_ovf[(head + j) % cap])) & m
                         for j in range(n)]

    def transferee(self):
        return int(self.ps.lead_transferee[0])

    def become_leader(self, term, bcast=True):
        """qe_become_leader on the one group."""
        ld = self.eng.Leader(self.ps, bcast=bcast)
        ld.term.fill_(term)
        self.eng.become_leader(self.ps, ld)
        if int(ld.result[0]) == 1:
            self.pci, self.unc = int(ld.pending_conf_index[0]), 0
        return {"result": int(ld.result[0]), "sent": int(ld.sent[0]), "snap": int(ld.snap[0])}

    def switch_config(self):
        """qe_switch_config on the one group."""
        sw = self.eng.switch_config(self.ps, self.eng.Switch(self.ps))
        return {"result": int(sw.result[0]), "sent": int(sw.sent[0]), "snap": int(sw.snap[0])}

    def send(self, want, sei):
        dt = torch.uint8 if self.sc["S"] <= 8 else torch.int16
        w = torch.tensor([want], dtype=dt, device=DEV)
        sent, snap = self.eng.progress_send(self.ps, w, sei)
        return {"sent": int(sent[0]), "snap": int(snap[0])}

    def last_index(self):
        return int(self.ps.last_index[0])

    def check_quorum(self):
        qa = self.eng.check_quorum(self.ps)
        w = self.ps.host()["peer"]
        ra = sum(1 << s for s in range(self.sc["S"]) if w[s * self.ps.stride] & 8)
        return int(qa[0]), ra

    def append(self):
        out = self.propose(1, append_only=True)
        assert out["result"] == 1, out

    def propose(self, n, payload=0, append_only=False, cc=None):
        """qe_propose on the one group (the backend holds pendingConfIndex,
        uncommittedSize and applied, as the oracle backend does)."""
        return gpu_propose(self, n, payload, append_only, cc)

    def set_outgoing(self, mask):
        """Voters[1] of the loaded JointConfig (0: a simple config again)."""
        self.ps.out.fill_(mask)

    def set_snapshot(self, index):
        """The index of the snapshot a MsgSnap sends (the applied index
        where the interaction traces take it)."""
        self.ps.snap_index.fill_(index)

    def set_config(self, tracked, inc):
        """A new configuration's tracked slots and Voters[0] (applied conf
        change; the Progress of a slot that stays keeps its state)."""
        self.ps.tracked.fill_(tracked)
        self.ps.inc.fill_(inc)

    def peer(self, s):
        h = self.ps.host()
        st = self.ps.stride
        sl = slice(0, self.sc["S"] * st, st)
        return peer_view(h["match"][sl], h["next"][sl], h["pending"][sl], h["flags"][sl],
                         h["icount"][sl], s)

    def committed(self):
        return int(self.ps.committed[0])


def test_progress_scenarios_on_gpu(eng):
    """The reference's leader-side tests (TestLeaderAppResp,
    TestSendAppendForProgress*, TestMsgAppRespWaitReset, TestProvideSnap,
    raft_snap_test.go, ...) through qe_progress_step / qe_progress_send."""
    for sc in scenarios():
        run_scenario(sc, GpuBackend(eng))


def test_readindex_and_checkquorum_scenarios_on_gpu(eng):
    """ReadIndex through qe_read_index and qe_progress_step's queue
    (TestReadOnlyOptionSafe / WithLearner / OptionLease, TestRaftFreesReadOnlyMem,
    TestReadOnlyForNewLeader, two requests in flight, the queue limit, the
    learner-ack rule), CheckQuorum (TestLeaderStepdownWhenQuorumActive /
    Lost, TestAddNodeCheckQuorum) and MsgTransferLeader (TestLeaderTransfer*)
    -- tests/leader_round_scenarios.py."""
    from tests.leader_round_scenarios import SCENARIOS
    for sc in SCENARIOS:
        sc(GpuBackend(eng))


@pytest.mark.parametrize("S,masks,extras", [(3, (), ()), (5, ("inc",), EXTRAS),
                                            (9, ("inc", "out"), EXTRAS), (16, (), EXTRAS)])
def test_check_quorum_matches_oracle(eng, S, masks, extras):
    """qe_check_quorum against the oracle on random Progress words, voter
    masks, tracked sets (voters without a Progress are missing) and leader
    slots (>= S: the leader removed itself), twice in a row (the second sees
    the reset RecentActive bits)."""
    rng = np.random.default_rng(900 + S)
    G = 5003
    pb = random_state(rng, G, S, 8, 2, masks, extras)
    ps = to_device(eng, pb, masks, extras)
    for rnd in range(2):
        st = eng.stats_buffer(DEV)
        qa = eng.check_quorum(ps, stats=st)
        got = eng.stats_reduce(st).cpu().numpy().view(np.uint64)
        o_qa, o_st = orc.check_quorum(pb)
        np.testing.assert_array_equal(qa.cpu().numpy(), o_qa)
        np.testing.assert_array_equal(got, o_st)
        assert_same(ps, pb)
        if rnd == 0 and S <= 5:  # random RecentActive bits: both outcomes occur
            assert 0 < int(o_qa.sum()) < G


def test_bytes_requested_equal_oracle_on_bench_state(eng):
    """The Progress step's roofline denominator (bench.py progress_step: the
    instrumented kernel's byte count per group) equals the oracle's
    independent count on the bench workload's own state and messages
    (bench.progress_round_state), here at 64K groups."""
    import bench
    bench.engine = eng
    G, S, F, R = 1 << 16, 5, 8, 4
    ps = eng.ProgressState(G, S, F, R, DEV, extras=("self_slot",), max_ents=16)
    msgs = eng.PeerMsgs(ps)
    msgs.snap = msgs.timeout_now = None
    bench.progress_round_state(ps, msgs)
    h = ps.host()
    pb = orc.ProgressBatch(G, S, F, R, stride=ps.stride, max_ents=16)
    for k in ("match", "next", "pending", "ibuf", "committed", "term_start", "first_index",
              "last_index", "run_first", "run_term", "run_count", "self_slot"):
        setattr(pb, k, h[k].copy())
    pb.pw = h["peer"] & ~RING_MASK
    mtype = msgs.type.cpu().numpy()
    mix = [msgs.index, msgs.reject_hint, msgs.log_term]
    mindex, mhint, mlogterm = (t.cpu().numpy().view(np.uint64) for t in mix)
    b = eng.progress_bytes_requested(ps, msgs)
    o = orc.StepOut(pb)
    m = orc.OrcMsgs(type=orc.P(mtype), index=orc.P(mindex), hint=orc.P(mhint),
                    logterm=orc.P(mlogterm), sent=orc.P(o.sent), bcast=orc.P(o.bcast),
                    msg_count=orc.P(o.msg_count), msg_index=orc.P(o.msg_index),
                    read_released=orc.P(o.read_released), term_commit=orc.P(o.term_commit),
                    term_commit_index=orc.P(o.term_commit_index), bytes=orc.P(o.bytes))
    import ctypes as C
    orc.lib().orc_progress_step_batch(C.byref(pb.struct()), C.byref(m), orc.P(o.stats), 0)
    assert_same(ps, pb)
    assert b == int(o.bytes[0]), (b / G, int(o.bytes[0]) / G)
    assert 300 * G < b < 700 * G  # the ~0.5 KB per group-round DESIGN.md quotes


def test_fast_log_rejection_on_gpu(eng):
    """TestFastLogRejection leader side: heartbeat response -> probe MsgApp
    (sent inside the step) -> rejection -> the next MsgApp's (Index,
    LogTerm)."""
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
        msgs.type.fill_(3)  # MsgHeartbeatResp -> sendAppend (probe)
        eng.progress_step(ps, msgs)
        assert int(msgs.sent[0]) == 1 and int(msgs.msg_index[0]) == l_last
        msgs = eng.PeerMsgs(ps)
        msgs.type.fill_(2)  # MsgAppResp reject of the probe at Index = l_last
        msgs.index.fill_(l_last)
        msgs.reject_hint.fill_(r["reject_hint_index"])
        msgs.log_term.fill_(r["reject_hint_term"])
        eng.progress_step(ps, msgs)
        assert int(msgs.msg_count[0]) == 1
        idx = int(msgs.msg_index[0])
        assert idx == int(ps.next[0]) - 1
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
        # the sendAppend after a decrease moves Next again only in Replicate
        # (BecomeProbe first), so check MaybeDecrTo's result through the
        # message it triggered: Index = Next - 1 after the decrease
        assert int(h["match"][i]) == r["match"], r
        sent = bool(int(msgs.sent[i]) & 1)
        assert sent == r["want"], r
        if r["want"] and r["state"] != 1:
            assert int(msgs.msg_index[i]) + 1 == r["want_next"], r


def test_send_if_empty_precedes_snapshot_on_gpu(eng):
    """raft.go:440-469: maybeSendAppend(to, false) with Next < firstIndex
    returns false before the snapshot branch (round-1 kernels sent a MsgSnap
    here)."""
    G = 64
    ps = eng.ProgressState(G, 1, 8, 1, DEV)
    ps.first_index.fill_(10)
    ps.last_index.fill_(20)
    ps.next.fill_(5)
    ps.match.fill_(4)
    ps.peer.fill_(8)  # Probe, RecentActive
    want = torch.ones(G, dtype=torch.uint8, device=DEV)
    sent, snap = eng.progress_send(ps, want, False)
    assert int(sent.sum()) == 0 and int(snap.sum()) == 0
    assert int((ps.peer[:G] & 3).sum()) == 0 and int(ps.pending[:G].sum()) == 0
    sent, snap = eng.progress_send(ps, want, True)
    assert int(sent.sum()) == G and int(snap.sum()) == G
    assert bool(((ps.peer[:G] & 3) == 2).all()) and bool((ps.pending[:G] == 9).all())


def test_bytes_requested_accounting(eng):
    """The instrumented variant gives the same results, and its byte count
    equals the oracle's exactly (no outputs requested: only the state)."""
    rng = np.random.default_rng(5)
    G, S, F, R = 4096, 5, 8, 4
    pb = random_state(rng, G, S, F, R, ())
    ps = to_device(eng, pb, ())
    mtype, mindex, mhint, mlogterm = random_msgs(rng, pb)
    msgs = load_msgs(eng, ps, mtype, mindex, mhint, mlogterm)
    for k in ("sent", "bcast", "snap", "timeout_now", "msg_count", "msg_index", "read_released",
              "term_commit", "term_commit_index"):
        setattr(msgs, k, None)
    b = eng.progress_bytes_requested(ps, msgs)
    o = orc.progress_step(pb, mtype, mindex, mhint, mlogterm, outputs=False, count_bytes=True)
    assert_same(ps, pb)
    assert b == int(o.bytes[0])
