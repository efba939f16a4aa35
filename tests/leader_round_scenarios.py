"""Leader-side transcriptions of the reference tests that pin the stepLeader
decisions fused onto the resident Progress state: ReadIndex as readOnly
keeps it (MsgReadIndex raft/raft.go:1078-1096, the queue of
raft/read_only.go:39-112, the heartbeat acks :1296-1309, the postponed
reads of a new leader :1259-1262 / :1813-1825), MsgCheckQuorum
(raft/raft.go:997-1018) and MsgTransferLeader (raft/raft.go:1339-1370).

Each reference test drives a small in-process cluster; the leader's view of
it is restated here as rounds of the batch engine on one group (slot s is
node id s+1, slot 0 is the leader), through the backend interface of
tests/progress_scenarios.py plus
  step(t, idx, hint, lt, ctx=None) -> out with "read_released",
      "term_commit", "term_commit_index", "timeout_now"
  read_index(lease_based=False) -> (QE_RI_* result, context number, index)
  queue() -> (pending count, head context number, acks of each entry)
  transferee() -> lead_transferee slot (0xFF none)
  check_quorum() -> (quorum_active, RecentActive bits of the slots).
The same functions drive the oracle (CPU tests) and the HIP engine (GPU
tests).  Expectations are what each reference test asserts; the rest of
its message flow (proposals, appends, acks) is executed, not assumed."""
import numpy as np

from tests.progress_scenarios import (F_CAP, PF_RECENT_ACTIVE, bits, initial_arrays,
                                      oracle_propose, peer_view)

REPLICATE = 1


def _peer(match, nxt, state, recent_active=False, probe_sent=False):
    return {"match": match, "next": nxt, "pending": 0, "state": state,
            "probe_sent": probe_sent, "recent_active": recent_active, "ring": []}


def _leader_after_hup(S):
    """A freshly elected leader (term 1) whose empty entry (index 1) every
    peer has acked: the state nt.send(MsgHup) leaves in the 3-node network
    of TestReadOnlyOptionSafe (raft_test.go:2186-2189) -- becomeLeader
    appends the empty entry, the followers' MsgAppResp move them to
    StateReplicate and commit index 1."""
    return {
        "name": "", "S": S, "self": 0, "max_ents": 0,
        "log": {"runs": [[0, 0], [1, 1]], "committed": 1, "term_start": 1, "first_index": 1,
                "last_index": 1},
        "peers": [_peer(1, 2, REPLICATE, True)] + [_peer(1, 2, REPLICATE, True)
                                                    for _ in range(S - 1)],
    }


def _propose(be, S, voters_acking):
    """One MsgProp (raft.go:1019-1076) through qe_propose: appendEntry
    (lastIndex + 1, the leader's own MaybeUpdate, maybeCommit) + bcastAppend
    to every follower, then the followers' MsgAppResp for the new entry --
    the network of the reference test delivers them synchronously."""
    out = be.propose(1)
    assert out["result"] == 1, out
    li = be.last_index()
    t = np.zeros(S, np.uint8)
    idx = np.zeros(S, np.uint64)
    for s in voters_acking:
        t[s], idx[s] = 1, li
    z = np.zeros(S, np.uint64)
    be.step(t, idx, z, z)


def _heartbeat_round(be, S, slots, ctx=None):
    """MsgHeartbeatResp from `slots`; ctx: None (each carries the newest
    pending context, as the heartbeats of bcastHeartbeat do), an int (every
    one carries that context number, 0 = none) or a per-slot dict."""
    t = np.zeros(S, np.uint8)
    for s in slots:
        t[s] = 3  # MsgHeartbeatResp
    z = np.zeros(S, np.uint64)
    c = None
    if ctx is not None:
        c = np.zeros(S, np.uint32)
        for s in slots:
            c[s] = ctx[s] if isinstance(ctx, dict) else ctx
    return be.step(t, z, z, z, ctx=c)


QUEUED, RESPOND, POSTPONED, FULL, DUPLICATE = 3, 1, 2, 4, 5


def read_only_option_safe(be):
    """TestReadOnlyOptionSafe (raft/raft_test.go:2177-2229), leader a's side:
    six rounds of 10 proposals, then a ReadIndex under ReadOnlySafe.  The
    leader adds the request at committed and acks it itself
    (sendMsgReadIndexResponse, raft.go:1827-1837); the heartbeat responses of
    b then c arrive; b's makes the acks a quorum of {1,2,3}, so the request
    is released with Index = committed (wri 11, 21, ..., 61); c's response
    finds it gone (recvAck returns nil) and records nothing."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    wri = [11, 21, 31, 41, 51, 61]
    for want in wri:
        for _ in range(10):
            _propose(be, S, (1, 2))
        res, ctx, index = be.read_index()
        assert (res, index) == (QUEUED, want), (res, index, want)
        assert be.queue()[0] == 1
        out = _heartbeat_round(be, S, (1, 2))
        assert out["read_released"] == 1, want
        assert be.queue()[0] == 0


def read_only_with_learner(be):
    """TestReadOnlyWithLearner (raft/raft_test.go:2231-2278): voters {1},
    learner {2}.  Ten proposals per round commit on the leader alone (the
    learner's MsgAppResp advances its Match, not the quorum); the leader is
    the only voting member, so r.prs.IsSingleton() answers the read at once
    at committed = 11, 21, 31, 41 (raft.go:1079-1085), without a heartbeat
    round."""
    S = 2
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc), inc=0b01)
    wri = [11, 21, 31, 41]
    for want in wri:
        for _ in range(10):
            _propose(be, S, (1,))
        assert be.committed() == want  # committed by the leader's own Match
        res, _, index = be.read_index()
        assert (res, index) == (RESPOND, want)
        assert be.queue()[0] == 0


def read_only_option_lease(be):
    """TestReadOnlyOptionLease (raft/raft_test.go:2282-2337), leader a's
    side: ReadOnlyLeaseBased answers at once at committed (11, ..., 61)."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    for want in [11, 21, 31, 41, 51, 61]:
        for _ in range(10):
            _propose(be, S, (1, 2))
        res, _, index = be.read_index(lease_based=True)
        assert (res, index) == (RESPOND, want)
        assert be.queue()[0] == 0


def raft_frees_read_only_mem(be):
    """TestRaftFreesReadOnlyMem (raft/raft_test.go:1359-1403): peers {1,2},
    the leader committed to its lastIndex; MsgReadIndex from 2 queues one
    request (readIndexQueue and pendingReadIndex of length 1); the
    heartbeat response from 2 carrying its context releases it and both
    are empty again."""
    S = 2
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    res, ctx, index = be.read_index()
    assert (res, index) == (QUEUED, 1)
    n, head, acks = be.queue()
    assert (n, head) == (1, ctx) and acks == [0b01]  # the leader's own ack
    out = _heartbeat_round(be, S, (1,), ctx=ctx)
    assert out["read_released"] == 1
    assert be.queue()[0] == 0


def read_only_for_new_leader(be):
    """TestReadOnlyForNewLeader (raft/raft_test.go:2341-2410), the leader's
    side.  Node 1 (log [1@1, 2@1], committed 1) wins term 2 and appends its
    empty entry 3@2; MsgApp is dropped, so nothing of term 2 commits and
    the ReadIndex is postponed (raft.go:1087-1092).  After recover: the
    heartbeat responses make the leader probe (sendAppend), a MsgProp
    appends 4@2 (the peers are paused: nothing sent), the followers' accept
    of [3, 4] commits 4 -- the first commit in the term -- and
    releasePendingReadIndexMessages answers the postponed read at index 4
    (windex): it is added to the queue at 4, and the heartbeat responses
    carrying its context release it.  A second ReadIndex is queued at once."""
    S = 3
    sc = {"name": "", "S": S, "self": 0, "max_ents": 0,
          "log": {"runs": [[0, 0], [1, 1], [3, 2]], "committed": 1, "term_start": 3,
                  "first_index": 1, "last_index": 3},
          # becomeLeader: reset() gives every Progress Match 0, Next =
          # lastIndex + 1 = 3 before the empty entry; the leader's own
          # Progress follows its appends (Replicate); bcastAppend's probes
          # went out (ProbeSent) and were dropped
          "peers": [_peer(3, 4, REPLICATE)] + [_peer(0, 3, 0, probe_sent=True)
                                              for _ in range(S - 1)]}
    be.load(sc, initial_arrays(sc))
    res, _, _ = be.read_index()
    assert res == POSTPONED
    # recover; heartbeat responses (no read pending: no context) -> probes
    out = _heartbeat_round(be, S, (1, 2))
    assert bits(out["sent"]) == [1, 2] and out["term_commit"] == 0
    out = be.propose(1)  # MsgProp: 4@2; the followers are paused again
    assert out["result"] == 1 and out["sent"] == 0
    # the followers append [3, 4] and accept; slot 1's accept commits 4
    t = np.array([0, 1, 1], np.uint8)
    idx = np.array([0, 4, 4], np.uint64)
    z = np.zeros(S, np.uint64)
    out = be.step(t, idx, z, z)
    assert be.committed() == 4
    assert out["term_commit"] == 1 and out["term_commit_index"] == 4
    # the postponed read: sendMsgReadIndexResponse -> addRequest(4)
    res, ctx, index = be.read_index()
    assert res == QUEUED and index == 4
    out = _heartbeat_round(be, S, (1, 2), ctx=ctx)
    assert out["read_released"] == 1 and out["term_commit"] == 0
    # a new ReadIndex is accepted at once
    res, ctx2, index = be.read_index()
    assert res == QUEUED and index == 4 and ctx2 == ctx + 1
    out = _heartbeat_round(be, S, (1, 2), ctx=ctx2)
    assert out["read_released"] == 1


def postponed_read_commit_advances_twice(be):
    """A postponed ReadIndex released in a round whose commit advances twice
    (derived from raft.go:1259-1262 and :1813-1825; no reference test has
    this round).  Entries 3..5 of the new term are in flight; slot 1's accept
    of 4 commits 4 -- the term's first commit, so maybeCommit's caller runs
    releasePendingReadIndexMessages there and addRequest takes committed = 4
    -- then slot 2's accept of 5 commits 5 in the same round.  The step
    reports term_commit_index 4 (the host re-adds the postponed read at it),
    while the committed index the round ends with, and the one a later
    MsgReadIndex is answered at, is 5."""
    S = 3
    sc = {"name": "", "S": S, "self": 0, "max_ents": 0,
          "log": {"runs": [[0, 0], [1, 1], [3, 2]], "committed": 1, "term_start": 3,
                  "first_index": 1, "last_index": 5},
          "peers": [_peer(5, 6, REPLICATE)] + [_peer(2, 6, REPLICATE, True)
                                              for _ in range(S - 1)]}
    be.load(sc, initial_arrays(sc))
    res, _, _ = be.read_index()
    assert res == POSTPONED
    t = np.array([0, 1, 1], np.uint8)
    idx = np.array([0, 4, 5], np.uint64)
    z = np.zeros(S, np.uint64)
    out = be.step(t, idx, z, z)
    assert out["term_commit"] == 1 and out["term_commit_index"] == 4, out
    assert be.committed() == 5
    # the re-added read: queued at the term_commit_index the host passes
    # on; qe_read_index itself reports the committed index of now (5)
    res, ctx, index = be.read_index()
    assert res == QUEUED and index == 5
    out = _heartbeat_round(be, S, (1, 2), ctx=ctx)
    assert out["read_released"] == 1 and out["term_commit"] == 0


def two_reads_in_flight(be):
    """Two pending requests (derived from readOnly.advance, read_only.go:
    81-112): a response carrying the older context releases only the older
    one; a later response carrying a released context records nothing
    (recvAck returns nil); a response carrying the newer context releases
    the newer one.  Then two more: a quorum on the newer one releases both
    at once (advance dequeues everything up to it)."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    _, a, _ = be.read_index()
    _, b, _ = be.read_index()
    assert b == a + 1 and be.queue()[0] == 2
    out = _heartbeat_round(be, S, (1,), ctx=a)  # acks(a) = {1, 2}: a quorum
    assert out["read_released"] == 1
    n, head, acks = be.queue()
    assert (n, head, acks) == (1, b, [0b001])
    out = _heartbeat_round(be, S, (2,), ctx=a)  # a is gone: nothing recorded
    assert out["read_released"] == 0 and be.queue() == (1, b, [0b001])
    out = _heartbeat_round(be, S, (2,), ctx=b)
    assert out["read_released"] == 1 and be.queue()[0] == 0
    _, c, _ = be.read_index()
    _, d, _ = be.read_index()
    out = _heartbeat_round(be, S, (1,), ctx=c)  # one round: 1 acks c ...
    assert out["read_released"] == 1
    _, e, _ = be.read_index()
    assert be.queue()[0] == 2  # d, e
    # slot 1 carries e, slot 2 carries d; slots go in order, so slot 1's ack
    # makes e's acks {1, 2} a quorum and advance releases d and e together;
    # slot 2's response then finds d gone
    out = _heartbeat_round(be, S, (1, 2), ctx={1: e, 2: d})
    assert out["read_released"] == 2 and be.queue()[0] == 0


def read_queue_deep_and_duplicates(be):
    """ABI 7: a queue longer than the word (readIndexQueue is unbounded in
    the reference, read_only.go:56-63; here a capacity of 8) and
    addRequest's duplicate drop (:57-60) by request key.  Eight requests
    queue (four in the word, four in the overflow ring); a ninth is over the
    capacity; a resent request (its key pending) is a duplicate naming the
    pending context, nothing queued.  A heartbeat response for the seventh
    request -- an overflow entry -- makes its acks a quorum: advance
    releases the seven oldest at once and the eighth moves into the word; a
    response for a released context records nothing; MsgBeat carries the
    newest context; the next response releases the last one."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc), read_cap=8)
    got = [be.read_index(key=100 + k) for k in range(8)]
    assert [r for r, _, _ in got] == [QUEUED] * 8
    ctxs = [c for _, c, _ in got]
    assert ctxs == list(range(ctxs[0], ctxs[0] + 8))
    assert be.read_index(key=200)[0] == FULL
    res, ctx, _ = be.read_index(key=103)  # resent: pending already
    assert (res, ctx) == (DUPLICATE, ctxs[3]) and be.queue()[0] == 8
    n, head, acks = be.queue()
    assert (n, head) == (8, ctxs[0]) and acks == [0b001] * 8  # the leader's own acks
    out = _heartbeat_round(be, S, (1,), ctx=ctxs[6])
    assert out["read_released"] == 7
    assert be.queue() == (1, ctxs[7], [0b001])
    out = _heartbeat_round(be, S, (2,), ctx=ctxs[5])  # released: nothing recorded
    assert out["read_released"] == 0 and be.queue() == (1, ctxs[7], [0b001])
    _, hctx, _ = be.heartbeat()
    assert hctx == ctxs[7]
    res, ctx, _ = be.read_index(key=103)  # released: a fresh request now
    assert (res, ctx) == (QUEUED, ctxs[7] + 1)
    out = _heartbeat_round(be, S, (2,), ctx=ctxs[7] + 1)
    assert out["read_released"] == 2 and be.queue()[0] == 0


def read_queue_full(be):
    """The engine keeps QE_READ_QUEUE = 4 pending requests per group; a fifth
    is refused (QE_RI_FULL, nothing changes) until a release makes room.
    The reference's queue is unbounded (read_only.go:56-63): this is the
    engine's limit, reported, never silent."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    ctxs = [be.read_index()[1] for _ in range(4)]
    assert ctxs == list(range(ctxs[0], ctxs[0] + 4))
    res, _, _ = be.read_index()
    assert res == FULL and be.queue()[0] == 4
    out = _heartbeat_round(be, S, (2,))  # the newest context: releases all 4
    assert out["read_released"] == 4
    assert be.read_index()[0] == QUEUED


def learner_ack_does_not_count(be):
    """Derived from TestReadOnlyWithLearner's rule that learners never count
    (VoteResult ranges over Voters only, raft.go:1300): voters {1,2},
    learner {3}; the learner's ack alone leaves the request pending, a
    response without a context (len(m.Context) == 0) is not an ack, the
    voter's ack releases it."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc), inc=0b011)
    res, ctx, _ = be.read_index()
    assert res == QUEUED
    out = _heartbeat_round(be, S, (2,), ctx=ctx)
    assert out["read_released"] == 0 and be.queue()[2] == [0b101]
    out = _heartbeat_round(be, S, (1,), ctx=0)  # no context
    assert out["read_released"] == 0 and be.queue()[2] == [0b101]
    out = _heartbeat_round(be, S, (1,), ctx=ctx)
    assert out["read_released"] == 1


def _transfer(be, S, slot):
    t = np.zeros(S, np.uint8)
    t[slot] = 7  # MsgTransferLeader from node slot+1
    z = np.zeros(S, np.uint64)
    return be.step(t, z, z, z)


def leader_transfer_to_up_to_date_node(be):
    """TestLeaderTransferToUpToDateNode (raft/raft_test.go:3435-3456), the
    leader's side: node 2 is caught up (Match == lastIndex), so the leader
    records it as leadTransferee and sends MsgTimeoutNow at once
    (raft.go:1363-1366), no MsgApp."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    out = _transfer(be, S, 1)
    assert bits(out["timeout_now"]) == [1] and out["sent"] == 0
    assert be.transferee() == 1


def leader_transfer_to_slow_follower(be):
    """TestLeaderTransferToSlowFollower (raft/raft_test.go:3523-3541), the
    leader's side: node 3 was isolated during a proposal (Match 1, its
    MsgApp for entry 2 lost: Replicate, Next 3, one inflight); the transfer
    to 3 sends an append instead (raft.go:1367-1369); node 3 rejects it,
    the leader probes from its Match, node 3's accept of 2 brings its Match
    to lastIndex and the leader sends MsgTimeoutNow (raft.go:1278-1281)."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    _propose(be, S, (1,))  # node 3 isolated: its MsgApp is lost
    z = np.zeros(S, np.uint64)
    out = _transfer(be, S, 2)
    assert be.transferee() == 2
    assert out["timeout_now"] == 0 and bits(out["sent"]) == [2]
    t = np.array([0, 0, 2], np.uint8)  # reject of Index 2, hint 1
    out = be.step(t, np.array([0, 0, 2], np.uint64), np.array([0, 0, 1], np.uint64), z)
    assert bits(out["sent"]) == [2] and out["timeout_now"] == 0
    out = be.step(np.array([0, 0, 1], np.uint8), np.array([0, 0, 2], np.uint64), z, z)
    assert bits(out["timeout_now"]) == [2]


def leader_transfer_after_snapshot(be):
    """TestLeaderTransferAfterSnapshot (raft/raft_test.go:3543-3587), the
    leader's side.  Node 1 leads term 1 of {1, 2, 3}; node 3 was isolated
    while entry 2 was proposed (its MsgApp lost: StateReplicate, Match 1,
    Next 3, one entry in flight); entry 2 committed with node 2; the leader's
    log compacted to the snapshot at 2 (firstIndex 3).  The transfer to 3
    finds it behind: sendAppend sends an empty MsgApp at Index 2; node 3
    rejects it (hint 1, LogTerm 1: findConflictByTerm over the compacted
    prefix gives 1); MaybeDecrTo(2, 1) moves Next to Match + 1 = 2 and
    BecomeProbe; the retry finds 2 compacted and sends the snapshot at 2
    (BecomeSnapshot) -- the leader is still the leader, the transfer
    pending.  Node 3's MsgAppResp after applying the snapshot (Index 2)
    ends StateSnapshot (Match >= PendingSnapshot: BecomeProbe +
    BecomeReplicate) and, its Match now lastIndex, the leader sends
    MsgTimeoutNow (raft.go:1275-1281)."""
    S = 3
    sc = {"name": "", "S": S, "self": 0, "max_ents": 0,
          "log": {"runs": [[2, 1]], "committed": 2, "term_start": 1, "first_index": 3,
                  "last_index": 2, "snap_index": 2},
          "peers": [_peer(2, 3, REPLICATE), _peer(2, 3, REPLICATE, True),
                    dict(_peer(1, 3, REPLICATE), ring=[2])]}
    be.load(sc, initial_arrays(sc), inc=0b111, tracked=0b111)
    out = _transfer(be, S, 2)
    assert be.transferee() == 2 and out["timeout_now"] == 0
    assert bits(out["sent"]) == [2] and int(out["msg_index"][2]) == 2 and out["snap"] == 0
    z = np.zeros(S, np.uint64)
    out = be.step(np.array([0, 0, 2], np.uint8), np.array([0, 0, 2], np.uint64),
                  np.array([0, 0, 1], np.uint64), np.array([0, 0, 1], np.uint64))
    assert bits(out["snap"]) == [2] and out["timeout_now"] == 0, out
    p = be.peer(2)
    assert (p["state"], p["pending"], p["match"]) == (2, 2, 1), p  # StateSnapshot(2)
    out = be.step(np.array([0, 0, 1], np.uint8), np.array([0, 0, 2], np.uint64), z, z)
    assert bits(out["timeout_now"]) == [2], out
    p = be.peer(2)
    assert (p["state"], p["match"], p["next"]) == (REPLICATE, 2, 3), p
    assert be.transferee() == 2


def leader_transfer_with_check_quorum(be):
    """TestLeaderTransferWithCheckQuorum (raft/raft_test.go:3488-3521), the
    side of the leader the transfers go to.  Node 2 has won term 2 after the
    first transfer (becomeLeader: reset() -- every Progress at Match 0, Next
    lastIndex + 1 = 2, the leader's own at Match 1 -- then its empty entry 2
    and the bcastAppend probes); nodes 1 and 3 accept 2.  The MsgProp of the
    test appends 3, which both followers accept: node 1 is up to date, so its
    MsgTransferLeader makes node 2 send MsgTimeoutNow at once -- CheckQuorum
    (the leader lease) does not hold the transfer back on the leader's side,
    and a MsgCheckQuorum in between keeps node 2 the leader (both followers
    active).  Node 1 is slot 0, node 2 slot 1."""
    S = 3
    sc = {"name": "", "S": S, "self": 1, "max_ents": 0,
          "log": {"runs": [[0, 0], [1, 1], [2, 2]], "committed": 1, "term_start": 2,
                  "first_index": 1, "last_index": 1},
          "peers": [_peer(0, 2, 0), _peer(1, 2, REPLICATE), _peer(0, 2, 0)]}
    be.load(sc, initial_arrays(sc), inc=0b111, tracked=0b111)
    out = be.propose(1, append_only=True)  # becomeLeader's empty entry at 2
    assert out["result"] == 1 and be.last_index() == 2
    out = be.send(0b101, 1)  # stepCandidate's bcastAppend: probes
    assert bits(out["sent"]) == [0, 2]
    z = np.zeros(S, np.uint64)
    be.step(np.array([1, 0, 1], np.uint8), np.array([2, 0, 2], np.uint64), z, z)
    assert be.committed() == 2  # the term's first entry commits
    out = be.propose(1)  # the test's MsgProp: entry 3, bcast to both
    assert out["result"] == 1 and bits(out["sent"]) == [0, 2]
    be.step(np.array([1, 0, 1], np.uint8), np.array([3, 0, 3], np.uint64), z, z)
    assert be.committed() == 3
    qa, _ = be.check_quorum()  # the lease: both followers were heard from
    assert qa == 1
    out = _transfer(be, S, 0)  # MsgTransferLeader from node 1
    assert bits(out["timeout_now"]) == [0] and out["sent"] == 0 and be.transferee() == 0


def leader_transfer_to_self(be):
    """TestLeaderTransferToSelf (raft/raft_test.go:3589-3598): a transfer to
    the leader itself is a no-op (raft.go:1355-1358)."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    out = _transfer(be, S, 0)
    assert out["timeout_now"] == 0 and out["sent"] == 0 and be.transferee() == 0xFF


def leader_transfer_to_non_existing_node(be):
    """TestLeaderTransferToNonExistingNode (raft/raft_test.go:3600-3608): a
    request from a node without a Progress is dropped (raft.go:1100-1104);
    slot 3 holds no Progress here."""
    S = 4
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc), tracked=0b0111, inc=0b0111)
    out = _transfer(be, S, 3)
    assert out["timeout_now"] == 0 and out["sent"] == 0 and be.transferee() == 0xFF


def leader_transfer_second_to_another_node(be):
    """TestLeaderTransferSecondTransferToAnotherNode (raft/raft_test.go:
    3754-3771): node 3 isolated (but caught up: MsgTimeoutNow is sent and
    lost), then a transfer to 2 aborts it (raft.go:1346-1353) and goes to 2."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    out = _transfer(be, S, 2)
    assert bits(out["timeout_now"]) == [2] and be.transferee() == 2
    out = _transfer(be, S, 1)
    assert bits(out["timeout_now"]) == [1] and be.transferee() == 1


def leader_transfer_second_to_same_node(be):
    """TestLeaderTransferSecondTransferToSameNode (raft/raft_test.go:
    3775-3799): a second request for the transfer in progress is ignored
    (raft.go:1347-1350): no MsgTimeoutNow, no MsgApp, leadTransferee kept."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    _transfer(be, S, 2)
    out = _transfer(be, S, 2)
    assert out["timeout_now"] == 0 and out["sent"] == 0 and be.transferee() == 2


def leader_transfer_back(be):
    """TestLeaderTransferBack (raft/raft_test.go:3733-3750): with a transfer
    to 3 pending, a transfer to the leader itself aborts it
    (abortLeaderTransfer, raft.go:1352) and is then ignored: no transfer is
    left in progress."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    _transfer(be, S, 2)
    out = _transfer(be, S, 0)
    assert be.transferee() == 0xFF and out["timeout_now"] == 0 and out["sent"] == 0


def leader_transfer_learner_ignored(be):
    """Derived from raft.go:1340-1343: a learner's MsgTransferLeader is
    ignored (voters {1,2}, learner {3})."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc), inc=0b011)
    out = _transfer(be, S, 2)
    assert out["timeout_now"] == 0 and out["sent"] == 0 and be.transferee() == 0xFF


def _stepdown_run(be, heartbeats):
    """newTestRaft(1, 5, 1, peers 1,2,3), checkQuorum, becomeCandidate +
    becomeLeader: term 1, the empty entry at index 1; reset() left every
    Progress at Match 0, Next 1, RecentActive false (raft.go:703-716), the
    leader's own one in StateReplicate at Match 1.  Then electionTimeout + 1
    = 6 times: (MsgHeartbeatResp from 2), tick() -- tickHeartbeat steps
    MsgCheckQuorum when electionElapsed reaches electionTimeout = 5
    (raft.go:657-667)."""
    S = 3
    sc = {"name": "", "S": S, "self": 0, "max_ents": 0,
          "log": {"runs": [[0, 0], [1, 1]], "committed": 0, "term_start": 1, "first_index": 1,
                  "last_index": 1},
          "peers": [_peer(1, 2, REPLICATE)] + [_peer(0, 1, 0) for _ in range(S - 1)]}
    be.load(sc, initial_arrays(sc))
    leader, elapsed, checks = True, 0, 0
    for _ in range(5 + 1):
        if heartbeats:
            t = np.array([0, 3, 0], np.uint8)
            z = np.zeros(S, np.uint64)
            be.step(t, z, z, z)
        elapsed += 1
        if leader and elapsed >= 5:
            elapsed = 0
            qa, ra = be.check_quorum()
            checks += 1
            # the leader marks itself active and resets every other peer
            assert ra & 1 and not ra & 0b110, ra
            if not qa:
                leader = False  # becomeFollower
    assert checks == 1
    return leader


def leader_stepdown_when_quorum_active(be):
    """TestLeaderStepdownWhenQuorumActive (raft/raft_test.go:1748-1764)."""
    assert _stepdown_run(be, heartbeats=True) is True


def leader_stepdown_when_quorum_lost(be):
    """TestLeaderStepdownWhenQuorumLost (raft/raft_test.go:1766-1781)."""
    assert _stepdown_run(be, heartbeats=False) is False


def add_node_check_quorum(be):
    """TestAddNodeCheckQuorum (raft/raft_test.go:3221-3251), from the conf
    change on: a single-voter leader (checkQuorum, electionTimeout 10) adds
    node 2 one tick before its quorum check.  initProgress gives the new
    Progress RecentActive = true (confchange.go:240-262), so the check at
    the next tick keeps the leader (and resets node 2's RecentActive); with
    no word from node 2 the check electionTimeout ticks later steps it
    down."""
    S = 2
    sc = {"name": "", "S": S, "self": 0, "max_ents": 0,
          "log": {"runs": [[0, 0], [1, 1]], "committed": 1, "term_start": 1, "first_index": 1,
                  "last_index": 1},
          "peers": [_peer(1, 2, REPLICATE), _peer(0, 1, 0, recent_active=True)]}
    be.load(sc, initial_arrays(sc))
    qa, ra = be.check_quorum()
    assert qa == 1 and ra == 0b01, (qa, ra)  # still the leader
    qa, ra = be.check_quorum()
    assert qa == 0, (qa, ra)  # steps down


SW_REMOVED, SW_BCAST, SW_PROBE, SW_ABORTED = 1, 3, 4, 0x10  # QE_SW_*


def commit_after_remove_node(be):
    """TestCommitAfterRemoveNode (raft/raft_test.go:3370-3431): peers {1, 2},
    node 1 made leader by becomeCandidate + becomeLeader (term 1; reset()
    leaves node 2 at Match 0, Next 1, StateProbe; the leader's empty entry
    at 1, no bcast).  A proposal of ConfChange{RemoveNode 2} appends 2 (its
    bcastAppend probes node 2), a normal entry "hello" appends 3 (node 2 is
    paused: nothing sent); nothing is committed.  Node 2's MsgAppResp for 2
    commits 1 and 2 (the empty entry and the conf change).  Applying the
    conf change (Voters {1}, node 2's Progress removed) and switchToConfig:
    maybeCommit under the new quorum commits 3 -- "This reduces quorum
    requirements so the pending command can now commit" -- and bcastAppend
    has nobody to send to."""
    S = 2
    sc = {"name": "", "S": S, "self": 0, "max_ents": 0,
          "log": {"runs": [[0, 0], [1, 1]], "committed": 0, "term_start": 1, "first_index": 1,
                  "last_index": 1},
          "peers": [_peer(1, 2, REPLICATE), _peer(0, 1, 0)]}
    be.load(sc, initial_arrays(sc), inc=0b11, tracked=0b11)
    be.pci, be.applied = 0, 0  # becomeLeader: pendingConfIndex = lastIndex before the empty entry
    out = be.propose(1, cc=[(0, False, 16)])  # EntryConfChange (RemoveNode 2) at 2
    assert out["result"] == 1 and out["cc_refused"] == 0 and bits(out["sent"]) == [1], out
    assert be.committed() == 0
    cc_index = be.last_index()
    assert cc_index == 2
    out = be.propose(1, payload=5)  # "hello" at 3; node 2 is paused (ProbeSent)
    assert out["result"] == 1 and out["sent"] == 0, out
    z = np.zeros(S, np.uint64)
    be.step(np.array([0, 1], np.uint8), np.array([0, cc_index], np.uint64), z, z)
    assert be.committed() == 2  # ents: the empty entry and the conf change
    be.set_config(tracked=0b01, inc=0b01)  # applyConfChange: Voters {1}
    out = be.switch_config()
    assert out["result"] == SW_BCAST and out["sent"] == 0, out
    assert be.committed() == 3  # "hello" commits under the new quorum


def leader_transfer_remove_node(be):
    """TestLeaderTransferRemoveNode (raft/raft_test.go:3681-3698): node 3 is
    caught up, so the transfer sends MsgTimeoutNow (ignored by the network)
    and leadTransferee = 3; then applyConfChange(RemoveNode 3):
    switchToConfig finds no commit to make (the probe of every peer sends
    nothing: all caught up) and aborts the transfer, since 3 is no voter
    (raft.go:1694-1697) -- checkLeaderTransferState(lead, StateLeader, 1)."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc), inc=0b111, tracked=0b111)
    out = _transfer(be, S, 2)
    assert bits(out["timeout_now"]) == [2] and be.transferee() == 2
    be.set_config(tracked=0b011, inc=0b011)
    out = be.switch_config()
    assert out["result"] == SW_PROBE | SW_ABORTED and out["sent"] == 0, out
    assert be.transferee() == 0xFF and be.committed() == 1


def leader_transfer_demote_node(be):
    """TestLeaderTransferDemoteNode (raft/raft_test.go:3700-3730): the
    transfer to 3 pending, ConfChangeV2{RemoveNode 3, AddLearnerNode 3}
    enters the joint config (1 2)&&(1 2 3) with 3 in LearnersNext: 3 is
    still in Voters.IDs(), so the transfer stays; the empty ConfChangeV2
    leaves it -- 3 becomes a learner (tracked, in neither half) -- and the
    transfer is aborted."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc), inc=0b111, tracked=0b111, out=0)
    _transfer(be, S, 2)
    assert be.transferee() == 2
    be.set_config(tracked=0b111, inc=0b011)  # EnterJoint: Voters[0] {1, 2}
    be.set_outgoing(0b111)                   # Voters[1] {1, 2, 3}
    out = be.switch_config()
    assert out["result"] == SW_PROBE and be.transferee() == 2, out
    be.set_outgoing(0)                       # LeaveJoint: 3 a learner
    out = be.switch_config()
    assert out["result"] == SW_PROBE | SW_ABORTED and be.transferee() == 0xFF, out


def switch_removed_or_demoted_leader(be):
    """switchToConfig returns at once for a leader that was removed
    (raft.go:1663-1674, the branch confchange_v1_remove_leader.txt takes) or
    demoted to a learner (the same branch, "we handle them the same way"):
    no commit, no sends, a pending transfer kept.  Derived: the reference
    has no test of the demotion ("It is untested at the time of writing")."""
    S = 3
    sc = _leader_after_hup(S)
    sc["peers"][1]["match"] = 2  # node 2 ahead of the commit
    sc["log"]["last_index"] = 2
    be.load(sc, initial_arrays(sc), inc=0b111, tracked=0b111)
    _transfer(be, S, 1)
    be.set_config(tracked=0b110, inc=0b110)  # node 1 removed
    out = be.switch_config()
    assert out["result"] == SW_REMOVED and out["sent"] == 0 and be.committed() == 1, out
    assert be.transferee() == 1
    be.set_config(tracked=0b111, inc=0b110)  # node 1 a learner
    out = be.switch_config()
    assert out["result"] == SW_REMOVED and out["sent"] == 0 and be.committed() == 1, out


SCENARIOS = [read_only_option_safe, read_only_with_learner, read_only_option_lease,
             raft_frees_read_only_mem, read_only_for_new_leader,
             postponed_read_commit_advances_twice, two_reads_in_flight,
             read_queue_full, read_queue_deep_and_duplicates, learner_ack_does_not_count,
             leader_stepdown_when_quorum_active, leader_stepdown_when_quorum_lost,
             add_node_check_quorum, leader_transfer_to_up_to_date_node,
             leader_transfer_to_slow_follower, leader_transfer_to_self,
             leader_transfer_to_non_existing_node, leader_transfer_second_to_another_node,
             leader_transfer_after_snapshot, leader_transfer_with_check_quorum,
             leader_transfer_second_to_same_node, leader_transfer_back,
             leader_transfer_learner_ignored, commit_after_remove_node,
             leader_transfer_remove_node, leader_transfer_demote_node,
             switch_removed_or_demoted_leader]


class OracleRoundBackend:
    """The oracle (oracle/quorum_oracle.c) over one group, with the ReadIndex
    queue, qe_read_index and CheckQuorum entry points."""

    def __init__(self, orc):
        self.orc = orc

    def load(self, sc, a, inc=None, tracked=None, out=None, read_cap=0):
        S = sc["S"]
        R = sc.get("log_runs", len(sc["log"]["runs"]))  # (room for new terms' runs)
        pb = self.orc.ProgressBatch(1, S, F_CAP, R, max_ents=sc["max_ents"])
        a = dict(a)
        pb.pw = self.orc.pack_word(a.pop("flags"), 0, a.pop("icount"))
        for k, v in a.items():
            if k in ("run_first", "run_term"):
                getattr(pb, k)[: v.size] = v
            else:
                setattr(pb, k, v.copy())
        md = self.orc.mask_dtype(S)
        if inc is not None:
            pb.inc = np.array([inc], md)
        if tracked is not None:
            pb.tracked = np.array([tracked], md)
        if out is not None:
            pb.out = np.array([out], md)
        pb.track_reads(read_cap, keys=True)
        self.pb, self.sc = pb, sc
        self.pci = self.unc = self.applied = self.max_unc = 0  # MsgProp state (qe_propose)

    def step(self, t, idx, hint, lt, ctx=None):
        o = self.orc.progress_step(self.pb, t, idx, hint, lt, read_ctx=ctx)
        return {"sent": o.sent[0], "bcast": o.bcast[0], "timeout_now": o.timeout_now[0],
                "snap": o.snap[0], "msg_count": o.msg_count, "msg_index": o.msg_index,
                "read_released": int(o.read_released[0]), "term_commit": int(o.term_commit[0]),
                "term_commit_index": int(o.term_commit_index[0])}

    def heartbeat(self):
        """MsgBeat (orc_heartbeat_batch) -> (commit per slot, ctx, sent mask)."""
        commit, ctx, sent = self.orc.heartbeat(self.pb)
        return [int(x) for x in commit[: self.sc["S"]]], int(ctx[0]), int(sent[0])

    def read_index(self, lease_based=False, key=None):
        k = None if key is None else np.array([key], np.uint64)
        r, c, i = self.orc.read_index(self.pb, np.ones(1, np.uint8), lease_based, key=k)
        return int(r[0]), int(c[0]), int(i[0])

    def queue(self):
        pb = self.pb
        n, head = int(pb.read_count[0]), int(pb.read_head[0])
        mb = 1 if self.sc["S"] <= 8 else 2
        w = int(pb.read_acks[0])
        cap = max(4, pb.read_cap)
        return n, head, [((w >> (8 * mb * j)) & ((1 << (8 * mb)) - 1)) if j < 4 else
                         int(pb.read_ovf[(head + j) % cap]) for j in range(n)]

    def transferee(self):
        return int(self.pb.lead_transferee[0])

    def set_outgoing(self, mask):
        """Voters[1] of the loaded JointConfig (0: a simple config again)."""
        self.pb.out[0] = mask

    def set_snapshot(self, index):
        """The index of the snapshot a MsgSnap sends (the applied index
        where the interaction traces take it)."""
        self.pb.snap_index[0] = index

    def set_config(self, tracked, inc):
        """A new configuration's tracked slots and Voters[0] (applied conf
        change; the Progress of a slot that stays keeps its state)."""
        self.pb.tracked[0] = tracked
        self.pb.inc[0] = inc

    def become_leader(self, term, bcast=True):
        """becomeLeader on the loaded group (orc_become_leader_batch)."""
        o = self.orc.become_leader(self.pb, np.array([term], np.uint64), bcast=bcast)
        if o.result[0] == 1:
            self.pci, self.unc = int(o.pending_conf_index[0]), 0
        return {"result": int(o.result[0]), "sent": int(o.sent[0]), "snap": int(o.snap[0])}

    def switch_config(self):
        """switchToConfig on the loaded group (orc_switch_config_batch)."""
        o = self.orc.switch_config(self.pb)
        return {"result": int(o.result[0]), "sent": int(o.sent[0]), "snap": int(o.snap[0])}

    def send(self, want, sei):
        w = np.array([want], self.orc.mask_dtype(self.sc["S"]))
        sent, snap = self.orc.progress_send(self.pb, w, sei)
        return {"sent": sent[0], "snap": snap[0]}

    def append(self):
        out = self.propose(1, append_only=True)
        assert out["result"] == 1, out

    def propose(self, n, payload=0, append_only=False, cc=None):
        return oracle_propose(self, n, payload, append_only, cc)

    def last_index(self):
        return int(self.pb.last_index[0])

    def peer(self, s):
        pb = self.pb
        return peer_view(pb.match, pb.next, pb.pending, pb.flags, pb.icount, s)

    def committed(self):
        return int(self.pb.committed[0])

    def check_quorum(self):
        qa, _ = self.orc.check_quorum(self.pb)
        ra = sum(1 << s for s in range(self.sc["S"]) if self.pb.pw[s] & PF_RECENT_ACTIVE)
        return int(qa[0]), ra
