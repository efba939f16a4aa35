"""Leader-side transcriptions of the reference tests that pin stepLeader's
MsgProp arm (raft/raft.go:1019-1076), appendEntry (:621-642, with
increaseUncommittedSize :1761-1779) and the bcastAppend after it
(:515-522): the entry point qe_propose (ABI 6).

As in tests/leader_round_scenarios.py, each reference test drives a small
in-process cluster; the leader's view is restated as rounds of the batch
engine on one group (slot s is node id s+1 unless a scenario says which slot
leads), through the backend interface there plus
  propose(n, payload=0, append_only=False, cc=None) -> {"result", "sent",
      "snap", "cc_refused"}   (cc: [(position, leave_joint, size), ...])
and the backend-held MsgProp state be.pci (pendingConfIndex), be.unc
(uncommittedSize), be.applied, be.max_unc (MaxUncommittedEntriesSize).
The same functions drive the oracle (CPU tests) and the HIP engine (GPU
tests).  Expectations are what each reference test asserts; the rest of
its message flow is executed, not assumed."""
import numpy as np

from tests.leader_round_scenarios import REPLICATE, _leader_after_hup, _peer
from tests.progress_scenarios import bits, initial_arrays

OK, NOT_MEMBER, TRANSFER, SIZE = 1, 2, 3, 4
ACCEPT, REJECT, HEARTBEAT, TRANSFER_LEADER = 1, 2, 3, 7


def _msgs(S, kinds):
    """kinds: {slot: (type, index[, hint, logterm])} -> step arrays."""
    t = np.zeros(S, np.uint8)
    idx = np.zeros(S, np.uint64)
    hint = np.zeros(S, np.uint64)
    lt = np.zeros(S, np.uint64)
    for s, m in kinds.items():
        t[s], idx[s] = m[0], m[1]
        if len(m) > 2:
            hint[s], lt[s] = m[2], m[3]
    return t, idx, hint, lt


def single_node_commit(be):
    """TestSingleNodeCommit (raft_test.go:705-715): a one-node cluster; the
    MsgHup makes it leader of term 1 and its empty entry 1 commits at once
    (a single voter); two MsgProp commit 2 and 3 on the leader's own
    MaybeUpdate + maybeCommit inside appendEntry."""
    sc = _leader_after_hup(1)
    be.load(sc, initial_arrays(sc))
    for want in (2, 3):
        out = be.propose(1, payload=9)
        assert out["result"] == OK and out["sent"] == 0, out
        assert be.last_index() == want and be.committed() == want
    assert be.committed() == 3


def uncommitted_entry_limit(be):
    """TestUncommittedEntryLimit (raft_test.go:179-270) with maxEntries = 200
    instead of 1024: the slot model's Inflights hold at most 255 entries
    (QE_MAX_INFLIGHT) where the test raises MaxInflightMsgs to 2048 "to avoid
    interference"; every figure below scales with maxEntries.  3 voters,
    testEntry payload 8 B, MaxUncommittedEntriesSize = maxEntries * 8.
    becomeLeader appended the empty entry 1 (not committed: 3 voters) and
    the two followers were moved to StateReplicate (Match 0, Next 1)."""
    n_max, esz = 200, 8
    S = 3
    sc = {"name": "", "S": S, "self": 0, "max_ents": 0,
          "log": {"runs": [[0, 0], [1, 1]], "committed": 0, "term_start": 1, "first_index": 1,
                  "last_index": 1},
          "peers": [_peer(1, 2, REPLICATE), _peer(0, 1, REPLICATE), _peer(0, 1, REPLICATE)]}
    be.load(sc, initial_arrays(sc))
    be.max_unc = n_max * esz
    msgs = 0
    for i in range(n_max):
        out = be.propose(1, payload=esz)
        assert out["result"] == OK, (i, out)
        msgs += len(bits(out["sent"]))
    out = be.propose(1, payload=esz)  # one more: rejected
    assert out["result"] == SIZE and out["sent"] == 0, out
    assert msgs == n_max * 2  # maxEntries * numFollowers
    # reduceUncommittedSize(propEnts) -- the host applies the entries
    be.unc = max(0, be.unc - n_max * esz)
    assert be.unc == 0
    # a single large proposal is accepted: the tail was empty before it
    out = be.propose(2 * n_max, payload=2 * n_max * esz)
    assert out["result"] == OK and len(bits(out["sent"])) == 2, out
    msgs = 2
    out = be.propose(1, payload=esz)  # rejected again
    assert out["result"] == SIZE, out
    out = be.propose(1, payload=0)  # an entry without Data is never refused
    assert out["result"] == OK, out
    msgs += len(bits(out["sent"]))
    assert msgs == 2 * 2  # 2 * numFollowers
    be.unc = max(0, be.unc - 2 * n_max * esz)
    assert be.unc == 0
    assert be.last_index() == 1 + n_max + 2 * n_max + 1


def step_ignore_config(be):
    """TestStepIgnoreConfig (raft_test.go:3120-3141): 2 voters; becomeLeader
    set pendingConfIndex = lastIndex (0) before appending its empty entry 1.
    A first EntryConfChange (empty Data: a V1 ConfChange, one change) is
    accepted at index 2; a second one while it is unapplied is replaced by
    an empty EntryNormal at index 3 and pendingConfIndex stays 2."""
    S = 2
    sc = {"name": "", "S": S, "self": 0, "max_ents": 0,
          "log": {"runs": [[0, 0], [1, 1]], "committed": 0, "term_start": 1, "first_index": 1,
                  "last_index": 1},
          "peers": [_peer(1, 2, REPLICATE), _peer(0, 2, 0)]}
    be.load(sc, initial_arrays(sc))
    out = be.propose(1, cc=[(0, False, 0)])
    assert out["result"] == OK and out["cc_refused"] == 0, out
    index, pending = be.last_index(), be.pci
    assert (index, pending) == (2, 2)
    out = be.propose(1, cc=[(0, False, 0)])
    assert out["result"] == OK and out["cc_refused"] == 1, out  # -> EntryNormal at 3
    assert be.last_index() == index + 1 == 3
    assert be.pci == pending


def new_leader_pending_config(be):
    """TestNewLeaderPendingConfig (raft_test.go:3144-3163): becomeLeader sets
    pendingConfIndex = lastIndex, then appends its empty entry through
    appendEntry (qe_propose, QE_PROP_APPEND_ONLY), which leaves it alone:
    0 for an empty log, 1 with one entry appended before."""
    for add_entry, want in ((False, 0), (True, 1)):
        li = 1 if add_entry else 0
        sc = {"name": "", "S": 2, "self": 0, "max_ents": 0,
              "log": {"runs": [[0, 0], [li + 1, 1]], "committed": 0, "term_start": li + 1,
                      "first_index": 1, "last_index": li},
              "peers": [_peer(li, li + 1, REPLICATE), _peer(0, li + 1, 0)]}
        be.load(sc, initial_arrays(sc))
        be.pci = li  # r.pendingConfIndex = r.raftLog.lastIndex()
        out = be.propose(1, append_only=True)  # emptyEnt
        assert out["result"] == OK and out["sent"] == 0
        assert be.pci == want and be.last_index() == li + 1
        assert be.peer(0)["match"] == li + 1


def leader_transfer_ignore_proposal(be):
    """TestLeaderTransferIgnoreProposal (raft_test.go:3637-3660): 3 nodes,
    node 3 isolated after the election.  Its MsgTransferLeader makes it the
    lead transferee (its Match equals lastIndex, so MsgTimeoutNow goes out
    and is lost); every MsgProp is then dropped and the leader's own Match
    stays 1."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    out = be.step(*_msgs(S, {2: (TRANSFER_LEADER, 0)}))
    assert bits(out["timeout_now"]) == [2] and be.transferee() == 2
    for _ in range(2):
        out = be.propose(1)
        assert out["result"] == TRANSFER and out["sent"] == 0, out
    assert be.last_index() == 1 and be.peer(0)["match"] == 1


def cannot_commit_without_new_term_entry(be):
    """TestCannotCommitWithoutNewTermEntry (raft_test.go:720-764), both
    leaders' views.  (a) Node 1 leads term 1 with 5 voters; cut from 3, 4, 5,
    it proposes twice: only node 2 acks, so 2 and 3 stay uncommitted
    (committed 1).  (b) Node 2 wins term 2 with log [1..3 @ 1], appends its
    empty entry 4@2, and its MsgApps are dropped: committed stays 1 -- no
    entry of term 1 commits on its own.  After recovery the heartbeat
    responses make it probe (the message flow the network delivers:
    node 1 holds [1..3] and accepts 4, nodes 3-5 hold [1] and reject with
    hint 1, then accept from 2), which commits 4; the MsgProp appends 5,
    bcastAppend reaches everyone and the acks commit 5 (the test's want)."""
    S = 5
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc))
    for li in (2, 3):
        out = be.propose(1, payload=9)
        assert out["result"] == OK and bits(out["sent"]) == [1, 2, 3, 4], out
        be.step(*_msgs(S, {1: (ACCEPT, li)}))  # only node 2 is reachable
    assert be.committed() == 1
    # (b) node 2 (slot 1) leads term 2
    sc = {"name": "", "S": S, "self": 1, "max_ents": 0,
          "log": {"runs": [[0, 0], [1, 1], [4, 2]], "committed": 1, "term_start": 4,
                  "first_index": 1, "last_index": 4},
          # reset(): Match 0, Next = lastIndex + 1 = 4 before the empty entry;
          # becomeLeader's bcastAppend probed everyone (dropped)
          "peers": [_peer(0, 4, 0, probe_sent=True), _peer(4, 5, REPLICATE),
                    _peer(0, 4, 0, probe_sent=True), _peer(0, 4, 0, probe_sent=True),
                    _peer(0, 4, 0, probe_sent=True)]}
    be.load(sc, initial_arrays(sc))
    assert be.committed() == 1
    out = be.step(*_msgs(S, {s: (HEARTBEAT, 0) for s in (0, 2, 3, 4)}))  # MsgBeat's round
    assert bits(out["sent"]) == [0, 2, 3, 4]
    out = be.step(*_msgs(S, {0: (ACCEPT, 4), 2: (REJECT, 3, 1, 1), 3: (REJECT, 3, 1, 1),
                             4: (REJECT, 3, 1, 1)}))
    assert be.committed() == 1 and [be.peer(s)["next"] for s in (2, 3, 4)] == [2, 2, 2]
    be.step(*_msgs(S, {s: (ACCEPT, 4) for s in (2, 3, 4)}))
    assert be.committed() == 4
    out = be.propose(1, payload=9)
    assert out["result"] == OK and bits(out["sent"]) == [0, 2, 3, 4], out
    be.step(*_msgs(S, {s: (ACCEPT, 5) for s in (0, 2, 3, 4)}))
    assert be.committed() == 5


def proposal(be):
    """TestProposal (raft_test.go:1030-1080), its rows where node 1 becomes
    leader (success = true): 3 nodes; 3 nodes with one nopStepper; 5 nodes
    with two.  The MsgProp's entry 2 commits once the live followers ack it
    (the wanted log has committed 2); a nopStepper never answers (its
    Progress stays where becomeLeader left it: Probe, Next 2, ProbeSent)."""
    for S, dead in ((3, ()), (3, (2,)), (5, (1, 2))):
        sc = _leader_after_hup(S)
        for s in dead:
            sc["peers"][s] = _peer(0, 2, 0, probe_sent=True)
        be.load(sc, initial_arrays(sc))
        out = be.propose(1, payload=8)
        live = [s for s in range(1, S) if s not in dead]
        assert out["result"] == OK and bits(out["sent"]) == live, (S, dead, out)
        be.step(*_msgs(S, {s: (ACCEPT, 2) for s in live}))
        assert be.committed() == 2 and be.last_index() == 2


def conf_change_gating(be):
    """The conf-change checks of the MsgProp arm (raft.go:1050-1069; derived
    from the code, no single reference test): outside a joint config an
    empty ConfChangeV2 (leave joint) is refused and a change is accepted;
    while that change is unapplied every further one is refused; once
    applied reaches it the next is accepted.  In a joint config a change
    with Changes is refused and the leave is accepted.  A refused entry keeps
    its place (an empty EntryNormal): lastIndex grows by the whole proposal,
    and its payload does not count toward uncommittedSize."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc), inc=0b111)
    out = be.propose(2, payload=5, cc=[(1, True, 7)])  # leave while not joint
    assert out["result"] == OK and out["cc_refused"] == 1 and be.pci == 0
    assert be.unc == 5 and be.last_index() == 3
    out = be.propose(3, cc=[(0, False, 4), (2, False, 6)])  # the second: pending
    assert out["cc_refused"] == 0b10 and be.pci == 4 and be.unc == 9
    out = be.propose(1, cc=[(0, False, 4)])
    assert out["cc_refused"] == 1 and be.pci == 4
    be.applied = 4
    out = be.propose(1, cc=[(0, False, 4)])
    assert out["cc_refused"] == 0 and be.pci == 8
    # joint (Voters[1] non-empty)
    be.load(sc, initial_arrays(sc), inc=0b011, out=0b101)
    out = be.propose(1, cc=[(0, False, 3)])
    assert out["cc_refused"] == 1 and be.pci == 0
    out = be.propose(1, cc=[(0, True, 0)])
    assert out["cc_refused"] == 0 and be.pci == 3
    # a dropped proposal (size) keeps the pendingConfIndex it set
    be.applied, be.max_unc, be.unc = 3, 10, 8
    out = be.propose(1, cc=[(0, True, 5)])
    assert out["result"] == SIZE and be.pci == 4 and be.last_index() == 3


SCENARIOS = [single_node_commit, uncommitted_entry_limit, step_ignore_config,
             new_leader_pending_config, leader_transfer_ignore_proposal,
             cannot_commit_without_new_term_entry, proposal, conf_change_gating]
