"""Leader-side transcriptions of the reference tests that pin the two
stepLeader decisions ABI 3 fuses onto the resident Progress state: the
ReadIndex ack on MsgHeartbeatResp (raft/raft.go:1296-1309,
raft/read_only.go:68-76) and MsgCheckQuorum (raft/raft.go:997-1018).

Each reference test drives a small in-process cluster; the leader's view of
it is restated here as rounds of the batch engine on one group (slot s is
node id s+1, slot 0 is the leader), through the backend interface of
tests/progress_scenarios.py plus
  step(t, idx, hint, lt, read=(acks, ctx) or None) -> out with "read_ok",
      "acks" when read is given
  check_quorum() -> (quorum_active, RecentActive bits of the slots).
The same functions drive the oracle (CPU tests) and the HIP engine (GPU
tests).  Expectations are what each reference test asserts; the rest of
its message flow (proposals, appends, acks) is executed, not assumed."""
import numpy as np

from tests.progress_scenarios import F_CAP, PF_RECENT_ACTIVE, initial_arrays

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
    """One MsgProp (raft.go:1070-1076): appendEntry (lastIndex + 1, the
    leader's own Match) + bcastAppend to every follower, then the followers'
    MsgAppResp for the new entry -- the network of the reference test
    delivers them synchronously."""
    be.append()
    li = be.last_index()
    be.send(sum(1 << s for s in range(1, S)), 1)
    t = np.zeros(S, np.uint8)
    idx = np.zeros(S, np.uint64)
    for s in voters_acking:
        t[s], idx[s] = 1, li
    z = np.zeros(S, np.uint64)
    be.step(t, idx, z, z)


def _heartbeat_round(be, S, slots, acks, ctx=None):
    t = np.zeros(S, np.uint8)
    for s in slots:
        t[s] = 3  # MsgHeartbeatResp
    z = np.zeros(S, np.uint64)
    return be.step(t, z, z, z, read=(acks, ctx))


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
        req_index = be.committed()  # readOnly.addRequest(r.raftLog.committed, m)
        out = _heartbeat_round(be, S, (1, 2), acks=0b001)
        assert out["read_ok"] == 1, want
        assert req_index == want
        assert out["acks"] == 0b011, out["acks"]  # c's ack came after the release


def read_only_with_learner(be):
    """TestReadOnlyWithLearner (raft/raft_test.go:2231-2278): voters {1},
    learner {2}.  Ten proposals per round commit on the leader alone (the
    learner's MsgAppResp advances its Match, not the quorum); the read is
    released at committed = 11, 21, 31, 41.  The reference answers a
    single-voter leader's ReadIndex at once (r.prs.IsSingleton,
    raft.go:1079-1085, a host-side shortcut); on the device the same
    release follows from the leader's own ack: VoteResult over Voters {1}
    is already won when the learner's heartbeat response arrives."""
    S = 2
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc), inc=0b01)
    wri = [11, 21, 31, 41]
    for want in wri:
        for _ in range(10):
            _propose(be, S, (1,))
        assert be.committed() == want  # committed by the leader's own Match
        out = _heartbeat_round(be, S, (1,), acks=0b01)
        assert out["read_ok"] == 1 and be.committed() == want


def learner_ack_does_not_count(be):
    """Derived from TestReadOnlyWithLearner's rule that learners never count
    (VoteResult ranges over Voters only, raft.go:1300): voters {1,2},
    learner {3}; the learner's ack alone leaves the request pending, the
    voter's ack releases it; a response without the context
    (len(m.Context) == 0) is not an ack."""
    S = 3
    sc = _leader_after_hup(S)
    be.load(sc, initial_arrays(sc), inc=0b011)
    out = _heartbeat_round(be, S, (2,), acks=0b001)
    assert out["read_ok"] == 0 and out["acks"] == 0b101
    out = _heartbeat_round(be, S, (1,), acks=0b101, ctx=0b000)  # no context
    assert out["read_ok"] == 0 and out["acks"] == 0b101
    out = _heartbeat_round(be, S, (1,), acks=0b101)
    assert out["read_ok"] == 1 and out["acks"] == 0b111


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


SCENARIOS = [read_only_option_safe, read_only_with_learner, learner_ack_does_not_count,
             leader_stepdown_when_quorum_active, leader_stepdown_when_quorum_lost,
             add_node_check_quorum]


class OracleRoundBackend:
    """The oracle (oracle/quorum_oracle.c) over one group, with the ReadIndex
    and CheckQuorum entry points."""

    def __init__(self, orc):
        self.orc = orc

    def load(self, sc, a, inc=None):
        S = sc["S"]
        pb = self.orc.ProgressBatch(1, S, F_CAP, len(sc["log"]["runs"]), max_ents=sc["max_ents"])
        a = dict(a)
        pb.pw = self.orc.pack_word(a.pop("flags"), 0, a.pop("icount"))
        for k, v in a.items():
            setattr(pb, k, v.copy())
        if inc is not None:
            pb.inc = np.array([inc], self.orc.mask_dtype(S))
        self.pb, self.sc = pb, sc

    def step(self, t, idx, hint, lt, read=None):
        md = self.orc.mask_dtype(self.sc["S"])
        acks = ctx = None
        if read is not None:
            acks = np.array([read[0]], md)
            ctx = None if read[1] is None else np.array([read[1]], md)
        o = self.orc.progress_step(self.pb, t, idx, hint, lt, read_acks=acks, read_ctx=ctx)
        out = {"sent": o.sent[0], "bcast": o.bcast[0]}
        if read is not None:
            out["read_ok"], out["acks"] = int(o.read_ok[0]), int(acks[0])
        return out

    def send(self, want, sei):
        w = np.array([want], self.orc.mask_dtype(self.sc["S"]))
        sent, snap = self.orc.progress_send(self.pb, w, sei)
        return {"sent": sent[0], "snap": snap[0]}

    def append(self):
        pb = self.pb
        pb.last_index[0] += 1
        s = self.sc["self"]
        pb.match[s] = pb.last_index[0]
        pb.next[s] = max(int(pb.next[s]), int(pb.last_index[0]) + 1)

    def last_index(self):
        return int(self.pb.last_index[0])

    def committed(self):
        return int(self.pb.committed[0])

    def check_quorum(self):
        qa, _ = self.orc.check_quorum(self.pb)
        ra = sum(1 << s for s in range(self.sc["S"]) if self.pb.pw[s] & PF_RECENT_ACTIVE)
        return int(qa[0]), ra
