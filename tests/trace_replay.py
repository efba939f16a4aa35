"""Replay of the reference's interaction traces (raft/testdata/*.txt, run by
raft/interaction_test.go:24-34) from the leader's side, through the batch
engine's entry points on one group:

  probe_and_replicate.txt            7 voters: election at term 8, then every
                                     follower probed back: rejections with
                                     hints, findConflictByTerm, MaybeDecrTo,
                                     the MsgApps that answer them
  snapshot_succeed_via_app_resp.txt  heartbeats, a MsgSnap for a compacted
                                     log, the MsgAppResp that ends it
  campaign.txt                       an election and the first commit
  campaign_learner_must_vote.txt     an election won with a voter the
                                     candidate's config has, then its catch-up
  confchange_v1_add_single.txt,      a voter added to a one-node cluster: the
  confchange_v2_add_single_auto.txt  new Progress (initProgress), the probe it
                                     gets when the config switches, its
                                     rejection, the MsgSnap, and the catch-up
  confchange_v2_add_double_implicit  the same through a joint config with
  .txt                               AutoLeave: the leave entry appended at
                                     apply time commits only with both halves
  confchange_v2_add_single_explicit  the joint config left by a proposal:
  .txt                               stepLeader's conf-change refusals
  confchange_v2_add_double_auto.txt  two voters added and removed through
                                     joint configs with AutoLeave
  confchange_v1_remove_leader.txt    a leader that removes itself: proposals
                                     through qe_propose, the commit quorum
                                     without it, its dropped proposal, its
                                     heartbeats

The fixture tests/golden/interaction_traces.json holds what the reference
printed (tests/golden/make_golden.py extracts it: no reference code runs).
Each leader's state at the point the printed part begins is restated from
the trace itself (raft-log dumps, status lines, HardState, the INFO lines of
the election) -- see the *_setup functions -- and the leader's transitions
run through the engine (becomeCandidate's term bump in the election
kernel; becomeLeader, with its reset() of every Progress, raft.go:590-613,
through qe_become_leader; the host's conf-change application between
Readies -- the new masks -- is written out where it occurs, and
switchToConfig runs through qe_switch_config).  Everything else is executed
by the engine and compared with the trace:

  * every "> L receiving messages" block is one or more rounds of
    qe_progress_step (messages in slot order; a block whose senders are not
    ascending is split where they descend, so the order is the trace's), or
    for MsgVoteResp one scripted qe_election_steps step;
  * every "> L handling Ready" block: per destination the number of
    MsgApp/MsgSnap sent since the previous Ready and the Log index of the
    first (msg_count / msg_index; a MsgSnap's snapshot index), the follower's
    Next after them (the entries they carried: Probe keeps Next at the
    probe, Replicate moves it past the last entry), the Commit they carry
    and the HardState commit; MsgHeartbeat commits (qe_heartbeat);
  * `status L` blocks: every Progress rendered as progress.go:214-236 does;
  * "decreased progress of X to [...]" DEBUG lines: X's state, match and next.
"""
import json
import os
import re

import numpy as np

from tests.golden_util import GOLDEN
from tests.progress_scenarios import initial_arrays

STATE = {"StateProbe": 0, "StateReplicate": 1, "StateSnapshot": 2}
STATE_NAME = {v: k for k, v in STATE.items()}
SW_REMOVED, SW_BCAST, SW_PROBE = 1, 3, 4  # QE_SW_* outcomes of qe_switch_config
# MaxInflightMsgs of the interaction env is math.MaxInt32 and MaxSizePerMsg
# math.MaxUint64 (raft/rafttest/interaction_env.go:96-97): no trace holds more
# than a few MsgApps in flight, so the slot model's 255 never binds
F_TRACE = 255


def traces():
    with open(os.path.join(GOLDEN, "interaction_traces.json"), encoding="utf-8") as f:
        return json.load(f)


def progress_string(p, F=F_TRACE):
    """tracker.Progress.String (raft/tracker/progress.go:214-236) of a peer
    view (tests/progress_scenarios.peer_view) with its Inflights capacity."""
    paused = (p["probe_sent"] if p["state"] == 0 else
              (p["inflights"] == F if p["state"] == 1 else True))
    s = f"{STATE_NAME[p['state']]} match={p['match']} next={p['next']}"
    if paused:
        s += " paused"
    if p["pending"] > 0:
        s += f" pendingSnap={p['pending']}"
    if not p["recent_active"]:
        s += " inactive"
    if p["inflights"] > 0:
        s += f" inflight={p['inflights']}"
        if p["inflights"] == F:
            s += "[full]"
    return s


def parse_progress(text):
    """The fields a Progress string shows -> a peer dict (scenario form)."""
    m = re.match(r"(State\w+) match=(\d+) next=(\d+)", text)
    state = STATE[m.group(1)]
    pend = re.search(r"pendingSnap=(\d+)", text)
    infl = re.search(r"inflight=(\d+)", text)
    paused = " paused" in text
    return {"match": int(m.group(2)), "next": int(m.group(3)),
            "pending": int(pend.group(1)) if pend else 0, "state": state,
            "probe_sent": paused and state == 0, "recent_active": " inactive" not in text,
            "ring": [0] * (int(infl.group(1)) if infl else 0)}


def log_runs(entries, dummy):
    """[[term, index], ...] of a log (ascending) after a dummy (snapshot)
    entry [term, index] -> term runs [[first, term], ...]."""
    runs = [[dummy[1], dummy[0]]]
    for t, i in entries:
        if t != runs[-1][1]:
            runs.append([i, t])
    return runs


class Leader:
    """The replayed leader: backend `be` (oracle or GPU, the interface of
    tests/leader_round_scenarios.py plus heartbeat() and election()), node
    id -> slot = id - 1.  The log's term runs end with the leader's own
    term (term_start = its first index: on a fresh cluster that can be the
    snapshot index, whose term the first leader shares)."""

    def __init__(self, be, node, S, F=F_TRACE):
        self.be, self.node, self.S, self.F = be, node, S, F
        self.self = node - 1
        self.pending = {}   # slot -> [(index, is_snap)] sent since the last Ready
        self.hb = {}        # slot -> heartbeat commit since the last Ready
        self.c_before = None
        self.checked = {"rounds": 0, "sends": 0, "status": 0, "heartbeats": 0, "progress": 0}

    def slot(self, node_id):
        return node_id - 1

    # -- state set-up ------------------------------------------------------
    def load(self, li, committed, runs, first_index, peers, snap_index=None, term_start=None,
             inc=None, out=None, tracked=None, spare_runs=0):
        lg = {"runs": runs, "committed": committed, "first_index": first_index,
              "last_index": li,
              "term_start": term_start if term_start is not None else runs[-1][0]}
        if snap_index is not None:
            lg["snap_index"] = snap_index
        sc = {"name": "", "S": self.S, "self": self.self, "max_ents": 0, "log": lg,
              "peers": peers, "log_runs": len(runs) + spare_runs}
        if inc is None and out is None and tracked is None:
            self.be.load(sc, initial_arrays(sc))
        else:  # a configuration given as slot masks (JointConfig: out too)
            self.be.load(sc, initial_arrays(sc), inc=inc, out=out, tracked=tracked)

    def become_leader(self, li, committed, runs, first_index, term):
        """becomeLeader (raft.go:724-759) after a won election, through the
        engine's qe_become_leader (QE_BL_BCAST): reset() (:590-613) of every
        Progress, the leader's own BecomeReplicate, pendingConfIndex =
        lastIndex, the log entering `term`, appendEntry of the empty entry and
        stepCandidate's bcastAppend (:1405-1407).  The Progress loaded
        before is the candidate's (arbitrary here: reset overwrites it) --
        only the log model (runs before the new term, lastIndex, committed,
        firstIndex) carries over."""
        peers = [{"match": 7 * s, "next": 1 + s, "pending": 0, "state": s % 2,
                  "probe_sent": bool(s % 3), "recent_active": True, "ring": []}
                 for s in range(self.S)]
        self.load(li, committed, runs, first_index, peers, spare_runs=1)
        out = self.be.become_leader(term)
        assert out["result"] == 1 and self.be.pci == li and self.be.last_index() == li + 1, out
        for s in range(self.S):
            if (out["sent"] >> s) & 1:
                snap = bool((out["snap"] >> s) & 1)
                p = self.be.peer(s)
                idx = p["pending"] if snap else p["next"] - 1  # a probe keeps Next
                self.pending.setdefault(s, []).append((idx, snap, self.be.last_index()))
        self.checked["elections"] = self.checked.get("elections", 0) + 1

    def bcast(self, sei=1):
        """bcastAppend: sendAppend to every peer but the leader (stepCandidate
        after a won election, raft.go:1405-1407)."""
        nxt = {s: self.be.peer(s)["next"] for s in range(self.S)}
        want = sum(1 << s for s in range(self.S) if s != self.self)
        out = self.be.send(want, sei)
        for s in range(self.S):
            if (out["sent"] >> s) & 1:
                snap = bool((out["snap"] >> s) & 1)
                idx = self.be.peer(s)["pending"] if snap else nxt[s] - 1
                self.pending.setdefault(s, []).append((idx, snap, self.be.last_index()))

    def switch(self, want):
        """switchToConfig (raft.go:1651-1700) after the host applied a conf
        change, through the engine's qe_switch_config: the removed-leader
        return, maybeCommit under the new config and bcastAppend, or the
        probe of every peer (maybeSendAppend(id, false)), the transfer
        abort.  `want`: the QE_SW_* outcome the trace implies (the Ready
        after it checks the sends and the commit)."""
        nxt = {s: self.be.peer(s)["next"] for s in range(self.S)}
        out = self.be.switch_config()
        assert out["result"] == want, ("switchToConfig", out, want)
        for s in range(self.S):
            if (out["sent"] >> s) & 1:
                snap = bool((out["snap"] >> s) & 1)
                idx = self.be.peer(s)["pending"] if snap else nxt[s] - 1
                self.pending.setdefault(s, []).append((idx, snap, self.be.last_index()))
        self.checked["switches"] = self.checked.get("switches", 0) + 1
        return out

    # -- replay --------------------------------------------------------------
    def recv(self, block):
        msgs = [m for m in block["msgs"] if m["to"] == self.node and m["type"] != "MsgVoteResp"]
        if not msgs:
            return
        rounds, cur = [], []
        for m in msgs:
            if cur and self.slot(m["from"]) <= self.slot(cur[-1]["from"]):
                rounds.append(cur)
                cur = []
            cur.append(m)
        rounds.append(cur)
        if self.c_before is None:
            self.c_before = self.be.committed()
        for rnd in rounds:
            t = np.zeros(self.S, np.uint8)
            idx = np.zeros(self.S, np.uint64)
            hint = np.zeros(self.S, np.uint64)
            lt = np.zeros(self.S, np.uint64)
            for m in rnd:
                s = self.slot(m["from"])
                if m["type"] == "MsgAppResp":
                    t[s] = 2 if m["reject"] else 1
                    idx[s], hint[s], lt[s] = m["index"], m["hint"], m["logterm"]
                elif m["type"] == "MsgHeartbeatResp":
                    t[s] = 3
                else:
                    raise AssertionError(f"unexpected message at the leader: {m}")
            out = self.be.step(t, idx, hint, lt)
            self.checked["rounds"] += 1
            for s in range(self.S):
                n = int(out["msg_count"][s])
                if n:
                    snap = bool((out["snap"] >> s) & 1)
                    li = self.be.last_index()
                    self.pending.setdefault(s, []).extend(
                        [(int(out["msg_index"][s]), snap, li)] + [(None, False, li)] * (n - 1))
        # the Progress a DEBUG line prints after the round's last change to
        # a peer: MaybeDecrTo's "decreased progress" (raft.go:1231), unless
        # the sendAppend after it turned the peer to StateSnapshot ("paused
        # sending replication messages", raft.go:466-470, printed after
        # BecomeSnapshot)
        last = {}
        for line in block.get("debug", []):
            d = (re.search(r"decreased progress of (\d+) to \[(.*)\]", line) or
                 re.search(r"paused sending replication messages to (\d+) \[(.*)\]", line))
            if d:
                last[int(d.group(1))] = (line, d.group(2))
        for node, (line, text) in last.items():
            want = parse_progress(text)
            got = self.be.peer(self.slot(node))
            for k in ("state", "match", "next", "pending"):
                assert got[k] == want[k], (line, got)
            self.checked["progress"] += 1

    def propose(self, c, where):
        """`propose L data` / `propose-conf-change L ...`: one MsgProp
        through qe_propose (stepLeader's arm, raft.go:1019-1076, and the
        bcastAppend after appendEntry) -- a conf-change entry for the
        latter; the trace prints "raft proposal dropped" or "ok"."""
        # a conf change with no changes listed is the empty ConfChangeV2
        # that leaves a joint config
        cc = ([(0, not c["input"], 0)] if c["cmd"].startswith("propose-conf-change") else None)
        nxt = {s: self.be.peer(s)["next"] for s in range(self.S)}
        out = self.be.propose(1, cc=cc)
        if c.get("dropped"):
            assert out["result"] in (2, 3, 4), (where, out)  # QE_PROP_DROPPED_*
            return
        assert out["result"] == 1, (where, out)  # QE_PROP_OK
        # refused conf changes become empty normal entries (raft.go:1050-1069)
        assert out["cc_refused"] == int(bool(c.get("ignored_cc"))), (where, out)
        for s in range(self.S):
            if (out["sent"] >> s) & 1:
                snap = bool((out["snap"] >> s) & 1)
                idx = self.be.peer(s)["pending"] if snap else nxt[s] - 1
                self.pending.setdefault(s, []).append((idx, snap, self.be.last_index()))
        self.checked["proposals"] = self.checked.get("proposals", 0) + 1

    def heartbeat(self):
        commit, _, sent = self.be.heartbeat()
        for s in range(self.S):
            if (sent >> s) & 1:
                self.hb[s] = int(commit[s])

    def ready(self, block, where):
        sends = {}
        hbs = {}
        for m in block["msgs"]:
            if m["from"] != self.node:
                continue
            s = self.slot(m["to"])
            if m["type"] in ("MsgApp", "MsgSnap"):
                sends.setdefault(s, []).append(m)
            elif m["type"] == "MsgHeartbeat":
                hbs[s] = m["commit"]
        got_slots = {s for s, v in self.pending.items() if v}
        assert got_slots == set(sends), (where, "destinations", sorted(got_slots), sorted(sends))
        for s, ms in sends.items():
            got = self.pending[s]
            assert len(got) == len(ms), (where, s, got, ms)
            first = ms[0]
            want_ix = first["snap_index"] if first["type"] == "MsgSnap" else first["index"]
            assert got[0][:2] == (want_ix, first["type"] == "MsgSnap"), (where, s, got[0], first)
            for m, g in zip(ms, got):
                # MaxSizePerMsg noLimit: a MsgApp carries every entry after its
                # Log index up to the lastIndex when it was sent
                if m["type"] == "MsgApp":
                    assert [e[1] for e in m["entries"]] == list(range(m["index"] + 1, g[2] + 1)), \
                        (where, s, m, g)
            p = self.be.peer(s)
            if first["type"] == "MsgSnap":
                assert p["state"] == 2 and p["pending"] == first["snap_index"], (where, p)
            elif p["state"] == 0:  # a probe does not move Next
                assert p["next"] == first["index"] + 1, (where, s, p)
            elif p["state"] == 1:  # Replicate: past the last entry sent
                last = ms[-1]
                end = last["entries"][-1][1] if last["entries"] else last["index"]
                assert p["next"] == end + 1, (where, s, p, last)
            self.checked["sends"] += len(ms)
        c = self.be.committed()
        apps = [m for ms in sends.values() for m in ms if m["type"] == "MsgApp"]
        if apps:
            assert max(m["commit"] for m in apps) == c, (where, c, apps)
        if block.get("commit") is not None and block.get("node") == self.node:
            assert block["commit"] == c, (where, block["commit"], c)
        assert self.hb == hbs, (where, self.hb, hbs)
        self.checked["heartbeats"] += len(hbs)
        self.pending, self.hb, self.c_before = {}, {}, None

    def status(self, block, where):
        for k, text in block["progress"].items():
            got = progress_string(self.be.peer(self.slot(int(k))), self.F)
            assert got == text, (where, k, got, text)
            self.checked["status"] += 1

    def replay(self, cmds, start_line, stop_line=None, on_election=None, after_ready=None,
               proposals=False):
        """Walk the commands of a trace from start_line: the leader's recv /
        Ready / status blocks and its tick-heartbeat commands.
        after_ready(block): the host's work after a Ready was handled (e.g.
        applying a committed conf change); proposals: run the leader's
        `propose` commands through qe_propose."""
        for c in cmds:
            if c["line"] < start_line or (stop_line is not None and c["line"] >= stop_line):
                continue
            where = f"line {c['line']} `{c['cmd']}`"
            if c["cmd"] == f"tick-heartbeat {self.node}":
                self.heartbeat()
            if proposals and c["cmd"].startswith(("propose ", "propose-conf-change ")) and \
                    c["cmd"].split()[1] == str(self.node):
                self.propose(c, where)
            for b in c["blocks"]:
                if b["kind"] == "status":
                    if c["cmd"] == f"status {self.node}":
                        self.status(b, where)
                    continue
                node = b["node"]
                if node is None and c["cmd"] == f"process-ready {self.node}":
                    node = self.node
                if node != self.node:
                    continue
                if b["kind"] == "recv":
                    votes = [m for m in b["msgs"] if m["type"] == "MsgVoteResp"]
                    if votes and on_election:
                        on_election(votes)
                    self.recv(b)
                else:
                    if any(m["type"] == "MsgVote" for m in b["msgs"]):
                        continue  # the candidate's vote requests
                    self.ready(b, where)
                    if after_ready:
                        after_ready(b)
        assert not any(self.pending.values()), ("sends never reported", self.pending)
        return self.checked


def command(cmds, text):
    return next(c for c in cmds if c["cmd"] == text)


def election(elector, S, self_slot, term0, votes, want_term):
    """The candidate side through scripted qe_election_steps on one group
    (a follower at term0, every slot a voter): a MsgHup step
    (becomeCandidate: term + 1, the self-vote), then one step with the vote
    responses the trace shows -> StateLeader at want_term.
    elector(S, self_slot, term0) -> step(resp, grant, hup) -> (term, state)."""
    step = elector(S, self_slot, term0)
    term, state = step(0, 0, 1)
    assert (term, state) == (want_term, 1), (term, state)  # StateCandidate
    resp = sum(1 << (m["from"] - 1) for m in votes)
    grant = sum(1 << (m["from"] - 1) for m in votes if not m["reject"])
    term, state = step(resp, grant, 0)
    assert (term, state) == (want_term, 2), (term, state)  # StateLeader


def _info(cmds, pattern):
    for c in cmds:
        for b in c["blocks"]:
            for line in b.get("debug", []):
                m = re.search(pattern, line)
                if m:
                    return m
    return None


def probe_and_replicate(leader_factory, elector):
    """raft/testdata/probe_and_replicate.txt from `campaign 1` (Figure 7 of
    the Raft paper, shifted by 10).  Node 1's log is the trace's `raft-log 1`
    dump after the snapshot at index 10 (term 1, add-nodes index=10);
    committed 18 is the HardState of the candidate's first Ready; the term
    before the campaign is 7 (its INFO line)."""
    cmds = traces()["probe_and_replicate.txt"]["commands"]
    log = command(cmds, "raft-log 1")["log"]
    li = log[-1][1]
    camp = command(cmds, "campaign 1")
    L = leader_factory(1, 7)
    runs = log_runs(log, [1, 10])
    assert runs == [[10, 1], [14, 4], [16, 5], [18, 6]] and li == 20
    state = {}

    def won(votes):
        election(elector, 7, 0, 7, votes, 8)
        L.become_leader(li, 18, runs, 11, term=8)
        state["won"] = True

    checked = L.replay(cmds, camp["line"] + 1, on_election=won)
    assert state.get("won")
    return checked


def snapshot_succeed_via_app_resp(leader_factory, elector):
    """raft/testdata/snapshot_succeed_via_app_resp.txt from its first
    `status 1`: the state is the one that status prints (3 voters, node 3
    paused in StateProbe, inactive); node 1's log is the snapshot at 10
    (term 1) plus its empty entry 11 (term 1), compacted through 11
    (`compact 1 11`: firstIndex 12, snapshot index 11), committed 11."""
    cmds = traces()["snapshot_succeed_via_app_resp.txt"]["commands"]
    st = command(cmds, "status 1")
    L = leader_factory(1, 3)
    peers = [parse_progress(st["blocks"][0]["progress"][str(k)]) for k in (1, 2, 3)]
    L.load(11, 11, [[11, 1]], 12, peers, snap_index=11, term_start=11)
    return L.replay(cmds, st["line"])


def campaign(leader_factory, elector):
    """raft/testdata/campaign.txt: 3 voters, each log the snapshot at 2
    (term 1; newRaft's INFO: commit 2, lastindex 2, lastterm 1), node 1
    campaigns from term 0."""
    cmds = traces()["campaign.txt"]["commands"]
    L = leader_factory(1, 3)
    state = {}

    def won(votes):
        election(elector, 3, 0, 0, votes, 1)
        L.become_leader(2, 2, [[2, 1]], 3, term=1)  # (the snapshot's term: the term starts at 2)
        state["won"] = True

    checked = L.replay(cmds, command(cmds, "campaign 1")["line"], on_election=won)
    assert state.get("won")
    return checked


def campaign_learner_must_vote(leader_factory, elector):
    """raft/testdata/campaign_learner_must_vote.txt from `campaign 2`: node
    2's config has voters 1, 2, 3 (the promotion of 3 is applied), its log
    the snapshot at 2 (term 1), 3@1 (node 1's empty entry) and 4@1 (the
    conf change), committed 4; it campaigns from term 1 (its INFO line) and
    node 1 is down."""
    cmds = traces()["campaign_learner_must_vote.txt"]["commands"]
    L = leader_factory(2, 3)
    state = {}

    def won(votes):
        election(elector, 3, 1, 1, votes, 2)
        L.become_leader(4, 4, [[2, 1]], 3, term=2)
        state["won"] = True

    checked = L.replay(cmds, command(cmds, "campaign 2")["line"], on_election=won)
    assert state.get("won")
    return checked


def _confchange_add_single(name):
    def run(leader_factory, elector):
        """raft/testdata/{name} from `stabilize`: node 1, bootstrapped alone
        with the snapshot at 2 (term 1; newRaft's INFO line), won term 1 by
        itself, appended its empty entry 3 and the conf change 4 and
        committed both alone (the first Ready's HardState Commit:4).  The
        state is restated as it is after that Ready applies 4: node 2 added
        by initProgress (raft/confchange/confchange.go:259-274: Match 0,
        Next = lastIndex 4, RecentActive); the leader's own Progress at
        match 4.  switchToConfig then runs through qe_switch_config right
        after the Ready that prints the switch: maybeCommit under {{1, 2}}
        finds nothing to commit, so every peer gets maybeSendAppend(id,
        false) (raft.go:1682-1692).  The snapshot a compacted log sends is
        the applied index 4 (the trace's MsgSnap)."""
        cmds = traces()[name]["commands"]
        st = command(cmds, "stabilize")
        L = leader_factory(1, 2)
        peers = [{"match": 4, "next": 5, "pending": 0, "state": 1, "probe_sent": False,
                  "recent_active": True, "ring": []},
                 {"match": 0, "next": 4, "pending": 0, "state": 0, "probe_sent": False,
                  "recent_active": True, "ring": []}]
        L.load(4, 4, [[2, 1]], 3, peers, snap_index=4)
        switched = []

        def after(block):
            if any("switched to configuration voters=(1 2)" in x for x in block["debug"]):
                L.switch(SW_PROBE)
                switched.append(block)

        checked = L.replay(cmds, st["line"], after_ready=after)
        assert len(switched) == 1
        return checked
    run.__name__ = name[:-4]
    run.__doc__ = run.__doc__.format(name=name)
    return run


def confchange_v2_add_double_implicit(leader_factory, elector):
    """raft/testdata/confchange_v2_add_double_implicit.txt from `stabilize 1
    2`: as the add_single traces, but the V2 change enters a joint config
    with AutoLeave (voters (1 2)&&(1)): applying 4 switches to it, the new
    voter gets its probe (switchToConfig, raft.go:1682-1692), and advance()
    then appends the empty EntryConfChangeV2 that leaves it (raft.go:
    apply-time auto-leave: appendEntry alone, no bcast -- qe_propose with
    QE_PROP_APPEND_ONLY) at 5.  Index 5 commits only when both halves hold
    it: on node 2's ack of 5 (the commit rule of the joint config), whose
    bcast carries Commit:5; applying 5 leaves the joint config (Voters[1]
    empty: the same quorum as the simple config) and probes again, which
    sends nothing."""
    cmds = traces()["confchange_v2_add_double_implicit.txt"]["commands"]
    st = command(cmds, "stabilize 1 2")
    L = leader_factory(1, 2)
    peers = [{"match": 4, "next": 5, "pending": 0, "state": 1, "probe_sent": False,
              "recent_active": True, "ring": []},
             {"match": 0, "next": 4, "pending": 0, "state": 0, "probe_sent": False,
              "recent_active": True, "ring": []}]
    L.load(4, 4, [[2, 1]], 3, peers, snap_index=4, inc=0b11, out=0b01)
    seen = []

    def after(block):
        for x in block["debug"]:
            if "switched to configuration voters=(1 2)&&(1) autoleave" in x:
                L.switch(SW_PROBE)
                out = L.be.propose(1, append_only=True)  # the auto-leave entry
                assert out["result"] == 1 and L.be.last_index() == 5, out
                seen.append("enter")
            elif x.endswith("switched to configuration voters=(1 2)"):
                L.be.set_outgoing(0)
                L.switch(SW_PROBE)
                seen.append("leave")

    checked = L.replay(cmds, st["line"], after_ready=after)
    assert seen == ["enter", "leave"] and L.be.committed() == 5
    return checked


def confchange_v1_remove_leader(leader_factory, elector):
    """raft/testdata/confchange_v1_remove_leader.txt from `log-level debug`:
    3 voters bootstrapped with the snapshot at 2 (term 1), node 1 elected at
    term 1 and everything stabilized (quietly): its empty entry 3 committed
    and acked, every follower in StateReplicate at match 3 with nothing in
    flight; pendingConfIndex 2 (becomeLeader takes lastIndex before the
    empty entry, raft.go:745-757), applied 3.  Node 1 then proposes its own
    removal (a conf-change entry at 4) and entries 5 and 6; applying 4
    removes its Progress (tracked and Voters lose slot 0) and
    switchToConfig returns early for a removed leader (raft.go:1663-1674).
    From then on the commit quorum is {2, 3} alone (6 waits for node 3),
    its proposals are dropped (no Progress of its own, raft.go:1023-1028),
    and it still heartbeats both followers."""
    cmds = traces()["confchange_v1_remove_leader.txt"]["commands"]
    st = command(cmds, "log-level debug")
    L = leader_factory(1, 3)
    rep = {"match": 3, "next": 4, "pending": 0, "state": 1, "probe_sent": False,
           "recent_active": True, "ring": []}
    L.load(3, 3, [[2, 1]], 3, [dict(rep) for _ in range(3)], tracked=0b111, inc=0b111)
    L.be.pci, L.be.applied = 2, 3
    seen = []

    def after(block):
        if any(x.endswith("switched to configuration voters=(2 3)") for x in block["debug"]):
            L.be.set_config(tracked=0b110, inc=0b110)
            L.switch(SW_REMOVED)  # the removed leader returns at once (raft.go:1663-1674)
            seen.append(block)

    checked = L.replay(cmds, st["line"], after_ready=after, proposals=True)
    assert len(seen) == 1 and L.be.committed() == 6 and checked.get("proposals") == 3
    return checked


def confchange_v2_add_single_explicit(leader_factory, elector):
    """raft/testdata/confchange_v2_add_single_explicit.txt from `stabilize 1
    2`: the joint config (1 2)&&(1) entered explicitly (no AutoLeave), set up
    as in the implicit trace (pendingConfIndex 4, applied 4).  Then three
    conf-change proposals through qe_propose's MsgProp arm: "v3 v4 v5" while
    joint (refused: must leave first -> an empty normal entry at 5), the
    empty one that leaves (accepted at 6; pendingConfIndex 6), and, once
    that is applied, an empty one outside a joint config (refused: an empty
    entry at 7) -- the trace prints the refusals as INFO lines."""
    cmds = traces()["confchange_v2_add_single_explicit.txt"]["commands"]
    st = command(cmds, "stabilize 1 2")
    L = leader_factory(1, 2)
    peers = [{"match": 4, "next": 5, "pending": 0, "state": 1, "probe_sent": False,
              "recent_active": True, "ring": []},
             {"match": 0, "next": 4, "pending": 0, "state": 0, "probe_sent": False,
              "recent_active": True, "ring": []}]
    L.load(4, 4, [[2, 1]], 3, peers, snap_index=4, inc=0b11, out=0b01)
    L.be.pci, L.be.applied = 4, 4
    seen = []

    def after(block):
        for x in block["debug"]:
            if x.endswith("switched to configuration voters=(1 2)&&(1)"):
                L.switch(SW_PROBE)
                seen.append("enter")
            elif x.endswith("switched to configuration voters=(1 2)"):
                L.be.set_outgoing(0)
                L.be.applied = 6
                L.switch(SW_PROBE)
                seen.append("leave")

    checked = L.replay(cmds, st["line"], after_ready=after, proposals=True)
    assert seen == ["enter", "leave"] and L.be.committed() == 7 and checked.get("proposals") == 3
    return checked


def confchange_v2_add_double_auto(leader_factory, elector):
    """raft/testdata/confchange_v2_add_double_auto.txt from `process-ready
    1`: voters 2 and 3 added through the joint config (1 2 3)&&(1) with
    AutoLeave, then both removed again through (1)&&(1 2 3).  Restated at
    the first Ready's application of 4 (as the add_single traces, two new
    peers; pendingConfIndex 4, applied 4); the host work after each Ready
    that switches configs is the reference's: switchToConfig's probe of
    every peer (raft.go:1682-1692), advance()'s auto-leave appendEntry with
    pendingConfIndex at it (raft.go:549-569), the new voter masks, and the
    snapshot index, which the interaction env takes at the applied index.
    The removals' proposal and two entries go through qe_propose; the joint
    quorum (1)&&(1 2 3) commits 7 and 8 one ack at a time; after the last
    switch the responses of the removed peers are not stepped (RawNode.Step:
    no Progress for a response's sender, rawnode.go:108-119) -- here, slots
    no longer tracked."""
    cmds = traces()["confchange_v2_add_double_auto.txt"]["commands"]
    st = command(cmds, "process-ready 1")
    L = leader_factory(1, 3)
    new = {"match": 0, "next": 4, "pending": 0, "state": 0, "probe_sent": False,
           "recent_active": True, "ring": []}
    peers = [{"match": 4, "next": 5, "pending": 0, "state": 1, "probe_sent": False,
              "recent_active": True, "ring": []}, dict(new), dict(new)]
    L.load(4, 4, [[2, 1]], 3, peers, snap_index=4, tracked=0b111, inc=0b111, out=0b001)
    L.be.pci, L.be.applied = 4, 4
    seen = []

    def auto_leave():
        out = L.be.propose(1, append_only=True)
        assert out["result"] == 1, out
        L.be.pci = L.be.last_index()

    def after(block):
        for x in block["debug"]:
            if x.endswith("switched to configuration voters=(1 2 3)&&(1) autoleave"):
                L.switch(SW_PROBE)
                auto_leave()  # at 5
                seen.append(x)
            elif x.endswith("switched to configuration voters=(1 2 3)"):
                L.be.set_outgoing(0)
                L.be.applied = 5
                L.be.set_snapshot(5)
                L.switch(SW_PROBE)
                seen.append(x)
            elif x.endswith("switched to configuration voters=(1)&&(1 2 3) autoleave"):
                L.be.set_config(tracked=0b111, inc=0b001)
                L.be.set_outgoing(0b111)
                L.be.applied = 6
                L.be.set_snapshot(6)
                L.switch(SW_PROBE)
                auto_leave()  # at 9
                seen.append(x)
            elif x.endswith("switched to configuration voters=(1)"):
                L.be.set_config(tracked=0b001, inc=0b001)
                L.be.set_outgoing(0)
                L.be.applied = 9
                L.switch(SW_PROBE)
                seen.append(x)

    checked = L.replay(cmds, st["line"], after_ready=after, proposals=True)
    assert len(seen) == 4 and L.be.committed() == 9 and checked.get("proposals") == 3
    return checked


confchange_v1_add_single = _confchange_add_single("confchange_v1_add_single.txt")
confchange_v2_add_single_auto = _confchange_add_single("confchange_v2_add_single_auto.txt")

TRACES = [probe_and_replicate, snapshot_succeed_via_app_resp, campaign,
          campaign_learner_must_vote, confchange_v1_add_single, confchange_v2_add_single_auto,
          confchange_v2_add_double_implicit, confchange_v2_add_single_explicit,
          confchange_v2_add_double_auto, confchange_v1_remove_leader]
