"""The Progress state-machine oracle (oracle/quorum_oracle.c, SURVEY.md
§8(f) rows 3-4) pinned to the reference's own tables: TestProgressMaybeDecr,
IsPaused, BecomeProbe/Replicate/Snapshot, Resume, the Inflights tests and the
leader side of TestFastLogRejection."""
import numpy as np

from oracle import orc
from tests.golden_util import raft_tables

T = raft_tables()
PF_PROBE_SENT, PF_RECENT_ACTIVE = 4, 8


def log_runs(entries, extra=None):
    """[(index, term)] (+ an appended entry) -> run_first, run_term arrays with
    run 0 at the dummy index 0 (term 0), as MemoryStorage starts."""
    ents = sorted(entries + ([extra] if extra else []))
    first, term = [0], [0]
    for i, t in ents:
        if t != term[-1]:
            first.append(i)
            term.append(t)
    return np.array(first, np.uint64), np.array(term, np.uint64), ents[-1][0]


def test_maybe_decr_table(orc):
    L = orc.lib()
    for r in T["TestProgressMaybeDecr"]["rows"]:
        m = np.array([r["match"]], np.uint64)
        n = np.array([r["next"]], np.uint64)
        ok = L.orc_pr_maybe_decr_to(r["state"], orc.P(m), orc.P(n), r["rejected"], r["last"])
        assert (bool(ok), int(m[0]), int(n[0])) == (r["want"], r["match"], r["want_next"]), r


def test_is_paused_table(orc):
    for r in T["TestProgressIsPaused"]["rows"]:
        assert bool(orc.lib().orc_pr_is_paused(r["state"], r["probe_sent"], 0, 256)) == r["want"], r


def test_become_probe_table(orc):
    for r in T["TestProgressBecomeProbe"]["rows"]:
        assert orc.lib().orc_pr_become_probe(r["state"], r["match"], r["next"], r["pending"]) == r["want_next"]


def test_inflights_tables(orc):
    for case in T["Inflights"]["rows"]:
        size = case["size"]
        start = np.array([case["start"]], np.uint32)
        count = np.array([0], np.uint32)
        buf = np.zeros(size, np.uint64)
        for st in case["steps"]:
            ops = np.array(st["ops"], np.int64)
            orc.lib().orc_inflights_ops(size, orc.P(start), orc.P(count), orc.P(buf), orc.P(ops),
                                        len(ops))
            assert (int(start[0]), int(count[0])) == (st["start"], st["count"]), case["name"]
            assert buf.tolist() == st["buffer"], case["name"]


def _one_group(F=16):
    pb = orc.ProgressBatch(1, 1, F, 16)
    return pb


def test_fast_log_rejection_leader_side(orc):
    """raft_test.go TestFastLogRejection, leader side, through the batch
    runner: becomeLeader appends an empty entry at term 1 (the test's fresh
    raft is at term 0 -> campaign -> term 1); the follower's heartbeat
    response triggers a probe MsgApp at Index = lastIndex-1; its rejection
    (hint index / log term) goes through findConflictByTerm + MaybeDecrTo and
    the sendAppend inside the step emits the next MsgApp, whose (Index,
    LogTerm) must match the test."""
    L = orc.lib()
    for r in T["TestFastLogRejection"]["rows"]:
        lead = [tuple(e) for e in r["leader_log"]]
        l_last = max(i for i, _ in lead)
        rf, rt, last = log_runs(lead, (l_last + 1, 1))
        pb = _one_group()
        pb.run_first[: len(rf)] = rf
        pb.run_term[: len(rt)] = rt
        pb.run_count[0] = len(rf)
        pb.first_index[0], pb.last_index[0] = 1, last
        pb.term_start[0] = l_last + 1
        pb.next[0], pb.match[0] = l_last + 1, 0  # reset(): Next = lastIndex+1 before the append
        z = lambda v: np.array([v], np.uint64)
        # heartbeat response -> sendAppend: probe at Index = Next-1 = l_last
        o = orc.progress_step(pb, np.array([3], np.uint8), z(0), z(0), z(0))
        assert o.sent[0] == 1 and o.msg_count[0] == 1 and o.msg_index[0] == l_last
        assert pb.flags[0] & PF_PROBE_SENT
        # rejection of that probe -> next MsgApp
        o = orc.progress_step(pb, np.array([2], np.uint8), z(l_last),
                              z(r["reject_hint_index"]), z(r["reject_hint_term"]))
        assert o.sent[0] == 1 and o.msg_count[0] == 1
        idx = int(o.msg_index[0])
        assert idx == int(pb.next[0]) - 1
        term = L.orc_log_term(len(rf), orc.P(rf), orc.P(rt), last, idx)
        assert (idx, term) == (r["next_append_index"], r["next_append_term"]), r


def test_progress_scenarios_on_oracle(orc):
    """Every leader-side scenario of tests/golden/progress_scenarios.json
    (TestLeaderAppResp, TestSendAppendForProgress*, TestProvideSnap, the
    raft_snap_test.go tests, ...) through the oracle."""
    from tests.progress_scenarios import OracleBackend, run_scenario, scenarios
    names = []
    for sc in scenarios():
        run_scenario(sc, OracleBackend(orc))
        names.append(sc["name"])
    assert len(names) == 23


def test_send_if_empty_precedes_snapshot(orc):
    """raft.go:440-469: with sendIfEmpty=false and Next < firstIndex there are
    no entries, so maybeSendAppend returns false BEFORE the snapshot branch
    (no MsgSnap, the Progress stays in its state)."""
    pb = orc.ProgressBatch(1, 1, 8, 1)
    pb.first_index[0], pb.last_index[0] = 10, 20
    pb.next[0], pb.match[0] = 5, 4
    pb.set_peer(flags=0 | PF_RECENT_ACTIVE)  # Probe, recently active
    w = np.array([1], np.uint8)
    sent, snap = orc.progress_send(pb, w, 0, 0)
    assert sent[0] == 0 and snap[0] == 0 and pb.flags[0] & 3 == 0 and pb.pending[0] == 0
    sent, snap = orc.progress_send(pb, w, 1, 0)
    assert sent[0] == 1 and snap[0] == 1 and pb.flags[0] & 3 == 2 and pb.pending[0] == 9


def test_find_conflict_by_term_jump_equals_walk(orc):
    """The device walks term runs instead of single indexes; restate that
    jump form here and check it against the linear loop of log.go:147-168."""
    rng = np.random.default_rng(1)
    L = orc.lib()
    for _ in range(2000):
        R = int(rng.integers(1, 6))
        first = np.sort(rng.choice(np.arange(0, 40), R, replace=False)).astype(np.uint64)
        term = rng.integers(0, 8, R).astype(np.uint64)
        last = int(first[-1] + rng.integers(0, 5))
        index = int(rng.integers(0, last + 3))
        t = int(rng.integers(1, 9))
        walk = L.orc_find_conflict_by_term(R, orc.P(first), orc.P(term), last, index, t)
        # jump form (qe_kernels.hpp find_conflict_by_term)
        if index > last or index < first[0]:
            jump = index
        else:
            r = R - 1
            while r > 0 and first[r] > index:
                r -= 1
            jump = None
            while r >= 0:
                if term[r] <= t:
                    jump = index
                    break
                index = int(first[r]) - 1 if first[r] > 0 else (1 << 64) - 1
                r -= 1
            if jump is None:
                jump = index
        assert walk == jump


def test_readindex_and_checkquorum_scenarios_on_oracle(orc):
    """TestReadOnlyOptionSafe, TestReadOnlyWithLearner (+ the learner-ack
    rule), TestLeaderStepdownWhenQuorumActive / ...Lost, leader side,
    through the oracle's ReadIndex ack and CheckQuorum
    (tests/leader_round_scenarios.py)."""
    from tests.leader_round_scenarios import SCENARIOS, OracleRoundBackend
    for sc in SCENARIOS:
        sc(OracleRoundBackend(orc))


def test_byte_accounting_rules_on_oracle(orc):
    """The oracle's algorithmic byte count of a round on a hand-checked
    state: one group, S = 2 (leader slot 0, one follower in StateReplicate
    with an empty ring), the follower acks index 5 of a 5-entry log in the
    leader's term.  Reads: self_slot 1 + the log model and commit 32, per
    slot Match 8 + message kind 1 (both tracked), the follower's m.Index 8
    and its Next + packed word 12; writes: its Match 8 (Next stays 6, the
    word stays Replicate|RecentActive with an empty ring) and the commit 8;
    no optional outputs."""
    pb = orc.ProgressBatch(1, 2, 8, 1, max_ents=0)
    pb.first_index[0], pb.last_index[0], pb.term_start[0] = 1, 5, 1
    pb.run_count[0] = 1
    pb.match[:] = [5, 3]
    pb.next[:] = [6, 6]
    pb.set_peer(flags=np.array([1 | 8, 1 | 8], np.uint8), istart=0, icount=np.array([0, 0]))
    pb.self_slot = np.array([0], np.uint8)
    z = np.zeros(2, np.uint64)
    o = orc.progress_step(pb, np.array([0, 1], np.uint8), np.array([0, 5], np.uint64), z, z,
                          outputs=False, count_bytes=True)
    # commit advanced 0 -> 5: bcastAppend to slot 1 (Next 6 > lastIndex: an
    # empty MsgApp, nothing appended); the ack's FreeLE on an empty ring
    # reads nothing; the word is unchanged (Replicate, RecentActive, empty)
    want = (1 + 32) + (8 + 1) + (8 + 1 + 8) + 12 + 8 + 8
    assert int(pb.committed[0]) == 5 and int(pb.match[1]) == 5
    assert int(o.bytes[0]) == want, (int(o.bytes[0]), want)
