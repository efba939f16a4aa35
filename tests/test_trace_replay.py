"""The reference's interaction traces (raft/testdata/probe_and_replicate.txt,
snapshot_succeed_via_app_resp.txt, campaign.txt,
campaign_learner_must_vote.txt, confchange_v1_add_single.txt,
confchange_v2_add_single_auto.txt, confchange_v2_add_double_implicit.txt) replayed from the leader's side through the
oracle (tests/trace_replay.py); tests/test_gpu_trace_replay.py runs the same
replay through the HIP engine."""
import numpy as np
import pytest

from tests.leader_round_scenarios import OracleRoundBackend
from tests.trace_replay import (F_TRACE, TRACES, Leader, parse_progress, progress_string,
                                traces)


def oracle_elector(orc):
    def make(S, self_slot, term0):
        md = orc.mask_dtype(S)
        term = np.array([term0], np.uint64)
        state = np.zeros(1, np.uint8)
        voted, granted = np.zeros(1, md), np.zeros(1, md)
        self_a = np.array([self_slot], np.uint8)
        inc = np.array([(1 << S) - 1], md)
        k = [0]

        def step(resp, grant, hup):
            script = (np.array([resp], md), np.array([grant], md), np.array([hup], np.uint8), 1)
            orc.election_steps(1, 0, S, term, state, voted, granted, self_a, inc, None,
                               np.zeros(1, md), 0, k[0], 1, 0, 0, script=script)
            k[0] += 1
            return int(term[0]), int(state[0])
        return step
    return make


@pytest.mark.parametrize("trace", TRACES, ids=lambda f: f.__name__)
def test_trace_replay_on_oracle(orc, trace):
    checked = trace(lambda node, S: Leader(OracleRoundBackend(orc), node, S),
                    oracle_elector(orc))
    assert checked["rounds"] > 0 and checked["sends"] > 0


def test_trace_fixture_counts():
    t = traces()
    assert set(t) == {"probe_and_replicate.txt", "snapshot_succeed_via_app_resp.txt",
                      "campaign.txt", "campaign_learner_must_vote.txt",
                      "confchange_v1_add_single.txt", "confchange_v2_add_single_auto.txt",
                      "confchange_v2_add_double_implicit.txt", "confchange_v1_remove_leader.txt",
                      "confchange_v2_add_single_explicit.txt", "confchange_v2_add_double_auto.txt"}
    pr = t["probe_and_replicate.txt"]["commands"]
    rejects = [m for c in pr for b in c["blocks"] if b["kind"] == "recv" and b["node"] == 1
               for m in b["msgs"] if m["type"] == "MsgAppResp" and m["reject"]]
    # followers 2, 3, 5, 6, 7 reject the new leader's first probe (4 accepts)
    assert sorted(m["from"] for m in rejects) >= [2, 3, 5, 6, 7]


def test_progress_string_round_trip():
    """progress_string restates tracker.Progress.String; the status lines of
    the snapshot trace parse and render back to themselves."""
    for c in traces()["snapshot_succeed_via_app_resp.txt"]["commands"]:
        for b in c["blocks"]:
            if b["kind"] == "status":
                for text in b["progress"].values():
                    p = parse_progress(text)
                    view = dict(p, inflights=len(p["ring"]))
                    assert progress_string(view, F_TRACE) == text


def _mutated(monkeypatch, name, edit):
    """The fixture with one printed value changed (a deep copy), installed
    where the replay reads it."""
    import copy

    import tests.trace_replay as tr
    t = copy.deepcopy(traces())
    edit(t[name]["commands"])
    monkeypatch.setattr(tr, "traces", lambda: t)


def _first(cmds, pred):
    for c in cmds:
        for b in c["blocks"]:
            for m in b.get("msgs", []):
                if pred(b, m):
                    return m
    raise LookupError("no such message in the fixture")


@pytest.mark.parametrize("what", ["reply_index", "reject_hint", "status_line", "snap_index",
                                  "paused_line", "dropped_proposal", "ignored_cc"])
def test_trace_replay_detects_a_changed_value(orc, monkeypatch, what):
    """Negative controls: the replay fails when one printed value differs
    from what the engine computes -- the index of the MsgApp answering a
    rejection, the hint a rejection carries (the engine then answers from a
    different probe), a Progress line of a `status` block, the snapshot
    index of the MsgSnap to a newly added voter, the Progress a "paused
    sending" DEBUG line prints, a removed leader's proposal printed as
    accepted, a refused conf change printed as accepted."""
    from tests.trace_replay import (confchange_v1_add_single, confchange_v1_remove_leader,
                                    confchange_v2_add_single_explicit, probe_and_replicate,
                                    snapshot_succeed_via_app_resp)
    if what == "ignored_cc":
        def edit(cmds):
            c = next(c for c in cmds if c.get("ignored_cc"))
            c["ignored_cc"] = False
        name, trace = "confchange_v2_add_single_explicit.txt", confchange_v2_add_single_explicit
    elif what == "dropped_proposal":
        def edit(cmds):
            c = next(c for c in cmds if c.get("dropped"))
            c["dropped"] = False
        name, trace = "confchange_v1_remove_leader.txt", confchange_v1_remove_leader
    elif what == "snap_index":
        def edit(cmds):
            m = _first(cmds, lambda b, m: b["kind"] == "ready" and b["node"] == 1
                       and m["type"] == "MsgSnap")
            m["snap_index"] = 3
        name, trace = "confchange_v1_add_single.txt", confchange_v1_add_single
    elif what == "paused_line":
        def edit(cmds):
            for c in cmds:
                for b in c["blocks"]:
                    for i, x in enumerate(b.get("debug", [])):
                        if "paused sending replication messages to 2" in x:
                            b["debug"][i] = x.replace("pendingSnap=4", "pendingSnap=3")
                            return
            raise LookupError("paused line not found")
        name, trace = "confchange_v1_add_single.txt", confchange_v1_add_single
    elif what == "reply_index":
        def edit(cmds):
            m = _first(cmds, lambda b, m: b["kind"] == "ready" and b["node"] == 1
                       and m["type"] == "MsgApp" and m["to"] == 2 and m["index"] == 19)
            m["index"] = 18
        name, trace = "probe_and_replicate.txt", probe_and_replicate
    elif what == "reject_hint":
        def edit(cmds):
            m = _first(cmds, lambda b, m: b["kind"] == "recv" and b["node"] == 1
                       and m["type"] == "MsgAppResp" and m["reject"])
            m["hint"] = m["hint"] - 2
        name, trace = "probe_and_replicate.txt", probe_and_replicate
    else:
        def edit(cmds):
            for c in cmds:
                for b in c["blocks"]:
                    if b["kind"] == "status" and "pendingSnap=11" in b["progress"].get("3", ""):
                        b["progress"]["3"] = b["progress"]["3"].replace("pendingSnap=11",
                                                                        "pendingSnap=12")
                        return
            raise LookupError("status line not found")
        name, trace = "snapshot_succeed_via_app_resp.txt", snapshot_succeed_via_app_resp
    _mutated(monkeypatch, name, edit)  # (LookupError, not a pass, if the value moved)
    with pytest.raises(AssertionError):
        trace(lambda node, S: Leader(OracleRoundBackend(orc), node, S), oracle_elector(orc))


@pytest.mark.parametrize("trace", TRACES, ids=lambda f: f.__name__)
def test_trace_replay_in_tiles_on_oracle(trace):
    """The tile replay of tests/test_gpu_trace_tiles.py with the oracle alone:
    the trace's group at lane 37 of a 192-group batch of random groups with
    F = 8 (the GPU test compares the engine with this, group by group)."""
    from tests.test_gpu_trace_tiles import TileBackend
    checked = trace(lambda node, S: Leader(TileBackend(None, 37, seed=5), node, S),
                    oracle_elector(__import__("oracle.orc", fromlist=["orc"])))
    assert checked["rounds"] > 0 and checked["sends"] > 0
