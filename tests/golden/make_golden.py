#!/usr/bin/env python3
"""Extract the reference's own golden vectors for the quorum hot path into
small data fixtures under tests/golden/.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box):  python tests/golden/make_golden.py

Sources (read as text; nothing from the reference is executed):
  * raft/quorum/testdata/{majority_commit,majority_vote,joint_commit,
    joint_vote}.txt -- the datadriven cases of TestDataDriven
    (raft/quorum/datadriven_test.go:36-250).  File format is that of
    github.com/cockroachdb/datadriven v0.0.0-20200714090401-bf6692d28da5
    (raft/go.mod:7, not vendored): a command line, "----", then output lines
    up to the first blank line.  Value->voter mapping follows makeLookuper
    (datadriven_test.go:122-150): values go to cfg ids then unseen cfgj ids;
    "_" (idx) / "_" (votes) means absent; 0 is forbidden as an idx (:87).
  * TestCommit table, raft/raft_test.go:1127-1152.
  * TestLeaderElectionInOneRoundRPC table, raft/raft_paper_test.go:192-216.
  * TestProgressUpdate table, raft/tracker/progress_test.go:149-161.
  * TestProgressMaybeDecr / IsPaused / BecomeProbe / BecomeReplicate /
    BecomeSnapshot / Resume, raft/tracker/progress_test.go:40-245.
  * TestInflightsAdd / TestInflightFreeTo / TestInflightFreeFirstOne
    (raft/tracker/inflights_test.go:22-190), transcribed as op sequences.
  * TestFastLogRejection leader-side rows, raft/raft_test.go:4319-4540.
  * raft/confchange/testdata/*.txt -- TestConfChangeDataDriven
    (raft/confchange/datadriven_test.go:29-98): per file, the command
    sequence (simple / enter-joint [autoleave=..] / leave-joint), its input
    tokens (vN voter, lN learner, rN remove, uN update) and the expected
    output lines (Config.String + ProgressMap.String, or the error text).

Outputs (data only: inputs + expected outputs):
  tests/golden/quorum_testdata.jsonl   127 rows
  tests/golden/raft_tables.json        the three tables
  tests/golden/confchange_testdata.json  9 files of confchange steps
  tests/golden/confchange_testdata.txt   the same, tab-separated (C++ test)
  tests/golden/progress_scenarios.json  leader-side Progress scenarios:
    TestLeaderAppResp (table), TestSendAppendForProgressProbe/Replicate/
    Snapshot, TestLeaderIncreaseNext, TestRecvMsgUnreachable,
    TestMsgAppRespWaitReset, TestProvideSnap, TestIgnoreProvidingSnap,
    raft_snap_test.go's five tests, and the leader side of
    TestLeaderTransferToSlowFollower -- state set up by the tests' code is
    restated per scenario (see progress_scenarios()).
  tests/golden/interaction_traces.json  raft/testdata/{probe_and_replicate,
    snapshot_succeed_via_app_resp,campaign,campaign_learner_must_vote}.txt
    (raft/interaction_test.go): per command its printed blocks -- the
    messages each node received, the Ready it handled (HardState commit,
    entries, messages sent: DescribeMessage fields) and `status` Progress
    strings; tests/trace_replay.py replays the leaders' side.
  tests/golden/election_scenarios.json  scripted election steps:
    TestLeaderElectionInOneRoundRPC (table), TestLeaderStepdownWhenQuorumLost,
    TestPreVoteWithSplitVote (node views derived from the test's flow).
"""
import json
import os
import re
import sys

REF = "/root/reference/raft"
HERE = os.path.dirname(os.path.abspath(__file__))
INF = (1 << 64) - 1
VOTES = {"VotePending": 1, "VoteLost": 2, "VoteWon": 3}


def parse_args(line):
    """`committed cfg=(1,2) cfgj=zero idx=(_, 5)` -> (cmd, {key: [vals]})."""
    cmd, _, rest = line.partition(" ")
    args = {}
    for m in re.finditer(r"(\w+)=(\([^)]*\)|\S+)", rest):
        key, val = m.group(1), m.group(2)
        if val.startswith("("):
            vals = [v.strip() for v in val[1:-1].split(",") if v.strip() != ""]
        else:
            vals = [val]
        args[key] = vals
    return cmd, args


def parse_datadriven(path):
    with open(path, encoding="utf-8") as f:
        lines = f.read().split("\n")
    cases = []
    i = 0
    while i < len(lines):
        line = lines[i]
        if line.startswith("committed") or line.startswith("vote"):
            lineno = i + 1
            assert lines[i + 1] == "----", (path, lineno)
            j = i + 2
            out = []
            while j < len(lines) and lines[j] != "":
                out.append(lines[j])
                j += 1
            cases.append((lineno, line, out))
            i = j
        else:
            i += 1
    return cases


def resolve(cmd, args):
    ids = [int(v) for v in args.get("cfg", [])]
    joint = "cfgj" in args
    idsj = [] if args.get("cfgj") == ["zero"] else [int(v) for v in args.get("cfgj", [])]
    key = "idx" if cmd == "committed" else "votes"
    raw = args.get(key, [])
    if cmd == "committed":
        vals = [0 if v == "_" else int(v) for v in raw]
        assert all(v != 0 for v, r in zip(vals, raw) if r != "_")
    else:
        vals = [{"y": 2, "n": 1, "_": 0}[v] for v in raw]
    # makeLookuper: ids then idsj, skipping repeats, zero entries dropped.
    lookup = {}
    p = 0
    for vid in ids + idsj:
        if vid in lookup:
            continue
        if p < len(vals):
            lookup[vid] = vals[p]
            p += 1
    lookup = {k: v for k, v in lookup.items() if v != 0}
    voters = set(ids) | set(idsj)
    assert len(voters) == len(vals), "mismatched input"
    return ids, idsj, joint, lookup


def expected(cmd, out):
    last = out[-1]
    assert "<--" not in "\n".join(out), "golden case carries a mismatch annotation"
    assert not last.startswith("error"), last
    if cmd == "committed":
        if last.endswith("∞"):
            return INF, last
        return int(last.split()[-1]), last
    return VOTES[last.strip()], last


def datadriven_rows():
    rows = []
    for name in ["majority_commit.txt", "majority_vote.txt", "joint_commit.txt", "joint_vote.txt"]:
        for lineno, line, out in parse_datadriven(os.path.join(REF, "quorum", "testdata", name)):
            cmd, args = parse_args(line)
            ids, idsj, joint, lookup = resolve(cmd, args)
            exp, text = expected(cmd, out)
            row = {
                "source": f"raft/quorum/testdata/{name}:{lineno}",
                "cmd": cmd,
                "cfg": ids,
                "cfgj": idsj,
                "joint": joint,
                "expect": exp,
                "expect_text": text,
            }
            if cmd == "committed":
                row["acked"] = sorted([k, v] for k, v in lookup.items())
                # the harness prints c.Describe(l) and then the index
                # (datadriven_test.go:172, :216): every line but the last
                # is Describe's text (for the empty config the two share it)
                if out[-1].startswith("<empty majority quorum>"):
                    row["describe"] = "<empty majority quorum>"
                else:
                    row["describe"] = "\n".join(out[:-1]) + "\n"
            else:
                row["votes"] = sorted([k, v == 2] for k, v in lookup.items())
            rows.append(row)
    return rows


def test_commit_table():
    src = open(os.path.join(REF, "raft_test.go"), encoding="utf-8").read()
    start = src.index("func TestCommit(t *testing.T)")
    body = src[start:src.index("for i, tt := range tests", start)]
    rows = []
    for m in re.finditer(r"\{\[\]uint64\{([\d, ]+)\}, \[\]pb\.Entry\{(.*)\}, (\d+), (\d+)\},", body):
        matches = [int(x) for x in m.group(1).split(",")]
        ents = [[int(a), int(b)] for a, b in re.findall(r"\{Index: (\d+), Term: (\d+)\}", m.group(2))]
        rows.append({"matches": matches, "logs": ents, "sm_term": int(m.group(3)), "want": int(m.group(4))})
    assert len(rows) == 14, len(rows)
    return rows


def election_table():
    src = open(os.path.join(REF, "raft_paper_test.go"), encoding="utf-8").read()
    start = src.index("func TestLeaderElectionInOneRoundRPC(t *testing.T)")
    body = src[start:src.index("for i, tt := range tests", start)]
    rows = []
    for m in re.finditer(r"\{(\d+), map\[uint64\]bool\{([^}]*)\}, (State\w+)\},", body):
        votes = [[int(a), b == "true"] for a, b in re.findall(r"(\d+): (true|false)", m.group(2))]
        rows.append({"size": int(m.group(1)), "votes": votes, "state": m.group(3)})
    assert len(rows) == 13, len(rows)
    return rows


def progress_update_table():
    src = open(os.path.join(REF, "tracker", "progress_test.go"), encoding="utf-8").read()
    start = src.index("func TestProgressUpdate(t *testing.T)")
    body = src[start:src.index("for i, tt := range tests", start)]
    pm = int(re.search(r"prevM, prevN := uint64\((\d+)\), uint64\((\d+)\)", body).group(1))
    pn = int(re.search(r"prevM, prevN := uint64\((\d+)\), uint64\((\d+)\)", body).group(2))

    def ev(expr):
        expr = expr.replace("prevM", str(pm)).replace("prevN", str(pn)).replace(" ", "")
        toks = re.findall(r"[+-]?\d+", expr)
        return sum(int(t) for t in toks)

    rows = []
    for m in re.finditer(r"\{(prev[MN][^,]*), (prev[MN][^,]*), (prev[MN][^,]*), (true|false)\}", body):
        rows.append({"prev_match": pm, "prev_next": pn, "update": ev(m.group(1)),
                     "want_match": ev(m.group(2)), "want_next": ev(m.group(3)),
                     "want_ok": m.group(4) == "true"})
    assert len(rows) == 4, len(rows)
    return rows


STATES = {"StateProbe": 0, "StateReplicate": 1, "StateSnapshot": 2}


def _body(path, fn):
    src = open(os.path.join(REF, path), encoding="utf-8").read()
    start = src.index(f"func {fn}(t *testing.T)")
    end = src.index("\n}\n", start)
    return src[start:end]


def progress_tables():
    out = {}
    b = _body("tracker/progress_test.go", "TestProgressMaybeDecr")
    rows = []
    for m in re.finditer(r"(State\w+), (\d+), (\d+), (\d+), (\d+), (true|false), (\d+),", b):
        rows.append({"state": STATES[m.group(1)], "match": int(m.group(2)), "next": int(m.group(3)),
                     "rejected": int(m.group(4)), "last": int(m.group(5)),
                     "want": m.group(6) == "true", "want_next": int(m.group(7))})
    assert len(rows) == 10, len(rows)
    out["TestProgressMaybeDecr"] = {"source": "raft/tracker/progress_test.go:181-245", "rows": rows}
    b = _body("tracker/progress_test.go", "TestProgressIsPaused")
    rows = [{"state": STATES[a], "probe_sent": p == "true", "want": w == "true"}
            for a, p, w in re.findall(r"\{(State\w+), (true|false), (true|false)\}", b)]
    assert len(rows) == 6, len(rows)
    out["TestProgressIsPaused"] = {"source": "raft/tracker/progress_test.go:40-66", "rows": rows}
    b = _body("tracker/progress_test.go", "TestProgressBecomeProbe")
    match = int(re.search(r"match := uint64\((\d+)\)", b).group(1))
    rows = []
    for m in re.finditer(r"&Progress\{State: (State\w+), Match: match, Next: (\d+),"
                         r"(?: PendingSnapshot: (\d+),)? Inflights: NewInflights\(256\)\},\s*(\d+),", b):
        rows.append({"state": STATES[m.group(1)], "match": match, "next": int(m.group(2)),
                     "pending": int(m.group(3) or 0), "want_next": int(m.group(4))})
    assert len(rows) == 3, len(rows)
    out["TestProgressBecomeProbe"] = {"source": "raft/tracker/progress_test.go:84-117", "rows": rows}
    # single-case tests, transcribed (progress_test.go:68-82, :119-147)
    out["TestProgressBecomeReplicate"] = {"source": "raft/tracker/progress_test.go:119-132",
                                          "rows": [{"state": 0, "match": 1, "next": 5,
                                                    "want_state": 1, "want_next": 2}]}
    out["TestProgressBecomeSnapshot"] = {"source": "raft/tracker/progress_test.go:134-147",
                                         "rows": [{"state": 0, "match": 1, "next": 5, "snap": 10,
                                                   "want_state": 2, "want_pending": 10}]}
    out["TestProgressResume"] = {"source": "raft/tracker/progress_test.go:68-82",
                                 "rows": [{"next": 2, "decr_rejected": 1, "decr_hint": 1,
                                           "update": 2, "want_probe_sent": False}]}
    return out


def inflights_tables():
    """inflights_test.go:22-190 as op sequences: op >= 0 Add(op), -1
    FreeFirstOne, -(k+2) FreeLE(k); each check lists the expected
    (start, count, buffer)."""
    return {"source": "raft/tracker/inflights_test.go:22-190", "rows": [
        {"name": "TestInflightsAdd/no-rotate", "size": 10, "start": 0,
         "steps": [{"ops": [0, 1, 2, 3, 4], "start": 0, "count": 5,
                    "buffer": [0, 1, 2, 3, 4, 0, 0, 0, 0, 0]},
                   {"ops": [5, 6, 7, 8, 9], "start": 0, "count": 10,
                    "buffer": [0, 1, 2, 3, 4, 5, 6, 7, 8, 9]}]},
        {"name": "TestInflightsAdd/rotate", "size": 10, "start": 5,
         "steps": [{"ops": [0, 1, 2, 3, 4], "start": 5, "count": 5,
                    "buffer": [0, 0, 0, 0, 0, 0, 1, 2, 3, 4]},
                   {"ops": [5, 6, 7, 8, 9], "start": 5, "count": 10,
                    "buffer": [5, 6, 7, 8, 9, 0, 1, 2, 3, 4]}]},
        {"name": "TestInflightFreeTo", "size": 10, "start": 0,
         "steps": [{"ops": list(range(10)) + [-(4 + 2)], "start": 5, "count": 5,
                    "buffer": list(range(10))},
                   {"ops": [-(8 + 2)], "start": 9, "count": 1, "buffer": list(range(10))},
                   {"ops": [10, 11, 12, 13, 14, -(12 + 2)], "start": 3, "count": 2,
                    "buffer": [10, 11, 12, 13, 14, 5, 6, 7, 8, 9]},
                   {"ops": [-(14 + 2)], "start": 0, "count": 0,
                    "buffer": [10, 11, 12, 13, 14, 5, 6, 7, 8, 9]}]},
        {"name": "TestInflightFreeFirstOne", "size": 10, "start": 0,
         "steps": [{"ops": list(range(10)) + [-1], "start": 1, "count": 9,
                    "buffer": list(range(10))}]},
    ]}


def fast_log_rejection_table():
    b = _body("raft_test.go", "TestFastLogRejection")
    table = b[:b.index("for i, test := range tests")]
    rows = []
    for case in re.split(r"\n\t\t\{\n", table)[1:]:
        lead = case[case.index("leaderLog:"):case.index("followerLog:")]
        ents = [[int(i), int(t)] for t, i in re.findall(r"\{Term: (\d+), Index: (\d+)\}", lead)]
        def val(k):
            return int(re.search(k + r":\s+(\d+)", case).group(1))
        rows.append({"leader_log": ents, "reject_hint_index": val("rejectHintIndex"),
                     "reject_hint_term": val("rejectHintTerm"),
                     "next_append_index": val("nextAppendIndex"),
                     "next_append_term": val("nextAppendTerm")})
    assert len(rows) == 8, len(rows)
    return {"source": "raft/raft_test.go:4319-4600 (leader side: heartbeat resp -> probe MsgApp "
                      "-> rejection -> next MsgApp)", "rows": rows}


# ---------------------------------------------------------------------------
# Leader-side Progress scenarios (stepLeader + maybeSendAppend).  These tests
# build their state with code (newTestRaft, becomeLeader, restore ...) rather
# than tables, so each scenario below restates the state that code produces
# (raft.go reset :590-619, becomeLeader :724-758, appendEntry :621-642,
# restore) for a single group: slot s is node id s+1, slot 0 is the leader.
# Inflights capacity: the tests use 256 (newTestConfig); the slot model caps it
# at 255, and no scenario fills the ring.  max_ents 0 = noLimit (the tests'
# MaxSizePerMsg).  Expectations are exactly what each test asserts, except
# where a scenario says "derived" (then they follow the test's message flow).
# ---------------------------------------------------------------------------
def _peer(match, nxt, state, probe_sent=False, recent_active=False, pending=0, ring=()):
    return {"match": match, "next": nxt, "state": STATES[state], "probe_sent": probe_sent,
            "recent_active": recent_active, "pending": pending, "ring": list(ring)}


def leader_app_resp_rows():
    b = _body("raft_test.go", "TestLeaderAppResp")
    rows = [(int(a), r == "true", int(wm), int(wn), int(k), int(wi), int(wc))
            for a, r, wm, wn, k, wi, wc in re.findall(
                r"\{(\d+), (true|false), (\d+), (\d+), (\d+), (\d+), (\d+)\},", b)]
    assert len(rows) == 4, rows
    return rows


def progress_scenarios():
    sc = []
    # TestLeaderAppResp (raft_test.go:2426-2480): log [1:t0, 2:t1] in storage,
    # becomeCandidate -> Term 1, becomeLeader appends 3:t1.  Peers reset to
    # Match 0 / Next 3 (Probe); the leader's own Progress Match 3 (Replicate).
    for i, (idx, rej, wm, wn, k, wi, wc) in enumerate(leader_app_resp_rows()):
        exp = {"peers": {"1": {"match": wm, "next": wn}}, "messages": k, "committed": wc}
        if k:
            exp["msg_index_all"] = wi
        sc.append({
            "name": f"TestLeaderAppResp#{i}", "source": "raft/raft_test.go:2426-2480",
            "S": 3, "self": 0, "max_ents": 0,
            "log": {"first_index": 1, "last_index": 3, "term_start": 2, "committed": 0,
                    "runs": [[0, 0], [2, 1]]},
            "peers": [_peer(3, 4, "StateReplicate"), _peer(0, 3, "StateProbe"),
                      _peer(0, 3, "StateProbe")],
            "steps": [{"op": "step", "msgs": {"1": {"type": "reject" if rej else "accept",
                                                    "index": idx, "hint": idx}},
                       "expect": exp}]})
    # TestSendAppendForProgressProbe (raft_test.go:2613-2678): fresh log,
    # becomeLeader appends 1:t1; node 2 in StateProbe, Next 1.
    steps = [{"op": "append"}, {"op": "send", "want": [1], "send_if_empty": 1,
                                 "expect": {"sent": [1], "peers": {"1": {"probe_sent": True}}}}]
    for _ in range(3):
        for _ in range(10):
            steps += [{"op": "append"}, {"op": "send", "want": [1], "send_if_empty": 1,
                                          "expect": {"sent": []}}]
        steps += [{"op": "check", "expect": {"peers": {"1": {"probe_sent": True}}}}]
    steps += [{"op": "step", "msgs": {"1": {"type": "heartbeat"}},
               "expect": {"messages": 1, "msg_index": {"1": 0},
                          "peers": {"1": {"probe_sent": True}}}}]
    base = {"S": 2, "self": 0, "max_ents": 0,
            "log": {"first_index": 1, "last_index": 1, "term_start": 1, "committed": 0,
                    "runs": [[0, 0], [1, 1]]}}
    sc.append(dict(base, name="TestSendAppendForProgressProbe",
                   source="raft/raft_test.go:2613-2678",
                   peers=[_peer(1, 2, "StateReplicate"), _peer(0, 1, "StateProbe")], steps=steps))
    # TestSendAppendForProgressReplicate (:2680-2695): BecomeReplicate -> Next 1
    steps = []
    for _ in range(10):
        steps += [{"op": "append"}, {"op": "send", "want": [1], "send_if_empty": 1,
                                      "expect": {"sent": [1]}}]
    sc.append(dict(base, name="TestSendAppendForProgressReplicate",
                   source="raft/raft_test.go:2680-2695",
                   peers=[_peer(1, 2, "StateReplicate"), _peer(0, 1, "StateReplicate")],
                   steps=steps))
    # TestSendAppendForProgressSnapshot (:2697-2712): BecomeSnapshot(10)
    steps = []
    for _ in range(10):
        steps += [{"op": "append"}, {"op": "send", "want": [1], "send_if_empty": 1,
                                      "expect": {"sent": []}}]
    sc.append(dict(base, name="TestSendAppendForProgressSnapshot",
                   source="raft/raft_test.go:2697-2712",
                   peers=[_peer(1, 2, "StateReplicate"), _peer(0, 1, "StateSnapshot", pending=10)],
                   steps=steps))
    # TestLeaderIncreaseNext (:2581-2611): log 1..3:t1, Term 1, becomeLeader
    # appends 4:t1; node 2 forced to (state, Next 2); MsgProp appends 5 ->
    # bcastAppend.
    b = _body("raft_test.go", "TestLeaderIncreaseNext")
    rows = re.findall(r"\{tracker\.(State\w+), (\d+), ([^}]+)\}", b)
    assert len(rows) == 2, rows
    for st, nxt, want in rows:
        want = eval(want.replace("uint64(len(previousEnts) + 1 + 1 + 1)", "3 + 1 + 1 + 1"))
        sc.append({"name": f"TestLeaderIncreaseNext/{st}", "source": "raft/raft_test.go:2581-2611",
                   "S": 2, "self": 0, "max_ents": 0,
                   "log": {"first_index": 1, "last_index": 4, "term_start": 1, "committed": 0,
                           "runs": [[0, 0], [1, 1]]},
                   "peers": [_peer(4, 5, "StateReplicate"), _peer(0, int(nxt), st)],
                   "steps": [{"op": "append"},
                             {"op": "send", "want": [1], "send_if_empty": 1,
                              "expect": {"peers": {"1": {"next": want}}}}]})
    # TestRecvMsgUnreachable (:2714-2735): log 1..3:t1 + 4:t1; node 2 Match 3,
    # BecomeReplicate (Next 4), OptimisticUpdate(5) (Next 6).
    sc.append({"name": "TestRecvMsgUnreachable", "source": "raft/raft_test.go:2714-2735",
               "S": 2, "self": 0, "max_ents": 0,
               "log": {"first_index": 1, "last_index": 4, "term_start": 1, "committed": 0,
                       "runs": [[0, 0], [1, 1]]},
               "peers": [_peer(4, 5, "StateReplicate"), _peer(3, 6, "StateReplicate")],
               "steps": [{"op": "step", "msgs": {"1": {"type": "unreachable"}},
                          "expect": {"peers": {"1": {"state": 0, "next": 4}}}}]})
    # TestMsgAppRespWaitReset (:1407-1465): 3 peers, becomeLeader appends 1:t1;
    # bcastAppend probes nodes 2 and 3; node 2 acks 1 (commit 1); MsgProp
    # appends 2 and broadcasts (only node 2 is not paused); node 3 acks 1.
    sc.append({"name": "TestMsgAppRespWaitReset", "source": "raft/raft_test.go:1407-1465",
               "S": 3, "self": 0, "max_ents": 0,
               "log": {"first_index": 1, "last_index": 1, "term_start": 1, "committed": 0,
                       "runs": [[0, 0], [1, 1]]},
               "peers": [_peer(1, 2, "StateReplicate"), _peer(0, 1, "StateProbe"),
                         _peer(0, 1, "StateProbe")],
               "steps": [{"op": "send", "want": [1, 2], "send_if_empty": 1, "expect": {}},
                         {"op": "step", "msgs": {"1": {"type": "accept", "index": 1}},
                          "expect": {"committed": 1}},
                         {"op": "append"},
                         {"op": "send", "want": [1, 2], "send_if_empty": 1,
                          "expect": {"sent": [1]}},
                         {"op": "step", "msgs": {"2": {"type": "accept", "index": 1}},
                          "expect": {"messages": 1, "msg_index": {"2": 1}}}]})
    # Snapshot tests: restore(snapshot index 11, term 11) -> committed 11,
    # firstIndex 12, lastIndex 11; becomeCandidate Term 1; becomeLeader appends
    # 12:t1 (node 2: Match 0, Next 12, Probe).
    snap_log = {"first_index": 12, "last_index": 12, "term_start": 12, "committed": 11,
                "runs": [[11, 11], [12, 1]], "snap_index": 11}
    lead = _peer(12, 13, "StateReplicate")
    # TestProvideSnap (:2986-3014) / TestSendingSnapshotSetPendingSnapshot
    # (raft_snap_test.go:33-49): Next forced to firstIndex; rejection of Index
    # Next-1 (hint 0) -> MaybeDecrTo -> Next 1 -> sendAppend -> MsgSnap.
    sc.append({"name": "TestProvideSnap", "source": "raft/raft_test.go:2986-3014",
               "S": 2, "self": 0, "max_ents": 0, "log": snap_log,
               "peers": [lead, _peer(0, 12, "StateProbe")],
               "steps": [{"op": "step", "msgs": {"1": {"type": "reject", "index": 11}},
                          "expect": {"messages": 1, "snap": [1]}}]})
    sc.append({"name": "TestSendingSnapshotSetPendingSnapshot",
               "source": "raft/raft_snap_test.go:33-49",
               "S": 2, "self": 0, "max_ents": 0, "log": snap_log,
               "peers": [lead, _peer(0, 12, "StateProbe")],
               "steps": [{"op": "step", "msgs": {"1": {"type": "reject", "index": 11}},
                          "expect": {"peers": {"1": {"pending": 11}}}}]})
    # TestIgnoreProvidingSnap (:3016-3043): Next = firstIndex-1, not
    # RecentActive; MsgProp -> bcastAppend sends nothing.
    sc.append({"name": "TestIgnoreProvidingSnap", "source": "raft/raft_test.go:3016-3043",
               "S": 2, "self": 0, "max_ents": 0, "log": snap_log,
               "peers": [lead, _peer(0, 11, "StateProbe")],
               "steps": [{"op": "append"},
                         {"op": "send", "want": [1], "send_if_empty": 1,
                          "expect": {"sent": []}}]})
    # TestPendingSnapshotPauseReplication (raft_snap_test.go:51-66)
    sc.append({"name": "TestPendingSnapshotPauseReplication",
               "source": "raft/raft_snap_test.go:51-66",
               "S": 2, "self": 0, "max_ents": 0, "log": snap_log,
               "peers": [lead, _peer(0, 12, "StateSnapshot", pending=11)],
               "steps": [{"op": "append"},
                         {"op": "send", "want": [1], "send_if_empty": 1,
                          "expect": {"sent": []}}]})
    # TestSnapshotFailure / Succeed / Abort (raft_snap_test.go:68-141): node 2
    # Next 1, BecomeSnapshot(11).
    snap_peer = _peer(0, 1, "StateSnapshot", pending=11)
    sc.append({"name": "TestSnapshotFailure", "source": "raft/raft_snap_test.go:68-89",
               "S": 2, "self": 0, "max_ents": 0, "log": snap_log, "peers": [lead, snap_peer],
               "steps": [{"op": "step", "msgs": {"1": {"type": "snap_status_reject"}},
                          "expect": {"peers": {"1": {"pending": 0, "next": 1,
                                                     "probe_sent": True}}}}]})
    sc.append({"name": "TestSnapshotSucceed", "source": "raft/raft_snap_test.go:91-112",
               "S": 2, "self": 0, "max_ents": 0, "log": snap_log, "peers": [lead, snap_peer],
               "steps": [{"op": "step", "msgs": {"1": {"type": "snap_status"}},
                          "expect": {"peers": {"1": {"pending": 0, "next": 12,
                                                     "probe_sent": True}}}}]})
    sc.append({"name": "TestSnapshotAbort", "source": "raft/raft_snap_test.go:114-141",
               "S": 2, "self": 0, "max_ents": 0, "log": snap_log, "peers": [lead, snap_peer],
               "steps": [{"op": "step", "msgs": {"1": {"type": "accept", "index": 11}},
                          "expect": {"peers": {"1": {"pending": 0, "next": 13,
                                                     "inflights": 1}}}}]})
    # TestLeaderTransferToSlowFollower (:3523-3541), leader side, derived from
    # the test's message flow: entries 1, 2 (Term 1) committed; node 3 missed
    # entry 2 (Match 1, Next 3, entry 2 in flight).  MsgTransferLeader ->
    # sendAppend(3) (empty MsgApp at Index 2); node 3 rejects (hint 1, log term
    # 1) -> Probe at Index 1; node 3 acks 2 -> Match == lastIndex ->
    # MsgTimeoutNow (the test then finds the leader stepped down for node 3).
    sc.append({"name": "TestLeaderTransferToSlowFollower (leader side, derived)",
               "source": "raft/raft_test.go:3523-3541, raft.go:1275-1281",
               "S": 3, "self": 0, "max_ents": 0, "transferee": 2,
               "log": {"first_index": 1, "last_index": 2, "term_start": 1, "committed": 2,
                       "runs": [[0, 0], [1, 1]]},
               "peers": [_peer(2, 3, "StateReplicate"),
                         _peer(2, 3, "StateReplicate", recent_active=True),
                         _peer(1, 3, "StateReplicate", recent_active=True, ring=[2])],
               "steps": [{"op": "send", "want": [2], "send_if_empty": 1, "expect": {"sent": [2]}},
                         {"op": "step", "msgs": {"2": {"type": "reject", "index": 2, "hint": 1,
                                                       "logterm": 1}},
                          "expect": {"messages": 1, "msg_index": {"2": 1}, "timeout_now": [],
                                     "peers": {"2": {"state": 0, "next": 2,
                                                     "probe_sent": True}}}},
                         {"op": "step", "msgs": {"2": {"type": "accept", "index": 2}},
                          "expect": {"timeout_now": [2],
                                     "peers": {"2": {"state": 1, "match": 2, "next": 3}}}}]})
    # TestProgressPaused (raft_test.go:97-109): two peers, becomeLeader
    # appends 1:t1 (node 2: Probe, Next 1); three MsgProp -> appendEntry +
    # bcastAppend each: one MsgApp in all (the probe pauses node 2).
    base = {"S": 2, "self": 0, "max_ents": 0,
            "log": {"first_index": 1, "last_index": 1, "term_start": 1, "committed": 0,
                    "runs": [[0, 0], [1, 1]]}}
    steps = []
    for i in range(3):
        steps += [{"op": "append"}, {"op": "send", "want": [1], "send_if_empty": 1,
                                      "expect": {"sent": [1] if i == 0 else []}}]
    sc.append(dict(base, name="TestProgressPaused", source="raft/raft_test.go:97-109",
                   peers=[_peer(1, 2, "StateReplicate"), _peer(0, 1, "StateProbe")], steps=steps))
    # TestProgressResumeByHeartbeatResp (:78-95): node 2 ProbeSent = true
    # stays so through MsgBeat (heartbeats only, no Progress change: the
    # check); then BecomeReplicate (the state below) and MsgHeartbeatResp
    # -> ProbeSent false.
    sc.append(dict(base, name="TestProgressResumeByHeartbeatResp",
                   source="raft/raft_test.go:78-95",
                   peers=[_peer(1, 2, "StateReplicate"), _peer(0, 1, "StateReplicate")],
                   steps=[{"op": "step", "msgs": {"1": {"type": "heartbeat"}},
                           "expect": {"peers": {"1": {"probe_sent": False}}}}]))
    # TestProgressFlowControl (:111-177): MaxInflightMsgs 3 (inflight_cap),
    # MaxSizePerMsg 2048 over 1000-byte entries = 2 entries per MsgApp
    # (max_ents; the first MsgApp, [1:empty, 2], also carries 2).  Node 2
    # BecomeProbe (Next 1); ten MsgProp: one MsgApp (probe).  Ack of 2 ->
    # Replicate, commit 2, bcast + send loop: three MsgApps of 2 entries
    # ([3,4] [5,6] [7,8]: Next 9, ring full).  Ack of 8: two MsgApps, of 2
    # and 1 entries ([9,10] [11]: Next 12).
    steps = []
    for i in range(10):
        steps += [{"op": "append"},
                  {"op": "send", "want": [1], "send_if_empty": 1,
                   "expect": {"sent": [1] if i == 0 else [],
                              "peers": {"1": {"probe_sent": True, "next": 1}}}}]
    steps += [{"op": "step", "msgs": {"1": {"type": "accept", "index": 2}},
               "expect": {"messages": 3, "msg_index": {"1": 2}, "committed": 2,
                          "peers": {"1": {"state": 1, "match": 2, "next": 9, "inflights": 3}}}},
              {"op": "step", "msgs": {"1": {"type": "accept", "index": 8}},
               "expect": {"messages": 2, "msg_index": {"1": 8}, "committed": 8,
                          "peers": {"1": {"match": 8, "next": 12, "inflights": 2}}}}]
    sc.append(dict(base, name="TestProgressFlowControl", source="raft/raft_test.go:111-177",
                   max_ents=2, inflight_cap=3,
                   peers=[_peer(1, 2, "StateReplicate"), _peer(0, 1, "StateProbe")], steps=steps))
    # TestHandleHeartbeatResp (:1312-1354): storage 1:t1 2:t2 3:t3, Term 1,
    # becomeLeader appends 4:t1 (node 2: Probe, Next 4), commitTo(4).  Two
    # heartbeat responses each re-send the probe MsgApp (Index 3); the ack of
    # 4 (its sendAppend is consumed unchecked); then a heartbeat response
    # sends nothing.  The log model's term_start is 4 (the commit never moves
    # here, so index 1's term-1 entry plays no part).
    sc.append({"name": "TestHandleHeartbeatResp", "source": "raft/raft_test.go:1312-1354",
               "S": 2, "self": 0, "max_ents": 0,
               "log": {"first_index": 1, "last_index": 4, "term_start": 4, "committed": 4,
                       "runs": [[0, 0], [1, 1], [2, 2], [3, 3], [4, 1]]},
               "peers": [_peer(4, 5, "StateReplicate"), _peer(0, 4, "StateProbe")],
               "steps": [{"op": "step", "msgs": {"1": {"type": "heartbeat"}},
                          "expect": {"messages": 1, "msg_index": {"1": 3}}},
                         {"op": "step", "msgs": {"1": {"type": "heartbeat"}},
                          "expect": {"messages": 1, "msg_index": {"1": 3}}},
                         {"op": "step", "msgs": {"1": {"type": "accept", "index": 4}}},
                         {"op": "step", "msgs": {"1": {"type": "heartbeat"}},
                          "expect": {"messages": 0}}]})
    return sc


# ---------------------------------------------------------------------------
# Election scenarios for qe_election_steps' scripted mode: one group per
# node view, slot s = node id s+1.  Each step is one qe_election_steps step
# with the responses the test's message flow delivers (resp = slots whose
# response arrives, grant = those granting, hup = election timeout fires).
# ---------------------------------------------------------------------------
STATE_IDS = {"StateFollower": 0, "StateCandidate": 1, "StateLeader": 2, "StatePreCandidate": 3}


def election_scenarios():
    sc = []
    # TestLeaderElectionInOneRoundRPC (raft_paper_test.go:192-232): MsgHup
    # (campaign, Term 1), then one MsgVoteResp per entry of the votes map.
    for i, r in enumerate(election_table()):
        steps = [{}]
        if r["size"] > 1:
            steps.append({"resp": [vid - 1 for vid, _ in r["votes"]],
                          "grant": [vid - 1 for vid, v in r["votes"] if v]})
        steps[-1]["expect"] = {"state": STATE_IDS[r["state"]], "term": 1}
        sc.append({"name": f"TestLeaderElectionInOneRoundRPC#{i}",
                   "source": "raft/raft_paper_test.go:192-232", "S": r["size"], "self": 0,
                   "flags": 0, "term": 0, "state": 0, "steps": steps})
    # TestLeaderStepdownWhenQuorumLost (raft_test.go:1766-1781): a CheckQuorum
    # leader of {1,2,3} at Term 1 hears from nobody for an election timeout.
    sc.append({"name": "TestLeaderStepdownWhenQuorumLost", "source": "raft/raft_test.go:1766-1781",
               "S": 3, "self": 0, "flags": 2, "term": 1, "state": 2,
               "steps": [{"resp": [], "expect": {"state": 0, "term": 1}}]})
    # ... and one that hears from a quorum stays leader (the converse, derived).
    sc.append({"name": "CheckQuorum keeps a leader that hears from a quorum (derived)",
               "source": "raft/raft.go:997-1018", "S": 3, "self": 0, "flags": 2, "term": 1,
               "state": 2, "steps": [{"resp": [2], "expect": {"state": 2, "term": 1}}]})
    # TestPreVoteWithSplitVote (raft_test.go:3925-3998), derived from the
    # test's message flow: n1 won Term 2 and is isolated; n2 and n3 (both
    # Term 2 followers) pre-vote for each other, both win the pre-vote, both
    # campaign at Term 3 and reject each other (split vote: candidates at
    # Term 3).  n2 times out first: pre-vote granted by n3, election at Term
    # 4 granted by n3 -> n2 leads Term 4.  n3's view is followed up to the
    # split (its step down to follower comes from n2's higher-term MsgVote,
    # which is not a vote response).
    n2 = [{"hup": 1},
          {"resp": [2], "grant": [2]},
          {"resp": [2], "grant": [], "expect": {"term": 3, "state": 1}},
          {"hup": 1, "expect": {"term": 3, "state": 3}},
          {"resp": [2], "grant": [2], "expect": {"term": 4, "state": 1}},
          {"resp": [2], "grant": [2], "expect": {"term": 4, "state": 2}}]
    sc.append({"name": "TestPreVoteWithSplitVote/n2 (derived)",
               "source": "raft/raft_test.go:3925-3998", "S": 3, "self": 1, "flags": 1,
               "term": 2, "state": 0, "steps": n2})
    n3 = [{"hup": 1},
          {"resp": [1], "grant": [1]},
          {"resp": [1], "grant": [], "expect": {"term": 3, "state": 1}}]
    sc.append({"name": "TestPreVoteWithSplitVote/n3 (derived)",
               "source": "raft/raft_test.go:3925-3998", "S": 3, "self": 2, "flags": 1,
               "term": 2, "state": 0, "steps": n3})
    return sc


def confchange_files():
    """datadriven blocks: `cmd [args]`, input lines, `----`, output up to a
    blank line."""
    d = os.path.join(REF, "confchange", "testdata")
    files = {}
    for name in sorted(os.listdir(d)):
        lines = open(os.path.join(d, name), encoding="utf-8").read().split("\n")
        steps, i = [], 0
        while i < len(lines):
            line = lines[i]
            if line.split(" ")[0] in ("simple", "enter-joint", "leave-joint"):
                cmd, _, args = line.partition(" ")
                j, inp = i + 1, []
                while lines[j] != "----":
                    inp.append(lines[j])
                    j += 1
                j += 1
                out = []
                while j < len(lines) and lines[j] != "":
                    out.append(lines[j])
                    j += 1
                steps.append({"line": i + 1, "cmd": cmd, "args": args,
                              "input": " ".join(inp).strip(), "expect": out})
                i = j
            else:
                i += 1
        files[name] = {"source": f"raft/confchange/testdata/{name}", "steps": steps}
    return files


# ---------------------------------------------------------------------------
# raft/testdata/*.txt interaction traces (raft/interaction_test.go:24-34,
# raft/rafttest/interaction_env*.go): what every node received and sent, as
# the reference printed it.  Only the printed data is extracted; the
# replay (tests/trace_replay.py) restates each leader's side.
# ---------------------------------------------------------------------------
TRACE_FILES = ("probe_and_replicate.txt", "snapshot_succeed_via_app_resp.txt", "campaign.txt",
               "campaign_learner_must_vote.txt", "confchange_v1_add_single.txt",
               "confchange_v2_add_single_auto.txt", "confchange_v2_add_double_implicit.txt",
               "confchange_v1_remove_leader.txt", "confchange_v2_add_single_explicit.txt",
               "confchange_v2_add_double_auto.txt")
_MSG_RE = re.compile(r"^([0-9a-f]+)->([0-9a-f]+) (Msg\w+) Term:(\d+) Log:(\d+)/(\d+)(.*)$")


def parse_message(text):
    """A DescribeMessage line (raft/util.go:133-156) -> dict."""
    m = _MSG_RE.match(text)
    assert m, text
    rest = m.group(7)
    d = {"from": int(m.group(1), 16), "to": int(m.group(2), 16), "type": m.group(3),
         "term": int(m.group(4)), "logterm": int(m.group(5)), "index": int(m.group(6)),
         "reject": False, "hint": 0, "commit": 0, "entries": [], "snap_index": None}
    r = re.search(r" Rejected \(Hint: (\d+)\)", rest)
    if r:
        d["reject"], d["hint"] = True, int(r.group(1))
    c = re.search(r" Commit:(\d+)", rest)
    if c:
        d["commit"] = int(c.group(1))
    e = re.search(r" Entries:\[(.*)\]", rest)
    if e:
        d["entries"] = [[int(a), int(b)] for a, b in re.findall(r"(\d+)/(\d+) Entry\w+", e.group(1))]
    sn = re.search(r" Snapshot: Index:(\d+) Term:(\d+)", rest)
    if sn:
        d["snap_index"] = int(sn.group(1))
    return d


def parse_trace_output(out):
    """The output lines of one command -> blocks: recv (messages a node
    received, with its DEBUG progress lines), ready (HardState commit, state,
    entries, messages sent) and status (Progress strings)."""
    blocks, cur = [], None
    for raw in out:
        line = raw.strip()
        h = re.match(r"^> (\d+) (receiving messages|handling Ready)$", line)
        if h:
            cur = {"node": int(h.group(1)),
                   "kind": "recv" if h.group(2).startswith("receiving") else "ready",
                   "msgs": [], "debug": []}
            blocks.append(cur)
            continue
        if line.startswith("Ready MustSync") and (cur is None or cur["kind"] != "ready"):
            cur = {"node": None, "kind": "ready", "msgs": [], "debug": []}  # process-ready
            blocks.append(cur)
            continue
        st = re.match(r"^(\d+): (State\w+ match=\d+ next=\d+.*)$", line)
        if st and not raw.startswith(" "):
            if cur is None or cur["kind"] != "status":
                cur = {"node": None, "kind": "status", "progress": {}}
                blocks.append(cur)
            cur["progress"][st.group(1)] = st.group(2)
            continue
        if cur is None or cur["kind"] == "status":
            continue
        if _MSG_RE.match(line):
            cur["msgs"].append(parse_message(line))
        elif line.startswith("HardState"):
            cur["commit"] = int(re.search(r"Commit:(\d+)", line).group(1))
            t = re.search(r"Term:(\d+)", line)
            cur["term"] = int(t.group(1)) if t else None
        elif line.startswith("Lead:"):
            cur["lead_state"] = line
        elif re.match(r"^\d+/\d+ Entry\w+", line):
            cur.setdefault("entries", []).append([int(x) for x in line.split()[0].split("/")])
        elif line.startswith("DEBUG") or line.startswith("INFO"):
            cur["debug"].append(line)
    return blocks


def interaction_traces():
    out = {}
    for name in TRACE_FILES:
        path = os.path.join(REF, "testdata", name)
        with open(path, encoding="utf-8") as f:
            lines = f.read().split("\n")
        cmds, i = [], 0
        while i < len(lines):
            if lines[i] == "----":
                # the command is the non-comment block above, its output the
                # lines up to the next blank line
                j = i - 1
                cmd = []
                while j >= 0 and lines[j] != "" and not lines[j].startswith("#"):
                    cmd.insert(0, lines[j])
                    j -= 1
                k = i + 1
                body = []
                while k < len(lines) and lines[k] != "":
                    body.append(lines[k])
                    k += 1
                c = {"line": j + 2, "cmd": cmd[0], "input": cmd[1:],
                     "blocks": parse_trace_output(body)}
                if cmd[0].startswith("propose"):  # "ok", "raft proposal dropped" or the
                    # INFO line of a conf change stepLeader turns into an empty entry
                    c["dropped"] = any("raft proposal dropped" in x for x in body)
                    c["ignored_cc"] = any("ignoring conf change" in x for x in body)
                if cmd[0].startswith("raft-log"):  # the node's log: term/index per entry
                    c["log"] = [[int(a), int(b)] for a, b in
                                (re.match(r"^(\d+)/(\d+) Entry", x).groups() for x in body
                                 if re.match(r"^\d+/\d+ Entry", x))]
                cmds.append(c)
                i = k
            else:
                i += 1
        out[name] = {"source": f"raft/testdata/{name}", "commands": cmds}
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not present; fixtures are already committed")
    rows = datadriven_rows()
    assert len(rows) == 127, len(rows)
    with open(os.path.join(HERE, "quorum_testdata.jsonl"), "w", encoding="utf-8") as f:
        for r in rows:
            f.write(json.dumps(r, ensure_ascii=False) + "\n")
    # the same cases in a line format the C++ test reads without a JSON parser:
    # <cmd> <joint> <expect> cfg=a,b cfgj=c acked=id:idx,.. votes=id:0|1,.. <source>
    with open(os.path.join(HERE, "quorum_testdata.txt"), "w", encoding="utf-8") as f:
        for r in rows:
            acked = ",".join(f"{k}:{v}" for k, v in r.get("acked", []))
            votes = ",".join(f"{k}:{int(v)}" for k, v in r.get("votes", []))
            f.write(f"{r['cmd']} {int(r['joint'])} {r['expect']} "
                    f"cfg={','.join(map(str, r['cfg']))} cfgj={','.join(map(str, r['cfgj']))} "
                    f"acked={acked} votes={votes} {r['source']}\n")
    # Describe texts for the C++ test: cfg|cfgj|acked|text with newlines as \\n
    with open(os.path.join(HERE, "describe_testdata.txt"), "w", encoding="utf-8") as f:
        for r in rows:
            if "describe" not in r:
                continue
            acked = ",".join(f"{k}:{v}" for k, v in r["acked"])
            f.write(f"{','.join(map(str, r['cfg']))}|{','.join(map(str, r['cfgj']))}|{acked}|"
                    + r["describe"].replace("\n", "\\n") + "\n")
    tables = {
        "TestCommit": {"source": "raft/raft_test.go:1127-1152", "rows": test_commit_table()},
        "TestLeaderElectionInOneRoundRPC": {"source": "raft/raft_paper_test.go:192-216", "rows": election_table()},
        "TestProgressUpdate": {"source": "raft/tracker/progress_test.go:149-161", "rows": progress_update_table()},
        **progress_tables(),
        "Inflights": inflights_tables(),
        "TestFastLogRejection": fast_log_rejection_table(),
    }
    with open(os.path.join(HERE, "raft_tables.json"), "w", encoding="utf-8") as f:
        json.dump(tables, f, indent=1)
    with open(os.path.join(HERE, "progress_scenarios.json"), "w", encoding="utf-8") as f:
        json.dump(progress_scenarios(), f, indent=1)
    with open(os.path.join(HERE, "election_scenarios.json"), "w", encoding="utf-8") as f:
        json.dump(election_scenarios(), f, indent=1)
    # election table in a line format for the C++ test: <size> <state> id:0|1,..
    with open(os.path.join(HERE, "election_table.txt"), "w", encoding="utf-8") as f:
        for r in tables["TestLeaderElectionInOneRoundRPC"]["rows"]:
            votes = ",".join(f"{i}:{int(v)}" for i, v in r["votes"])
            f.write(f"{r['size']} {r['state']} votes={votes}\n")
    traces = interaction_traces()
    with open(os.path.join(HERE, "interaction_traces.json"), "w", encoding="utf-8") as f:
        json.dump(traces, f, indent=1)
    print("wrote", sum(len(v["commands"]) for v in traces.values()), "trace commands from",
          len(traces), "interaction files")
    cc = confchange_files()
    with open(os.path.join(HERE, "confchange_testdata.json"), "w", encoding="utf-8") as f:
        json.dump(cc, f, indent=1)
    # the same steps in a tab-separated line format for the C++ test:
    # <file> <line> <cmd> <args> <input> <expected lines joined by '|'>
    with open(os.path.join(HERE, "confchange_testdata.txt"), "w", encoding="utf-8") as f:
        for name, v in cc.items():
            for st in v["steps"]:
                f.write("\t".join([name, str(st["line"]), st["cmd"], st["args"], st["input"],
                                   "|".join(st["expect"])]) + "\n")
    print("wrote", sum(len(v["steps"]) for v in cc.values()), "confchange steps in", len(cc), "files")
    counts = {}
    for r in rows:
        k = r["source"].split("/")[-1].split(":")[0]
        counts[k] = counts.get(k, 0) + 1
    print("wrote", len(rows), "datadriven cases", counts)


if __name__ == "__main__":
    main()
