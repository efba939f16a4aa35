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
    # election table in a line format for the C++ test: <size> <state> id:0|1,..
    with open(os.path.join(HERE, "election_table.txt"), "w", encoding="utf-8") as f:
        for r in tables["TestLeaderElectionInOneRoundRPC"]["rows"]:
            votes = ",".join(f"{i}:{int(v)}" for i, v in r["votes"])
            f.write(f"{r['size']} {r['state']} votes={votes}\n")
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
