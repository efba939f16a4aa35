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

Outputs (data only: inputs + expected outputs):
  tests/golden/quorum_testdata.jsonl   127 rows
  tests/golden/raft_tables.json        the three tables
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


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not present; fixtures are already committed")
    rows = datadriven_rows()
    assert len(rows) == 127, len(rows)
    with open(os.path.join(HERE, "quorum_testdata.jsonl"), "w", encoding="utf-8") as f:
        for r in rows:
            f.write(json.dumps(r, ensure_ascii=False) + "\n")
    tables = {
        "TestCommit": {"source": "raft/raft_test.go:1127-1152", "rows": test_commit_table()},
        "TestLeaderElectionInOneRoundRPC": {"source": "raft/raft_paper_test.go:192-216", "rows": election_table()},
        "TestProgressUpdate": {"source": "raft/tracker/progress_test.go:149-161", "rows": progress_update_table()},
    }
    with open(os.path.join(HERE, "raft_tables.json"), "w", encoding="utf-8") as f:
        json.dump(tables, f, indent=1)
    counts = {}
    for r in rows:
        k = r["source"].split("/")[-1].split(":")[0]
        counts[k] = counts.get(k, 0) + 1
    print("wrote", len(rows), "datadriven cases", counts)


if __name__ == "__main__":
    main()
