"""Loading helpers for the committed golden fixtures (tests/golden/)."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
INF = (1 << 64) - 1


def datadriven_cases():
    with open(os.path.join(GOLDEN, "quorum_testdata.jsonl"), encoding="utf-8") as f:
        return [json.loads(line) for line in f if line.strip()]


def raft_tables():
    with open(os.path.join(GOLDEN, "raft_tables.json"), encoding="utf-8") as f:
        return json.load(f)


def case_acked(case):
    return {int(k): int(v) for k, v in case.get("acked", [])}


def case_votes(case):
    return {int(k): bool(v) for k, v in case.get("votes", [])}


def case_id(case):
    return case["source"].split("/")[-1]
