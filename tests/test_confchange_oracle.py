"""The confchange oracle (oracle/confchange_ref.py) against the reference's
golden vectors: every step of raft/confchange/testdata/*.txt
(TestConfChangeDataDriven, raft/confchange/datadriven_test.go:29-98),
compared as text."""
import json
import os

import pytest

from oracle import confchange_ref as cc

HERE = os.path.dirname(os.path.abspath(__file__))
FILES = json.load(open(os.path.join(HERE, "golden", "confchange_testdata.json")))


def test_fixture_counts():
    assert len(FILES) == 9
    assert sum(len(f["steps"]) for f in FILES.values()) == 58


@pytest.mark.parametrize("name", sorted(FILES))
def test_oracle_reproduces_testdata(name):
    for st, out in cc.replay(FILES[name]["steps"]):
        assert out == st["expect"], f"{name}:{st['line']} {st['cmd']} {st['input']}"


def test_change_batch_refuses_more_than_255_changes():
    """qe_conf_changes.count is a u8 per group: the Python mirror refuses a
    longer list up front instead of truncating it."""
    import pytest
    from etcd_amd import confchange as C
    from etcd_amd.tracker import ProgressTracker
    ch = C.Changer(ProgressTracker(), LastIndex=1, device="cpu")
    with pytest.raises(ValueError):
        C.ChangeBatch([ch], [1], [[C.ConfChangeSingle(0, 1)] * 256], device="cpu")
