"""qe_propose's oracle (orc_propose_batch, oracle/quorum_oracle.c) pinned to
the reference tests of the MsgProp arm, appendEntry and the uncommitted
size limit (tests/propose_scenarios.py), plus the properties the kernel's
random differential (tests/test_gpu_propose.py) relies on."""
import numpy as np
import pytest

from tests.leader_round_scenarios import OracleRoundBackend
from tests.propose_scenarios import SCENARIOS


@pytest.mark.parametrize("sc", SCENARIOS, ids=lambda f: f.__name__)
def test_propose_scenarios_on_oracle(orc, sc):
    sc(OracleRoundBackend(orc))


def test_no_proposal_changes_nothing(orc):
    """num_entries 0: result NONE and no state is touched."""
    pb = orc.ProgressBatch(4, 3, 8, 2)
    pb.last_index[:] = 7
    pb.match[:] = 3
    before = pb.copy()
    o = orc.propose(pb, np.zeros(4, np.uint32))
    assert not o.result.any() and not o.sent.any()
    for k in ("match", "next", "pw", "ibuf", "committed", "last_index"):
        np.testing.assert_array_equal(getattr(pb, k), getattr(before, k))
    assert o.stats[0] == 4  # groups counted


def test_append_only_sends_nothing_and_skips_gates(orc):
    """QE_PROP_APPEND_ONLY (appendEntry alone): no bcast, no transfer gate,
    conf-change lists ignored; the leader's own Progress still gates."""
    pb = orc.ProgressBatch(2, 3, 8, 2)
    pb.self_slot = np.array([0, 0xFF], np.uint8)
    pb.lead_transferee = np.array([1, 0xFF], np.uint8)
    pb.pw[:] = orc.pack_word(1, 0, 0)  # StateReplicate
    pb.next[:] = 1
    o = orc.propose(pb, np.array([2, 2], np.uint32), flags=1,
                    cc=(1, np.array([1, 1], np.uint8), np.zeros(2, np.uint32),
                        np.ones(2, np.uint8), np.zeros(2, np.uint32)),
                    applied=np.zeros(2, np.uint64), pending_conf_index=np.zeros(2, np.uint64))
    assert list(o.result) == [1, 2] and not o.sent.any() and not o.cc_refused.any()
    assert list(pb.last_index) == [2, 0] and pb.match[0] == 2
