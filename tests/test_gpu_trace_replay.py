"""The reference's interaction traces replayed from the leader's side through
the HIP engine (qe_election_steps scripted, qe_propose, qe_progress_send,
qe_progress_step, qe_heartbeat) -- the same replay the oracle passes in
tests/test_trace_replay.py (tests/trace_replay.py)."""
import pytest
import torch

from tests.test_gpu_progress import DEV, GpuBackend
from tests.trace_replay import TRACES, Leader

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from etcd_amd import engine
    return engine


def gpu_elector(eng):
    def make(S, self_slot, term0):
        b = eng.SlotBatch(1, S, DEV, masks=("inc", "learner"), votes=False)
        b.inc.fill_((1 << S) - 1)
        est = eng.ElectionState(b, torch.tensor([self_slot], dtype=torch.uint8, device=DEV))
        est.term.fill_(term0)
        est.state.fill_(0)
        dt = torch.uint8 if S <= 8 else torch.int16
        k = [0]

        def step(resp, grant, hup):
            script = (torch.tensor([resp], dtype=dt, device=DEV),
                      torch.tensor([grant], dtype=dt, device=DEV),
                      torch.tensor([hup], dtype=torch.uint8, device=DEV), 1)
            eng.election_steps(est, 0, k[0], 1, p_drop=0, p_grant=0, script=script)
            k[0] += 1
            return int(est.term[0]), int(est.state[0])
        return step
    return make


@pytest.mark.parametrize("trace", TRACES, ids=lambda f: f.__name__)
def test_trace_replay_on_gpu(eng, trace):
    checked = trace(lambda node, S: Leader(GpuBackend(eng), node, S), gpu_elector(eng))
    assert checked["rounds"] > 0 and checked["sends"] > 0
