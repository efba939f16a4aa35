"""Runner for tests/golden/election_scenarios.json: one group per scenario,
each step one qe_election_steps step in scripted mode (responses given, no
RNG).  The same runner drives the oracle (CPU) and the HIP kernel (GPU)."""
import json
import os

import numpy as np

from tests.golden_util import GOLDEN


def scenarios():
    with open(os.path.join(GOLDEN, "election_scenarios.json"), encoding="utf-8") as f:
        return json.load(f)


def script_arrays(sc):
    """[steps][1] resp / grant masks and hup bytes."""
    n = len(sc["steps"])
    md = np.uint8 if sc["S"] <= 8 else np.uint16
    resp = np.zeros(n, md)
    grant = np.zeros(n, md)
    hup = np.zeros(n, np.uint8)
    for k, st in enumerate(sc["steps"]):
        resp[k] = sum(1 << s for s in st.get("resp", []))
        grant[k] = sum(1 << s for s in st.get("grant", []))
        hup[k] = st.get("hup", 0)
    return resp, grant, hup


def run_scenario(sc, step_fn):
    """step_fn(k) runs step k and returns (term, state)."""
    for k, st in enumerate(sc["steps"]):
        term, state = step_fn(k)
        exp = st.get("expect")
        if exp:
            assert (term, state) == (exp["term"], exp["state"]), (sc["name"], k, term, state)


def oracle_runner(orc, sc):
    S = sc["S"]
    md = np.uint8 if S <= 8 else np.uint16
    term = np.array([sc["term"]], np.uint64)
    state = np.array([sc["state"]], np.uint8)
    voted = np.zeros(1, md)
    granted = np.zeros(1, md)
    self_slot = np.array([sc["self"]], np.uint8)
    inc = np.array([(1 << S) - 1], md)
    learner = np.zeros(1, md)
    resp, grant, hup = script_arrays(sc)

    def step(k):
        orc.election_steps(1, 0, S, term, state, voted, granted, self_slot, inc, None, learner,
                           0, k, 1, 0, 0, flags=sc["flags"],
                           script=(resp[k:k + 1], grant[k:k + 1], hup[k:k + 1], 1))
        return int(term[0]), int(state[0])
    return step
