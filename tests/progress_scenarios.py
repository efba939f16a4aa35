"""Runner for tests/golden/progress_scenarios.json (leader-side Progress
scenarios transcribed from the reference's raft tests, see
tests/golden/make_golden.py progress_scenarios()).

A scenario is one group: slot s is node id s+1 and `self` is the leader's
slot.  Ops:
  step    one round of peer messages through qe_progress_step (stepLeader)
  send    qe_progress_send: sendAppend / bcastAppend to the `want` slots
  append  appendEntry of one empty entry (qe_propose with
          QE_PROP_APPEND_ONLY: lastIndex + 1, the leader's own MaybeUpdate,
          maybeCommit; no bcast -- the tests call sendAppend themselves)
  check   expectations only
The same runner drives the oracle (CPU tests) and the HIP engine (GPU tests)
through a small backend interface.
"""
import json
import os

import numpy as np

from tests.golden_util import GOLDEN

KIND = {"accept": 1, "reject": 2, "heartbeat": 3, "snap_status": 4, "snap_status_reject": 5,
        "unreachable": 6}
F_CAP = 255  # the tests' MaxInflightMsgs is 256; the slot model caps it at 255


def cap(sc):
    """The scenario's Inflights capacity (MaxInflightMsgs): F_CAP unless the
    test sets its own (TestProgressFlowControl: 3)."""
    return int(sc.get("inflight_cap", F_CAP))
PF_PROBE_SENT, PF_RECENT_ACTIVE = 4, 8


def scenarios():
    with open(os.path.join(GOLDEN, "progress_scenarios.json"), encoding="utf-8") as f:
        return json.load(f)


def initial_arrays(sc):
    """Host arrays (G = 1, stride = 1) of the scenario's initial state."""
    S, lg = sc["S"], sc["log"]
    R = len(lg["runs"])
    a = {
        "match": np.array([p["match"] for p in sc["peers"]], np.uint64),
        "next": np.array([p["next"] for p in sc["peers"]], np.uint64),
        "pending": np.array([p["pending"] for p in sc["peers"]], np.uint64),
        "flags": np.array([p["state"] | (PF_PROBE_SENT if p["probe_sent"] else 0) |
                           (PF_RECENT_ACTIVE if p["recent_active"] else 0)
                           for p in sc["peers"]], np.uint8),
        "icount": np.array([len(p["ring"]) for p in sc["peers"]], np.uint8),
        "ibuf": np.zeros(S * cap(sc), np.uint64),
        "committed": np.array([lg["committed"]], np.uint64),
        "term_start": np.array([lg["term_start"]], np.uint64),
        "first_index": np.array([lg["first_index"]], np.uint64),
        "last_index": np.array([lg["last_index"]], np.uint64),
        "run_first": np.array([r[0] for r in lg["runs"]], np.uint64),
        "run_term": np.array([r[1] for r in lg["runs"]], np.uint64),
        "run_count": np.array([R], np.uint8),
        "self_slot": np.array([sc["self"]], np.uint8),
        "lead_transferee": np.array([sc.get("transferee", 0xFF)], np.uint8),
    }
    if lg.get("snap_index") is not None:
        a["snap_index"] = np.array([lg["snap_index"]], np.uint64)
    for s, p in enumerate(sc["peers"]):
        for k, v in enumerate(p["ring"]):
            a["ibuf"][s * cap(sc) + k] = v
    return a


def msg_arrays(sc, msgs):
    S = sc["S"]
    t = np.zeros(S, np.uint8)
    idx = np.zeros(S, np.uint64)
    hint = np.zeros(S, np.uint64)
    lt = np.zeros(S, np.uint64)
    for k, m in msgs.items():
        s = int(k)
        t[s] = KIND[m["type"]]
        idx[s] = m.get("index", 0)
        hint[s] = m.get("hint", 0)
        lt[s] = m.get("logterm", 0)
    return t, idx, hint, lt


def bits(mask):
    return [s for s in range(16) if (int(mask) >> s) & 1]


def check_expect(sc, exp, be, out, where):
    for k, want in exp.get("peers", {}).items():
        got = be.peer(int(k))
        for f, v in want.items():
            assert got[f] == v, f"{where}: peer {k} {f} = {got[f]}, want {v}"
    if "committed" in exp:
        assert be.committed() == exp["committed"], where
    for key in ("sent", "snap", "timeout_now"):
        if key in exp:
            assert bits(out[key]) == exp[key], f"{where}: {key} {bits(out[key])} != {exp[key]}"
    if "messages" in exp:
        assert int(np.sum(out["msg_count"])) == exp["messages"], f"{where}: {out['msg_count']}"
    for k, v in exp.get("msg_index", {}).items():
        s = int(k)
        assert out["msg_count"][s] > 0 and int(out["msg_index"][s]) == v, where
    if "msg_index_all" in exp:
        for s in range(sc["S"]):
            if out["msg_count"][s]:
                assert int(out["msg_index"][s]) == exp["msg_index_all"], where


def run_scenario(sc, be):
    """be: backend with load(arrays), step(t, idx, hint, lt) -> out dict,
    send(want_mask, sei) -> out dict, append(), peer(s), committed()."""
    be.load(sc, initial_arrays(sc))
    for i, st in enumerate(sc["steps"]):
        where = f"{sc['name']} step {i} ({st['op']})"
        out = {}
        if st["op"] == "step":
            out = be.step(*msg_arrays(sc, st["msgs"]))
        elif st["op"] == "send":
            want = sum(1 << s for s in st["want"])
            out = be.send(want, st["send_if_empty"])  # MaxSizePerMsg: the state's max_ents
        elif st["op"] == "append":
            be.append()
        check_expect(sc, st.get("expect", {}), be, out, where)


def cc_arrays(cc, max_cc=2):
    """(max_cc, count[1], pos[max_cc], leave[max_cc], size[max_cc]) of one
    group's conf-change entries [(position, leave_joint, size), ...]."""
    cc = cc or []
    m = max(max_cc, len(cc))
    pos = np.zeros(m, np.uint32)
    lv = np.zeros(m, np.uint8)
    sz = np.zeros(m, np.uint32)
    for k, (p, leave, size) in enumerate(cc):
        pos[k], lv[k], sz[k] = p, int(bool(leave)), size
    return m, np.array([len(cc)], np.uint8), pos, lv, sz


def oracle_propose(be, n, payload=0, append_only=False, cc=None):
    """Backend helper: orc_propose_batch on be.pb (one group) with the
    backend-held pendingConfIndex / uncommittedSize / applied."""
    for k, v in (("pci", 0), ("unc", 0), ("applied", 0), ("max_unc", 0)):
        if not hasattr(be, k):
            setattr(be, k, v)
    pci = np.array([be.pci], np.uint64)
    unc = np.array([be.unc], np.uint64)
    o = be.orc.propose(be.pb, np.array([n], np.uint32), np.array([payload], np.uint64),
                       cc=cc_arrays(cc), applied=np.array([be.applied], np.uint64),
                       pending_conf_index=pci, uncommitted_size=unc,
                       max_uncommitted=be.max_unc, flags=1 if append_only else 0)
    be.pci, be.unc = int(pci[0]), int(unc[0])
    return {"result": int(o.result[0]), "sent": int(o.sent[0]), "snap": int(o.snap[0]),
            "cc_refused": int(o.cc_refused[0])}


def peer_view(match, nxt, pending, flags, icount, s):
    f = int(flags[s])
    return {"match": int(match[s]), "next": int(nxt[s]), "pending": int(pending[s]),
            "state": f & 3, "probe_sent": bool(f & PF_PROBE_SENT),
            "recent_active": bool(f & PF_RECENT_ACTIVE), "inflights": int(icount[s])}


class OracleBackend:
    """Drives the oracle (oracle/quorum_oracle.c) over one group."""

    def __init__(self, orc):
        self.orc = orc

    def load(self, sc, a):
        S = sc["S"]
        pb = self.orc.ProgressBatch(1, S, cap(sc), len(sc["log"]["runs"]), max_ents=sc["max_ents"])
        a = dict(a)
        pb.pw = self.orc.pack_word(a.pop("flags"), 0, a.pop("icount"))
        for k, v in a.items():
            setattr(pb, k, v.copy())
        self.pb, self.sc = pb, sc
        self.pci = self.unc = self.applied = self.max_unc = 0  # MsgProp state (qe_propose)

    def step(self, t, idx, hint, lt):
        o = self.orc.progress_step(self.pb, t, idx, hint, lt)
        return {"sent": o.sent[0], "snap": o.snap[0], "timeout_now": o.timeout_now[0],
                "msg_count": o.msg_count, "msg_index": o.msg_index, "bcast": o.bcast[0]}

    def send(self, want, sei):
        w = np.array([want], self.orc.mask_dtype(self.sc["S"]))
        sent, snap = self.orc.progress_send(self.pb, w, sei)
        return {"sent": sent[0], "snap": snap[0]}

    def append(self):
        out = self.propose(1, append_only=True)
        assert out["result"] == 1, out

    def propose(self, n, payload=0, append_only=False, cc=None):
        """One MsgProp (or appendEntry alone) through the oracle's
        orc_propose_batch; cc: list of (position, leave_joint, size).
        pendingConfIndex / uncommittedSize / applied live in the backend
        (self.pci, self.unc, self.applied, self.max_unc)."""
        return oracle_propose(self, n, payload, append_only, cc)

    def peer(self, s):
        pb = self.pb
        return peer_view(pb.match, pb.next, pb.pending, pb.flags, pb.icount, s)

    def committed(self):
        return int(self.pb.committed[0])
