"""Python mirror of etcd's raft/confchange Changer
(raft/confchange/confchange.go) whose transitions run on the MI355X
(qe_confchange, one group per lane).

    c = Changer(Tracker=MakeProgressTracker(256), LastIndex=0)
    cfg, prs, err = c.Simple([ConfChangeSingle(ConfChangeAddNode, 1)])

Each method returns (tracker.Config, ProgressMap, error) as the Go methods
do; err is None or a ConfChangeError carrying the reference's message.
ChangeBatch runs one operation per Changer in a single launch.
"""
import numpy as np
import torch

from . import _lib, engine
from .quorum import JointConfig
from .tracker import Config, Progress, StateProbe

# raftpb.ConfChangeType (raft/raftpb/raft.pb.go:224-227)
ConfChangeAddNode, ConfChangeRemoveNode, ConfChangeUpdateNode, ConfChangeAddLearnerNode = \
    0, 1, 2, 3

_ERRORS = {
    1: "invalid input configuration (checkInvariants)",
    2: "config is already joint",
    3: "can't make a zero-voter config joint",
    4: "can't leave a non-joint config",
    5: "can't apply simple config change in joint config",
    6: "unexpected conf type",
    7: "removed all voters",
    8: "more than one voter changed without entering joint config",
    9: "invalid resulting configuration (checkInvariants)",
    10: "more than 16 peers",
}


class ConfChangeError(Exception):
    def __init__(self, code):
        super().__init__(_ERRORS.get(code, f"confchange error {code}"))
        self.code = code


class ConfChangeSingle:
    """raftpb.ConfChangeSingle (Type, NodeID)."""

    __slots__ = ("Type", "NodeID")

    def __init__(self, Type, NodeID):
        self.Type, self.NodeID = int(Type), int(NodeID)


class Changer:
    """confchange.Changer{Tracker, LastIndex} (confchange.go:31-34)."""

    def __init__(self, Tracker, LastIndex=0, device=None):
        self.Tracker, self.LastIndex = Tracker, LastIndex
        self.device = device

    def EnterJoint(self, autoLeave, ccs):  # confchange.go:49-76
        op = _lib.QE_CC_OP_ENTER_JOINT_AUTO if autoLeave else _lib.QE_CC_OP_ENTER_JOINT
        return ChangeBatch([self], [op], [ccs], self.device)[0]

    def LeaveJoint(self):  # confchange.go:92-123
        return ChangeBatch([self], [_lib.QE_CC_OP_LEAVE_JOINT], [[]], self.device)[0]

    def Simple(self, ccs):  # confchange.go:130-147
        return ChangeBatch([self], [_lib.QE_CC_OP_SIMPLE], [ccs], self.device)[0]


def ChangeBatch(changers, ops, ccs, device=None):
    """One qe_confchange launch for all changers; returns [(Config,
    ProgressMap, error)].  A tracker's peers take slots in ascending ID
    order; S = the largest (peers + changes) of the batch, capped at 16."""
    dev = torch.device(device if device is not None else "cuda")
    G = len(changers)
    if G == 0:
        return []
    if any(len(x) > 255 for x in ccs):
        # qe_conf_changes.count is a u8 per group (the reference Changer has
        # no limit): refuse rather than apply a truncated change list
        raise ValueError("ChangeBatch: more than 255 changes in one group")
    S = max(1, min(_lib.QE_MAX_SLOTS,
                   max(len(c.Tracker.Progress) + len(x) for c, x in zip(changers, ccs))))
    C = max(1, max(len(x) for x in ccs))
    cs = engine.ConfState(G, S, dev)
    ch = engine.ConfChanges(G, S, C, dev)
    md = engine.mask_np_dtype(S)
    ids = np.zeros((G, S), np.uint64)
    masks = {k: np.zeros(G, np.int64) for k in cs.MASKS}
    al = np.zeros(G, np.uint8)
    op = np.zeros(G, np.uint8)
    cnt = np.zeros(G, np.uint8)
    typ = np.zeros((C, G), np.uint8)
    node = np.zeros((C, G), np.uint64)
    li = np.zeros(G, np.uint64)
    pre = {}
    for g, c in enumerate(changers):
        t = c.Tracker
        peers = sorted(t.Progress)
        members = t.Voters.IDs() | set(t.Learners or ()) | set(t.LearnersNext or ())
        if len(peers) > S:
            pre[g] = 10
            continue
        if not members <= set(peers):  # "no progress for %d"
            pre[g] = 1
            continue
        for s, i in enumerate(peers):
            ids[g, s] = i
            b = 1 << s
            masks["inc"][g] |= b if i in t.Voters[0] else 0
            masks["out"][g] |= b if i in t.Voters[1] else 0
            masks["learner"][g] |= b if i in (t.Learners or ()) else 0
            masks["learners_next"][g] |= b if i in (t.LearnersNext or ()) else 0
            masks["is_learner"][g] |= b if t.Progress[i].IsLearner else 0
            masks["tracked"][g] |= b
        al[g] = bool(t.AutoLeave)
        op[g] = ops[g]
        cnt[g] = len(ccs[g])
        for k, cc in enumerate(ccs[g]):
            typ[k, g], node[k, g] = cc.Type, cc.NodeID
        li[g] = c.LastIndex
    cs.slot_ids.copy_(torch.from_numpy(np.ascontiguousarray(ids.T).reshape(-1).view(np.int64)))
    for k, v in masks.items():
        a = v.astype(md)
        getattr(cs, k).copy_(torch.from_numpy(a.view(np.int16) if md == np.uint16 else a))
    cs.auto_leave.copy_(torch.from_numpy(al))
    ch.op.copy_(torch.from_numpy(op))
    ch.count.copy_(torch.from_numpy(cnt))
    ch.type.copy_(torch.from_numpy(typ.reshape(-1)))
    ch.node_id.copy_(torch.from_numpy(node.reshape(-1).view(np.int64)))
    ch.last_index.copy_(torch.from_numpy(li.view(np.int64)))
    engine.confchange(cs, ch)
    h = cs.host()
    res = ch.result.cpu().numpy()
    newp = ch.new_progress.cpu().numpy().view(md)
    out = []
    for g, c in enumerate(changers):
        rc = pre.get(g, int(res[g]))
        if rc != 0:
            out.append((None, None, ConfChangeError(rc)))
            continue

        def ids_of(mask):
            m = int(h[mask][g])
            return {int(h["slot_ids"][g, s]) for s in range(S) if (m >> s) & 1}
        cfg = Config(Voters=JointConfig(ids_of("inc"), ids_of("out")),
                     Learners=ids_of("learner") or None,
                     LearnersNext=ids_of("learners_next") or None,
                     AutoLeave=bool(h["auto_leave"][g]))
        prs = {}
        trk, isl = int(h["tracked"][g]), int(h["is_learner"][g])
        for s in range(S):
            if not (trk >> s) & 1:
                continue
            i = int(h["slot_ids"][g, s])
            old = c.Tracker.Progress.get(i)
            if (int(newp[g]) >> s) & 1 or old is None:
                p = Progress(Match=0, Next=c.LastIndex, RecentActive=True)  # initProgress
                p.State = StateProbe
            else:
                p = Progress(old.Match, old.Next, old.IsLearner, old.RecentActive)
                p.State, p.PendingSnapshot, p.ProbeSent = (old.State, old.PendingSnapshot,
                                                           old.ProbeSent)
            p.IsLearner = bool((isl >> s) & 1)
            prs[i] = p
        out.append((cfg, prs, None))
    return out
