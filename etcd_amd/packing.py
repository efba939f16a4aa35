"""Host-side ID -> slot packing: turns per-group reference objects (voter-ID
sets, AckedIndexer lookups, vote maps) into the slot-SoA arrays of
include/etcd_quorum.h.

Every quorum function is an order-free set function of (voter set,
per-voter value) (raft/quorum/majority.go:155-161 iterates a map and sorts),
so any injective ID -> slot assignment is legal.  We assign the union of
JointConfig.IDs() (raft/quorum/joint.go:30-38) in ascending ID order, then
learners, so a group's slots are [voters..., learners...].
"""
import numpy as np

MAX_SLOTS = 16


class PackedGroups:
    """Slot-SoA host arrays for G groups plus the slot -> ID map."""

    def __init__(self, G, S):
        md = np.uint8 if S <= 8 else np.uint16
        self.G, self.S = G, S
        self.match = np.zeros((S, G), dtype=np.uint64)
        self.inc = np.zeros(G, md)
        self.out = np.zeros(G, md)
        self.learner = np.zeros(G, md)
        self.voted = np.zeros(G, md)
        self.granted = np.zeros(G, md)
        self.recent = np.zeros(G, md)
        self.slot_ids = np.zeros((G, S), dtype=np.uint64)  # 0 = unused slot
        self.joint = False


def slot_order(c0, c1, learners=()):
    voters = sorted(set(c0) | set(c1))
    lrn = sorted(set(learners) - set(voters))
    return voters + lrn


def pack(groups, num_slots=None):
    """groups: iterable of dicts with keys
         c0, c1      voter-ID iterables (JointConfig halves; c1 may be empty)
         learners    learner IDs (optional)
         acked       callable id -> (index, found) or dict id -> index (optional)
         votes       dict id -> bool (optional)
         recent      set of RecentActive ids (optional)
    Returns PackedGroups.  Raises ValueError if a group needs > 16 slots."""
    groups = list(groups)
    orders = [slot_order(g.get("c0", ()), g.get("c1", ()), g.get("learners", ())) for g in groups]
    need = max([len(o) for o in orders] + [1])
    S = int(num_slots) if num_slots else need
    if need > S or S > MAX_SLOTS:
        raise ValueError(f"group needs {need} slots; engine supports at most {MAX_SLOTS}")
    p = PackedGroups(len(groups), S)
    for gi, (g, order) in enumerate(zip(groups, orders)):
        c0, c1 = set(g.get("c0", ())), set(g.get("c1", ()))
        lrn = set(g.get("learners", ()))
        acked = g.get("acked")
        votes = g.get("votes") or {}
        recent = g.get("recent") or set()
        if c1:
            p.joint = True
        mi = mo = ml = vd = gr = ra = 0
        for s, vid in enumerate(order):
            p.slot_ids[gi, s] = vid
            bit = 1 << s
            if vid in c0:
                mi |= bit
            if vid in c1:
                mo |= bit
            if vid in lrn:
                ml |= bit
            if acked is not None:
                if callable(acked):
                    idx, found = acked(vid)
                else:
                    found = vid in acked
                    idx = acked.get(vid, 0)
                p.match[s, gi] = int(idx) if found else 0
            if vid in votes:
                vd |= bit
                if votes[vid]:
                    gr |= bit
            if vid in recent:
                ra |= bit
        p.inc[gi], p.out[gi], p.learner[gi] = mi, mo, ml
        p.voted[gi], p.granted[gi], p.recent[gi] = vd, gr, ra
    return p
