"""Host-side ID -> slot packing: turns per-group reference objects (voter-ID
sets, AckedIndexer lookups, vote maps) into the slot-SoA arrays of
include/etcd_quorum.h.

Every quorum function is an order-free set function of (voter set,
per-voter value) (raft/quorum/majority.go:155-161 iterates a map and sorts),
so any injective ID -> slot assignment is legal.  We assign the union of
JointConfig.IDs() (raft/quorum/joint.go:30-38) in ascending ID order, then
learners, so a group's slots are [voters..., learners...].
"""
import ctypes

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
        # ID-major [S][G] (the C ABI's layout); slot_ids is its [G][S] view
        self.slot_ids_sg = np.zeros((S, G), dtype=np.uint64)  # 0 = unused slot
        self.slot_ids = self.slot_ids_sg.T
        self.perm = None  # packed position -> caller group (qe_pack_order)
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


# ---------------------------------------------------------------------------
# Native (C++) packer: the wire-format path used at scale.
# ---------------------------------------------------------------------------
def _csr(lists):
    """list of id-iterables -> (ids uint64, off uint64[G+1])."""
    lens = np.fromiter((len(x) for x in lists), dtype=np.uint64, count=len(lists))
    off = np.zeros(len(lists) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    ids = np.fromiter((i for x in lists for i in x), dtype=np.uint64, count=int(off[-1]))
    return ids, off


class ConfStates:
    """G raftpb.ConfState messages (raft/raftpb/raft.proto:115-130) in CSR
    form: each field is (ids uint64, off uint64[G+1]) or None.  `perm`
    (uint64[G] or None) is the packing order: packed position i takes group
    perm[i] (qe_pack_order)."""

    def __init__(self, voters, voters_outgoing=None, learners=None, learners_next=None,
                 auto_leave=None):
        self.G = len(voters)
        self.voters = _csr(voters)
        self.voters_outgoing = _csr(voters_outgoing) if voters_outgoing is not None else None
        self.learners = _csr(learners) if learners is not None else None
        self.learners_next = _csr(learners_next) if learners_next is not None else None
        self.auto_leave = (None if auto_leave is None else
                           np.ascontiguousarray(np.asarray(auto_leave, dtype=np.uint8)))
        self.perm = None

    @classmethod
    def from_csr(cls, G, voters, voters_outgoing=None, learners=None, learners_next=None,
                 auto_leave=None):
        """Build from ready CSR pairs (ids uint64, off uint64[G+1]) without
        going through Python lists (large batches)."""
        c = cls.__new__(cls)
        c.G = int(G)
        c.voters, c.voters_outgoing = voters, voters_outgoing
        c.learners, c.learners_next = learners, learners_next
        c.auto_leave = auto_leave
        c.perm = None
        return c

    def struct(self):
        from ._lib import QeConfStateCSR

        def p(x, i):
            return None if x is None else x[i].ctypes.data_as(ctypes.c_void_p)
        return QeConfStateCSR(self.G, p(self.voters, 0), p(self.voters, 1),
                              p(self.voters_outgoing, 0), p(self.voters_outgoing, 1),
                              p(self.learners, 0), p(self.learners, 1),
                              p(self.learners_next, 0), p(self.learners_next, 1),
                              _np_ptr(self.auto_leave), _np_ptr(self.perm))


def _np_ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def pack_order(cs, num_slots):
    """Native qe_pack_order: the shape-bucketed packing order (perm[i] = the
    caller's group at packed position i) and the number of distinct shapes."""
    from . import _lib
    perm = np.zeros(cs.G, dtype=np.uint64)
    nshape = ctypes.c_uint64(0)
    st = cs.struct()
    _lib.check("qe_pack_order", _lib.lib().qe_pack_order(ctypes.byref(st), num_slots,
                                                         _np_ptr(perm), ctypes.byref(nshape)))
    return perm, int(nshape.value)


def pack_confstates(cs, num_slots, bucketed=False):
    """Native qe_pack_confstate -> PackedGroups (masks, slot_ids) + flags.
    bucketed: pack in qe_pack_order's shape order (p.perm maps packed
    positions back to cs's groups); otherwise in cs.perm's order (identity
    when None)."""
    from . import _lib
    if bucketed:
        cs.perm = pack_order(cs, num_slots)[0]
    p = PackedGroups(cs.G, num_slots)
    p.perm = cs.perm
    flags = np.zeros(cs.G, dtype=np.uint32)
    nflag = ctypes.c_uint64(0)
    st = cs.struct()
    _lib.check("qe_pack_confstate", _lib.lib().qe_pack_confstate(
        ctypes.byref(st), num_slots, _np_ptr(p.inc), _np_ptr(p.out), _np_ptr(p.learner),
        _np_ptr(p.slot_ids_sg), _np_ptr(flags), ctypes.byref(nflag)))
    p.flags = flags
    p.num_flagged = int(nflag.value)
    p.joint = cs.voters_outgoing is not None
    return p


def pack_conf(cs, num_slots):
    """Native qe_pack_conf: the full tracker.Config of every group (slot
    ids, Voters[0], Voters[1], Learners, LearnersNext, IsLearner, tracked,
    AutoLeave) as host arrays -- what qe_confchange consumes
    (confchange/restore.go).  Returns (dict of numpy arrays, flags)."""
    from . import _lib
    G, S = cs.G, int(num_slots)
    md = np.uint8 if S <= 8 else np.uint16
    arr = {"slot_ids": np.zeros(S * G, np.uint64), "auto_leave": np.zeros(G, np.uint8)}  # [S][G]
    for k in ("inc", "out", "learner", "learners_next", "is_learner", "tracked"):
        arr[k] = np.zeros(G, md)
    st = cs.struct()
    c = _lib.QeConf(G, S, 0, _np_ptr(arr["slot_ids"]), _np_ptr(arr["inc"]), _np_ptr(arr["out"]),
                    _np_ptr(arr["learner"]), _np_ptr(arr["learners_next"]),
                    _np_ptr(arr["is_learner"]), _np_ptr(arr["tracked"]),
                    _np_ptr(arr["auto_leave"]))
    flags = np.zeros(G, dtype=np.uint32)
    nflag = ctypes.c_uint64(0)
    _lib.check("qe_pack_conf", _lib.lib().qe_pack_conf(ctypes.byref(st), ctypes.byref(c),
                                                       _np_ptr(flags), ctypes.byref(nflag)))
    return arr, flags


def pack_progress(p, progress, stride=None):
    """progress: list (per caller group) of {id: Match} -> p.match (packed
    order, through p.perm) via qe_pack_match."""
    from . import _lib
    ids, off = _csr([list(d.keys()) for d in progress])
    vals = np.fromiter((v for d in progress for v in d.values()), dtype=np.uint64,
                       count=int(off[-1]))
    stride = stride or p.G
    match = np.zeros(p.S * stride, dtype=np.uint64)
    unknown = ctypes.c_uint64(0)
    _lib.check("qe_pack_match", _lib.lib().qe_pack_match(
        p.G, p.S, _np_ptr(p.slot_ids_sg), _np_ptr(p.perm), _np_ptr(off), _np_ptr(ids),
        _np_ptr(vals), _np_ptr(match), stride, ctypes.byref(unknown)))
    p.match = match.reshape(p.S, stride)[:, : p.G]
    return int(unknown.value)


def pack_votes(p, votes):
    """votes: list (per caller group) of [(id, bool), ...] in arrival order."""
    from . import _lib
    ids, off = _csr([[i for i, _ in v] for v in votes])
    vals = np.fromiter((int(b) for v in votes for _, b in v), dtype=np.uint8, count=int(off[-1]))
    _lib.check("qe_pack_votes", _lib.lib().qe_pack_votes(
        p.G, p.S, _np_ptr(p.slot_ids_sg), _np_ptr(p.perm), _np_ptr(off), _np_ptr(ids),
        _np_ptr(vals), _np_ptr(p.voted), _np_ptr(p.granted)))


def slot_lookup(p, group, ids):
    from . import _lib
    group = np.ascontiguousarray(group, dtype=np.uint64)
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    out = np.zeros(len(ids), dtype=np.int8)
    _lib.check("qe_slot_lookup", _lib.lib().qe_slot_lookup(
        p.G, p.S, _np_ptr(p.slot_ids_sg), len(ids), _np_ptr(group), _np_ptr(ids), _np_ptr(out)))
    return out
