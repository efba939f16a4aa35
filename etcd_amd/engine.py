"""Device-buffer layer over the C ABI: slot-SoA batches held in HBM as torch
tensors (torch is plumbing here: allocation, streams, distributed), and thin
callers of every qe_* entry point.

Layout: match is [S][stride] uint64 (stored as int64 bits),
masks/bitmaps are uint8 for S <= 8 and uint16 (stored as int16) for S <= 16.
`stride` is rounded up to 64 groups so every slot row starts 512-byte aligned
and the 16-byte vector path is always taken.
"""
import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import (QeElectionParams, QeElectionState, QeGenParams, QeGroups, QeOutputs,
                   QeReplMsgs, QeReplState, check)

ROW_ALIGN = 64


def mask_torch_dtype(S):
    return torch.uint8 if S <= 8 else torch.int16


def mask_np_dtype(S):
    return np.uint8 if S <= 8 else np.uint16


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _np_u64(t):
    return t.detach().cpu().numpy().view(np.uint64)


class SlotBatch:
    """G Raft groups in slot-SoA form on one device (the qe_groups view)."""

    def __init__(self, G, S, device="cuda", masks=("inc", "out", "learner"), votes=True,
                 group_offset=0, stride=None):
        if not 1 <= S <= _lib.QE_MAX_SLOTS:
            raise ValueError(f"num_slots must be 1..{_lib.QE_MAX_SLOTS}")
        self.G, self.S = int(G), int(S)
        self.device = torch.device(device)
        self.group_offset = int(group_offset)
        self.stride = int(stride) if stride else max(ROW_ALIGN, -(-self.G // ROW_ALIGN) * ROW_ALIGN)
        md = mask_torch_dtype(S)
        dev = self.device
        self.match = torch.zeros(self.S * self.stride, dtype=torch.int64, device=dev)
        self.inc = torch.zeros(self.G, dtype=md, device=dev) if "inc" in masks else None
        self.out = torch.zeros(self.G, dtype=md, device=dev) if "out" in masks else None
        self.learner = torch.zeros(self.G, dtype=md, device=dev) if "learner" in masks else None
        self.voted = torch.zeros(self.G, dtype=md, device=dev) if votes else None
        self.granted = torch.zeros(self.G, dtype=md, device=dev) if votes else None

    # -- views --------------------------------------------------------------
    def struct(self):
        return QeGroups(self.G, self.group_offset, self.S, 0, self.stride, _ptr(self.match),
                        _ptr(self.inc), _ptr(self.out), _ptr(self.learner), _ptr(self.voted),
                        _ptr(self.granted))

    def bytes_per_group(self, with_outputs=True):
        """Algorithmic bytes one qe_commit_vote evaluation moves per group."""
        mb = 1 if self.S <= 8 else 2
        b = 8 * self.S
        b += mb * sum(x is not None for x in (self.inc, self.out, self.learner, self.voted,
                                                self.granted))
        if with_outputs:
            b += 8 + 1
        return b

    def match_rows(self):
        """[S][G] view of the match array."""
        return self.match.view(self.S, self.stride)[:, : self.G]

    # -- host transfer ------------------------------------------------------
    def load_host(self, match, inc=None, out=None, learner=None, voted=None, granted=None):
        """match: uint64 array [S][G] (or [S][stride]); masks: [G] arrays."""
        m = np.ascontiguousarray(np.asarray(match, dtype=np.uint64)).reshape(self.S, -1)
        rows = self.match_rows()
        rows.copy_(torch.from_numpy(m[:, : self.G].view(np.int64).copy()).to(self.device))
        md = mask_np_dtype(self.S)
        for name, arr in (("inc", inc), ("out", out), ("learner", learner), ("voted", voted),
                          ("granted", granted)):
            dst = getattr(self, name)
            if arr is None or dst is None:
                continue
            a = np.ascontiguousarray(np.asarray(arr).astype(md))
            if md == np.uint16:
                a = a.view(np.int16)
            dst.copy_(torch.from_numpy(a).to(self.device))
        return self

    def host(self):
        """Return a dict of numpy arrays (match as [S][G] uint64)."""
        md = mask_np_dtype(self.S)
        out = {"match": self.match_rows().cpu().numpy().view(np.uint64)}
        for name in ("inc", "out", "learner", "voted", "granted"):
            t = getattr(self, name)
            out[name] = None if t is None else t.cpu().numpy().view(md)
        return out


def stats_buffer(device="cuda"):
    return torch.zeros(_lib.QE_STATS_WORDS, dtype=torch.int64, device=device)


def stats_reduce(stats):
    """Fold the shards of a stats buffer on device -> int64[16] tensor."""
    out = torch.empty(_lib.QE_STATS_COUNTERS, dtype=torch.int64, device=stats.device)
    check("qe_stats_reduce", _lib.lib().qe_stats_reduce(_ptr(stats), _ptr(out),
                                                         _stream(stats.device)))
    return out


def collect(flags, values=None, group_offset=0, scratch=None, perm=None):
    """qe_collect: the groups with flags[g] != 0 in ascending position order
    (the Ready-style delta of a batch step, e.g. qe_replication_round's `adv`
    with `committed` as values) -> (groups int64[n], values int64[n] or None).
    perm (device int64[G], qe_pack_order) maps packed positions back to the
    caller's group ids.  One int64 count is read back to size the result."""
    G = flags.numel()
    dev = flags.device
    lib = _lib.lib()
    if scratch is None:
        scratch = torch.empty((lib.qe_collect_scratch_bytes(G) + 7) // 8, dtype=torch.int64,
                              device=dev)
    groups = torch.empty(max(1, G), dtype=torch.int64, device=dev)
    vals = torch.empty(max(1, G), dtype=torch.int64, device=dev) if values is not None else None
    count = torch.empty(1, dtype=torch.int64, device=dev)
    check("qe_collect", lib.qe_collect(G, group_offset, _ptr(perm), _ptr(flags), _ptr(values),
                                       _ptr(groups),
                                       _ptr(vals), _ptr(count), _ptr(scratch), _stream(dev)))
    n = int(count.item())
    return groups[:n], (vals[:n] if vals is not None else None)


def stats_dict(folded):
    v = folded.detach().cpu().numpy().view(np.uint64)
    return {name: int(v[i]) for i, name in enumerate(_lib.STAT_NAMES)}


def gen_groups(batch, seed, dist=0, p_absent=3277, p_voted=52429, p_granted=39322, n_inc=0,
               n_out=0, mask_mode=0, values_only=False):
    """Fill `batch` with the counter-based synthetic generator.
    values_only: Match and votes only, the batch's masks are left as they are
    (e.g. as a packer wrote them)."""
    p = QeGenParams(seed, 0, dist, p_absent, p_voted, p_granted, n_inc, n_out, mask_mode, 0)
    g = batch.struct()
    if values_only:
        g.inc_mask = g.out_mask = g.learner_mask = None
    check("qe_gen_groups", _lib.lib().qe_gen_groups(C.byref(g), C.byref(p),
                                                     _stream(batch.device)))
    return batch


class Outputs:
    def __init__(self, G, device, commit=True, vote=True, tally=True):
        self.commit = torch.empty(G, dtype=torch.int64, device=device) if commit else None
        self.vote = torch.empty(G, dtype=torch.uint8, device=device) if vote else None
        self.granted = torch.empty(G, dtype=torch.uint8, device=device) if tally else None
        self.rejected = torch.empty(G, dtype=torch.uint8, device=device) if tally else None

    def struct(self, stats=None):
        return QeOutputs(_ptr(self.commit), _ptr(self.vote), _ptr(self.granted),
                         _ptr(self.rejected), _ptr(stats))


def commit_vote(batch, outputs=None, stats=None):
    """ProgressTracker.Committed + TallyVotes for every group (qe_commit_vote)."""
    if outputs is None:
        outputs = Outputs(batch.G, batch.device)
    g = batch.struct()
    o = outputs.struct(stats)
    check("qe_commit_vote", _lib.lib().qe_commit_vote(C.byref(g), C.byref(o),
                                                       _stream(batch.device)))
    return outputs


def committed_index(batch, commit=None):
    commit = torch.empty(batch.G, dtype=torch.int64, device=batch.device) if commit is None else commit
    g = batch.struct()
    check("qe_committed_index", _lib.lib().qe_committed_index(C.byref(g), _ptr(commit),
                                                               _stream(batch.device)))
    return commit


def vote_result(batch, vote=None):
    vote = torch.empty(batch.G, dtype=torch.uint8, device=batch.device) if vote is None else vote
    g = batch.struct()
    check("qe_vote_result", _lib.lib().qe_vote_result(C.byref(g), _ptr(vote),
                                                       _stream(batch.device)))
    return vote


def quorum_active(batch, recent_active, active=None):
    active = torch.empty(batch.G, dtype=torch.uint8, device=batch.device) if active is None else active
    g = batch.struct()
    check("qe_quorum_active", _lib.lib().qe_quorum_active(C.byref(g), _ptr(recent_active),
                                                           _ptr(active), _stream(batch.device)))
    return active


def record_votes(batch, resp_mask, resp_value):
    check("qe_record_votes", _lib.lib().qe_record_votes(
        batch.G, batch.S, _ptr(batch.voted), _ptr(batch.granted), _ptr(resp_mask),
        _ptr(resp_value), _stream(batch.device)))


class ReplicationState:
    """Leader-side Progress state of G groups for qe_replication_round."""

    def __init__(self, batch, committed, term_start, last_index, nxt=None):
        self.batch = batch
        self.match = batch.match
        self.next = nxt if nxt is not None else batch.match.clone() + 1
        self.committed = committed
        self.term_start = term_start
        self.last_index = last_index

    def struct(self):
        b = self.batch
        return QeReplState(b.G, b.group_offset, b.S, 0, b.stride, _ptr(self.match),
                           _ptr(self.next), _ptr(self.committed), _ptr(self.term_start),
                           _ptr(self.last_index), _ptr(b.inc), _ptr(b.out))


def replication_round(state, resp_index, resp_mask, read_acks=None, read_ok=None, adv=None,
                      stats=None):
    m = QeReplMsgs(_ptr(resp_index), _ptr(resp_mask), _ptr(read_acks), _ptr(read_ok), _ptr(adv))
    s = state.struct()
    check("qe_replication_round", _lib.lib().qe_replication_round(
        C.byref(s), C.byref(m), _ptr(stats), _stream(state.batch.device)))


class ElectionState:
    """Per-group candidate state for qe_election_steps."""

    def __init__(self, batch, self_slot):
        G, dev = batch.G, batch.device
        self.batch = batch
        self.term = torch.zeros(G, dtype=torch.int64, device=dev)
        self.state = torch.zeros(G, dtype=torch.uint8, device=dev)
        self.voted = torch.zeros(G, dtype=mask_torch_dtype(batch.S), device=dev)
        self.granted = torch.zeros(G, dtype=mask_torch_dtype(batch.S), device=dev)
        self.self_slot = self_slot

    def struct(self):
        b = self.batch
        return QeElectionState(b.G, b.group_offset, b.S, 0, _ptr(self.term), _ptr(self.state),
                               _ptr(self.voted), _ptr(self.granted), _ptr(self.self_slot),
                               _ptr(b.inc), _ptr(b.out), _ptr(b.learner))


def first_voter_slot(batch):
    """self_slot = lowest slot of JointConfig[0] (device computation)."""
    inc = batch.inc.to(torch.int32) & ((1 << batch.S) - 1)
    slot = torch.zeros(batch.G, dtype=torch.uint8, device=batch.device)
    found = torch.zeros(batch.G, dtype=torch.bool, device=batch.device)
    for s in range(batch.S):
        bit = ((inc >> s) & 1).bool() & ~found
        slot = torch.where(bit, torch.full_like(slot, s), slot)
        found |= bit
    return slot


def election_steps(est, seed, step0, steps, p_drop=13107, p_grant=32768, stats=None, flags=0,
                   p_active=0, script=None):
    """script: None or (resp, grant, hup, stride) device tensors [steps][stride]
    (hup may be None) replacing the RNG (qe_election_params scripted mode)."""
    sr, sg, sh, ss = script if script is not None else (None, None, None, 0)
    p = QeElectionParams(seed, step0, steps, p_drop, p_grant, flags, p_active, 0, _ptr(sr),
                         _ptr(sg), _ptr(sh), ss)
    s = est.struct()
    check("qe_election_steps", _lib.lib().qe_election_steps(C.byref(s), C.byref(p), _ptr(stats),
                                                             _stream(est.batch.device)))


def tune(key, value):
    check("qe_tune", _lib.lib().qe_tune(key.encode(), int(value)))


def pack_peer_word(flags, start=0, count=0):
    """The packed per-peer word (include/etcd_quorum.h QE_PW_*): flag bits
    (StateType | ProbeSent << 2 | RecentActive << 3), Inflights.start << 8,
    Inflights.count << 16.  numpy arrays or ints."""
    return ((np.asarray(flags, np.uint32) & 0xF) | (np.asarray(start, np.uint32) << 8) |
            (np.asarray(count, np.uint32) << 16)).astype(np.uint32)


class ProgressState:
    """Device-resident leader-side Progress of G groups (qe_progress):
    match/next/pending [S][stride], the packed per-peer words `peer` [S][stride]
    (int32 storage of the u32 QE_PW_* words), Inflights rings as 32-bit entry
    words `ilo` / `ihi` [S][stride][QE_RING_PITCH(F)] (lane-major, ABI 4: the
    upper words come from the peer word's epoch unless QE_PF_RING_WIDE),
    committed, and the leader-log model (term runs).  `extras`
    allocates the optional per-group arrays: "tracked" (slot mask),
    "self_slot", "lead_transferee" (u8, 0xFF = none), "snap_index" (u64),
    "reads" (ABI 5: the ReadIndex queue -- read_acks [G][QE_READ_QUEUE]
    mask-typed, read_head u32 (starting at context 1), read_count u8; ABI 7:
    read_cap > QE_READ_QUEUE adds the overflow ring read_ovf [G][read_cap]
    mask-typed), "read_keys" (ABI 7: [G][cap] u64 request keys, for
    qe_read_index's duplicate check).  ring16 (ABI 8): the rings in the
    16-bit form, `infl16` [S][stride][8] offsets below Next (F <= 8, S <= 9,
    R <= 4; ilo / ihi then hold the wide peers)."""

    def __init__(self, G, S, F, R, device="cuda", masks=(), group_offset=0, stride=None,
                 extras=(), max_ents=0, read_cap=0, ring16=False):
        if not 1 <= S <= _lib.QE_MAX_SLOTS or not 1 <= F <= _lib.QE_MAX_INFLIGHT:
            raise ValueError("bad num_slots / inflight_cap")
        if not 1 <= R <= _lib.QE_MAX_LOG_RUNS:
            raise ValueError("bad log_runs")
        self.G, self.S, self.F, self.R = int(G), int(S), int(F), int(R)
        self.max_ents = int(max_ents)
        self.device = torch.device(device)
        self.group_offset = int(group_offset)
        self.stride = int(stride) if stride else max(ROW_ALIGN, -(-self.G // ROW_ALIGN) * ROW_ALIGN)
        dev, n = self.device, self.S * self.stride
        i64, u8 = torch.int64, torch.uint8
        self.match = torch.zeros(n, dtype=i64, device=dev)
        self.next = torch.ones(n, dtype=i64, device=dev)
        self.pending = torch.zeros(n, dtype=i64, device=dev)
        self.peer = torch.zeros(n, dtype=torch.int32, device=dev)
        self.FP = _lib.QE_RING_PITCH(self.F)
        self.ilo = torch.zeros(n * self.FP, dtype=torch.int32, device=dev)
        self.ihi = torch.zeros(n * self.FP, dtype=torch.int32, device=dev)
        self.committed = torch.zeros(self.G, dtype=i64, device=dev)
        self.term_start = torch.zeros(self.G, dtype=i64, device=dev)
        self.first_index = torch.ones(self.G, dtype=i64, device=dev)
        self.last_index = torch.zeros(self.G, dtype=i64, device=dev)
        self.run_first = torch.zeros(self.R * self.stride, dtype=i64, device=dev)
        self.run_term = torch.zeros(self.R * self.stride, dtype=i64, device=dev)
        self.run_count = torch.zeros(self.G, dtype=u8, device=dev)
        md = mask_torch_dtype(S)
        self.inc = torch.zeros(self.G, dtype=md, device=dev) if "inc" in masks else None
        self.out = torch.zeros(self.G, dtype=md, device=dev) if "out" in masks else None
        self.tracked = torch.zeros(self.G, dtype=md, device=dev) if "tracked" in extras else None
        self.self_slot = (torch.full((self.G,), 0xFF, dtype=u8, device=dev)
                          if "self_slot" in extras else None)
        self.lead_transferee = (torch.full((self.G,), 0xFF, dtype=u8, device=dev)
                                if "lead_transferee" in extras else None)
        self.snap_index = (torch.zeros(self.G, dtype=i64, device=dev)
                           if "snap_index" in extras else None)
        rq = _lib.QE_READ_QUEUE
        self.read_acks = (torch.zeros(self.G * rq, dtype=md, device=dev)
                          if "reads" in extras else None)
        self.read_head = (torch.ones(self.G, dtype=torch.int32, device=dev)
                          if "reads" in extras else None)
        self.read_count = (torch.zeros(self.G, dtype=u8, device=dev)
                           if "reads" in extras else None)
        self.read_cap = int(read_cap)
        cap = max(rq, self.read_cap)
        self.read_ovf = (torch.zeros(self.G * cap, dtype=md, device=dev)
                         if "reads" in extras and cap > rq else None)
        self.read_keys = (torch.zeros(self.G * cap, dtype=i64, device=dev)
                          if "read_keys" in extras else None)
        if ring16 and (self.F > _lib.QE_RING16_MAX_F or self.S > _lib.QE_RING16_MAX_SLOTS or self.R > 4):
            raise ValueError("the 16-bit Inflights form needs F <= 8, S <= 9, R <= 4")
        self.infl16 = (torch.zeros(n * _lib.QE_RING16_MAX_F, dtype=torch.int16, device=dev)
                       if ring16 else None)

    def struct(self):
        return _lib.QeProgress(
            self.G, self.group_offset, self.S, self.F, self.stride, _ptr(self.match),
            _ptr(self.next), _ptr(self.pending), _ptr(self.peer), _ptr(self.ilo), _ptr(self.ihi),
            _ptr(self.committed), _ptr(self.term_start),
            _ptr(self.first_index), _ptr(self.last_index), self.R, 0, _ptr(self.run_first),
            _ptr(self.run_term), _ptr(self.run_count), _ptr(self.inc), _ptr(self.out),
            _ptr(self.tracked), _ptr(self.self_slot), _ptr(self.lead_transferee),
            _ptr(self.snap_index), self.max_ents, 0, _ptr(self.read_acks), _ptr(self.read_head),
            _ptr(self.read_count), self.read_cap, 0, _ptr(self.read_ovf), _ptr(self.read_keys),
            _ptr(self.infl16))

    ARRAYS = ("match", "next", "pending", "peer", "ilo", "ihi", "committed",
              "term_start", "first_index", "last_index", "run_first", "run_term", "run_count",
              "inc", "out", "tracked", "self_slot", "lead_transferee", "snap_index",
              "read_acks", "read_head", "read_count", "read_ovf", "read_keys", "infl16")

    def load_host(self, **arrays):
        """numpy arrays (uint64 as uint64, masks as uint8/uint16, peer words
        as uint32).  flags / istart / icount (uint8 arrays, any subset) are
        packed into the peer words (absent fields 0).  `ibuf` takes plain
        uint64 Inflights rings, entry-major [S][F][stride] (the oracle's
        layout), converted through qe_ring_pack after the peer words are in
        place (their ring representation bits are recomputed).  Without
        `ibuf`, rewritten peer words keep describing the resident rings: the
        rings are decoded with the old words and packed again with the new
        ones (a new Inflights.start / count selects other live entries) --
        unless raw `ilo` / `ihi` words are passed too, which are then taken
        as they are."""
        ibuf = arrays.pop("ibuf", None)
        fields = {k: arrays.pop(k) for k in ("flags", "istart", "icount") if k in arrays}
        raw_rings = "ilo" in arrays or "ihi" in arrays or "infl16" in arrays  # the caller's words stand
        # (the 16-bit form's entries are offsets below Next: a new Next re-bases them)
        rebase = fields or "peer" in arrays or (self.infl16 is not None and "next" in arrays)
        if ibuf is None and not raw_rings and rebase:
            ibuf = self.rings()  # decoded with the words (and Next) in place now
        if fields:
            n = max(np.asarray(v).size for v in fields.values())
            z = np.zeros(n, np.uint32)
            arrays["peer"] = pack_peer_word(fields.get("flags", z), fields.get("istart", z),
                                            fields.get("icount", z))
        for k, a in arrays.items():
            dst = getattr(self, k)
            if dst is None or a is None:
                continue
            a = np.ascontiguousarray(a)
            if a.dtype == np.uint64:
                a = a.view(np.int64)
            elif a.dtype == np.uint16:
                a = a.view(np.int16)
            elif a.dtype == np.uint32:
                a = a.view(np.int32)
            a = a.reshape(-1)[: dst.numel()]
            dst[: a.size].copy_(torch.from_numpy(a.copy()).to(self.device))
        if ibuf is not None:
            self.load_rings(ibuf)
        if "pending" in arrays or "peer" in arrays:
            self.check_pending_precondition()
        return self

    def check_pending_precondition(self):
        """The ABI's precondition (include/etcd_quorum.h qe_progress.
        pending_snapshot): PendingSnapshot is 0 for every peer not in
        StateSnapshot -- ResetState clears it on each state change
        (raft/tracker/progress.go:84-89), and the kernels write it only where
        its value changes.  Raises ValueError on a host-loaded state that
        violates it (results would be unspecified)."""
        pend = self.pending.view(self.S, self.stride)[:, : self.G].cpu().numpy()
        state = self.peer.view(self.S, self.stride)[:, : self.G].cpu().numpy() & 3
        bad = (pend != 0) & (state != _lib.QE_PR_SNAPSHOT)
        if bad.any():
            s, g = (int(x[0]) for x in np.nonzero(bad))
            raise ValueError(f"PendingSnapshot != 0 outside StateSnapshot (slot {s}, group {g}): "
                             "the qe_progress precondition")

    def load_rings(self, ibuf):
        """Plain uint64 rings, entry-major [S][F][stride] -> ilo / ihi and the
        peer words' representation bits (qe_ring_pack, host side)."""
        S, F, st = self.S, self.F, self.stride
        e = np.zeros(S * F * st, np.uint64)
        a = np.asarray(ibuf, np.uint64).reshape(-1)[: e.size]
        e[: a.size] = a
        ent = np.ascontiguousarray(e.reshape(S, F, st).transpose(0, 2, 1))  # [S][stride][F]
        peer = self.peer.cpu().numpy().view(np.uint32).copy()
        lo = np.zeros(S * st * self.FP, np.uint32)
        hi = np.zeros_like(lo)
        if self.infl16 is not None:  # ABI 8: offsets below Next, wide where they do not fit
            nxt = self.next.cpu().numpy().view(np.uint64).copy()
            o16 = np.zeros(S * st * _lib.QE_RING16_MAX_F, np.uint16)
            check("qe_ring_pack16", _lib.lib().qe_ring_pack16(
                self.G, S, F, st, ent.ctypes.data, nxt.ctypes.data, peer.ctypes.data,
                o16.ctypes.data, lo.ctypes.data, hi.ctypes.data))
            self.infl16.copy_(torch.from_numpy(o16.view(np.int16)).to(self.device))
        else:
            check("qe_ring_pack", _lib.lib().qe_ring_pack(
                self.G, S, F, st, ent.ctypes.data, peer.ctypes.data, lo.ctypes.data, hi.ctypes.data))
        for dst, v in ((self.peer, peer), (self.ilo, lo), (self.ihi, hi)):
            dst.copy_(torch.from_numpy(v.view(np.int32)).to(self.device))

    def set_ring_slot(self, s, ent):
        """Slot s's rings from a device int64 tensor [stride][F] (uint64
        entries), in place on the device: the 32-bit words, and the peer
        words' representation bits in canonical form (the rule of
        qe_ring_pack) from their Inflights.start / count."""
        S, F, st, FP = self.S, self.F, self.stride, self.FP
        ent = ent.view(st, F)
        lo = ent & 0xFFFFFFFF
        hi = (ent >> 32) & 0xFFFFFFFF
        as_i32 = lambda v: torch.where(v >= (1 << 31), v - (1 << 32), v).to(torch.int32)  # noqa: E731
        rows = slice(s * st, (s + 1) * st)
        self.ilo.view(S * st, FP)[rows, :F] = as_i32(lo)
        self.ihi.view(S * st, FP)[rows, :F] = as_i32(hi)
        w = self.peer[rows].to(torch.int64) & 0xFFFFFFFF
        start, count = (w >> 8) & 0xFF, (w >> 16) & 0xFF
        k = torch.arange(F, device=self.device).view(1, F)
        live = torch.remainder(k - start.view(st, 1), F) < count.view(st, 1)
        if self.infl16 is not None:  # ABI 8: offsets below Next (the rule of qe_ring_pack16)
            top = (self.next[rows] - 1).view(st, 1)
            d = top - ent  # int64; entries and Next below 2^63 here
            off = d & 0xFFFF
            fits = ((d >= 0) & (d <= 0xFFFF)) | ~live
            o = torch.zeros(st, _lib.QE_RING16_MAX_F, dtype=torch.int64, device=self.device)
            o[:, :F] = off
            self.infl16.view(S * st, _lib.QE_RING16_MAX_F)[rows] = torch.where(
                o >= (1 << 15), o - (1 << 16), o).to(torch.int16)
            rep = torch.where(fits.all(1), 0, _lib.QE_PF_RING_WIDE)
            w = (w & ~_lib.QE_PW_RING_MASK & 0xFFFFFFFF) | rep
            self.peer[rows] = as_i32(w)
            return
        hmin = torch.where(live, hi, 1 << 40).amin(1)
        hmax = torch.where(live, hi, -1).amax(1)
        uni = (hmin == hmax) & (hmax <= _lib.QE_RING_EPOCH_MAX)
        h = torch.where(uni, hmin, 0)
        ep_bits = ((h & 7) << 5) | ((h & 0x7F8) << 21)
        rep = torch.where(count == 0, 0, torch.where(uni, ep_bits, _lib.QE_PF_RING_WIDE))
        w = (w & ~_lib.QE_PW_RING_MASK & 0xFFFFFFFF) | rep
        self.peer[rows] = as_i32(w)

    def rings(self, peer=None):
        """Every ring position decoded to uint64 (qe_ring_unpack), entry-major
        [S][F][stride] flattened (groups >= G are 0)."""
        S, F, st = self.S, self.F, self.stride
        if peer is None:
            peer = self.peer.cpu().numpy().view(np.uint32)
        lo = self.ilo.cpu().numpy().view(np.uint32)
        hi = self.ihi.cpu().numpy().view(np.uint32)
        ent = np.zeros(S * st * F, np.uint64)
        if self.infl16 is not None:  # ABI 8
            o16 = self.infl16.cpu().numpy().view(np.uint16)
            nxt = self.next.cpu().numpy().view(np.uint64)
            check("qe_ring_unpack16", _lib.lib().qe_ring_unpack16(
                self.G, S, F, st, o16.ctypes.data, lo.ctypes.data, hi.ctypes.data,
                nxt.ctypes.data, np.ascontiguousarray(peer).ctypes.data, ent.ctypes.data))
        else:
            check("qe_ring_unpack", _lib.lib().qe_ring_unpack(
                self.G, S, F, st, lo.ctypes.data, hi.ctypes.data,
                np.ascontiguousarray(peer).ctypes.data, ent.ctypes.data))
        return np.ascontiguousarray(ent.reshape(S, st, F).transpose(0, 2, 1)).reshape(-1)

    def host(self):
        out = {}
        for k in self.ARRAYS:
            t = getattr(self, k)
            if t is None:
                out[k] = None
                continue
            a = t.cpu().numpy()
            out[k] = a.view(np.uint64) if a.dtype == np.int64 else (
                a.view(np.uint16) if a.dtype == np.int16 else (
                    a.view(np.uint32) if a.dtype == np.int32 else a))
        w = out["peer"]
        out["ibuf"] = self.rings(w)
        out["flags"] = (w & 0xF).astype(np.uint8)
        out["istart"] = ((w >> 8) & 0xFF).astype(np.uint8)
        out["icount"] = ((w >> 16) & 0xFF).astype(np.uint8)
        return out


class PeerMsgs:
    """One round of per-peer messages for qe_progress_step ([S][stride]) and
    its outputs (sent / snap / timeout_now masks and bcast count per group,
    msg_count / msg_index per peer)."""

    def __init__(self, ps, outputs=True):
        dev, n = ps.device, ps.S * ps.stride
        md = mask_torch_dtype(ps.S)
        self.type = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.index = torch.zeros(n, dtype=torch.int64, device=dev)
        self.reject_hint = torch.zeros(n, dtype=torch.int64, device=dev)
        self.log_term = torch.zeros(n, dtype=torch.int64, device=dev)
        self.sent = torch.zeros(ps.G, dtype=md, device=dev) if outputs else None
        self.bcast = torch.zeros(ps.G, dtype=torch.uint8, device=dev) if outputs else None
        self.snap = torch.zeros(ps.G, dtype=md, device=dev) if outputs else None
        self.timeout_now = torch.zeros(ps.G, dtype=md, device=dev) if outputs else None
        self.msg_count = torch.zeros(n, dtype=torch.uint8, device=dev) if outputs else None
        self.msg_index = torch.zeros(n, dtype=torch.int64, device=dev) if outputs else None
        self.bytes_requested = None
        # ReadIndex (ABI 5): contexts carried by heartbeat responses (None =
        # the newest pending at the start of the round) and the outputs
        self.read_ctx = None       # [S][stride] uint32 (int32 storage)
        self.read_released = torch.zeros(ps.G, dtype=torch.uint8, device=dev) if outputs else None
        self.term_commit = torch.zeros(ps.G, dtype=torch.uint8, device=dev) if outputs else None
        self.term_commit_index = (torch.zeros(ps.G, dtype=torch.int64, device=dev)
                                  if outputs else None)

    def set_read_ctx(self, ps, ctx):
        """Context numbers of the heartbeat responses: uint32 [S][stride]
        (numpy or tensor); None = every response carries the newest context
        pending when the round starts."""
        if ctx is None:
            self.read_ctx = None
            return self
        if not torch.is_tensor(ctx):
            a = np.ascontiguousarray(np.asarray(ctx, np.uint32)).view(np.int32)
            ctx = torch.from_numpy(a.copy())
        t = torch.zeros(ps.S * ps.stride, dtype=torch.int32, device=ps.device)
        t[: ctx.numel()].copy_(ctx.reshape(-1).to(torch.int32))
        self.read_ctx = t
        return self

    def struct(self):
        return _lib.QePeerMsgs(_ptr(self.type), _ptr(self.index), _ptr(self.reject_hint),
                               _ptr(self.log_term), _ptr(self.sent), _ptr(self.bcast),
                               _ptr(self.snap), _ptr(self.timeout_now), _ptr(self.msg_count),
                               _ptr(self.msg_index), _ptr(self.bytes_requested),
                               _ptr(self.read_ctx), _ptr(self.read_released),
                               _ptr(self.term_commit), _ptr(self.term_commit_index))


def progress_step(ps, msgs, stats=None):
    p, m = ps.struct(), msgs.struct()
    check("qe_progress_step", _lib.lib().qe_progress_step(C.byref(p), C.byref(m), _ptr(stats),
                                                           _stream(ps.device)))


def progress_bytes_requested(ps, msgs):
    """Run one round through the instrumented kernel variant and return the
    bytes it requested (reads + writes at field granularity): the
    algorithmic bytes of that round.  Mutates the state like progress_step."""
    acct = torch.zeros(1, dtype=torch.int64, device=ps.device)
    msgs.bytes_requested = acct
    try:
        progress_step(ps, msgs)
    finally:
        msgs.bytes_requested = None
    return int(acct.item())


def progress_send(ps, want, send_if_empty=False):
    """qe_progress_send: MaxSizePerMsg is ps.max_ents (ABI 3)."""
    sent = torch.zeros(ps.G, dtype=mask_torch_dtype(ps.S), device=ps.device)
    snap = torch.zeros(ps.G, dtype=mask_torch_dtype(ps.S), device=ps.device)
    p = ps.struct()
    check("qe_progress_send", _lib.lib().qe_progress_send(
        C.byref(p), _ptr(want), int(bool(send_if_empty)), _ptr(sent), _ptr(snap),
        _stream(ps.device)))
    return sent, snap


def read_index(ps, request, lease_based=False, key=None):
    """qe_read_index: MsgReadIndex on the leader of every group with
    request[g] != 0 (raft/raft.go:1078-1096) -> (result uint8[G] QE_RI_*,
    ctx int32[G] (the context number of a QUEUED request, or of the pending
    one a DUPLICATE key names), index int64[G] (the read index of RESPOND /
    QUEUED)).  key: int64[G] request keys (ABI 7, with ps.read_keys)."""
    G, dev = ps.G, ps.device
    result = torch.zeros(G, dtype=torch.uint8, device=dev)
    ctx = torch.zeros(G, dtype=torch.int32, device=dev)
    index = torch.zeros(G, dtype=torch.int64, device=dev)
    p = ps.struct()
    check("qe_read_index", _lib.lib().qe_read_index(
        C.byref(p), _ptr(request), _ptr(key), int(bool(lease_based)), _ptr(result), _ptr(ctx),
        _ptr(index),
        _stream(dev)))
    return result, ctx, index


def check_quorum(ps, quorum_active=None, stats=None):
    """qe_check_quorum: MsgCheckQuorum on every group's leader
    (raft/raft.go:997-1018) over the resident Progress words -> uint8[G]
    QuorumActive (0 = the leader steps down)."""
    if quorum_active is None:
        quorum_active = torch.empty(ps.G, dtype=torch.uint8, device=ps.device)
    p = ps.struct()
    check("qe_check_quorum", _lib.lib().qe_check_quorum(C.byref(p), _ptr(quorum_active),
                                                         _ptr(stats), _stream(ps.device)))
    return quorum_active


def heartbeat(ps, commit=None, ctx=None, sent=None):
    """qe_heartbeat: MsgBeat -> bcastHeartbeat (raft/raft.go:524-541) ->
    (commit int64 [S][stride]: min(Match, committed) of every slot sent to,
    ctx int32 [G]: the newest pending ReadIndex context, sent mask [G])."""
    if commit is None:
        commit = torch.zeros(ps.S * ps.stride, dtype=torch.int64, device=ps.device)
    if ctx is None:
        ctx = torch.zeros(ps.G, dtype=torch.int32, device=ps.device)
    if sent is None:
        sent = torch.zeros(ps.G, dtype=mask_torch_dtype(ps.S), device=ps.device)
    p = ps.struct()
    check("qe_heartbeat", _lib.lib().qe_heartbeat(C.byref(p), _ptr(commit), _ptr(ctx), _ptr(sent),
                                                   _stream(ps.device)))
    return commit, ctx, sent


class Proposals:
    """One MsgProp per group for qe_propose (qe_proposals, ABI 6):
    num_entries [G] (0 = none), payload [G] (sum of the non-conf-change
    entries' PayloadSize), up to max_cc conf-change entries per proposal
    ([max_cc][G]: position, leave-joint flag, size), applied /
    pending_conf_index / uncommitted_size [G], and the outputs result,
    cc_refused, sent, snap [G]."""

    def __init__(self, ps, max_cc=0, max_uncommitted=0, track_uncommitted=True, flags=0):
        G, dev = ps.G, ps.device
        self.G, self.max_cc, self.max_uncommitted = G, int(max_cc), int(max_uncommitted)
        self.flags = int(flags)  # QE_PROP_APPEND_ONLY: appendEntry alone
        i64 = torch.int64
        self.num_entries = torch.zeros(G, dtype=torch.int32, device=dev)
        self.payload = torch.zeros(G, dtype=i64, device=dev)
        c = max(1, self.max_cc)
        self.cc_count = torch.zeros(G, dtype=torch.uint8, device=dev)
        self.cc_pos = torch.zeros(c * G, dtype=torch.int32, device=dev)
        self.cc_leave = torch.zeros(c * G, dtype=torch.uint8, device=dev)
        self.cc_size = torch.zeros(c * G, dtype=torch.int32, device=dev)
        self.applied = torch.zeros(G, dtype=i64, device=dev)
        self.pending_conf_index = torch.zeros(G, dtype=i64, device=dev)
        self.uncommitted_size = torch.zeros(G, dtype=i64, device=dev) if track_uncommitted else None
        self.result = torch.zeros(G, dtype=torch.uint8, device=dev)
        self.cc_refused = torch.zeros(G, dtype=torch.uint8, device=dev)
        md = mask_torch_dtype(ps.S)
        self.sent = torch.zeros(G, dtype=md, device=dev)
        self.snap = torch.zeros(G, dtype=md, device=dev)
        self.bytes_requested = None

    def struct(self):
        cc = self.max_cc > 0
        return _lib.QeProposals(
            _ptr(self.num_entries), _ptr(self.payload), self.max_cc, self.flags, self.G,
            _ptr(self.cc_count) if cc else None, _ptr(self.cc_pos) if cc else None,
            _ptr(self.cc_leave) if cc else None, _ptr(self.cc_size) if cc else None,
            _ptr(self.applied), _ptr(self.pending_conf_index), _ptr(self.uncommitted_size),
            self.max_uncommitted, _ptr(self.result), _ptr(self.cc_refused), _ptr(self.sent),
            _ptr(self.snap), _ptr(self.bytes_requested))


def propose(ps, props, stats=None):
    """qe_propose: stepLeader's MsgProp + appendEntry + bcastAppend
    (raft/raft.go:1019-1076, :621-642, :515-522) for every group with
    num_entries > 0; advances ps.last_index."""
    p, q = ps.struct(), props.struct()
    check("qe_propose", _lib.lib().qe_propose(C.byref(p), C.byref(q), _ptr(stats),
                                               _stream(ps.device)))


def propose_bytes_requested(ps, props):
    """The algorithmic bytes of one qe_propose launch (instrumented variant,
    field granularity); mutates the state like propose."""
    acct = torch.zeros(1, dtype=torch.int64, device=ps.device)
    props.bytes_requested = acct
    try:
        propose(ps, props)
    finally:
        props.bytes_requested = None
    return int(acct.item())


class Switch:
    """One qe_switch_config call's per-group flags and outputs (qe_switch,
    ABI 7): switched [G] (None = every group), result [G] (QE_SW_*, bit
    QE_SW_TRANSFER_ABORTED), sent / snap masks [G]."""

    def __init__(self, ps, switched=None):
        G, dev = ps.G, ps.device
        self.switched = switched
        self.result = torch.zeros(G, dtype=torch.uint8, device=dev)
        md = mask_torch_dtype(ps.S)
        self.sent = torch.zeros(G, dtype=md, device=dev)
        self.snap = torch.zeros(G, dtype=md, device=dev)
        self.bytes_requested = None

    def struct(self):
        return _lib.QeSwitch(_ptr(self.switched), _ptr(self.result), _ptr(self.sent),
                             _ptr(self.snap), _ptr(self.bytes_requested))


def switch_config(ps, sw, stats=None):
    """qe_switch_config: raft.switchToConfig (raft/raft.go:1651-1700) on every
    group with sw.switched[g], the new configuration being ps's inc / out /
    tracked masks: maybeCommit under it, then bcastAppend or the probe of
    every peer, and abortLeaderTransfer for a transferee no longer a voter."""
    p, q = ps.struct(), sw.struct()
    check("qe_switch_config", _lib.lib().qe_switch_config(C.byref(p), C.byref(q), _ptr(stats),
                                                           _stream(ps.device)))
    return sw


def switch_bytes_requested(ps, sw):
    """The algorithmic bytes of one qe_switch_config launch (instrumented
    variant, field granularity); mutates the state like switch_config."""
    acct = torch.zeros(1, dtype=torch.int64, device=ps.device)
    sw.bytes_requested = acct
    try:
        switch_config(ps, sw)
    finally:
        sw.bytes_requested = None
    return int(acct.item())


class Leader:
    """One qe_become_leader call's per-group inputs and outputs (qe_leader,
    ABI 7): elected [G] (None = every group), term [G], pending_conf_index /
    uncommitted_size [G] outputs, result [G] (QE_BL_*), sent / snap masks."""

    def __init__(self, ps, elected=None, bcast=True):
        G, dev = ps.G, ps.device
        self.elected = elected
        self.term = torch.zeros(G, dtype=torch.int64, device=dev)
        self.flags = _lib.QE_BL_BCAST if bcast else 0
        self.pending_conf_index = torch.zeros(G, dtype=torch.int64, device=dev)
        self.uncommitted_size = torch.zeros(G, dtype=torch.int64, device=dev)
        self.result = torch.zeros(G, dtype=torch.uint8, device=dev)
        md = mask_torch_dtype(ps.S)
        self.sent = torch.zeros(G, dtype=md, device=dev)
        self.snap = torch.zeros(G, dtype=md, device=dev)

    def struct(self):
        return _lib.QeLeader(_ptr(self.elected), _ptr(self.term), self.flags, 0,
                             _ptr(self.pending_conf_index), _ptr(self.uncommitted_size),
                             _ptr(self.result), _ptr(self.sent), _ptr(self.snap))


def become_leader(ps, ld, stats=None):
    """qe_become_leader: raft.becomeLeader (raft/raft.go:724-759, reset
    :590-613) on every group with ld.elected[g] -- every Progress reset, the
    log model enters ld.term[g], the empty entry appended and (bcast)
    stepCandidate's bcastAppend."""
    p, q = ps.struct(), ld.struct()
    check("qe_become_leader", _lib.lib().qe_become_leader(C.byref(p), C.byref(q), _ptr(stats),
                                                           _stream(ps.device)))
    return ld


class ConfState:
    """Device-resident tracker.Config + ProgressMap key set of G groups in
    slot form (qe_conf): slot_ids ID-major [S][G], slot masks for Voters[0],
    Voters[1], Learners, LearnersNext, Progress.IsLearner and tracked slots,
    and AutoLeave."""

    MASKS = ("inc", "out", "learner", "learners_next", "is_learner", "tracked")

    def __init__(self, G, S, device="cuda"):
        if not 1 <= S <= _lib.QE_MAX_SLOTS:
            raise ValueError("bad num_slots")
        self.G, self.S, self.device = int(G), int(S), torch.device(device)
        md = mask_torch_dtype(S)
        self.slot_ids = torch.zeros(self.G * self.S, dtype=torch.int64, device=self.device)
        for k in self.MASKS:
            setattr(self, k, torch.zeros(self.G, dtype=md, device=self.device))
        self.auto_leave = torch.zeros(self.G, dtype=torch.uint8, device=self.device)

    def struct(self):
        return _lib.QeConf(self.G, self.S, 0, _ptr(self.slot_ids), _ptr(self.inc), _ptr(self.out),
                           _ptr(self.learner), _ptr(self.learners_next), _ptr(self.is_learner),
                           _ptr(self.tracked), _ptr(self.auto_leave))

    def host(self):
        md = mask_np_dtype(self.S)
        out = {"slot_ids": self.slot_ids.cpu().numpy().view(np.uint64).reshape(self.S, self.G).T,
               "auto_leave": self.auto_leave.cpu().numpy()}
        for k in self.MASKS:
            out[k] = getattr(self, k).cpu().numpy().view(md)
        return out


class ConfChanges:
    """One configuration-change operation per group (qe_conf_changes):
    op [G], count [G], type/node_id [C][stride], last_index [G]; result and
    new_progress are outputs."""

    def __init__(self, G, S, C_max, device="cuda"):
        self.G, self.C = int(G), int(C_max)
        self.stride = max(1, self.G)
        dev = torch.device(device)
        self.op = torch.zeros(self.G, dtype=torch.uint8, device=dev)
        self.count = torch.zeros(self.G, dtype=torch.uint8, device=dev)
        self.type = torch.zeros(max(1, self.C) * self.stride, dtype=torch.uint8, device=dev)
        self.node_id = torch.zeros(max(1, self.C) * self.stride, dtype=torch.int64, device=dev)
        self.last_index = torch.zeros(self.G, dtype=torch.int64, device=dev)
        self.result = torch.zeros(self.G, dtype=torch.uint8, device=dev)
        self.new_progress = torch.zeros(self.G, dtype=mask_torch_dtype(S), device=dev)

    def struct(self):
        return _lib.QeConfChanges(self.C, 0, self.stride, _ptr(self.op), _ptr(self.count),
                                  _ptr(self.type), _ptr(self.node_id), _ptr(self.last_index),
                                  _ptr(self.result), _ptr(self.new_progress))


def confchange(cs, ch, ps=None):
    """Changer.Simple / EnterJoint / LeaveJoint per group on the GPU
    (qe_confchange, raft/confchange/confchange.go:49-274)."""
    c, x = cs.struct(), ch.struct()
    p = C.byref(ps.struct()) if ps is not None else None
    check("qe_confchange", _lib.lib().qe_confchange(C.byref(c), C.byref(x), p,
                                                     _stream(cs.device)))
