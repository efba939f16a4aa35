"""ctypes wrapper over oracle/build/liborc.so (the C restatement in
oracle/quorum_oracle.c).  TEST INFRASTRUCTURE ONLY -- used by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker or the
CPU baseline, never by the product package etcd_amd/.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# QE_ORC_LIB: a sanitizer build of the same source (tests/test_sanitizers.py)
LIB_PATH = os.environ.get("QE_ORC_LIB", os.path.join(HERE, "build", "liborc.so"))
INF = (1 << 64) - 1
NSTAT = 16

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def _declare(L):
    u64, u32, i32, vp, dbl = C.c_uint64, C.c_uint32, C.c_int, C.c_void_p, C.c_double
    sig = {
        "orc_mix64": (u64, [u64]),
        "orc_hash": (u64, [u64, u64, u32, u32]),
        "orc_majority_committed": (u64, [u32, u32, vp]),
        "orc_alt_committed": (u64, [u32, u32, vp]),
        "orc_majority_vote": (C.c_uint8, [u32, u32, u32]),
        "orc_joint_committed": (u64, [u32, u32, u32, vp]),
        "orc_joint_vote": (C.c_uint8, [u32, u32, u32, u32]),
        "orc_quorum_active": (C.c_uint8, [u32, u32, u32, u32]),
        "orc_gen_batch": (None, [u64, u64, u32, u64, u64, u32, u32, u32, u32, u32, u32, u32,
                                 vp, vp, vp, vp, vp, vp, i32]),
        "orc_commit_vote_batch": (None, [u64, u64, u32, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                         vp, vp, i32, i32]),
        "orc_quorum_active_batch": (None, [u64, u32, vp, vp, vp, vp, vp]),
        "orc_record_votes_batch": (None, [u64, u32, vp, vp, vp, vp]),
        "orc_replication_round_batch": (None, [u64, u64, u32, u64, vp, vp, vp, vp, vp, vp, vp, vp,
                                               vp, vp, vp, vp, vp, i32]),
        "orc_election_steps_batch": (None, [u64, u64, u32, vp, vp, vp, vp, vp, vp, vp, vp, u64,
                                            u64, u32, u32, u32, u32, u32, vp, vp, vp, u64, vp,
                                            i32]),
        "orc_gf_build": (vp, [u64, u32, u64, vp, vp, vp, vp, vp, vp]),
        "orc_gf_free": (None, [vp]),
        "orc_gf_run": (dbl, [vp, vp, vp, i32, i32]),
        "orc_soa_run": (dbl, [u64, u32, u64, vp, vp, vp, vp, vp, vp, vp, i32, i32]),
        "orc_max_threads": (i32, []),
        "orc_progress_step_batch": (None, [C.POINTER(OrcProg), C.POINTER(OrcMsgs), vp, i32]),
        "orc_check_quorum_batch": (None, [C.POINTER(OrcProg), vp, vp]),
        "orc_read_index_batch": (None, [C.POINTER(OrcProg), vp, vp, u32, vp, vp, vp]),
        "orc_progress_send_batch": (None, [C.POINTER(OrcProg), vp, u32, u32, vp, vp]),
        "orc_propose_batch": (None, [C.POINTER(OrcProg), C.POINTER(OrcProps), vp]),
        "orc_checksum_prop": (u64, [u64, u32, u64, u64, u32]),
        "orc_heartbeat_batch": (None, [C.POINTER(OrcProg), vp, vp, vp]),
        "orc_switch_config_batch": (None, [C.POINTER(OrcProg), vp, vp, vp, vp, vp, vp]),
        "orc_become_leader_batch": (None, [C.POINTER(OrcProg), vp, vp, u32, vp, vp, vp, vp, vp,
                                           vp]),
        "orc_checksum_switch": (u64, [u64, u32, u64, u32, u32]),
        "orc_find_conflict_by_term": (u64, [u32, vp, vp, u64, u64, u64]),
        "orc_log_term": (u64, [u32, vp, vp, u64, u64]),
        "orc_pr_maybe_decr_to": (i32, [u32, vp, vp, u64, u64]),
        "orc_pr_is_paused": (i32, [u32, u32, u32, u32]),
        "orc_pr_become_probe": (u64, [u32, u64, u64, u64]),
        "orc_inflights_ops": (None, [u32, vp, vp, vp, vp, u32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


def P(a):
    """Pointer of a numpy array (or None)."""
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def mask_dtype(S):
    return np.uint8 if S <= 8 else np.uint16


class Batch:
    """Host slot-SoA batch (same layout as qe_groups)."""

    def __init__(self, G, S, stride=None, masks=("inc", "out", "learner"), votes=True):
        self.G, self.S = G, S
        self.stride = stride or G
        md = mask_dtype(S)
        self.match = np.zeros(S * self.stride, dtype=np.uint64)
        self.inc = np.zeros(G, md) if "inc" in masks else None
        self.out = np.zeros(G, md) if "out" in masks else None
        self.learner = np.zeros(G, md) if "learner" in masks else None
        self.voted = np.zeros(G, md) if votes else None
        self.granted = np.zeros(G, md) if votes else None


def gen_batch(b, seed, goff=0, dist=0, p_absent=3277, p_voted=52429, p_granted=39322,
              n_inc=0, n_out=0, mask_mode=0, threads=0):
    lib().orc_gen_batch(b.G, goff, b.S, b.stride, seed, dist, p_absent, p_voted, p_granted,
                        n_inc, n_out, mask_mode, P(b.match), P(b.inc), P(b.out), P(b.learner),
                        P(b.voted), P(b.granted), threads)
    return b


def commit_vote(b, goff=0, alg=0, threads=0):
    commit = np.zeros(b.G, np.uint64)
    vote = np.zeros(b.G, np.uint8)
    gc = np.zeros(b.G, np.uint8)
    rc = np.zeros(b.G, np.uint8)
    stats = np.zeros(NSTAT, np.uint64)
    lib().orc_commit_vote_batch(b.G, goff, b.S, b.stride, P(b.match), P(b.inc), P(b.out),
                                P(b.learner), P(b.voted), P(b.granted), P(commit), P(vote), P(gc),
                                P(rc), P(stats), alg, threads)
    return commit, vote, gc, rc, stats


def quorum_active(G, S, inc, out, learner, recent):
    active = np.zeros(G, np.uint8)
    lib().orc_quorum_active_batch(G, S, P(inc), P(out), P(learner), P(recent), P(active))
    return active


def record_votes(G, S, voted, granted, resp, value):
    lib().orc_record_votes_batch(G, S, P(voted), P(granted), P(resp), P(value))


def replication_round(G, goff, S, stride, match, nxt, committed, term_start, last_index, inc,
                      out, resp_index, resp_mask, read_acks, threads=0):
    read_ok = np.zeros(G, np.uint8)
    adv = np.zeros(G, np.uint8)
    stats = np.zeros(NSTAT, np.uint64)
    lib().orc_replication_round_batch(G, goff, S, stride, P(match), P(nxt), P(committed),
                                      P(term_start), P(last_index), P(inc), P(out), P(resp_index),
                                      P(resp_mask), P(read_acks), P(read_ok), P(adv), P(stats),
                                      threads)
    return read_ok, adv, stats


def election_steps(G, goff, S, term, state, voted, granted, self_slot, inc, out, learner, seed,
                   step0, steps, p_drop, p_grant, threads=0, flags=0, p_active=0, script=None):
    """script: None or (resp, grant, hup, stride) arrays [steps][stride]."""
    stats = np.zeros(NSTAT, np.uint64)
    sr, sg, sh, ss = script if script is not None else (None, None, None, 0)
    lib().orc_election_steps_batch(G, goff, S, P(term), P(state), P(voted), P(granted),
                                   P(self_slot), P(inc), P(out), P(learner), seed, step0, steps,
                                   p_drop, p_grant, flags, p_active, P(sr), P(sg), P(sh), ss,
                                   P(stats), threads)
    return stats


def max_threads():
    return lib().orc_max_threads()


class OrcProg(C.Structure):
    """orc_prog (oracle/quorum_oracle.c), the oracle's mirror of qe_progress."""
    _fields_ = [
        ("G", C.c_uint64), ("goff", C.c_uint64), ("S", C.c_uint32), ("F", C.c_uint32),
        ("stride", C.c_uint64), ("match", C.c_void_p), ("next", C.c_void_p),
        ("pending", C.c_void_p), ("pw", C.c_void_p), ("ibuf", C.c_void_p),
        ("committed", C.c_void_p),
        ("term_start", C.c_void_p), ("first_index", C.c_void_p), ("last_index", C.c_void_p),
        ("R", C.c_uint32), ("reserved", C.c_uint32), ("run_first", C.c_void_p),
        ("run_term", C.c_void_p), ("run_count", C.c_void_p), ("inc", C.c_void_p),
        ("out", C.c_void_p), ("tracked", C.c_void_p), ("self_slot", C.c_void_p),
        ("lead_transferee", C.c_void_p), ("snap_index", C.c_void_p), ("max_ents", C.c_uint32),
        ("reserved2", C.c_uint32), ("read_acks", C.c_void_p), ("read_head", C.c_void_p),
        ("read_count", C.c_void_p), ("read_cap", C.c_uint32), ("reserved3", C.c_uint32),
        ("read_ovf", C.c_void_p), ("read_keys", C.c_void_p),
        ("infl16", C.c_void_p),  # ABI 8: a flag here (the byte rules of 2-B entries)
    ]


class OrcMsgs(C.Structure):
    _fields_ = [("type", C.c_void_p), ("index", C.c_void_p), ("hint", C.c_void_p),
                ("logterm", C.c_void_p), ("sent", C.c_void_p), ("bcast", C.c_void_p),
                ("snap", C.c_void_p), ("timeout_now", C.c_void_p), ("msg_count", C.c_void_p),
                ("msg_index", C.c_void_p), ("read_ctx", C.c_void_p),
                ("read_released", C.c_void_p), ("term_commit", C.c_void_p),
                ("term_commit_index", C.c_void_p), ("bytes", C.c_void_p)]


class OrcProps(C.Structure):
    """orc_props (oracle/quorum_oracle.c), the oracle's mirror of qe_proposals."""
    _fields_ = [("num_entries", C.c_void_p), ("payload", C.c_void_p), ("max_cc", C.c_uint32),
                ("flags", C.c_uint32), ("cc_stride", C.c_uint64), ("cc_count", C.c_void_p),
                ("cc_pos", C.c_void_p), ("cc_leave", C.c_void_p), ("cc_size", C.c_void_p),
                ("applied", C.c_void_p), ("pending_conf_index", C.c_void_p),
                ("uncommitted_size", C.c_void_p), ("max_uncommitted", C.c_uint64),
                ("result", C.c_void_p), ("cc_refused", C.c_void_p), ("sent", C.c_void_p),
                ("snap", C.c_void_p), ("bytes", C.c_void_p)]


PF_STATE, PF_PROBE_SENT, PF_RECENT_ACTIVE = 3, 4, 8


def pack_word(flags, start, count):
    """Packed per-peer word (QE_PW_*): the flag bits (StateType, ProbeSent,
    RecentActive), Inflights.start << 8, Inflights.count << 16."""
    return (np.asarray(flags, np.uint32) & 0xF) | (np.asarray(start, np.uint32) << 8) | \
        (np.asarray(count, np.uint32) << 16)


class ProgressBatch:
    """Host mirror of qe_progress (numpy arrays, same layout).  Optional
    per-group arrays (tracked, self_slot, lead_transferee, snap_index) are
    None unless set.  `pw` holds the packed per-peer words; `flags`,
    `istart`, `icount` are read-only views of their fields (set_peer
    rewrites them)."""

    OPTIONAL = ("inc", "out", "tracked", "self_slot", "lead_transferee", "snap_index",
                "read_acks", "read_head", "read_count", "read_ovf", "read_keys")
    READ_QUEUE = 4

    def __init__(self, G, S, F, R, stride=None, max_ents=0):
        self.G, self.S, self.F, self.R = G, S, F, R
        self.stride = stride or G
        self.max_ents = max_ents
        n = S * self.stride
        self.match = np.zeros(n, np.uint64)
        self.next = np.ones(n, np.uint64)
        self.pending = np.zeros(n, np.uint64)
        self.pw = np.zeros(n, np.uint32)
        self.ibuf = np.zeros(S * F * self.stride, np.uint64)
        self.committed = np.zeros(G, np.uint64)
        self.term_start = np.zeros(G, np.uint64)
        self.first_index = np.ones(G, np.uint64)
        self.last_index = np.zeros(G, np.uint64)
        self.run_first = np.zeros(max(R, 1) * self.stride, np.uint64)
        self.run_term = np.zeros(max(R, 1) * self.stride, np.uint64)
        self.run_count = np.zeros(G, np.uint8)
        for k in self.OPTIONAL:
            setattr(self, k, None)
        self.read_cap = 0
        self.ring16 = False  # ABI 8: the device form is the 16-bit one (byte rules only)
        self._flag = np.ones(1, np.uint8)

    @property
    def flags(self):
        return (self.pw & 0xFF).astype(np.uint8)

    @property
    def istart(self):
        return ((self.pw >> 8) & 0xFF).astype(np.uint8)

    @property
    def icount(self):
        return ((self.pw >> 16) & 0xFF).astype(np.uint8)

    def set_peer(self, flags=None, istart=None, icount=None):
        """Rewrite fields of the packed words (None keeps a field)."""
        f = self.flags if flags is None else np.broadcast_to(flags, self.pw.shape)
        st = self.istart if istart is None else np.broadcast_to(istart, self.pw.shape)
        ct = self.icount if icount is None else np.broadcast_to(icount, self.pw.shape)
        self.pw[:] = pack_word(f, st, ct)

    def track_reads(self, cap=0, keys=False):
        """Allocate the ReadIndex queue (ABI 5): acks word per group (uint32
        for S <= 8, uint64 above: entry j in bits [8*mb*j, ...)), the
        context number of entry 0 (starting at 1) and the count; ABI 7: a
        capacity `cap` > 4 adds the overflow ring [G][cap] (mask type),
        `keys` the request keys [G][max(cap, 4)] (uint64)."""
        self.read_acks = np.zeros(self.G, np.uint32 if self.S <= 8 else np.uint64)
        self.read_head = np.ones(self.G, np.uint32)
        self.read_count = np.zeros(self.G, np.uint8)
        self.read_cap = int(cap)
        c = max(4, self.read_cap)
        self.read_ovf = np.zeros(self.G * c, mask_dtype(self.S)) if c > 4 else None
        self.read_keys = np.zeros(self.G * c, np.uint64) if keys else None
        return self

    def copy(self):
        c = ProgressBatch.__new__(ProgressBatch)
        for k, v in self.__dict__.items():
            setattr(c, k, v.copy() if isinstance(v, np.ndarray) else v)
        return c

    def struct(self, goff=0):
        return OrcProg(self.G, goff, self.S, self.F, self.stride, P(self.match), P(self.next),
                       P(self.pending), P(self.pw),
                       P(self.ibuf), P(self.committed), P(self.term_start), P(self.first_index),
                       P(self.last_index), self.R, 0, P(self.run_first), P(self.run_term),
                       P(self.run_count), P(self.inc), P(self.out), P(self.tracked),
                       P(self.self_slot), P(self.lead_transferee), P(self.snap_index),
                       self.max_ents, 0, P(self.read_acks), P(self.read_head),
                       P(self.read_count), self.read_cap, 0, P(self.read_ovf), P(self.read_keys),
                       P(self._flag) if self.ring16 else None)


class StepOut:
    """Outputs of one oracle progress_step round."""

    def __init__(self, pb):
        md = mask_dtype(pb.S)
        self.sent = np.zeros(pb.G, md)
        self.bcast = np.zeros(pb.G, np.uint8)
        self.snap = np.zeros(pb.G, md)
        self.timeout_now = np.zeros(pb.G, md)
        self.msg_count = np.zeros(pb.S * pb.stride, np.uint8)
        self.msg_index = np.zeros(pb.S * pb.stride, np.uint64)
        self.read_released = np.zeros(pb.G, np.uint8)
        self.term_commit = np.zeros(pb.G, np.uint8)
        self.term_commit_index = np.zeros(pb.G, np.uint64)
        self.stats = np.zeros(NSTAT, np.uint64)
        self.bytes = np.zeros(1, np.uint64)


def progress_step(pb, mtype, mindex, mhint, mlogterm, goff=0, threads=0, read_ctx=None,
                  outputs=True, count_bytes=False):
    """One round of stepLeader message handling (oracle).  Returns StepOut.
    The ReadIndex queue is pb's (pb.track_reads()); read_ctx (uint32
    [S][stride]) the contexts heartbeat responses carry (None: the newest
    pending).  outputs=False leaves the optional outputs NULL (as a kernel
    call without them); count_bytes: o.bytes[0] = the round's algorithmic
    bytes by the accounting rules."""
    o = StepOut(pb)
    opt = (lambda a: P(a)) if outputs else (lambda a: None)
    if read_ctx is not None:
        read_ctx = np.ascontiguousarray(read_ctx, np.uint32)
    m = OrcMsgs(P(mtype), P(mindex), P(mhint), P(mlogterm), opt(o.sent), opt(o.bcast),
                opt(o.snap), opt(o.timeout_now), opt(o.msg_count), opt(o.msg_index),
                P(read_ctx) if pb.read_acks is not None else None, opt(o.read_released),
                opt(o.term_commit), opt(o.term_commit_index),
                P(o.bytes) if count_bytes else None)
    s = pb.struct(goff)
    lib().orc_progress_step_batch(C.byref(s), C.byref(m), P(o.stats), threads)
    return o


def progress_send(pb, want, send_if_empty, max_ents=None):
    """max_ents: None = pb.max_ents (ABI 3 takes MaxSizePerMsg from the state)."""
    sent = np.zeros(pb.G, mask_dtype(pb.S))
    snap = np.zeros(pb.G, mask_dtype(pb.S))
    s = pb.struct()
    me = pb.max_ents if max_ents is None else max_ents
    lib().orc_progress_send_batch(C.byref(s), P(want), send_if_empty, me, P(sent), P(snap))
    return sent, snap


def read_index(pb, request, lease_based=False, key=None):
    """MsgReadIndex on the leader of every group with request[g] != 0
    (oracle) -> (result uint8[G], ctx uint32[G], index uint64[G]); key:
    uint64[G] request keys (ABI 7, with pb.read_keys)."""
    result = np.zeros(pb.G, np.uint8)
    ctx = np.zeros(pb.G, np.uint32)
    index = np.zeros(pb.G, np.uint64)
    s = pb.struct()
    k = None if key is None else np.ascontiguousarray(key, np.uint64)
    lib().orc_read_index_batch(C.byref(s), P(np.ascontiguousarray(request, np.uint8)), P(k),
                               int(bool(lease_based)), P(result), P(ctx), P(index))
    return result, ctx, index


def check_quorum(pb, goff=0):
    """MsgCheckQuorum on every group's leader (oracle).  Returns (quorum
    active uint8[G], stats)."""
    qa = np.zeros(pb.G, np.uint8)
    stats = np.zeros(NSTAT, np.uint64)
    s = pb.struct(goff)
    lib().orc_check_quorum_batch(C.byref(s), P(qa), P(stats))
    return qa, stats


class ProposeOut:
    def __init__(self, pb):
        md = mask_dtype(pb.S)
        self.result = np.zeros(pb.G, np.uint8)
        self.cc_refused = np.zeros(pb.G, np.uint8)
        self.sent = np.zeros(pb.G, md)
        self.snap = np.zeros(pb.G, md)
        self.stats = np.zeros(NSTAT, np.uint64)
        self.bytes = np.zeros(1, np.uint64)


def propose(pb, num_entries, payload=None, cc=None, applied=None, pending_conf_index=None,
            uncommitted_size=None, max_uncommitted=0, goff=0, flags=0):
    """MsgProp + appendEntry + bcastAppend on every group with
    num_entries[g] > 0 (oracle).  cc: None or (max_cc, count[G],
    pos[max_cc][G], leave[max_cc][G], size[max_cc][G]).  pending_conf_index
    and uncommitted_size (uint64[G]) and pb are updated in place.  Returns
    ProposeOut (o.bytes[0] = the algorithmic bytes).  flags 1: appendEntry
    alone (QE_PROP_APPEND_ONLY)."""
    o = ProposeOut(pb)
    ne = np.ascontiguousarray(num_entries, np.uint32)
    pl = None if payload is None else np.ascontiguousarray(payload, np.uint64)
    if cc is None:
        mc, cnt, pos, lv, sz = 0, None, None, None, None
    else:
        mc, cnt, pos, lv, sz = cc
        cnt = np.ascontiguousarray(cnt, np.uint8)
        pos = np.ascontiguousarray(pos, np.uint32)
        lv = np.ascontiguousarray(lv, np.uint8)
        sz = np.ascontiguousarray(sz, np.uint32)
    ap = None if applied is None else np.ascontiguousarray(applied, np.uint64)
    q = OrcProps(P(ne), P(pl), mc, flags, pb.G, P(cnt), P(pos), P(lv), P(sz), P(ap),
                 P(pending_conf_index), P(uncommitted_size), max_uncommitted, P(o.result),
                 P(o.cc_refused), P(o.sent), P(o.snap), P(o.bytes))
    s = pb.struct(goff)
    lib().orc_propose_batch(C.byref(s), C.byref(q), P(o.stats))
    return o


def heartbeat(pb):
    """MsgBeat -> bcastHeartbeat on every group's leader (oracle) ->
    (commit uint64 [S][stride] (0 where nothing was sent), ctx uint32 [G],
    sent mask [G])."""
    commit = np.zeros(pb.S * pb.stride, np.uint64)
    ctx = np.zeros(pb.G, np.uint32)
    sent = np.zeros(pb.G, mask_dtype(pb.S))
    s = pb.struct()
    lib().orc_heartbeat_batch(C.byref(s), P(commit), P(ctx), P(sent))
    return commit, ctx, sent


class SwitchOut:
    def __init__(self, pb):
        md = mask_dtype(pb.S)
        self.result = np.zeros(pb.G, np.uint8)
        self.sent = np.zeros(pb.G, md)
        self.snap = np.zeros(pb.G, md)
        self.stats = np.zeros(NSTAT, np.uint64)
        self.bytes = np.zeros(1, np.uint64)


def switch_config(pb, switched=None, goff=0):
    """raft.switchToConfig (raft/raft.go:1651-1700) on every group with
    switched[g] (None = every group), the new configuration being pb's inc /
    out / tracked (oracle).  pb is updated in place.  Returns SwitchOut
    (result: 0 none, 1 removed / demoted leader, 2 no voters, 3 bcastAppend,
    4 probe, | 0x10 transfer aborted; o.bytes[0] = the algorithmic bytes)."""
    o = SwitchOut(pb)
    sw = None if switched is None else np.ascontiguousarray(switched, np.uint8)
    s = pb.struct(goff)
    lib().orc_switch_config_batch(C.byref(s), P(sw), P(o.result), P(o.sent), P(o.snap),
                                  P(o.stats), P(o.bytes))
    return o


class LeaderOut:
    def __init__(self, pb):
        md = mask_dtype(pb.S)
        self.result = np.zeros(pb.G, np.uint8)
        self.pending_conf_index = np.zeros(pb.G, np.uint64)
        self.uncommitted_size = np.zeros(pb.G, np.uint64)
        self.sent = np.zeros(pb.G, md)
        self.snap = np.zeros(pb.G, md)
        self.stats = np.zeros(NSTAT, np.uint64)


def become_leader(pb, term, elected=None, bcast=True, goff=0):
    """raft.becomeLeader (raft/raft.go:724-759) on every group with
    elected[g] (None = every group), entering term[g] (oracle); pb is updated
    in place.  Returns LeaderOut (result: 0 none, 1 leader, 2 no Progress of
    its own, 3 run table full)."""
    o = LeaderOut(pb)
    el = None if elected is None else np.ascontiguousarray(elected, np.uint8)
    t = np.ascontiguousarray(term, np.uint64)
    s = pb.struct(goff)
    lib().orc_become_leader_batch(C.byref(s), P(el), P(t), 1 if bcast else 0,
                                  P(o.pending_conf_index), P(o.uncommitted_size), P(o.result),
                                  P(o.sent), P(o.snap), P(o.stats))
    return o
