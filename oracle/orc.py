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
LIB_PATH = os.path.join(HERE, "build", "liborc.so")
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
                                            u64, u32, u32, u32, vp, i32]),
        "orc_gf_build": (vp, [u64, u32, u64, vp, vp, vp, vp, vp, vp]),
        "orc_gf_free": (None, [vp]),
        "orc_gf_run": (dbl, [vp, vp, vp, i32, i32]),
        "orc_soa_run": (dbl, [u64, u32, u64, vp, vp, vp, vp, vp, vp, vp, i32, i32]),
        "orc_max_threads": (i32, []),
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
                   step0, steps, p_drop, p_grant, threads=0):
    stats = np.zeros(NSTAT, np.uint64)
    lib().orc_election_steps_batch(G, goff, S, P(term), P(state), P(voted), P(granted),
                                   P(self_slot), P(inc), P(out), P(learner), seed, step0, steps,
                                   p_drop, p_grant, P(stats), threads)
    return stats


def max_threads():
    return lib().orc_max_threads()
