"""The C-ABI boundary: the library loads, exports every symbol
include/etcd_quorum.h declares, its struct layouts agree with the ctypes
mirror (checked by compiling the header with gcc), and argument errors are
reported as status codes without touching the GPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

from etcd_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "etcd_quorum.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(qe_\w+)\s*\(", src)))


def test_header_declares_expected_surface():
    fns = declared_functions()
    for f in ["qe_commit_vote", "qe_committed_index", "qe_vote_result", "qe_quorum_active",
              "qe_record_votes", "qe_replication_round", "qe_election_steps",
              "qe_stats_reduce", "qe_gen_groups", "qe_abi_version", "qe_strerror",
              "qe_mask_bytes", "qe_tune", "qe_allreduce_stats", "qe_comm_init",
              "qe_comm_unique_id", "qe_comm_destroy", "qe_comm_id_bytes", "qe_check_quorum",
              "qe_pack_order", "qe_progress_step", "qe_progress_send", "qe_confchange",
              "qe_read_index", "qe_propose", "qe_comm_init_timeout", "qe_comm_abort",
              "qe_heartbeat", "qe_switch_config"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = set(re.findall(r"\s[TW]\s+(qe_\w+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    # ctypes prototypes cover the whole surface
    assert set(declared_functions()) == set(_lib.PROTOTYPES)


LAYOUT_PROG = r"""
#include <stdio.h>
#include <stddef.h>
#include "etcd_quorum.h"
#define F(T, m) printf(#T " " #m " %zu\n", offsetof(T, m));
#define Z(T) printf(#T " sizeof %zu\n", sizeof(T));
int main(void) {
  Z(qe_groups) F(qe_groups, num_groups) F(qe_groups, group_offset) F(qe_groups, num_slots)
  F(qe_groups, stride) F(qe_groups, match) F(qe_groups, granted)
  Z(qe_outputs) F(qe_outputs, stats)
  Z(qe_repl_state) F(qe_repl_state, stride) F(qe_repl_state, out_mask)
  Z(qe_repl_msgs) F(qe_repl_msgs, commit_advanced)
  Z(qe_election_state) F(qe_election_state, term) F(qe_election_state, learner_mask)
  Z(qe_election_params) F(qe_election_params, steps) F(qe_election_params, p_grant_q16)
  Z(qe_gen_params) F(qe_gen_params, dist) F(qe_gen_params, mask_mode)
  Z(qe_confstate_csr) F(qe_confstate_csr, learners_next_off) F(qe_confstate_csr, learners)
  F(qe_confstate_csr, auto_leave) F(qe_confstate_csr, perm)
  Z(qe_progress) F(qe_progress, peer) F(qe_progress, infl_lo) F(qe_progress, infl_hi) F(qe_progress, log_runs)
  F(qe_progress, out_mask) F(qe_progress, tracked) F(qe_progress, snap_index)
  F(qe_progress, max_ents) F(qe_progress, read_acks) F(qe_progress, read_head)
  F(qe_progress, read_count) F(qe_progress, lead_transferee) F(qe_progress, read_cap)
  F(qe_progress, read_ovf) F(qe_progress, read_keys)
  Z(qe_peer_msgs) F(qe_peer_msgs, bcast) F(qe_peer_msgs, timeout_now) F(qe_peer_msgs, msg_index)
  F(qe_peer_msgs, bytes_requested) F(qe_peer_msgs, read_ctx) F(qe_peer_msgs, read_released)
  F(qe_peer_msgs, term_commit) F(qe_peer_msgs, term_commit_index)
  Z(qe_conf) F(qe_conf, slot_ids) F(qe_conf, tracked) F(qe_conf, auto_leave)
  Z(qe_conf_changes) F(qe_conf_changes, stride) F(qe_conf_changes, node_id)
  F(qe_conf_changes, new_progress)
  Z(qe_proposals) F(qe_proposals, max_cc) F(qe_proposals, cc_stride) F(qe_proposals, cc_size)
  F(qe_proposals, max_uncommitted) F(qe_proposals, cc_refused) F(qe_proposals, bytes_requested)
  Z(qe_switch) F(qe_switch, result) F(qe_switch, snap) F(qe_switch, bytes_requested)
  return 0;
}
"""

CTYPES = {"qe_groups": _lib.QeGroups, "qe_outputs": _lib.QeOutputs,
          "qe_repl_state": _lib.QeReplState, "qe_repl_msgs": _lib.QeReplMsgs,
          "qe_election_state": _lib.QeElectionState,
          "qe_election_params": _lib.QeElectionParams, "qe_gen_params": _lib.QeGenParams,
          "qe_confstate_csr": _lib.QeConfStateCSR, "qe_progress": _lib.QeProgress,
          "qe_peer_msgs": _lib.QePeerMsgs, "qe_conf": _lib.QeConf,
          "qe_conf_changes": _lib.QeConfChanges, "qe_proposals": _lib.QeProposals,
          "qe_switch": _lib.QeSwitch}


def test_struct_layout_matches_header(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_PROG)
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)])
    for line in subprocess.check_output([str(exe)], text=True).splitlines():
        t, m, v = line.split()
        cls = CTYPES[t]
        if m == "sizeof":
            assert C.sizeof(cls) == int(v), t
        else:
            assert getattr(cls, m).offset == int(v), (t, m)


def test_constants_and_introspection():
    L = _lib.lib()
    assert L.qe_abi_version() == _lib.QE_ABI_VERSION == 8
    assert L.qe_mask_bytes(1) == 1 and L.qe_mask_bytes(8) == 1
    assert L.qe_mask_bytes(9) == 2 and L.qe_mask_bytes(16) == 2
    assert L.qe_mask_bytes(0) == 0 and L.qe_mask_bytes(17) == 0
    assert L.qe_strerror(0) == b"ok"
    assert L.qe_strerror(_lib.QE_EINVAL) == b"invalid argument"
    src = open(HEADER).read()
    for name, val in [("QE_VOTE_PENDING", 1), ("QE_VOTE_LOST", 2), ("QE_VOTE_WON", 3),
                      ("QE_STATS_COUNTERS", 16), ("QE_STATS_SHARDS", 64), ("QE_EINVAL", -22),
                      ("QE_PF_RECENT_ACTIVE", 8), ("QE_PW_START_SHIFT", 8),
                      ("QE_PW_COUNT_SHIFT", 16), ("QE_PF_RING_WIDE", 16),
                      ("QE_MSG_TRANSFER_LEADER", 7), ("QE_READ_QUEUE", 4), ("QE_RI_RESPOND", 1),
                      ("QE_RI_POSTPONED", 2), ("QE_RI_QUEUED", 3), ("QE_RI_FULL", 4),
                      ("QE_RI_DUPLICATE", 5), ("QE_READ_CAP_MAX", 255)]:
        m = re.search(rf"#define {name} \(?(-?\d+)u?\)?", src)
        assert m and int(m.group(1)) == val, name


def test_argument_errors_without_gpu():
    """Validation happens before any HIP call, so these run on CPU."""
    L = _lib.lib()
    o = _lib.QeOutputs()
    assert L.qe_commit_vote(None, C.byref(o), None) == _lib.QE_EINVAL
    g = _lib.QeGroups(num_groups=10, num_slots=0, stride=10)
    assert L.qe_commit_vote(C.byref(g), C.byref(o), None) == _lib.QE_EINVAL
    g = _lib.QeGroups(num_groups=10, num_slots=17, stride=10)
    assert L.qe_commit_vote(C.byref(g), C.byref(o), None) == _lib.QE_EINVAL
    g = _lib.QeGroups(num_groups=10, num_slots=5, stride=5)  # stride < G
    assert L.qe_commit_vote(C.byref(g), C.byref(o), None) == _lib.QE_EINVAL
    g = _lib.QeGroups(num_groups=0, num_slots=5, stride=0)  # empty batch is a no-op
    assert L.qe_commit_vote(C.byref(g), C.byref(o), None) == _lib.QE_OK
    g = _lib.QeGroups(num_groups=4, num_slots=5, stride=4, out_mask=C.c_void_p(64))
    assert L.qe_commit_vote(C.byref(g), C.byref(o), None) == _lib.QE_EINVAL  # out w/o inc
    assert L.qe_record_votes(4, 0, None, None, None, None, None) == _lib.QE_EINVAL
    assert L.qe_replication_round(None, None, None, None) == _lib.QE_EINVAL
    assert L.qe_election_steps(None, None, None, None) == _lib.QE_EINVAL
    assert L.qe_tune(b"blocks_per_cu", -1) == _lib.QE_ERANGE
    assert L.qe_tune(b"blocks_per_cu", 33) == _lib.QE_ERANGE
    assert L.qe_tune(b"nope", 1) == _lib.QE_EINVAL
    pr = _lib.QeProgress(num_groups=1, num_slots=3, inflight_cap=0, stride=1)
    assert L.qe_progress_step(C.byref(pr), C.byref(_lib.QePeerMsgs()), None, None) == _lib.QE_ERANGE
    pr = _lib.QeProgress(num_groups=1, num_slots=3, inflight_cap=4, stride=1, log_runs=17)
    assert L.qe_progress_send(C.byref(pr), None, 0, None, None, None) == _lib.QE_ERANGE
    assert L.qe_check_quorum(None, None, None, None) == _lib.QE_EINVAL
    pr = _lib.QeProgress(num_groups=4, num_slots=3, inflight_cap=4, stride=4)  # no peer words
    assert L.qe_check_quorum(C.byref(pr), None, None, None) == _lib.QE_EINVAL
    pr = _lib.QeProgress(num_groups=0, num_slots=3)  # empty batch is a no-op
    assert L.qe_check_quorum(C.byref(pr), None, None, None) == _lib.QE_OK
    assert L.qe_read_index(C.byref(pr), None, None, 0, None, None, None, None) == _lib.QE_OK
    assert L.qe_read_index(None, None, None, 0, None, None, None, None) == _lib.QE_EINVAL
    v = C.c_void_p(64)
    pr = _lib.QeProgress(num_groups=4, num_slots=3, inflight_cap=4, stride=4, committed=v,
                         term_start=v, last_index=v)
    # ReadOnlySafe needs the queue; LeaseBased does not
    assert L.qe_read_index(C.byref(pr), v, None, 0, v, None, None, None) == _lib.QE_EINVAL
    assert L.qe_read_index(C.byref(pr), None, None, 1, v, None, None, None) == _lib.QE_EINVAL
    # a queue comes whole or not at all (qe_progress_step)
    pr = _lib.QeProgress(num_groups=4, num_slots=3, inflight_cap=4, stride=4, log_runs=1,
                         match=v, next=v, pending_snapshot=v, peer=v, infl_lo=v, infl_hi=v,
                         committed=v, term_start=v, first_index=v, last_index=v, run_first=v,
                         run_term=v, run_count=v, read_acks=v)
    m = _lib.QePeerMsgs(type=v, index=v, reject_hint=v, log_term=v)
    assert L.qe_progress_step(C.byref(pr), C.byref(m), None, None) == _lib.QE_EINVAL
    assert L.qe_confchange(None, None, None, None) == _lib.QE_EINVAL
    cf = _lib.QeConf(num_groups=4, num_slots=17)
    assert L.qe_confchange(C.byref(cf), C.byref(_lib.QeConfChanges()), None, None) == _lib.QE_EINVAL
    cf = _lib.QeConf(num_groups=0, num_slots=5)  # empty batch is a no-op
    assert L.qe_confchange(C.byref(cf), C.byref(_lib.QeConfChanges()), None, None) == _lib.QE_OK
    p = _lib.QeElectionParams(p_drop_q16=70000)
    st = _lib.QeElectionState(num_groups=1, num_slots=3, term=C.c_void_p(64),
                              state=C.c_void_p(64), voted=C.c_void_p(64),
                              granted=C.c_void_p(64), self_slot=C.c_void_p(64))
    assert L.qe_election_steps(C.byref(st), C.byref(p), None, None) == _lib.QE_ERANGE


def test_comm_argument_errors_without_gpu():
    """qe_comm_* / qe_allreduce_stats validate before touching RCCL."""
    L = _lib.lib()
    assert L.qe_comm_id_bytes() == 128  # sizeof(ncclUniqueId)
    assert L.qe_comm_unique_id(None) == _lib.QE_EINVAL
    comm = C.c_void_p()
    idb = (C.c_uint8 * 128)()
    assert L.qe_comm_init(None, 1, 0, idb, 0) == _lib.QE_EINVAL
    assert L.qe_comm_init(C.byref(comm), 0, 0, idb, 0) == _lib.QE_EINVAL
    assert L.qe_comm_init(C.byref(comm), 2, 2, idb, 0) == _lib.QE_EINVAL  # rank >= nranks
    assert L.qe_comm_init(C.byref(comm), 1, 0, None, 0) == _lib.QE_EINVAL
    assert L.qe_comm_destroy(None) == _lib.QE_EINVAL
    assert L.qe_comm_abort(None) == _lib.QE_EINVAL
    assert L.qe_comm_init_timeout(None, 1, 0, idb, 0, 1000) == _lib.QE_EINVAL
    assert L.qe_comm_init_timeout(C.byref(comm), 2, 2, idb, 0, 1000) == _lib.QE_EINVAL
    assert L.qe_comm_init_timeout(C.byref(comm), 1, 0, None, 0, 1000) == _lib.QE_EINVAL
    assert L.qe_allreduce_stats(None, 16, C.c_void_p(64), None) == _lib.QE_EINVAL
    assert L.qe_allreduce_stats(C.c_void_p(64), 16, None, None) == _lib.QE_EINVAL
    assert L.qe_allreduce_stats(C.c_void_p(64), 0, C.c_void_p(64), None) == _lib.QE_EINVAL
    assert L.qe_allreduce_stats(C.c_void_p(64), 1025, C.c_void_p(64), None) == _lib.QE_EINVAL


def test_missing_library_fails_loudly(tmp_path):
    code = ("import os; os.environ['QE_LIB']='/nonexistent/lib.so'\n"
            "try:\n import etcd_amd\nexcept ImportError as e:\n print('IMPORTERROR', e)\n")
    out = subprocess.run(["python", "-c", code], capture_output=True, text=True, cwd=ROOT)
    assert "IMPORTERROR" in out.stdout, out.stdout + out.stderr


def _ring_case(rng, G, S, F):
    """Random peer words (start < F, count <= F) and uint64 rings mixing
    small indices, indices near 2^32 boundaries (rings that straddle one)
    and indices past the 11-bit epoch (2^43)."""
    import numpy as np
    n = S * G
    start = rng.integers(0, F, n)
    count = rng.integers(0, F + 1, n)
    w = (rng.integers(0, 16, n) | (start << 8) | (count << 16)).astype(np.uint32)
    kind = rng.integers(0, 4, n)
    base = np.where(kind == 0, rng.integers(0, 1 << 20, n),
                    np.where(kind == 1, (rng.integers(1, 1 << 11, n) << 32) - rng.integers(0, 6, n),
                             np.where(kind == 2, rng.integers(0, 1 << 43, n),
                                      rng.integers(1 << 43, 1 << 62, n)))).astype(np.uint64)
    ent = base.reshape(S, 1, G) + np.arange(F, dtype=np.uint64).reshape(1, F, 1)
    return w, np.ascontiguousarray(ent.transpose(0, 2, 1)).reshape(-1)  # [S][G][F]


@pytest.mark.parametrize("F", [1, 3, 8, 13, 255])
def test_ring_pack_unpack_roundtrip(F):
    """qe_ring_pack / qe_ring_unpack (host side, ABI 4): every live entry
    round-trips exactly; the representation is canonical (empty -> epoch 0,
    not wide; one upper word <= QE_RING_EPOCH_MAX -> that epoch; else wide);
    Progress bits of the word are kept."""
    import numpy as np
    rng = np.random.default_rng(F)
    G, S = 700, 3
    w, ent = _ring_case(rng, G, S, F)
    FP = _lib.QE_RING_PITCH(F)
    lo = np.zeros(S * G * FP, np.uint32)
    hi = np.zeros_like(lo)
    peer = w.copy()
    L = _lib.lib()
    assert L.qe_ring_pack(G, S, F, G, ent.ctypes.data, peer.ctypes.data, lo.ctypes.data,
                          hi.ctypes.data) == _lib.QE_OK
    assert np.array_equal(peer & ~np.uint32(_lib.QE_PW_RING_MASK), w & ~np.uint32(_lib.QE_PW_RING_MASK))
    back = np.zeros_like(ent)
    assert L.qe_ring_unpack(G, S, F, G, lo.ctypes.data, hi.ctypes.data, peer.ctypes.data,
                            back.ctypes.data) == _lib.QE_OK
    e2, b2 = ent.reshape(S * G, F), back.reshape(S * G, F)
    start, count = (w >> 8) & 0xFF, (w >> 16) & 0xFF
    wide = (peer & _lib.QE_PF_RING_WIDE) != 0
    epoch = ((peer >> 5) & 7) | ((peer >> 21) & 0x7F8)
    n_wide = 0
    for i in range(S * G):
        pos = [(int(start[i]) + j) % F for j in range(int(count[i]))]
        assert np.array_equal(b2[i, pos], e2[i, pos]), i
        his = {int(e2[i, q]) >> 32 for q in pos}
        if not pos:
            assert not wide[i] and epoch[i] == 0
        elif len(his) == 1 and max(his) <= _lib.QE_RING_EPOCH_MAX:
            assert not wide[i] and epoch[i] == his.pop()
        else:
            assert wide[i] and epoch[i] == 0
            assert np.array_equal(b2[i], e2[i])  # wide: both words of every position
            n_wide += 1
    assert n_wide > 0
    # argument checks
    assert L.qe_ring_pack(G, 0, F, G, None, None, None, None) == _lib.QE_EINVAL
    assert L.qe_ring_pack(G, S, 256, G, None, None, None, None) == _lib.QE_ERANGE
    assert L.qe_ring_unpack(G, S, F, G - 1, lo.ctypes.data, hi.ctypes.data, peer.ctypes.data,
                            back.ctypes.data) == _lib.QE_EINVAL


@pytest.mark.parametrize("F", [5, 8])
def test_set_ring_slot_matches_ring_pack(F):
    """engine.ProgressState.set_ring_slot (the bench's device-side ring
    builder, torch ops only -- run here on CPU tensors) writes the same
    32-bit words and representation bits as the host packer qe_ring_pack."""
    import numpy as np
    import torch

    from etcd_amd import engine
    rng = np.random.default_rng(40 + F)
    G, S = 300, 3
    ps = engine.ProgressState(G, S, F, 1, device="cpu", stride=320)
    st = ps.stride
    w, ent = _ring_case(rng, st, S, F)  # [S][st][F] uint64
    ps.peer.copy_(torch.from_numpy(w.view(np.int32)))
    for s in range(S):
        e = torch.from_numpy(ent.reshape(S, st, F)[s].copy().view(np.int64))
        ps.set_ring_slot(s, e)
    FP = _lib.QE_RING_PITCH(F)
    lo = np.zeros(S * st * FP, np.uint32)
    hi = np.zeros_like(lo)
    peer = w.copy()
    assert _lib.lib().qe_ring_pack(st, S, F, st, ent.ctypes.data, peer.ctypes.data,
                                   lo.ctypes.data, hi.ctypes.data) == _lib.QE_OK
    assert np.array_equal(ps.peer.numpy().view(np.uint32), peer)
    got_lo = ps.ilo.numpy().view(np.uint32).reshape(S * st, FP)[:, :F]
    got_hi = ps.ihi.numpy().view(np.uint32).reshape(S * st, FP)[:, :F]
    assert np.array_equal(got_lo, lo.reshape(S * st, FP)[:, :F])
    assert np.array_equal(got_hi, hi.reshape(S * st, FP)[:, :F])


def _ring16_case(rng, G, S, F):
    """Peer words and rings for the 16-bit form: Next just above the ring's
    entries (the window fits), far above it (more than 65536 indices: wide),
    below some entry (inconsistent: wide), indices near 2^32 and 2^43."""
    import numpy as np
    w, ent = _ring_case(rng, G, S, F)
    e = ent.reshape(S * G, F)
    hi = e.max(1)
    kind = rng.integers(0, 4, S * G)
    nxt = np.where(kind == 0, hi + 1 + rng.integers(0, 300, S * G),
                   np.where(kind == 1, hi + rng.integers(1, 40000, S * G),
                            np.where(kind == 2, hi + 70000 + rng.integers(0, 9, S * G),
                                     hi - rng.integers(0, F, S * G)))).astype(np.uint64)
    return w, ent, nxt


@pytest.mark.parametrize("F", [1, 3, 5, 8])
def test_ring16_pack_unpack_roundtrip(F):
    """qe_ring_pack16 / qe_ring_unpack16 (ABI 8): every position round-trips
    exactly; a peer is in the 16-bit form iff its live entries lie in
    [Next - 65536, Next - 1], else wide; Progress bits are kept, epoch 0."""
    import numpy as np
    rng = np.random.default_rng(160 + F)
    G, S = 700, 3
    w, ent, nxt = _ring16_case(rng, G, S, F)
    FP = _lib.QE_RING_PITCH(F)
    lo = np.zeros(S * G * FP, np.uint32)
    hi = np.zeros_like(lo)
    o16 = np.zeros(S * G * 8, np.uint16)
    peer = w.copy()
    L = _lib.lib()
    assert L.qe_ring_pack16(G, S, F, G, ent.ctypes.data, nxt.ctypes.data, peer.ctypes.data,
                            o16.ctypes.data, lo.ctypes.data, hi.ctypes.data) == _lib.QE_OK
    mask = np.uint32(_lib.QE_PW_RING_MASK)
    assert np.array_equal(peer & ~mask, w & ~mask)
    assert not ((peer & mask) & ~np.uint32(_lib.QE_PF_RING_WIDE)).any()  # no epoch bits
    back = np.zeros_like(ent)
    assert L.qe_ring_unpack16(G, S, F, G, o16.ctypes.data, lo.ctypes.data, hi.ctypes.data,
                              nxt.ctypes.data, peer.ctypes.data, back.ctypes.data) == _lib.QE_OK
    e2, b2 = ent.reshape(S * G, F), back.reshape(S * G, F)
    start, count = (w >> 8) & 0xFF, (w >> 16) & 0xFF
    wide = (peer & _lib.QE_PF_RING_WIDE) != 0
    n16 = 0
    for i in range(S * G):
        pos = [(int(start[i]) + j) % F for j in range(int(count[i]))]
        top = int(nxt[i]) - 1
        fits = all(int(e2[i, q]) <= top and top - int(e2[i, q]) <= 0xFFFF for q in pos)
        assert wide[i] == (not fits), i
        if wide[i]:
            assert np.array_equal(b2[i], e2[i])
        else:
            assert np.array_equal(b2[i, pos], e2[i, pos]), i
            n16 += bool(pos)
    assert n16 > 0 and wide.sum() > 0
    assert L.qe_ring_pack16(G, S, 9, G, None, None, None, None, None, None) == _lib.QE_ERANGE
    assert L.qe_ring_unpack16(G, S, F, G, None, lo.ctypes.data, hi.ctypes.data, nxt.ctypes.data,
                              peer.ctypes.data, back.ctypes.data) == _lib.QE_EINVAL


@pytest.mark.parametrize("F", [5, 8])
def test_set_ring_slot16_matches_ring_pack16(F):
    """ProgressState.set_ring_slot in the 16-bit form (torch ops, CPU
    tensors here) writes the same offsets and representation bits as
    qe_ring_pack16 (entries and Next below 2^63)."""
    import numpy as np
    import torch

    from etcd_amd import engine
    rng = np.random.default_rng(60 + F)
    G, S = 300, 3
    ps = engine.ProgressState(G, S, F, 1, device="cpu", stride=320, ring16=True)
    st = ps.stride
    w, ent, nxt = _ring16_case(rng, st, S, F)
    big = (ent.reshape(S * st, F) >= (1 << 62)).any(1) | (nxt >= (1 << 62))
    ent.reshape(S * st, F)[big] &= np.uint64((1 << 40) - 1)  # (torch int64 arithmetic)
    nxt[big] = ent.reshape(S * st, F)[big].max(1) + 1
    ps.peer.copy_(torch.from_numpy(w.view(np.int32)))
    ps.next.copy_(torch.from_numpy(nxt.view(np.int64)))
    for s in range(S):
        ps.set_ring_slot(s, torch.from_numpy(ent.reshape(S, st, F)[s].copy().view(np.int64)))
    FP = _lib.QE_RING_PITCH(F)
    lo = np.zeros(S * st * FP, np.uint32)
    hi = np.zeros_like(lo)
    o16 = np.zeros(S * st * 8, np.uint16)
    peer = w.copy()
    assert _lib.lib().qe_ring_pack16(st, S, F, st, ent.ctypes.data, nxt.ctypes.data,
                                     peer.ctypes.data, o16.ctypes.data, lo.ctypes.data,
                                     hi.ctypes.data) == _lib.QE_OK
    assert np.array_equal(ps.peer.numpy().view(np.uint32), peer)
    got = ps.infl16.numpy().view(np.uint16).reshape(S * st, 8)[:, :F]
    assert np.array_equal(got, o16.reshape(S * st, 8)[:, :F])
    back = ps.rings()  # decode through qe_ring_unpack16 (entry-major)
    e = ent.reshape(S, st, F).transpose(0, 2, 1).reshape(-1)
    start, count = (w >> 8) & 0xFF, (w >> 16) & 0xFF
    for i in range(0, S * st, 7):
        s, g = divmod(i, st)
        if g >= G:  # (rings() decodes groups < G)
            continue
        for j in range(int(count[i])):
            k = (int(start[i]) + j) % F
            assert back[(s * F + k) * st + g] == e[(s * F + k) * st + g]


def test_load_host_rejects_pending_outside_snapshot():
    """ProgressState.load_host checks the qe_progress precondition the
    kernels rely on (PendingSnapshot is 0 outside StateSnapshot, written only
    where it changes): a violating host state is refused (CPU tensors)."""
    import numpy as np

    from etcd_amd import engine
    G, S = 70, 3
    ps = engine.ProgressState(G, S, 4, 1, device="cpu")
    flags = np.full(S * ps.stride, 1, np.uint8)  # StateReplicate
    pend = np.zeros(S * ps.stride, np.uint64)
    ps.load_host(flags=flags, pending=pend)  # fine
    flags[5] = 2  # StateSnapshot: any PendingSnapshot
    pend[5] = 9
    ps.load_host(flags=flags, pending=pend)
    pend[ps.stride + 3] = 4  # slot 1, group 3 in StateReplicate
    with pytest.raises(ValueError, match="slot 1, group 3"):
        ps.load_host(flags=flags, pending=pend)
