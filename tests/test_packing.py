"""Host-side packing (the wire-format side of the boundary): the native C++
ConfState packer agrees with the Python packer, enforces the confchange
invariants as flags, and -- chained with the C oracle -- reproduces the
reference decisions computed on ID-keyed maps (oracle/quorum_ref.py)."""
import random

import numpy as np
import pytest

from etcd_amd import _lib
from etcd_amd.packing import (ConfStates, pack, pack_confstates, pack_order, pack_progress,
                              pack_votes, slot_lookup)
from oracle import quorum_ref as Q


def random_confstate(rng, max_voters=5, joint_p=0.5, learner_p=0.5):
    pool = rng.sample(range(1, 1 << 40), 12)
    nv = rng.randint(0, max_voters)
    voters = pool[:nv]
    outgoing = []
    if rng.random() < joint_p:
        k = rng.randint(1, max_voters)
        keep = rng.sample(voters, rng.randint(0, min(nv, k)))
        outgoing = keep + pool[nv:nv + k - len(keep)]
    used = set(voters) | set(outgoing)
    rest = [x for x in pool if x not in used]
    learners = rest[: rng.randint(0, 3)] if rng.random() < learner_p else []
    lnext = [x for x in outgoing if x not in voters][:1]
    return voters, outgoing, learners, lnext


def test_native_packer_matches_python_and_oracle(orc):
    rng = random.Random(7)
    G, S = 3000, 16
    confs = [random_confstate(rng) for _ in range(G)]
    cs = ConfStates([c[0] for c in confs], [c[1] for c in confs], [c[2] for c in confs],
                    [c[3] for c in confs])
    p = pack_confstates(cs, S)
    assert p.num_flagged == 0
    pyp = pack([{"c0": c[0], "c1": c[1], "learners": c[2]} for c in confs], num_slots=S)
    np.testing.assert_array_equal(p.slot_ids, pyp.slot_ids)
    np.testing.assert_array_equal(p.inc, pyp.inc)
    np.testing.assert_array_equal(p.out, pyp.out)
    np.testing.assert_array_equal(p.learner, pyp.learner)
    # Progress.Match for every peer (some absent), votes in arrival order
    progress, votes = [], []
    for c in confs:
        peers = list(dict.fromkeys(c[0] + c[1] + c[2]))
        progress.append({i: rng.choice([0, 5, 7, 9, rng.randrange(1 << 62)]) for i in peers
                         if rng.random() < 0.9})
        votes.append([(i, rng.random() < 0.6) for i in peers if rng.random() < 0.7])
        if votes[-1]:
            votes[-1].append((votes[-1][0][0], not votes[-1][0][1]))  # later vote ignored
    assert pack_progress(p, progress) == 0
    pack_votes(p, votes)
    b = orc.Batch(G, S)
    b.match[:] = np.ascontiguousarray(p.match).reshape(-1)
    b.inc[:], b.out[:], b.learner[:] = p.inc, p.out, p.learner
    b.voted[:], b.granted[:] = p.voted, p.granted
    commit, vote, gc, rc, _ = orc.commit_vote(b)
    for g, c in enumerate(confs):
        vmap = {}
        for i, v in votes[g]:
            Q.record_vote(vmap, i, v)
        assert int(commit[g]) == Q.joint_committed(c[0], c[1], progress[g])
        want_g, want_r, want_v = Q.tally_votes(c[0], c[1], set(c[2]), vmap)
        assert (int(gc[g]), int(rc[g]), int(vote[g])) == (want_g, want_r, want_v)


def test_packer_flags_invariant_violations():
    cs = ConfStates(
        voters=[[1, 2, 3], [1, 2], list(range(1, 20)), [0, 1]],
        voters_outgoing=[[], [2, 3], [], []],
        learners=[[3], [], [], []],
        learners_next=[[], [9], [], []])
    p = pack_confstates(cs, 16)
    assert p.flags[0] & _lib.QE_PACK_LEARNER_IS_VOTER
    assert p.flags[1] & _lib.QE_PACK_LEARNER_NEXT_NOT_OUTGOING
    assert p.flags[2] & _lib.QE_PACK_TOO_MANY_PEERS
    assert p.flags[3] & _lib.QE_PACK_ZERO_ID
    assert p.num_flagged == 4
    assert int(p.inc[2]) == 0 and not p.slot_ids[2].any()  # oversize group left empty


def test_slot_lookup_routes_deltas():
    cs = ConfStates(voters=[[10, 20, 30], [5]], voters_outgoing=[[30, 40], []],
                    learners=[[50], []])
    p = pack_confstates(cs, 8)
    assert p.slot_ids[0].tolist()[:5] == [10, 20, 30, 40, 50]
    got = slot_lookup(p, [0, 0, 0, 1, 1, 7], [40, 50, 99, 5, 0, 5])
    assert got.tolist() == [3, 4, -1, 0, -1, -1]


def test_pack_threads_knob_keeps_results():
    rng = random.Random(3)
    confs = [random_confstate(rng) for _ in range(20000)]
    cs = ConfStates([c[0] for c in confs], [c[1] for c in confs], [c[2] for c in confs])
    L = _lib.lib()
    try:
        L.qe_pack_threads(1)
        a = pack_confstates(cs, 16)
        L.qe_pack_threads(8)
        b = pack_confstates(cs, 16)
    finally:
        L.qe_pack_threads(0)
    np.testing.assert_array_equal(a.slot_ids, b.slot_ids)
    np.testing.assert_array_equal(a.inc, b.inc)
    assert L.qe_pack_threads(-1) == _lib.QE_ERANGE


def test_pack_conf_full_tracker_config():
    """qe_pack_conf writes the whole tracker.Config of a ConfState
    (confchange/restore.go): LearnersNext (outgoing voters only), IsLearner
    (= Learners), tracked (every placed peer) and AutoLeave."""
    from etcd_amd.packing import pack_conf
    cs = ConfStates(
        voters=[[1, 2, 3], [4, 5], [1], [7, 8]],
        voters_outgoing=[[], [4, 6], [], [8, 9]],
        learners=[[10], [7], [0], []],
        learners_next=[[], [6], [], [9]],
        auto_leave=[0, 1, 0, 1])
    arr, flags = pack_conf(cs, 8)
    ids = arr["slot_ids"].reshape(8, 4).T  # ID-major [S][G] (ABI 3)
    # group 0: voters 1,2,3 then learner 10
    assert ids[0].tolist() == [1, 2, 3, 10, 0, 0, 0, 0]
    assert int(arr["inc"][0]) == 0b0111 and int(arr["out"][0]) == 0
    assert int(arr["learner"][0]) == 0b1000 and int(arr["is_learner"][0]) == 0b1000
    assert int(arr["tracked"][0]) == 0b1111 and int(arr["learners_next"][0]) == 0
    # group 1: joint (4,5 | 4,6), learner 7, LearnersNext 6, AutoLeave
    assert ids[1].tolist()[:4] == [4, 5, 6, 7]
    assert int(arr["inc"][1]) == 0b0011 and int(arr["out"][1]) == 0b0101
    assert int(arr["learners_next"][1]) == 0b0100 and int(arr["is_learner"][1]) == 0b1000
    assert int(arr["tracked"][1]) == 0b1111 and arr["auto_leave"][1] == 1
    # group 2: a learner with ID 0 (raft.None) is flagged and the group left empty
    assert flags[2] & _lib.QE_PACK_ZERO_ID
    assert not ids[2].any() and int(arr["tracked"][2]) == 0 and arr["auto_leave"][2] == 0
    # group 3
    assert ids[3].tolist()[:3] == [7, 8, 9]
    assert int(arr["learners_next"][3]) == 0b100 and int(arr["out"][3]) == 0b110
    assert arr["auto_leave"][3] == 1 and flags[3] == 0


def test_zero_id_learner_flagged_by_pack_confstate():
    cs = ConfStates(voters=[[1, 2]], learners=[[0]])
    p = pack_confstates(cs, 4)
    assert p.flags[0] & _lib.QE_PACK_ZERO_ID
    assert not p.slot_ids.any() and int(p.learner[0]) == 0


def test_non_joint_auto_leave_restores_false():
    """restore.go:118-155: AutoLeave only takes effect through EnterJoint, so
    a non-joint ConfState restores AutoLeave = false (checkInvariants would
    reject AutoLeave without Voters[1]); a joint one keeps it."""
    from etcd_amd.packing import pack_conf
    cs = ConfStates(voters=[[1, 2, 3], [1, 2]], voters_outgoing=[[], [2, 3]],
                    auto_leave=[1, 1])
    arr, flags = pack_conf(cs, 4)
    assert not flags.any()
    assert arr["auto_leave"].tolist() == [0, 1]


def shape_key(c):
    v0, v1, lrn = set(c[0]), set(c[1]), set(c[2]) - set(c[0]) - set(c[1])
    return (len(v0 | v1), len(v0), len(v1), len(lrn))


def test_pack_order_buckets_by_shape():
    """qe_pack_order (ABI 3): a stable sort of the groups by configuration
    shape; packing in that order gives, at packed position i, exactly the
    identity packing of the caller's group perm[i] (masks, ID-major slot
    ids, flags, Match, votes)."""
    rng = random.Random(11)
    G, S = 5000, 16
    confs = [random_confstate(rng) for _ in range(G)]
    confs[7] = ([1, 2], [], [0], [])  # flagged (ID 0): sorts last
    lists = [[c[k] for c in confs] for k in range(4)]
    cs = ConfStates(*lists)
    perm, nshape = pack_order(cs, S)
    assert sorted(perm.tolist()) == list(range(G))
    keys = [shape_key(confs[int(g)]) for g in perm]
    assert int(perm[-1]) == 7
    assert keys[:-1] == sorted(keys[:-1])  # shape-ascending
    assert nshape == len(set(keys[:-1])) + 1
    for a, b in zip(range(G - 2), range(1, G - 1)):  # stable within a shape
        if keys[a] == keys[b]:
            assert perm[a] < perm[b]
    ident = pack_confstates(ConfStates(*lists), S)
    cs.perm = perm
    buck = pack_confstates(cs, S)
    np.testing.assert_array_equal(buck.perm, perm)
    for k in ("inc", "out", "learner", "flags"):
        np.testing.assert_array_equal(getattr(buck, k), getattr(ident, k)[perm], err_msg=k)
    np.testing.assert_array_equal(buck.slot_ids_sg, ident.slot_ids_sg[:, perm])
    progress = [{i: rng.randrange(1 << 62) for i in dict.fromkeys(c[0] + c[1] + c[2])}
                for c in confs]
    votes = [[(i, rng.random() < 0.5) for i in dict.fromkeys(c[0] + c[1])] for c in confs]
    assert pack_progress(ident, progress) == pack_progress(buck, progress)
    np.testing.assert_array_equal(buck.match, ident.match[:, perm])
    pack_votes(ident, votes)
    pack_votes(buck, votes)
    np.testing.assert_array_equal(buck.voted, ident.voted[perm])
    np.testing.assert_array_equal(buck.granted, ident.granted[perm])
    # packed voters sit in the low slots, so within a shape bucket the union
    # occupies the same slots in every group
    for i in range(G - 1):
        u, mask = keys[i][0], int(buck.inc[i]) | int(buck.out[i])
        assert mask == (1 << u) - 1
    # a perm entry out of range is refused
    bad = perm.copy()
    bad[3] = G
    cs.perm = bad
    with pytest.raises(_lib.QuorumEngineError):
        pack_confstates(cs, S)


def test_pack_order_threads_agree():
    rng = random.Random(5)
    confs = [random_confstate(rng) for _ in range(30000)]
    cs = ConfStates([c[0] for c in confs], [c[1] for c in confs], [c[2] for c in confs])
    L = _lib.lib()
    try:
        L.qe_pack_threads(1)
        a, na = pack_order(cs, 16)
        L.qe_pack_threads(7)
        b, nb = pack_order(cs, 16)
    finally:
        L.qe_pack_threads(0)
    np.testing.assert_array_equal(a, b)
    assert na == nb
