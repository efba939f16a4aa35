"""The native packer's multi-threaded paths (qe_pack.cpp parallel_for: more
than one worker from 4096 groups up) give exactly the single-threaded
result -- the packing the sanitizer builds (tests/test_sanitizers.py,
TSan) watch for races."""
import random

import numpy as np

from etcd_amd import _lib
from etcd_amd.packing import ConfStates, pack_confstates, pack_order


def _confs(G, seed=11):
    rng = random.Random(seed)
    v, o, l, n = [], [], [], []
    for g in range(G):
        ids = rng.sample(range(1, 1 << 30), 10)
        nv = rng.randint(1, 5)
        v.append(ids[:nv])
        if rng.random() < 0.4:
            out = ids[: rng.randint(0, nv)] + ids[nv: nv + rng.randint(0, 2)]
            o.append(out)
            n.append([x for x in out if x not in ids[:nv]][:1])
        else:
            o.append([])
            n.append([])
        l.append(ids[7: 7 + rng.randint(0, 2)])
    return ConfStates(v, o, l, n)


def test_threads_match_single_thread():
    L = _lib.lib()
    G, S = 40_000, 10
    cs = _confs(G)
    res = {}
    try:
        for nt in (1, 8):
            L.qe_pack_threads(nt)
            cs.perm = None
            plain = pack_confstates(cs, S)
            bucketed = pack_confstates(cs, S, bucketed=True)  # + qe_pack_order's sort
            res[nt] = (plain, bucketed, np.asarray(pack_order(cs, S)[0]))
    finally:
        L.qe_pack_threads(0)
        cs.perm = None
    for i in (0, 1):
        for k in ("inc", "out", "learner", "slot_ids", "flags"):
            np.testing.assert_array_equal(np.asarray(getattr(res[1][i], k)),
                                          np.asarray(getattr(res[8][i], k)), err_msg=k)
    np.testing.assert_array_equal(res[1][2], res[8][2])
    assert not np.array_equal(res[1][2], np.arange(G))  # the shapes were reordered
