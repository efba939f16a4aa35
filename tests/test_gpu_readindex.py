"""ReadIndex queues longer than the word (ABI 7; readOnly.readIndexQueue is
unbounded in the reference, raft/read_only.go:56-63) and addRequest's
duplicate check in the engine (:57-60), on the GPU against the oracle's
list (orc_ro, up to read_cap entries): random queue depths up to 64 and up
to the 255-entry maximum, heartbeat responses carrying contexts anywhere in
the queue (the overflow ring's entries, released ones, unknown ones), new
requests with fresh and duplicate keys, MsgBeat's newest context, and the
instrumented variant's byte count."""
import numpy as np
import pytest
import torch

from oracle import orc
from tests.test_gpu_progress import (DEV, EXTRAS, assert_outputs, assert_same, load_msgs,
                                     random_msgs, random_state, to_device)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from etcd_amd import engine
    return engine


def deep_queue(rng, pb, cap):
    """Random queues of 0..cap pending requests (most past the word), random
    acks in the word and the ring (dead slots hold garbage), context numbers
    near 1 and near 2^32, random keys (distinct within a group's queue)."""
    pb.track_reads(cap, keys=True)
    G = pb.G
    deep = rng.random(G) < 0.7
    pb.read_count[:] = np.where(deep, rng.integers(5, cap + 1, G), rng.integers(0, 5, G))
    pb.read_head[:] = np.where(rng.random(G) < 0.8, rng.integers(1, 1000, G),
                               rng.integers(1, 1 << 32, G, dtype=np.uint64)).astype(np.uint32)
    wbits = 32 if pb.S <= 8 else 64
    pb.read_acks[:] = rng.integers(0, 1 << 62, G, dtype=np.uint64).astype(
        np.uint32 if wbits == 32 else np.uint64)
    pb.read_ovf[:] = rng.integers(0, 1 << 16, pb.read_ovf.size).astype(pb.read_ovf.dtype)
    pb.read_keys[:] = rng.integers(0, 1 << 62, pb.read_keys.size, dtype=np.uint64)


def check_queue(ps, pb, where):
    """assert_same, with the first diverging groups' queues printed first."""
    h = ps.host()
    G = pb.G
    gw, ow = h["read_acks"].reshape(G, 4), pb.read_acks.view(orc.mask_dtype(pb.S)).reshape(G, 4)
    bad = np.nonzero((gw != ow).any(1) | (h["read_head"] != pb.read_head) |
                     (h["read_count"] != pb.read_count))[0]
    for g in bad[:4]:
        print(where, "group", g, "gpu", gw[g], h["read_head"][g], h["read_count"][g],
              "oracle", ow[g], pb.read_head[g], pb.read_count[g])
    assert_same(ps, pb)


def deep_ctx(rng, pb):
    """Contexts the heartbeat responses carry: mostly pending (word or ring),
    some released, some never assigned, some none."""
    n = pb.S * pb.G
    head = np.tile(pb.read_head, pb.S).astype(np.int64)
    cnt = np.tile(pb.read_count, pb.S).astype(np.int64)
    pick = rng.integers(0, 6, n)
    ctx = np.where(pick == 0, 0,
                   np.where(pick == 1, head - rng.integers(1, 4, n),
                            np.where(pick == 2, head + cnt + rng.integers(0, 3, n),
                                     head + rng.integers(0, 1 << 20, n) % np.maximum(cnt, 1))))
    return (ctx & 0xFFFFFFFF).astype(np.uint32)


@pytest.mark.parametrize("S,masks,cap", [(3, (), 16), (5, ("inc",), 64), (5, (), 255),
                                         (7, ("inc", "out"), 64), (10, ("inc",), 32),
                                         (16, ("inc", "out"), 255)])
@pytest.mark.parametrize("F", [8, 32])
def test_deep_readindex_queues_match_oracle(eng, S, masks, cap, F):
    rng = np.random.default_rng(9100 + 13 * S + cap + F)
    G = 3001
    pb = random_state(rng, G, S, F, 3, masks, EXTRAS, max_ents=1)
    deep_queue(rng, pb, cap)
    ps = to_device(eng, pb, masks, EXTRAS + ("reads",))
    md = orc.mask_dtype(S)
    for rnd in range(8):
        if rnd % 2 == 1:  # new requests: fresh keys, and keys already pending
            req = (rng.random(G) < 0.7).astype(np.uint8)
            key = rng.integers(0, 1 << 62, G, dtype=np.uint64)
            dup = rng.random(G) < 0.3
            cnt = pb.read_count.astype(np.int64)
            pick = (pb.read_head.astype(np.int64) + rng.integers(0, 1 << 20, G) % np.maximum(cnt, 1)) % cap
            key = np.where(dup & (cnt > 0), pb.read_keys.reshape(G, cap)[np.arange(G), pick], key)
            r_g, c_g, i_g = eng.read_index(ps, torch.from_numpy(req).to(DEV), False,
                                           key=torch.from_numpy(key.view(np.int64)).to(DEV))
            r_o, c_o, i_o = orc.read_index(pb, req, False, key=key)
            np.testing.assert_array_equal(r_g.cpu().numpy(), r_o, err_msg="result")
            w = (r_o == 3) | (r_o == 5)
            np.testing.assert_array_equal(c_g.cpu().numpy().view(np.uint32)[w], c_o[w], err_msg="ctx")
            w = (r_o == 1) | (r_o == 3)
            np.testing.assert_array_equal(i_g.cpu().numpy().view(np.uint64)[w], i_o[w])
            check_queue(ps, pb, f"read_index rnd {rnd}")
            assert (r_o == 5).any() and (r_o == 3).any()
        mtype, mindex, mhint, mlogterm = random_msgs(rng, pb)
        hb = rng.random(mtype.size) < 0.6  # mostly heartbeat responses
        mtype[hb] = 3
        msgs = load_msgs(eng, ps, mtype, mindex, mhint, mlogterm)
        ctx = None if rnd % 4 == 3 else deep_ctx(rng, pb)  # every fourth: the newest context
        msgs.set_read_ctx(ps, ctx)
        stats = eng.stats_buffer(DEV)
        acct = rnd % 2 == 0
        if acct:
            msgs.bytes_requested = torch.zeros(1, dtype=torch.int64, device=DEV)
        eng.progress_step(ps, msgs, stats)
        got = eng.stats_reduce(stats).cpu().numpy().view(np.uint64)
        o = orc.progress_step(pb, mtype, mindex, mhint, mlogterm, read_ctx=ctx, count_bytes=True)
        check_queue(ps, pb, f"step rnd {rnd}")
        assert_outputs(msgs, o, S)
        np.testing.assert_array_equal(got, o.stats)
        if acct:
            assert int(msgs.bytes_requested.item()) == int(o.bytes[0]), rnd
        assert o.read_released.any()
        # MsgBeat: the newest pending context, however deep the queue
        commit, hctx, sent = eng.heartbeat(ps)
        _, o_ctx, o_sent = orc.heartbeat(pb)
        np.testing.assert_array_equal(hctx.cpu().numpy().view(np.uint32), o_ctx)
        np.testing.assert_array_equal(sent.cpu().numpy().view(md), o_sent)
    assert (pb.read_count > 4).any()


def test_queue_capacity_argument_errors(eng):
    import ctypes as C
    L = eng._lib.lib()
    ps = eng.ProgressState(64, 3, 8, 2, DEV, extras=("self_slot", "reads"), read_cap=16)
    req = torch.ones(64, dtype=torch.uint8, device=DEV)
    res = torch.zeros(64, dtype=torch.uint8, device=DEV)
    p = ps.struct()
    p.read_cap = 3  # below the word
    assert L.qe_read_index(C.byref(p), eng._ptr(req), None, 0, eng._ptr(res), None, None,
                           None) == eng._lib.QE_ERANGE
    p = ps.struct()
    p.read_cap = 256
    assert L.qe_read_index(C.byref(p), eng._ptr(req), None, 0, eng._ptr(res), None, None,
                           None) == eng._lib.QE_ERANGE
    p = ps.struct()
    p.read_ovf = None  # a queue past the word needs the ring
    assert L.qe_read_index(C.byref(p), eng._ptr(req), None, 0, eng._ptr(res), None, None,
                           None) == eng._lib.QE_EINVAL
    p = ps.struct()
    p.reserved3 = 1
    assert L.qe_read_index(C.byref(p), eng._ptr(req), None, 0, eng._ptr(res), None, None,
                           None) == eng._lib.QE_EINVAL
