"""The timed kernels pinned at the bench's own sizes.

bench.py times qe_progress_step (progress_step / _n7 / _joint), qe_propose
(propose) and qe_switch_config (switch_config) on 16M groups with their
production kernels: the pipelined row-ring k_progress_step without byte
accounting or ReadIndex, k_propose / k_switch_config without accounting.
Here each of those launches runs on the bench's full 16M-group state
(bench.progress_round_state / psend_state / the switch_config set-up, the
same launch geometry), and 512 sampled 64-group tiles -- spread over the
whole batch, the first and the last among them -- are checked group by group
against the oracle run on the same tiles' starting state: every Progress
field, every live Inflights entry, committed and lastIndex, and every
per-group and per-peer output.  Groups are independent, so the oracle on
the sample is the oracle on the batch, restricted."""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import orc
from tests.test_gpu_progress import DEV, RING_MASK, live_entries

pytestmark = pytest.mark.gpu

G_FULL = 1 << 24
N_TILES = 512


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import bench
    from etcd_amd import engine
    bench.engine = engine
    return engine


def sample_groups(G, seed):
    rng = np.random.default_rng(seed)
    tiles = np.unique(np.concatenate([[0, (G - 1) // 64], rng.choice(G // 64, N_TILES - 2,
                                                                     replace=False)]))
    return (tiles[:, None] * 64 + np.arange(64)[None, :]).reshape(-1)


def rows(t, S, stride, idx):
    """[S][stride] device rows -> [S][len(idx)] host (numpy, native dtype)."""
    v = t.view(S, stride)[:, torch.from_numpy(idx).to(t.device)]
    return v.cpu().numpy()


def gather(ps, idx):
    """The sampled groups of ProgressState `ps` as an oracle ProgressBatch
    (rings decoded with qe_ring_unpack), plus the raw peer words."""
    S, F, R, st, Gs = ps.S, ps.F, ps.R, ps.stride, idx.size
    dev_idx = torch.from_numpy(idx).to(ps.device)
    pb = orc.ProgressBatch(Gs, S, F, R, max_ents=ps.max_ents)
    u64 = lambda t: rows(t, S, st, idx).view(np.uint64).reshape(-1)  # noqa: E731
    pb.match, pb.next, pb.pending = u64(ps.match), u64(ps.next), u64(ps.pending)
    peer = rows(ps.peer, S, st, idx).view(np.uint32).reshape(-1)
    pb.pw = peer & ~RING_MASK
    FP = ps.FP
    ring_rows = (torch.arange(S, device=ps.device).view(S, 1) * st + dev_idx.view(1, -1)).reshape(-1)
    lo = ps.ilo.view(S * st, FP)[ring_rows].cpu().numpy().view(np.uint32).reshape(-1)
    hi = ps.ihi.view(S * st, FP)[ring_rows].cpu().numpy().view(np.uint32).reshape(-1)
    ent = np.zeros(S * Gs * F, np.uint64)
    from etcd_amd import _lib
    if ps.infl16 is not None:  # ABI 8: offsets below each peer's Next
        o16 = ps.infl16.view(S * st, 8)[ring_rows].cpu().numpy().view(np.uint16).reshape(-1)
        nxt = np.ascontiguousarray(pb.next)
        assert _lib.lib().qe_ring_unpack16(Gs, S, F, Gs, o16.ctypes.data, lo.ctypes.data,
                                           hi.ctypes.data, nxt.ctypes.data,
                                           np.ascontiguousarray(peer).ctypes.data,
                                           ent.ctypes.data) == 0
        pb.ring16 = True
    else:
        assert _lib.lib().qe_ring_unpack(Gs, S, F, Gs, lo.ctypes.data, hi.ctypes.data,
                                         np.ascontiguousarray(peer).ctypes.data,
                                         ent.ctypes.data) == 0
    pb.ibuf = np.ascontiguousarray(ent.reshape(S, Gs, F).transpose(0, 2, 1)).reshape(-1)
    g1 = lambda t: t[dev_idx].cpu().numpy()  # noqa: E731
    for k in ("committed", "term_start", "first_index", "last_index"):
        setattr(pb, k, g1(getattr(ps, k)).view(np.uint64).copy())
    pb.run_first = rows(ps.run_first, R, st, idx).view(np.uint64).reshape(-1)
    pb.run_term = rows(ps.run_term, R, st, idx).view(np.uint64).reshape(-1)
    pb.run_count = g1(ps.run_count).copy()
    for k in ("self_slot", "lead_transferee"):
        if getattr(ps, k) is not None:
            setattr(pb, k, g1(getattr(ps, k)).copy())
    for k in ("inc", "out", "tracked"):
        if getattr(ps, k) is not None:
            setattr(pb, k, g1(getattr(ps, k)).view(orc.mask_dtype(S)).copy())
    if ps.snap_index is not None:
        pb.snap_index = g1(ps.snap_index).view(np.uint64).copy()
    return pb


def assert_sample_equal(got, want, tag):
    for k in ("match", "next", "pending", "committed", "last_index"):
        np.testing.assert_array_equal(getattr(got, k), getattr(want, k), err_msg=f"{tag} {k}")
    np.testing.assert_array_equal(got.pw, want.pw, err_msg=f"{tag} peer words")
    live = live_entries(want.pw, want.S, want.F, want.G)
    np.testing.assert_array_equal(got.ibuf[live], want.ibuf[live], err_msg=f"{tag} rings")
    if want.lead_transferee is not None:
        np.testing.assert_array_equal(got.lead_transferee, want.lead_transferee, err_msg=tag)


@pytest.mark.parametrize("wl", ["progress_step", "progress_step_n7", "progress_step_joint"])
def test_progress_step_full_size_sampled(eng, wl):
    """The production qe_progress_step at the bench's 16M groups, on the
    bench's own state and messages."""
    import bench
    _, G, S, kind = bench.WORKLOADS[wl]
    assert G == G_FULL
    joint = kind == "progress_joint"
    ps = eng.ProgressState(G, S, 8, 4, DEV, extras=("self_slot",), max_ents=16,
                           masks=("inc", "out") if joint else (), ring16=bench.RING16)
    if joint:
        ps.inc.fill_(0b101111)
        ps.out.fill_(0b011111)
    msgs = eng.PeerMsgs(ps)
    msgs.snap = msgs.timeout_now = None  # the bench's output set
    msgs.read_released = msgs.term_commit = msgs.term_commit_index = None
    bench.progress_round_state(ps, msgs)
    idx = sample_groups(G, 77 + S)
    pb = gather(ps, idx)
    st = ps.stride
    mtype = rows(msgs.type, S, st, idx).reshape(-1)
    mindex, mhint, mlogterm = (rows(t, S, st, idx).view(np.uint64).reshape(-1)
                               for t in (msgs.index, msgs.reject_hint, msgs.log_term))
    eng.progress_step(ps, msgs)
    torch.cuda.synchronize()
    o = orc.progress_step(pb, mtype, mindex, mhint, mlogterm)
    got = gather(ps, idx)
    assert_sample_equal(got, pb, wl)
    dev_idx = torch.from_numpy(idx).to(DEV)
    np.testing.assert_array_equal(msgs.sent[dev_idx].cpu().numpy(), o.sent, err_msg="sent")
    np.testing.assert_array_equal(msgs.bcast[dev_idx].cpu().numpy(), o.bcast, err_msg="bcast")
    cnt = rows(msgs.msg_count, S, st, idx).reshape(-1)
    np.testing.assert_array_equal(cnt, o.msg_count, err_msg="msg_count")
    ix = rows(msgs.msg_index, S, st, idx).view(np.uint64).reshape(-1)
    np.testing.assert_array_equal(ix[cnt > 0], o.msg_index[cnt > 0], err_msg="msg_index")
    assert o.bcast.any() and (cnt > 1).any()


def test_propose_full_size_sampled(eng):
    """The production qe_propose on the bench's propose state (16M groups,
    3 entries each, bcast to 4 followers)."""
    import bench
    _, G, S, _ = bench.WORKLOADS["propose"]
    ps = eng.ProgressState(G, S, 8, 1, DEV, extras=("self_slot",), max_ents=0, ring16=bench.RING16)
    bench.psend_state(ps)
    ps.self_slot.fill_(0)
    ps.term_start.copy_(ps.last_index)
    pr = eng.Proposals(ps, max_uncommitted=1 << 30)
    pr.num_entries.fill_(3)
    pr.payload.fill_(24)
    pr.uncommitted_size.fill_(100)
    idx = sample_groups(G, 91)
    pb = gather(ps, idx)
    dev_idx = torch.from_numpy(idx).to(DEV)
    Gs = idx.size
    unc = np.full(Gs, 100, np.uint64)
    pci = np.zeros(Gs, np.uint64)
    eng.propose(ps, pr)
    torch.cuda.synchronize()
    o = orc.propose(pb, np.full(Gs, 3, np.uint32), np.full(Gs, 24, np.uint64),
                    applied=np.zeros(Gs, np.uint64), pending_conf_index=pci,
                    uncommitted_size=unc, max_uncommitted=1 << 30)
    got = gather(ps, idx)
    assert_sample_equal(got, pb, "propose")
    np.testing.assert_array_equal(pr.result[dev_idx].cpu().numpy(), o.result)
    np.testing.assert_array_equal(pr.sent[dev_idx].cpu().numpy(), o.sent)
    np.testing.assert_array_equal(pr.uncommitted_size[dev_idx].cpu().numpy().view(np.uint64), unc)
    assert (o.result == 1).all() and (o.sent == 0b11110).all()


def test_switch_config_full_size_sampled(eng):
    """The production qe_switch_config on the bench's switch_config state."""
    import bench
    desc, G, S, kind = bench.WORKLOADS["switch_config"]

    class D:
        dev = torch.device(DEV)
        rank = 0
    stats = eng.stats_buffer(DEV)
    _, _, _, _, keep = bench.setup("switch_config", G, S, kind, D, stats)
    ps, sw = keep["ps"], keep["sw"]
    keep["prepare"]()
    idx = sample_groups(G, 93)
    pb = gather(ps, idx)
    eng.switch_config(ps, sw)
    torch.cuda.synchronize()
    o = orc.switch_config(pb)
    got = gather(ps, idx)
    assert_sample_equal(got, pb, "switch_config")
    dev_idx = torch.from_numpy(idx).to(DEV)
    np.testing.assert_array_equal(sw.result[dev_idx].cpu().numpy(), o.result)
    np.testing.assert_array_equal(sw.sent[dev_idx].cpu().numpy(), o.sent)
    out = o.result & 0xF
    assert (out == 3).any() and (out == 4).any() and (o.result & 0x10).any()
