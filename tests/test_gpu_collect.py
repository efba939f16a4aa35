"""qe_collect (Ready-style deltas, raft/node.go:571-573) on the GPU against
numpy: the selected groups in ascending order with their values, for every
density, ragged and chunk-boundary sizes, unaligned flag arrays, a group
offset, NULL outputs, and the commit delta of a real replication round."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def eng():
    from etcd_amd import engine
    return engine


def check(eng, flags_np, values_np=None, goff=0, offset=0):
    G = flags_np.size
    buf = torch.zeros(G + offset, dtype=torch.uint8, device=DEV)
    flags = buf[offset:]
    flags.copy_(torch.from_numpy(flags_np))
    values = torch.from_numpy(values_np).to(DEV) if values_np is not None else None
    groups, vals = eng.collect(flags, values, group_offset=goff)
    torch.cuda.synchronize()
    want = np.nonzero(flags_np)[0]
    np.testing.assert_array_equal(groups.cpu().numpy(), want + goff)
    if values_np is not None:
        np.testing.assert_array_equal(vals.cpu().numpy(), values_np[want])
    return want.size


@pytest.mark.parametrize("G", [1, 63, 100, 4095, 4096, 4097, 3 * 4096 + 17, 1_000_003])
@pytest.mark.parametrize("density", [0.0, 0.001, 0.3, 1.0])
def test_collect_matches_numpy(eng, G, density):
    rng = np.random.default_rng(G + int(density * 1000))
    flags = (rng.random(G) < density).astype(np.uint8) * rng.integers(1, 256, G).astype(np.uint8)
    values = rng.integers(-(1 << 62), 1 << 62, G, dtype=np.int64)
    n = check(eng, flags, values, goff=12345)
    assert n == {0.0: 0, 1.0: G}.get(density, n)


@pytest.mark.parametrize("offset", [1, 3, 8])
def test_collect_unaligned_flags(eng, offset):
    """A flag array that is not 16-B aligned takes the byte path."""
    rng = np.random.default_rng(offset)
    G = 2 * 4096 + 333
    flags = (rng.random(G) < 0.5).astype(np.uint8)
    check(eng, flags, rng.integers(0, 1 << 40, G, dtype=np.int64), offset=offset)


def test_collect_empty_and_no_values(eng):
    import ctypes as C
    lib = eng._lib.lib()
    count = torch.full((1,), 7, dtype=torch.int64, device=DEV)
    eng.check("qe_collect", lib.qe_collect(0, 0, None, None, None, None, None, eng._ptr(count), None,
                                           eng._stream(torch.device(DEV))))
    torch.cuda.synchronize()
    assert int(count.item()) == 0
    flags = np.zeros(5000, np.uint8)
    flags[[0, 4095, 4096, 4999]] = 1
    check(eng, flags, None)
    # values requested without a values array: refused
    out = torch.empty(8, dtype=torch.int64, device=DEV)
    f = torch.ones(8, dtype=torch.uint8, device=DEV)
    scratch = torch.empty(64, dtype=torch.int64, device=DEV)
    rc = lib.qe_collect(8, 0, None, eng._ptr(f), None, None, eng._ptr(out), eng._ptr(count),
                        eng._ptr(scratch), eng._stream(torch.device(DEV)))
    assert rc != 0
    del C


@pytest.mark.parametrize("G", [100, 4097, 3 * 4096 + 17])
def test_collect_with_perm(eng, G):
    """Packed batches (qe_pack_order): out_groups[i] = goff + perm[g] for the
    i-th selected packed position g, values taken at g."""
    rng = np.random.default_rng(G)
    flags = (rng.random(G) < 0.4).astype(np.uint8)
    values = rng.integers(0, 1 << 62, G, dtype=np.int64)
    perm = rng.permutation(G).astype(np.int64)
    groups, vals = eng.collect(torch.from_numpy(flags).to(DEV), torch.from_numpy(values).to(DEV),
                               group_offset=77, perm=torch.from_numpy(perm).to(DEV))
    torch.cuda.synchronize()
    want = np.nonzero(flags)[0]
    np.testing.assert_array_equal(groups.cpu().numpy(), perm[want] + 77)
    np.testing.assert_array_equal(vals.cpu().numpy(), values[want])


def test_collect_full_size(eng):
    """64M groups (config 2's batch) at half density, every entry compared."""
    G = 1 << 26
    rng = np.random.default_rng(7)
    flags = (rng.random(G) < 0.5).astype(np.uint8)
    values = rng.integers(0, 1 << 62, G, dtype=np.int64)
    check(eng, flags, values)


def test_collect_above_register_scan(eng):
    """More than 16K chunks (64M groups): the scan's register path no longer
    holds a thread's counts, the looped path takes over."""
    G = (1 << 26) + 3 * 4096 + 5
    rng = np.random.default_rng(11)
    flags = (rng.random(G) < 0.01).astype(np.uint8)
    check(eng, flags, None, goff=5)


def test_collect_replication_commit_delta(eng):
    """The commit delta of a replication round: the groups whose `adv` flag
    is set, with their new committed index, equal numpy's selection of the
    same outputs."""
    G, S = 300_001, 5
    b = eng.SlotBatch(G, S, DEV, masks=(), votes=False)
    eng.gen_groups(b, 0x5EED, p_absent=0)
    rows = b.match_rows()
    lo, hi = rows.min(dim=0).values, rows.max(dim=0).values
    st = eng.ReplicationState(b, lo.clone(), lo + (hi - lo) // 2, hi + 1024)
    rb = eng.SlotBatch(G, S, DEV, masks=(), votes=False)
    eng.gen_groups(rb, 0xACC, p_absent=0)
    resp = b.match.clone() + (rb.match & 1023)
    rm = torch.from_numpy(np.random.default_rng(3).integers(0, 32, G).astype(np.uint8)).to(DEV)
    adv = torch.zeros(G, dtype=torch.uint8, device=DEV)
    eng.replication_round(st, resp, rm, adv=adv)
    groups, commits = eng.collect(adv, st.committed, group_offset=b.group_offset)
    torch.cuda.synchronize()
    a = adv.cpu().numpy()
    want = np.nonzero(a)[0]
    assert 0 < want.size < G
    np.testing.assert_array_equal(groups.cpu().numpy(), want + b.group_offset)
    np.testing.assert_array_equal(commits.cpu().numpy(), st.committed.cpu().numpy()[want])
