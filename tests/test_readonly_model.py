"""The oracle's ReadIndex queue (oracle/quorum_oracle.c: ro_load / ro_advance,
orc_read_index_batch, the MsgHeartbeatResp arm of orc_progress_step_batch) in
its device form -- the acks word, the overflow ring at context mod read_cap,
the request keys (ABI 7) -- checked against an independent restatement of
raft/read_only.go kept here as Python lists, the way the reference keeps it:

  readIndexQueue   []string              -> a list of context numbers
  pendingReadIndex map[string]*readIndexStatus (acks map[uint64]bool)
                                          -> per context an acks bit set and
                                             the request key (m.Entries[0].Data)
  addRequest (:56-63): a pending context (here: key) is ignored
  recvAck    (:68-76): acks of the request with that context, nil if none
  advance    (:81-112): release every request up to and including it

driven by the leader's arms of raft.go: MsgReadIndex (:1078-1096, with the
engine's capacity: a request past read_cap is QE_RI_FULL) and
MsgHeartbeatResp (:1296-1309: recvAck, then advance when
Voters.VoteResult(acks) == VoteWon).  Random queues up to 255 deep with
garbage in the dead slots, contexts pending / released / unknown / absent,
and the newest-context default -- CPU only.  (The GPU's queue is compared
with the oracle in tests/test_gpu_readindex.py; this pins the oracle
itself past the word, where the reference's own tests hold at most two
requests.)"""
import numpy as np
import pytest

from etcd_amd import _lib
from oracle import orc
from tests.test_gpu_progress import EXTRAS, random_msgs, random_state

M32 = 0xFFFFFFFF


class Model:
    """One group's readOnly (read_only.go:39-63), ReadOnlySafe."""

    def __init__(self, head, entries):
        self.head = head            # context number of the oldest pending request
        self.q = list(entries)      # [ctx, acks, key] in arrival order

    def add(self, self_bit, key, cap):
        for c, _, k in self.q:
            if k == key:
                return _lib.QE_RI_DUPLICATE, c
        if not self.q and self.head == 0:  # context numbers start at 1 (0: no context)
            self.head = 1
        ctx = (self.head + len(self.q)) & M32
        if len(self.q) >= cap or ctx == 0:
            return _lib.QE_RI_FULL, None
        self.q.append([ctx, self_bit, key])
        return _lib.QE_RI_QUEUED, ctx

    def ack(self, slot, ctx, voters):
        """recvAck + advance on a won vote; returns how many were released."""
        if ctx == 0:  # len(m.Context) == 0 (raft.go:1296)
            return 0
        for j, e in enumerate(self.q):
            if e[0] == ctx:
                e[1] |= 1 << slot
                if bin(e[1] & voters).count("1") >= bin(voters).count("1") // 2 + 1:
                    del self.q[:j + 1]
                    self.head = (self.head + j + 1) & M32
                    return j + 1
                return 0
        return 0


def device_queue(pb, g):
    """Group g's queue from the oracle's device form: [ctx, acks, key]."""
    G, cap = pb.G, max(4, pb.read_cap)
    head, n = int(pb.read_head[g]), min(int(pb.read_count[g]), cap)
    word = pb.read_acks.view(orc.mask_dtype(pb.S)).reshape(G, 4)[g]
    ring = pb.read_ovf.reshape(G, cap)[g]
    keys = pb.read_keys.reshape(G, cap)[g]
    out = []
    for j in range(n):
        c = (head + j) & M32
        out.append([c, int(word[j]) if j < 4 else int(ring[c % cap]), int(keys[c % cap])])
    return head, out


@pytest.mark.parametrize("S,cap", [(3, 16), (5, 64), (5, 255), (10, 32), (16, 255)])
def test_oracle_queue_matches_read_only_model(S, cap):
    rng = np.random.default_rng(5100 + 17 * S + cap)
    G = 257
    pb = random_state(rng, G, S, 8, 3, (), EXTRAS, max_ents=1)
    full = (1 << S) - 1
    pb.tracked[:] = full
    pb.self_slot[:] = rng.integers(0, S, G)
    pb.term_start[:] = np.minimum(pb.term_start, pb.last_index)
    pb.committed[:] = pb.last_index  # an entry of the term committed: requests queue
    pb.track_reads(cap, keys=True)
    deep = rng.random(G) < 0.7
    pb.read_count[:] = np.where(deep, rng.integers(5, cap + 1, G), rng.integers(0, 5, G))
    pb.read_head[:] = np.where(rng.random(G) < 0.8, rng.integers(1, 1000, G),
                               rng.integers(1, 1 << 32, G, dtype=np.uint64)).astype(np.uint32)
    pb.read_acks[:] = rng.integers(0, 1 << 62, G, dtype=np.uint64).astype(pb.read_acks.dtype)
    pb.read_ovf[:] = rng.integers(0, 1 << 16, pb.read_ovf.size).astype(pb.read_ovf.dtype)
    # keys distinct within each queue (a repeated one is a duplicate request)
    pb.read_keys[:] = rng.permutation(pb.read_keys.size).astype(np.uint64) * 7919 + 1
    models = [Model(*device_queue(pb, g)) for g in range(G)]
    assert (pb.read_count > 4).sum() > G // 2  # most queues start past the word
    seen = set()
    for rnd in range(16):
        if rnd % 3 == 1:  # MsgReadIndex: fresh keys and keys already pending
            req = (rng.random(G) < 0.8).astype(np.uint8)
            key = rng.integers(1 << 40, 1 << 62, G, dtype=np.uint64)
            for g in range(G):
                if models[g].q and rng.random() < 0.3:
                    key[g] = models[g].q[int(rng.integers(0, len(models[g].q)))][2]
            res, ctx, _ = orc.read_index(pb, req, False, key=key)
            for g in range(G):
                if not req[g]:
                    assert res[g] == _lib.QE_RI_NONE
                    continue
                r, c = models[g].add(1 << int(pb.self_slot[g]), int(key[g]), cap)
                assert res[g] == r, (rnd, g, res[g], r)
                if c is not None:
                    assert int(ctx[g]) == c, (rnd, g)
                seen.add(int(res[g]))
        else:  # one round of MsgHeartbeatResp from random peers
            mtype, mindex, mhint, mlogterm = random_msgs(rng, pb)
            mtype[:] = np.where(rng.random(mtype.size) < 0.7, 3, 0).astype(mtype.dtype)
            default = rnd % 4 == 3
            cx = np.zeros(S * G, np.uint32)
            if not default:
                for g in range(G):
                    h, n = models[g].head, len(models[g].q)
                    for s in range(S):
                        pick = rng.integers(0, 5)
                        cx[s * G + g] = (0 if pick == 0 else
                                         (h - int(rng.integers(1, 4))) & M32 if pick == 1 else
                                         (h + n + int(rng.integers(0, 3))) & M32 if pick == 2 else
                                         (h + int(rng.integers(0, max(n, 1)))) & M32)
            o = orc.progress_step(pb, mtype, mindex, mhint, mlogterm,
                                  read_ctx=None if default else cx)
            for g in range(G):
                m = models[g]
                newest = m.q[-1][0] if m.q else 0  # lastPendingRequestCtx at the round's start
                rel = 0
                for s in range(S):
                    if mtype[s * G + g] == 3:
                        rel += m.ack(s, newest if default else int(cx[s * G + g]), full)
                assert int(o.read_released[g]) == rel, (rnd, g)
                seen.add(100 + min(rel, 9))
        for g in range(G):
            h, q = device_queue(pb, g)
            assert h == models[g].head, (rnd, g)
            assert q == models[g].q, (rnd, g, q[:6], models[g].q[:6])
    # the run covered queued and duplicate requests and releases past the word
    assert {_lib.QE_RI_QUEUED, _lib.QE_RI_DUPLICATE} <= seen
    assert any(v >= 105 for v in seen), sorted(seen)
