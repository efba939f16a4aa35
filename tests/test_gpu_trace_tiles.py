"""The reference's interaction traces (tests/trace_replay.py) replayed through
the production kernel instantiations the bench times, with the trace's group
placed at one lane of a 64-group tile among random groups.

tests/test_gpu_trace_replay.py replays each trace on a batch of ONE group
with the trace's Inflights capacity (255): qe_progress_step then takes its
memory-ring kernel.  Here the batch is three tiles (G = 192) with F = 8 and
no ReadIndex queue, so qe_progress_step takes the pipelined row-ring kernel
(qe_inst_prog.hip launch_progress_step: S <= 9, F <= 8, a run table of <= 4
-- every trace but probe_and_replicate.txt, whose 5 term runs take the
8-run kernel) with the untouched-slot skip and the cross-slot prefetch
running over 63 random neighbours.  Every engine call runs on the whole
batch and on the oracle (oracle/quorum_oracle.c) over the same batch, and
every group's state and outputs are compared after each call -- the
neighbours carry random states and random messages each round -- while the
trace's own group is checked against what the reference printed.  (No trace
holds more than a few MsgApps in flight, so F = 8 does not bind: the
replays' Progress lines would show it.)"""
import numpy as np
import pytest
import torch

from oracle import orc
from tests.progress_scenarios import bits, cc_arrays, peer_view  # noqa: F401
from tests.test_gpu_progress import (DEV, EXTRAS, assert_outputs, assert_same, load_msgs,
                                     random_msgs, random_state, to_device)
from tests.test_gpu_propose import load_props
from tests.test_gpu_trace_replay import gpu_elector
from tests.trace_replay import TRACES, Leader

pytestmark = pytest.mark.gpu

G_TILES = 192  # three 64-group tiles
F_TILE = 8     # row-form rings: the pipelined kernel


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from etcd_amd import engine
    return engine


class TileBackend:
    """The trace-replay backend over a G_TILES batch: group `pos` is the
    trace's, the others random; the GPU and the oracle run every call on the
    whole batch and must agree on every group (eng None: the oracle alone,
    tests/test_trace_replay.py)."""

    def __init__(self, eng, pos, seed, ring16=False):
        self.eng, self.pos, self.ring16 = eng, pos, ring16
        self.rng = np.random.default_rng(seed)
        self.calls = {"step": 0, "send": 0, "propose": 0, "heartbeat": 0, "switch": 0}

    # -- state ------------------------------------------------------------
    def load(self, sc, a, inc=None, tracked=None, out=None):
        S, G, g = sc["S"], G_TILES, self.pos
        R = sc.get("log_runs", len(sc["log"]["runs"]))
        masks = ("inc",) + (("out",) if out is not None else ())
        pb = random_state(self.rng, G, S, F_TILE, R, masks, EXTRAS, max_ents=sc["max_ents"])
        if self.ring16 and R <= 4 and S <= 9:  # ABI 8 (a trace with 5 term runs keeps 32 bits)
            from tests.test_gpu_progress import ring16_state
            ring16_state(self.rng, pb)
        full = (1 << S) - 1
        col = lambda s: s * G + g  # noqa: E731
        for s in range(S):
            pb.match[col(s)] = a["match"][s]
            pb.next[col(s)] = a["next"][s]
            pb.pending[col(s)] = a["pending"][s]
            pb.pw[col(s)] = orc.pack_word(a["flags"][s], 0, a["icount"][s])
            cap = a["ibuf"].size // S
            for k in range(int(a["icount"][s])):
                pb.ibuf[(s * F_TILE + k) * G + g] = a["ibuf"][s * cap + k]
        for k in ("committed", "term_start", "first_index", "last_index", "self_slot",
                  "lead_transferee"):
            getattr(pb, k)[g] = a[k][0]
        nr = int(a["run_count"][0])
        for r in range(nr):
            pb.run_first[r * G + g] = a["run_first"][r]
            pb.run_term[r * G + g] = a["run_term"][r]
        pb.run_count[g] = nr
        pb.snap_index[g] = a["snap_index"][0] if "snap_index" in a else a["first_index"][0] - 1
        pb.inc[g] = full if inc is None else inc
        if out is not None:
            pb.out[g] = out
        pb.tracked[g] = full if tracked is None else tracked
        self.masks, self.pb, self.sc = masks, pb, sc
        self.ps = to_device(self.eng, pb, masks, EXTRAS) if self.eng else None
        self.pci = self.unc = self.applied = self.max_unc = 0

    def _set(self, name, value):
        getattr(self.pb, name)[self.pos] = value
        v = int(value)
        if name in ("inc", "out", "tracked") and self.sc["S"] > 8 and v >= 1 << 15:
            v -= 1 << 16  # int16 storage of a u16 mask
        if self.ps is not None:
            getattr(self.ps, name)[self.pos] = v

    def set_outgoing(self, mask):
        self._set("out", mask)

    def set_snapshot(self, index):
        self._set("snap_index", index)

    def set_config(self, tracked, inc):
        self._set("tracked", tracked)
        self._set("inc", inc)

    # -- calls (whole batch, GPU and oracle) --------------------------------
    def _mask(self, a):
        md = orc.mask_dtype(self.sc["S"])
        return torch.from_numpy(a.astype(md).view(np.int16) if md == np.uint16 else a.astype(md)).to(DEV)

    def step(self, t, idx, hint, lt, ctx=None):
        assert ctx is None  # the traces carry no ReadIndex contexts
        pb, S, G, g = self.pb, self.sc["S"], G_TILES, self.pos
        mt, mi, mh, ml = random_msgs(self.rng, pb)
        for s in range(S):
            mt[s * G + g], mi[s * G + g], mh[s * G + g], ml[s * G + g] = t[s], idx[s], hint[s], lt[s]
        if self.eng:
            msgs = load_msgs(self.eng, self.ps, mt, mi, mh, ml)
            self.eng.progress_step(self.ps, msgs)
        o = orc.progress_step(pb, mt, mi, mh, ml)
        if self.eng:
            assert_outputs(msgs, o, S)
            assert_same(self.ps, pb)
        self.calls["step"] += 1
        return {"sent": int(o.sent[g]), "snap": int(o.snap[g]), "timeout_now": int(o.timeout_now[g]),
                "msg_count": o.msg_count[g::G][:S], "msg_index": o.msg_index[g::G][:S],
                "bcast": int(o.bcast[g]), "read_released": 0, "term_commit": int(o.term_commit[g]),
                "term_commit_index": int(o.term_commit_index[g])}

    def send(self, want, sei):
        pb, G, g = self.pb, G_TILES, self.pos
        w = self.rng.integers(0, 1 << self.sc["S"], G)
        w[g] = want
        if self.eng:
            sent, snap = self.eng.progress_send(self.ps, self._mask(w), sei)
        o_sent, o_snap = orc.progress_send(pb, w.astype(orc.mask_dtype(self.sc["S"])), sei)
        if self.eng:
            md = orc.mask_dtype(self.sc["S"])
            np.testing.assert_array_equal(sent.cpu().numpy().view(md), o_sent)
            np.testing.assert_array_equal(snap.cpu().numpy().view(md), o_snap)
            assert_same(self.ps, pb)
        self.calls["send"] += 1
        return {"sent": int(o_sent[g]), "snap": int(o_snap[g])}

    def propose(self, n, payload=0, append_only=False, cc=None):
        pb, G, g = self.pb, G_TILES, self.pos
        m, cnt1, pos1, lv1, sz1 = cc_arrays(cc)
        ne = self.rng.integers(0, 4, G).astype(np.uint32)
        ne[g] = n
        pl = self.rng.integers(0, 30, G).astype(np.uint64)
        pl[g] = payload
        cnt = np.zeros(G, np.uint8)
        cnt[g] = cnt1[0]
        pos = np.zeros((m, G), np.uint32)
        lv = np.zeros((m, G), np.uint8)
        sz = np.zeros((m, G), np.uint32)
        pos[:, g], lv[:, g], sz[:, g] = pos1, lv1, sz1
        cc_g = (m, cnt, pos.reshape(-1), lv.reshape(-1), sz.reshape(-1))
        applied = np.zeros(G, np.uint64)
        pci = np.zeros(G, np.uint64)
        unc = np.zeros(G, np.uint64)
        applied[g], pci[g], unc[g] = self.applied, self.pci, self.unc
        flags = 1 if append_only else 0
        if self.eng:
            pr = load_props(self.eng, self.ps, ne, pl, cc_g, applied, pci, unc, self.max_unc,
                            flags)
            self.eng.propose(self.ps, pr)
        o = orc.propose(pb, ne, pl, cc=cc_g, applied=applied, pending_conf_index=pci,
                        uncommitted_size=unc, max_uncommitted=self.max_unc, flags=flags)
        if self.eng:
            md = orc.mask_dtype(self.sc["S"])
            np.testing.assert_array_equal(pr.result.cpu().numpy(), o.result)
            np.testing.assert_array_equal(pr.cc_refused.cpu().numpy(), o.cc_refused)
            np.testing.assert_array_equal(pr.sent.cpu().numpy().view(md), o.sent)
            np.testing.assert_array_equal(pr.snap.cpu().numpy().view(md), o.snap)
            np.testing.assert_array_equal(pr.pending_conf_index.cpu().numpy().view(np.uint64), pci)
            np.testing.assert_array_equal(pr.uncommitted_size.cpu().numpy().view(np.uint64), unc)
            np.testing.assert_array_equal(self.ps.last_index.cpu().numpy().view(np.uint64),
                                          pb.last_index)
            assert_same(self.ps, pb)
        self.pci, self.unc = int(pci[g]), int(unc[g])
        self.calls["propose"] += 1
        return {"result": int(o.result[g]), "sent": int(o.sent[g]), "snap": int(o.snap[g]),
                "cc_refused": int(o.cc_refused[g])}

    def heartbeat(self):
        pb, S, G, g = self.pb, self.sc["S"], G_TILES, self.pos
        o_commit, o_ctx, o_sent = orc.heartbeat(pb)
        if self.eng:
            commit, ctx, sent = self.eng.heartbeat(self.ps)
            md = orc.mask_dtype(S)
            np.testing.assert_array_equal(sent.cpu().numpy().view(md), o_sent)
            got = commit.cpu().numpy().view(np.uint64)
            to = np.concatenate([(o_sent.astype(np.int64) >> s) & 1 for s in range(S)]) == 1
            np.testing.assert_array_equal(got[: S * G][to], o_commit[: S * G][to])
        self.calls["heartbeat"] += 1
        return [int(x) for x in o_commit[g::G][:S]], int(o_ctx[g]), int(o_sent[g])

    def become_leader(self, term, bcast=True):
        pb, G, g = self.pb, G_TILES, self.pos
        el = (self.rng.random(G) < 0.5).astype(np.uint8)
        el[g] = 1
        terms = pb.last_index + self.rng.integers(0, 3, G).astype(np.uint64)  # (neighbours: any)
        terms[g] = term
        if self.eng:
            ld = self.eng.Leader(self.ps, torch.from_numpy(el).to(DEV), bcast=bcast)
            ld.term.copy_(torch.from_numpy(terms.view(np.int64)).to(DEV))
            self.eng.become_leader(self.ps, ld)
        o = orc.become_leader(pb, terms, elected=el, bcast=bcast)
        if self.eng:
            md = orc.mask_dtype(self.sc["S"])
            np.testing.assert_array_equal(ld.result.cpu().numpy(), o.result)
            np.testing.assert_array_equal(ld.sent.cpu().numpy().view(md), o.sent)
            np.testing.assert_array_equal(ld.snap.cpu().numpy().view(md), o.snap)
            lv = o.result == 1
            np.testing.assert_array_equal(ld.pending_conf_index.cpu().numpy().view(np.uint64)[lv],
                                          o.pending_conf_index[lv])
            for k in ("term_start", "last_index", "run_count"):
                np.testing.assert_array_equal(getattr(self.ps, k).cpu().numpy().view(
                    getattr(pb, k).dtype), getattr(pb, k), err_msg=k)
            assert_same(self.ps, pb)
        self.calls["leader"] = self.calls.get("leader", 0) + 1
        if o.result[g] == 1:
            self.pci, self.unc = int(o.pending_conf_index[g]), 0
        return {"result": int(o.result[g]), "sent": int(o.sent[g]), "snap": int(o.snap[g])}

    def switch_config(self):
        pb, g = self.pb, self.pos
        if self.eng:
            sw = self.eng.switch_config(self.ps, self.eng.Switch(self.ps))
        o = orc.switch_config(pb)
        if self.eng:
            md = orc.mask_dtype(self.sc["S"])
            np.testing.assert_array_equal(sw.result.cpu().numpy(), o.result)
            np.testing.assert_array_equal(sw.sent.cpu().numpy().view(md), o.sent)
            np.testing.assert_array_equal(sw.snap.cpu().numpy().view(md), o.snap)
            assert_same(self.ps, pb)
        self.calls["switch"] += 1
        return {"result": int(o.result[g]), "sent": int(o.sent[g]), "snap": int(o.snap[g])}

    # -- views of the trace's group -----------------------------------------
    def peer(self, s):
        pb, G, g = self.pb, G_TILES, self.pos
        return peer_view(pb.match[g::G], pb.next[g::G], pb.pending[g::G], pb.flags[g::G],
                         pb.icount[g::G], s)

    def committed(self):
        return int(self.pb.committed[self.pos])

    def last_index(self):
        return int(self.pb.last_index[self.pos])

    def transferee(self):
        return int(self.pb.lead_transferee[self.pos])


@pytest.mark.parametrize("ring16", [False, True])
@pytest.mark.parametrize("pos", [0, 37, 127, 191])
@pytest.mark.parametrize("trace", TRACES, ids=lambda f: f.__name__)
def test_trace_replay_in_tiles(eng, trace, pos, ring16):
    """ring16: the batch in the 16-bit Inflights form (ABI 8; the bench's),
    the traces' own rings in it and most neighbours' too."""
    be = [None]

    def make(node, S):
        be[0] = TileBackend(eng, pos, seed=1000 + 7 * pos + S, ring16=ring16)
        return Leader(be[0], node, S)

    checked = trace(make, gpu_elector(eng))
    assert checked["rounds"] > 0 and checked["sends"] > 0
    assert be[0].calls["step"] == checked["rounds"]
