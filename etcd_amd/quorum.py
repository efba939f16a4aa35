"""Python mirror of etcd's raft/quorum package API (raft/quorum/*.go), backed
by the MI355X batch engine.

Same names, argument meaning and results as the Go package:
  Index, VoteResult (VotePending=1, VoteLost=2, VoteWon=3), AckedIndexer,
  MapAckIndexer, MajorityConfig, JointConfig.
Per-group methods (CommittedIndex / VoteResult) evaluate a batch of one on
the GPU; CommittedIndexBatch / VoteResultBatch evaluate many groups in one
launch -- the drop-in batch entry point of BASELINE.json's north star.
There is no CPU implementation here: without the HIP library the import
fails (etcd_amd/_lib.py).
"""
import enum

import numpy as np
import torch

from . import engine
from .packing import pack

INF = (1 << 64) - 1


class Index(int):
    """quorum.Index (raft/quorum/quorum.go:23-30); MaxUint64 prints as ∞."""

    def __str__(self):
        return "∞" if int(self) == INF else str(int(self))


class VoteResult(enum.IntEnum):
    """quorum.VoteResult (raft/quorum/quorum.go:48-58, voteresult_string.go)."""

    VotePending = 1
    VoteLost = 2
    VoteWon = 3

    def __str__(self):
        return self.name


VotePending, VoteLost, VoteWon = VoteResult.VotePending, VoteResult.VoteLost, VoteResult.VoteWon


class AckedIndexer:
    """quorum.AckedIndexer (raft/quorum/quorum.go:34-36)."""

    def AckedIndex(self, voter_id):  # -> (Index, bool)
        raise NotImplementedError


class MapAckIndexer(dict, AckedIndexer):
    """mapAckIndexer (raft/quorum/quorum.go:38-43)."""

    def AckedIndex(self, voter_id):
        if voter_id in self:
            return Index(self[voter_id]), True
        return Index(0), False


def _device(device):
    return torch.device(device if device is not None else "cuda")


class MajorityConfig(set):
    """quorum.MajorityConfig (raft/quorum/majority.go:25): a set of voter IDs."""

    def String(self):
        return "(" + " ".join(str(i) for i in sorted(self)) + ")"

    __str__ = String

    def Slice(self):
        return sorted(self)

    def Describe(self, l):
        """majority.go:45-101: the commit indexes of the voters as a bar
        chart (text only, host side).  The voter of the i-th smallest index
        gets a bar of i (0 when its index equals its predecessor's)."""
        if len(self) == 0:
            return "<empty majority quorum>"
        n = len(self)
        info = []
        for vid in self:
            idx, ok = l.AckedIndex(vid)
            info.append([vid, int(idx), ok, 0])
        info.sort(key=lambda t: (t[1], t[0]))
        for i in range(1, n):
            if info[i - 1][1] < info[i][1]:
                info[i][3] = i
        info.sort(key=lambda t: t[0])
        out = [" " * n + "    idx\n"]
        for vid, idx, ok, bar in info:
            out.append("?" + " " * n if not ok else "x" * bar + ">" + " " * (n - bar))
            out.append(f" {idx:5d}    (id={vid})\n")
        return "".join(out)

    def CommittedIndex(self, l, device=None):
        """majority.go:126-172, evaluated on the GPU."""
        return CommittedIndexBatch([JointConfig(self, MajorityConfig())], [l], device)[0]

    def VoteResult(self, votes, device=None):
        """majority.go:178-210, evaluated on the GPU."""
        return VoteResultBatch([JointConfig(self, MajorityConfig())], [votes], device)[0]


class JointConfig(tuple):
    """quorum.JointConfig (raft/quorum/joint.go:19): (incoming, outgoing)."""

    def __new__(cls, c0=None, c1=None):
        return super().__new__(cls, (MajorityConfig(c0 or ()), MajorityConfig(c1 or ())))

    def String(self):
        if len(self[1]) > 0:
            return self[0].String() + "&&" + self[1].String()
        return self[0].String()

    __str__ = String

    def IDs(self):
        """joint.go:30-38."""
        return set(self[0]) | set(self[1])

    def Describe(self, l):
        """joint.go:40-44: Describe of the union of the halves."""
        return MajorityConfig(self.IDs()).Describe(l)

    def CommittedIndex(self, l, device=None):
        """joint.go:49-56, evaluated on the GPU."""
        return CommittedIndexBatch([self], [l], device)[0]

    def VoteResult(self, votes, device=None):
        """joint.go:61-75, evaluated on the GPU."""
        return VoteResultBatch([self], [votes], device)[0]


def _as_joint(c):
    if isinstance(c, JointConfig):
        return c
    if isinstance(c, (set, frozenset, list)) and not (len(c) == 2 and all(isinstance(x, (set, frozenset)) for x in c)):
        return JointConfig(c, ())
    return JointConfig(c[0], c[1])


def _acked_fn(l):
    if hasattr(l, "AckedIndex"):
        return l.AckedIndex
    return lambda vid: (l[vid], True) if vid in l else (0, False)


def CommittedIndexBatch(configs, indexers, device=None):
    """JointConfig.CommittedIndex for many groups in one GPU launch.
    Returns a list of Index."""
    cfgs = [_as_joint(c) for c in configs]
    groups = [{"c0": c[0], "c1": c[1], "acked": _acked_fn(l)} for c, l in zip(cfgs, indexers)]
    if not groups:
        return []
    p = pack(groups)
    b = engine.SlotBatch(p.G, p.S, _device(device), masks=("inc", "out"), votes=False)
    b.load_host(p.match, inc=p.inc, out=p.out)
    commit = engine.committed_index(b)
    return [Index(int(x)) for x in commit.cpu().numpy().view(np.uint64)]


def VoteResultBatch(configs, votes_list, device=None):
    """JointConfig.VoteResult for many groups in one GPU launch."""
    cfgs = [_as_joint(c) for c in configs]
    groups = [{"c0": c[0], "c1": c[1], "votes": v} for c, v in zip(cfgs, votes_list)]
    if not groups:
        return []
    p = pack(groups)
    b = engine.SlotBatch(p.G, p.S, _device(device), masks=("inc", "out"), votes=True)
    b.load_host(p.match, inc=p.inc, out=p.out, voted=p.voted, granted=p.granted)
    vote = engine.vote_result(b)
    return [VoteResult(int(x)) for x in vote.cpu().numpy()]
