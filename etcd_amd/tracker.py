"""Python mirror of etcd's raft/tracker ProgressTracker API
(raft/tracker/tracker.go, progress.go) whose quorum decisions -- Committed,
TallyVotes, QuorumActive -- run on the MI355X batch engine.

Host-side bookkeeping (the Config sets, the Progress map, RecordVote's
first-vote-sticks map insert) mirrors the Go structs; the *Batch functions
evaluate many trackers in one GPU launch.
"""
import numpy as np
import torch

from . import engine
from .packing import pack
from .quorum import JointConfig, MajorityConfig, VoteResult

StateProbe, StateReplicate, StateSnapshot = 0, 1, 2


class Progress:
    """tracker.Progress fields used by the hot path (progress.go:30-80)."""

    __slots__ = ("Match", "Next", "State", "PendingSnapshot", "RecentActive", "ProbeSent",
                 "IsLearner")

    def __init__(self, Match=0, Next=1, IsLearner=False, RecentActive=False):
        self.Match, self.Next = Match, Next
        self.State = StateProbe
        self.PendingSnapshot = 0
        self.RecentActive = RecentActive
        self.ProbeSent = False
        self.IsLearner = IsLearner


class Config:
    """tracker.Config (tracker.go:27-78)."""

    def __init__(self, Voters=None, Learners=None, LearnersNext=None, AutoLeave=False):
        self.Voters = Voters if Voters is not None else JointConfig()
        self.Learners = Learners
        self.LearnersNext = LearnersNext
        self.AutoLeave = AutoLeave

    def String(self):
        s = f"voters={self.Voters.String()}"
        if self.Learners is not None:
            s += f" learners={MajorityConfig(self.Learners).String()}"
        if self.LearnersNext is not None:
            s += f" learners_next={MajorityConfig(self.LearnersNext).String()}"
        if self.AutoLeave:
            s += " autoleave"
        return s


class ProgressTracker(Config):
    """tracker.ProgressTracker (tracker.go:117-125)."""

    def __init__(self, MaxInflight=256):
        super().__init__()
        self.Progress = {}
        self.Votes = {}
        self.MaxInflight = MaxInflight

    # -- bookkeeping (host) ---------------------------------------------------
    def IsSingleton(self):
        return len(self.Voters[0]) == 1 and len(self.Voters[1]) == 0

    def VoterNodes(self):
        return sorted(self.Voters.IDs())

    def LearnerNodes(self):
        return sorted(self.Learners) if self.Learners else None

    def ConfState(self):
        return {"voters": self.Voters[0].Slice(), "voters_outgoing": self.Voters[1].Slice(),
                "learners": sorted(self.Learners or ()),
                "learners_next": sorted(self.LearnersNext or ()), "auto_leave": self.AutoLeave}

    def Visit(self, f):
        for vid in sorted(self.Progress):
            f(vid, self.Progress[vid])

    def ResetVotes(self):
        """tracker.go:252-254."""
        self.Votes = {}

    def RecordVote(self, vid, v):
        """tracker.go:258-263: the first vote sticks."""
        if vid not in self.Votes:
            self.Votes[vid] = bool(v)

    # -- quorum decisions (GPU) ----------------------------------------------
    def Committed(self, device=None):
        """tracker.go:177-179."""
        return CommittedBatch([self], device)[0]

    def TallyVotes(self, device=None):
        """tracker.go:267-288 -> (granted, rejected, VoteResult)."""
        return TallyVotesBatch([self], device)[0]

    def QuorumActive(self, device=None):
        """tracker.go:215-225."""
        return QuorumActiveBatch([self], device)[0]


def MakeProgressTracker(maxInflight):
    return ProgressTracker(maxInflight)


def _group(pt):
    learners = {vid for vid, pr in pt.Progress.items() if pr.IsLearner}
    return {
        "c0": pt.Voters[0], "c1": pt.Voters[1], "learners": learners,
        "acked": {vid: pr.Match for vid, pr in pt.Progress.items()},
        "votes": pt.Votes,
        "recent": {vid for vid, pr in pt.Progress.items() if pr.RecentActive},
    }


def _batch(trackers, device):
    p = pack([_group(t) for t in trackers])
    dev = torch.device(device if device is not None else "cuda")
    b = engine.SlotBatch(p.G, p.S, dev)
    b.load_host(p.match, inc=p.inc, out=p.out, learner=p.learner, voted=p.voted,
                granted=p.granted)
    return p, b


def CommittedBatch(trackers, device=None):
    if not trackers:
        return []
    _, b = _batch(trackers, device)
    out = engine.commit_vote(b, engine.Outputs(b.G, b.device, vote=False, tally=False))
    return [int(x) for x in out.commit.cpu().numpy().view(np.uint64)]


def TallyVotesBatch(trackers, device=None):
    if not trackers:
        return []
    _, b = _batch(trackers, device)
    out = engine.commit_vote(b, engine.Outputs(b.G, b.device, commit=False))
    gr, rj, vt = (x.cpu().numpy() for x in (out.granted, out.rejected, out.vote))
    return [(int(g), int(r), VoteResult(int(v))) for g, r, v in zip(gr, rj, vt)]


def QuorumActiveBatch(trackers, device=None):
    if not trackers:
        return []
    p, b = _batch(trackers, device)
    md = engine.mask_torch_dtype(p.S)
    rec = p.recent if p.S <= 8 else p.recent.view(np.int16)
    recent = torch.from_numpy(np.ascontiguousarray(rec)).to(b.device, dtype=md)
    act = engine.quorum_active(b, recent)
    return [bool(x) for x in act.cpu().numpy()]
