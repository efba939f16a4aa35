"""etcd_amd — MI355X-native batched Raft quorum engine.

Drop-in batch path for etcd's raft/quorum + raft/tracker hot path
(CommittedIndex, VoteResult, JointConfig, TallyVotes, QuorumActive,
MaybeUpdate-driven commit advance) evaluated over millions of independent
Raft groups with hand-written HIP kernels for gfx950.  The C ABI lives in
include/etcd_quorum.h; this package is its Python host side.
"""
from . import _lib, engine  # noqa: F401  (raises if the HIP library is missing)
from .quorum import (INF, AckedIndexer, CommittedIndexBatch, Index, JointConfig,  # noqa: F401
                     MajorityConfig, MapAckIndexer, VoteLost, VotePending, VoteResult,
                     VoteResultBatch, VoteWon)
from .tracker import (CommittedBatch, MakeProgressTracker, Progress,  # noqa: F401
                      ProgressTracker, QuorumActiveBatch, TallyVotesBatch)
from . import confchange  # noqa: F401  (raft/confchange mirror)

__version__ = "0.1.0"
