"""Pure-Python restatement of etcd raft/quorum + raft/tracker semantics over
maps, exactly as the Go code is written (TEST INFRASTRUCTURE ONLY).

This is the small-case oracle: it consumes voter-ID sets and ID-keyed maps,
the reference's own data model, so it can be checked directly against the
golden fixtures without any slot packing.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import anything under oracle/.

Parity pin: tests/test_oracle_golden.py runs every case of
tests/golden/quorum_testdata.jsonl (127 cases extracted from
raft/quorum/testdata/*.txt) and the raft_tables.json tables through it.
"""
INF = (1 << 64) - 1
VOTE_PENDING, VOTE_LOST, VOTE_WON = 1, 2, 3
VOTE_NAMES = {1: "VotePending", 2: "VoteLost", 3: "VoteWon"}


def majority_committed(cfg, acked):
    """MajorityConfig.CommittedIndex, raft/quorum/majority.go:126-172.

    cfg: iterable of voter ids; acked: dict id -> index (absent = no key)."""
    cfg = set(cfg)
    n = len(cfg)
    if n == 0:
        return INF  # :128-132
    srt = [0] * n
    i = n - 1  # fill from the right, :150-161
    for vid in cfg:
        if vid in acked:
            srt[i] = acked[vid]
            i -= 1
    # insertionSort, :115-122
    for a in range(1, n):
        j = a
        while j > 0 and srt[j] < srt[j - 1]:
            srt[j], srt[j - 1] = srt[j - 1], srt[j]
            j -= 1
    return srt[n - (n // 2 + 1)]  # :170-171


def alternative_committed(cfg, acked):
    """alternativeMajorityCommittedIndex, raft/quorum/quick_test.go:85-122."""
    cfg = set(cfg)
    if not cfg:
        return INF
    id_to_idx = {vid: acked[vid] for vid in cfg if vid in acked}
    idx_to_votes = {idx: 0 for idx in id_to_idx.values()}
    for idx in id_to_idx.values():
        for idy in list(idx_to_votes):
            if idy > idx:
                continue
            idx_to_votes[idy] += 1
    q = len(cfg) // 2 + 1
    best = 0
    for idx, cnt in idx_to_votes.items():
        if cnt >= q and idx > best:
            best = idx
    return best


def majority_vote(cfg, votes):
    """MajorityConfig.VoteResult, raft/quorum/majority.go:178-210."""
    cfg = set(cfg)
    if not cfg:
        return VOTE_WON
    ny = [0, 0]
    missing = 0
    for vid in cfg:
        if vid not in votes:
            missing += 1
            continue
        ny[1 if votes[vid] else 0] += 1
    q = len(cfg) // 2 + 1
    if ny[1] >= q:
        return VOTE_WON
    if ny[1] + missing >= q:
        return VOTE_PENDING
    return VOTE_LOST


def joint_committed(c0, c1, acked):
    """JointConfig.CommittedIndex, raft/quorum/joint.go:49-56."""
    return min(majority_committed(c0, acked), majority_committed(c1, acked))


def joint_vote(c0, c1, votes):
    """JointConfig.VoteResult, raft/quorum/joint.go:61-75."""
    r1 = majority_vote(c0, votes)
    r2 = majority_vote(c1, votes)
    if r1 == r2:
        return r1
    if VOTE_LOST in (r1, r2):
        return VOTE_LOST
    return VOTE_PENDING


def tally_votes(c0, c1, learners, votes):
    """ProgressTracker.TallyVotes, raft/tracker/tracker.go:267-288.
    Progress entries = voters of both halves + learners."""
    granted = rejected = 0
    for vid in set(c0) | set(c1) | set(learners):
        if vid in learners:
            continue
        if vid not in votes:
            continue
        if votes[vid]:
            granted += 1
        else:
            rejected += 1
    return granted, rejected, joint_vote(c0, c1, votes)


def quorum_active(c0, c1, learners, recent_active):
    """ProgressTracker.QuorumActive, raft/tracker/tracker.go:215-225."""
    votes = {}
    for vid in set(c0) | set(c1) | set(learners):
        if vid in learners:
            continue
        votes[vid] = vid in recent_active
    return joint_vote(c0, c1, votes) == VOTE_WON


def record_vote(votes, vid, v):
    """ProgressTracker.RecordVote, raft/tracker/tracker.go:258-263."""
    if vid not in votes:
        votes[vid] = v


def maybe_update(match, nxt, n):
    """Progress.MaybeUpdate, raft/tracker/progress.go:144-153 -> (ok, m, n)."""
    updated = False
    if match < n:
        match = n
        updated = True
    nxt = max(nxt, n + 1)
    return updated, match, nxt


def log_term_range(logs, sm_term):
    """Synthetic log model of DESIGN.md §5: entries (index, term) with
    non-decreasing terms; the current term's entries are [term_start,
    last_index].  Returns (term_start, last_index)."""
    last = max((i for i, _ in logs), default=0)
    starts = [i for i, t in logs if t == sm_term]
    return (min(starts) if starts else last + 1), last


def maybe_commit(mci, committed, term_start, last_index):
    """raft.maybeCommit -> raftLog.maybeCommit -> commitTo
    (raft/raft.go:585-588, raft/log.go:325-331, :233-241); term(i) is 0 for
    i > lastIndex (raft/log.go:265-271)."""
    if mci > committed and term_start <= mci <= last_index:
        return True, mci
    return False, committed
