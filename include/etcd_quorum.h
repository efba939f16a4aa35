/*
 * etcd_quorum.h — C ABI of the MI355X batched Raft quorum engine.
 *
 * This is the drop-in boundary for etcd's raft/quorum + raft/tracker hot path
 * (reference: /root/reference/raft, etcd 3.6.0-pre).  The per-group Go API
 * (MajorityConfig / JointConfig / ProgressTracker) stays the semantic
 * reference; every entry point below evaluates the same decision for G
 * independent Raft groups in one call on the GPU.  See INTEGRATION.md for the
 * cgo binding a maintainer adds next to raft/quorum.
 *
 * Data model ("slot SoA")
 *   A group's peers (voters of both halves, learners) are packed into S <= 16
 *   slots.  Slot order is arbitrary: every function here is an order-free set
 *   function of the (voter set, per-voter value) pairs, exactly like the Go
 *   code which iterates maps (raft/quorum/majority.go:155-161 fills then sorts).
 *
 *   match    uint64 [S][stride]   Progress.Match per slot; "absent" (no acked
 *                                 index, AckedIndexer.found == false) is 0,
 *                                 which CommittedIndex treats identically
 *                                 (raft/quorum/majority.go:150-161).
 *   masks    per-group slot bitmaps; element type is uint8_t when S <= 8 and
 *            uint16_t when 9 <= S <= 16 (qe_mask_bytes(S)).
 *            inc_mask  = JointConfig[0] (incoming voters)
 *            out_mask  = JointConfig[1] (outgoing voters; NULL = not joint)
 *            learner_mask = tracker.Config.Learners (optional)
 *            voted / granted = ProgressTracker.Votes: bit s of voted set iff
 *            slot s has a recorded vote, bit s of granted = that vote's value.
 *            A NULL inc_mask means "all S slots are voters" (fixed-size
 *            MajorityConfig, the BenchmarkMajorityConfig_CommittedIndex shape).
 *
 * Conventions
 *   - Index infinity (math.MaxUint64, raft/quorum/quorum.go:25-30) is
 *     QE_INDEX_INF.
 *   - VoteResult uses the reference's numeric encoding
 *     VotePending=1, VoteLost=2, VoteWon=3 (raft/quorum/quorum.go:48-58).
 *   - All pointers are DEVICE pointers (hipMalloc / torch CUDA tensors) unless
 *     the parameter says host.  The library allocates nothing and retains
 *     nothing; `stream` is a hipStream_t (NULL = default stream).  Calls are
 *     asynchronous on `stream` and reentrant on distinct buffers.
 *   - Return value: QE_OK or a negative QE_E* code.  num_groups == 0 is a
 *     successful no-op.  Semantic "panics" of the reference become counters
 *     in the optional stats buffer, never aborts.
 *   - Alignment: match/next/commit arrays 16-byte aligned and stride even
 *     take the vectorised path; anything else is still correct (scalar path).
 */
#ifndef ETCD_QUORUM_H
#define ETCD_QUORUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QE_ABI_VERSION 8  /* 8: see INTEGRATION.md "ABI 8" (changes listed there) */

#define QE_INDEX_INF UINT64_MAX
#define QE_MAX_SLOTS 16

/* quorum.VoteResult (raft/quorum/quorum.go:48-58) */
#define QE_VOTE_PENDING 1
#define QE_VOTE_LOST 2
#define QE_VOTE_WON 3

/* Raft StateType subset used by the election simulation (raft/raft.go:
 * StateFollower=0, StateCandidate=1, StateLeader=2, StatePreCandidate=3). */
#define QE_STATE_FOLLOWER 0
#define QE_STATE_CANDIDATE 1
#define QE_STATE_LEADER 2
#define QE_STATE_PRE_CANDIDATE 3

/* Status codes */
#define QE_OK 0
#define QE_EINVAL (-22)  /* null pointer / bad size / S out of range   */
#define QE_ERANGE (-34)  /* value out of supported range                */
#define QE_EHIP (-1000)  /* HIP launch / runtime error                  */
#define QE_ECOMM (-1001) /* RCCL error (qe_comm_*, qe_allreduce_stats)    */

/* Aggregate statistics.  A stats buffer is uint64[QE_STATS_WORDS]; kernels
 * add into QE_STATS_SHARDS shards of QE_STATS_COUNTERS counters (one 128-byte
 * line per shard) to avoid a single hot atomic line.  qe_stats_reduce() folds
 * the shards.  Counters accumulate across calls until the caller zeroes the
 * buffer, so one all-reduce at the end of a run aggregates a whole job. */
#define QE_STATS_COUNTERS 16
#define QE_STATS_SHARDS 64
#define QE_STATS_WORDS (QE_STATS_COUNTERS * QE_STATS_SHARDS)
enum qe_stat {
  QE_STAT_GROUPS = 0,        /* groups evaluated                              */
  QE_STAT_COMMIT_INF = 1,    /* CommittedIndex == inf (empty config)          */
  QE_STAT_COMMIT_SUM = 2,    /* sum of finite committed indexes (mod 2^64)    */
  QE_STAT_COMMIT_ZERO = 3,   /* CommittedIndex == 0 (nothing committed)       */
  QE_STAT_VOTE_WON = 4,
  QE_STAT_VOTE_LOST = 5,
  QE_STAT_VOTE_PENDING = 6,
  QE_STAT_GRANTED = 7,       /* sum of TallyVotes granted                      */
  QE_STAT_REJECTED = 8,      /* sum of TallyVotes rejected                     */
  QE_STAT_COMMIT_ADVANCED = 9,   /* replication: commit advanced this round    */
  QE_STAT_READ_RELEASED = 10,    /* ReadIndex requests released (a request count,
                                    * not groups; replication: quorum reached)  */
  QE_STAT_ELECTIONS = 11,        /* election sim: campaigns started            */
  QE_STAT_LEADERS = 12,          /* election sim: elections won                */
  QE_STAT_STEPDOWNS = 13,        /* election sim: elections lost               */
  QE_STAT_INVARIANT_VIOLATIONS = 14, /* learner∩voter≠∅, mci>lastIndex, ...  */
  QE_STAT_CHECKSUM = 15          /* mixed hash of all outputs (order-free)     */
};

/* A batch of G groups in slot-SoA form (see header comment). */
typedef struct qe_groups {
  uint64_t num_groups;       /* G                                            */
  uint64_t group_offset;     /* global id of group 0 (checksum key; shards)  */
  uint32_t num_slots;        /* S, 1..16                                     */
  uint32_t reserved;         /* must be 0                                    */
  uint64_t stride;           /* elements between slot rows of match (>= G)   */
  const uint64_t *match;     /* [S][stride] acked index per slot, 0 = absent */
  const void *inc_mask;      /* [G] JointConfig[0]; NULL = all S slots       */
  const void *out_mask;      /* [G] JointConfig[1]; NULL = non-joint         */
  const void *learner_mask;  /* [G] Learners; NULL = none                    */
  const void *voted;         /* [G] vote recorded bitmap; NULL = no votes    */
  const void *granted;       /* [G] vote value bitmap; NULL = all "no"       */
} qe_groups;

/* Outputs of the fused evaluation.  Any pointer may be NULL to skip it. */
typedef struct qe_outputs {
  uint64_t *commit;          /* [G] JointConfig.CommittedIndex               */
  uint8_t *vote;             /* [G] JointConfig.VoteResult (1/2/3)           */
  uint8_t *granted_count;    /* [G] TallyVotes granted                       */
  uint8_t *rejected_count;   /* [G] TallyVotes rejected                      */
  uint64_t *stats;           /* uint64[QE_STATS_WORDS] accumulated, or NULL  */
} qe_outputs;

/* ---- introspection ---------------------------------------------------- */
int qe_abi_version(void);
const char *qe_strerror(int status);
size_t qe_mask_bytes(uint32_t num_slots); /* 1 for S<=8, 2 for S<=16, 0 bad */

/* Optional launch tuning (no reference counterpart; never changes results):
 *   "blocks_per_cu"  cap on persistent-grid workgroups per CU, 0..32
 *                    (default 0 = the kernel's occupancy)
 *   "tiles_per_wave" -1 = per-kernel default (measured best), 0 =
 *                    persistent grid, T > 0: each wave walks T tiles
 *   "nontemporal"    bit 0: non-temporal loads, bit 1: non-temporal stores
 *                    of qe_commit_vote                                     */
int qe_tune(const char *key, int value);

/* ---- quorum decisions -------------------------------------------------- */

/* Fused ProgressTracker.Committed + TallyVotes for every group:
 *   commit[g] = Voters.CommittedIndex(match)           tracker.go:177-179,
 *               joint.go:49-56, majority.go:126-172
 *   vote[g]   = Voters.VoteResult(votes)               tracker.go:286,
 *               joint.go:61-75, majority.go:178-210
 *   granted/rejected_count[g] = TallyVotes counts over non-learner voters
 *               tracker.go:267-285
 * Replaces one AckedIndexer-driven CommittedIndex call plus one
 * VoteResult(map) call per group (raft/quorum/majority.go:126, :178). */
int qe_commit_vote(const qe_groups *groups, const qe_outputs *out,
                   void *stream);

/* JointConfig.CommittedIndex only (MajorityConfig when out_mask == NULL).
 * raft/quorum/joint.go:49-56, raft/quorum/majority.go:126-172. */
int qe_committed_index(const qe_groups *groups, uint64_t *commit,
                       void *stream);

/* JointConfig.VoteResult only; `voted`/`granted` give the votes map.
 * raft/quorum/joint.go:61-75, raft/quorum/majority.go:178-210. */
int qe_vote_result(const qe_groups *groups, uint8_t *vote, void *stream);

/* ProgressTracker.QuorumActive (raft/tracker/tracker.go:215-225): every
 * non-learner voter votes Progress.RecentActive; active[g] = 1 iff the
 * result is VoteWon.  `recent_active` is a [G] slot bitmap (mask type). */
int qe_quorum_active(const qe_groups *groups, const void *recent_active,
                     uint8_t *active, void *stream);

/* ProgressTracker.RecordVote (raft/tracker/tracker.go:258-263) for a batch of
 * vote responses: for each group, slots in `resp_mask` cast vote
 * `resp_value`; the first recorded vote per slot sticks.  Updates
 * voted/granted in place (mask-typed [G] arrays). */
int qe_record_votes(uint64_t num_groups, uint32_t num_slots, void *voted,
                    void *granted, const void *resp_mask,
                    const void *resp_value, void *stream);

/* ---- lockstep replication round (BASELINE config 4) -------------------- */

/* Device-resident leader-side state of G groups. */
typedef struct qe_repl_state {
  uint64_t num_groups;
  uint64_t group_offset;     /* global id of group 0 (checksum key)          */
  uint32_t num_slots;
  uint32_t reserved;
  uint64_t stride;           /* slot-row stride of match/next               */
  uint64_t *match;           /* [S][stride] Progress.Match (rw)             */
  uint64_t *next;            /* [S][stride] Progress.Next  (rw)             */
  uint64_t *committed;       /* [G] raftLog.committed (rw)                  */
  const uint64_t *term_start;/* [G] first index of the leader's term         */
  const uint64_t *last_index;/* [G] raftLog.lastIndex()                      */
  const void *inc_mask;      /* [G] as in qe_groups                          */
  const void *out_mask;      /* [G] or NULL                                  */
} qe_repl_state;

/* One round of MsgAppResp / MsgHeartbeatResp handling per group. */
typedef struct qe_repl_msgs {
  const uint64_t *resp_index;/* [S][stride] MsgAppResp.Index per slot        */
  const void *resp_mask;     /* [G] slots whose (non-reject) MsgAppResp came */
  const void *read_acks;     /* [G] ReadIndex heartbeat acks (incl. self), or NULL */
  uint8_t *read_ok;          /* [G] out: VoteResult(acks)==VoteWon, or NULL */
  uint8_t *commit_advanced;  /* [G] out: maybeCommit() returned true, or NULL */
} qe_repl_msgs;

/* For each group: Progress.MaybeUpdate(resp) on every responding slot
 * (raft/tracker/progress.go:144-153), then raft.maybeCommit
 * (raft/raft.go:585-588 -> raft/log.go:325-331 -> commitTo log.go:233-241)
 * with the synthetic log model term(i)==Term <=> term_start<=i<=last_index,
 * then the ReadIndex quorum check VoteResult(acks)==VoteWon
 * (raft/raft.go:1300, raft/read_only.go:68-76). */
int qe_replication_round(const qe_repl_state *st, const qe_repl_msgs *msgs,
                         uint64_t *stats, void *stream);

/* ---- randomized election simulation (BASELINE config 5) ---------------- */

typedef struct qe_election_state {
  uint64_t num_groups;
  uint64_t group_offset;     /* global id of group 0 (RNG key; sharding)     */
  uint32_t num_slots;
  uint32_t reserved;
  uint64_t *term;            /* [G] rw                                       */
  uint8_t *state;            /* [G] rw QE_STATE_*                            */
  void *voted;               /* [G] rw mask-typed                            */
  void *granted;             /* [G] rw mask-typed                            */
  const uint8_t *self_slot;  /* [G] candidate's own slot                     */
  const void *inc_mask;      /* [G]                                          */
  const void *out_mask;      /* [G] or NULL                                  */
  const void *learner_mask;  /* [G] or NULL (learners vote; never counted)   */
} qe_election_state;

typedef struct qe_election_params {
  uint64_t seed;
  uint64_t step0;            /* global step number of the first step         */
  uint32_t steps;            /* fused steps per launch (state in registers)  */
  uint32_t p_drop_q16;       /* P(response dropped) * 65536                  */
  uint32_t p_grant_q16;      /* P(vote granted | delivered) * 65536          */
  uint32_t flags;            /* QE_ELEC_* (ABI 1: reserved, 0)                */
  uint32_t p_active_q16;     /* CheckQuorum: P(a leader heard from a peer
                                within an election timeout) * 65536        */
  uint32_t reserved;
  /* Scripted mode (replaying a recorded or test message flow): when
   * script_resp is non-NULL, step k of group g takes its responses from
   * [k*script_stride + g] of these arrays instead of the RNG. */
  const void *script_resp;   /* mask-typed: peers whose (pre)vote response
                                arrives / that were active (CheckQuorum)   */
  const void *script_grant;  /* mask-typed: the responses that grant        */
  const uint8_t *script_hup; /* 1: the election timeout fires this step
                                (a (pre)candidate campaigns again); NULL
                                = never                                     */
  uint64_t script_stride;    /* >= num_groups                                */
} qe_election_params;

#define QE_ELEC_PREVOTE 1u       /* raft.Config.PreVote                      */
#define QE_ELEC_CHECK_QUORUM 2u  /* raft.Config.CheckQuorum                  */

/* `steps` election steps per group:
 *   Leader: CheckQuorum on -> one CheckQuorum round (raft/raft.go:997-1018):
 *     the leader sees itself active, each other voter active with
 *     p_active; !QuorumActive (tracker.go:215-225) -> becomeFollower (term
 *     kept).  CheckQuorum off -> the leader is deposed and campaigns.
 *   Follower (or a (pre)candidate whose timeout fires, script_hup): hup ->
 *     campaign (raft.go:785-803): PreVote on -> becomePreCandidate (term
 *     kept), else becomeCandidate (term+1); self-vote; a won tally moves on
 *     (pre-vote -> election -> leader).
 *   PreCandidate / Candidate: one round of responses from every other voter
 *     (drops/grants from a counter-based RNG) -> RecordVote -> TallyVotes
 *     (raft.go:837-845, :1399-1414): won -> campaign(campaignElection) /
 *     becomeLeader; lost -> becomeFollower (term kept); pending -> stay.
 * Invariant checks go to stats. */
int qe_election_steps(const qe_election_state *st,
                      const qe_election_params *p, uint64_t *stats,
                      void *stream);

/* ---- Progress state machine ------------------ */

/* tracker.StateType (raft/tracker/state.go) and the packed per-peer word
 * (ABI 3: one u32 per peer replaces the flags / Inflights.start /
 * Inflights.count byte rows of ABI 2, so a peer's small fields move in one
 * 4-byte access; ABI 4 adds the ring representation bits):
 *   bits 0-1   StateType (QE_PR_*)          bit 2  Progress.ProbeSent
 *   bit 3      Progress.RecentActive        bit 4  QE_PF_RING_WIDE
 *   bits 5-7   ring epoch bits 0-2          bits 8-15  Inflights.start
 *   bits 16-23 Inflights.count              bits 24-31 ring epoch bits 3-10
 * Inflights entries are stored as 32-bit words (infl_lo); the upper 32 bits
 * of an entry are the peer's 11-bit ring epoch H (QE_PW_EPOCH) unless
 * QE_PF_RING_WIDE is set, in which case they are infl_hi's word:
 *   entry k = ((wide ? infl_hi[k] : H) << 32) | infl_lo[k].
 * The form is canonical when count == 0 -> H = 0, not wide; else not wide
 * iff every live entry's upper word is the same value < 2^11 (entries below
 * 2^43 within one 2^32-aligned window: every realistic in-flight window),
 * which is then H.  qe_ring_pack produces it and the kernels restore it
 * whenever they append (a ring they only free entries from may stay wide).
 * qe_ring_pack / qe_ring_unpack convert plain uint64 rings.  Ring
 * representation bits are not Progress state: QE_PW_RING_MASK selects them.
 *
 * ABI 8, the 16-bit form (qe_progress.infl16 non-NULL; F <= QE_RING16_MAX_F):
 * the rings live in infl16 [S][stride][8] as offsets below Next,
 *   entry k = Progress.Next - 1 - infl16[k]        (not wide)
 *   entry k = (infl_hi[k] << 32) | infl_lo[k]       (QE_PF_RING_WIDE)
 * -- 16 bytes per peer, two peers per 32-byte HBM sector.  Live Inflights
 * entries are the last indices of MsgApps sent, all below Next; Next moves
 * only when an append rewrites the ring (OptimisticUpdate), or when the ring
 * empties (MaybeUpdate past every sent index, ResetState).  A peer is wide
 * iff some live entry lies outside [Next - 65536, Next - 1] (a window of
 * more than 65536 indices, or an inconsistent input); the epoch bits are 0.
 * The kernels re-encode a peer's ring whenever they append to it or change
 * its Next while entries are live.  Entry points that write Next without
 * knowing the rings (qe_apply_append_resps, a host) must not be used on the
 * Next rows of such a state while entries are live: they would re-base the
 * entries.  qe_ring_pack16 / qe_ring_unpack16 convert plain uint64 rings. */
#define QE_PR_PROBE 0
#define QE_PR_REPLICATE 1
#define QE_PR_SNAPSHOT 2
#define QE_PF_STATE 3u          /* word & QE_PF_STATE = StateType            */
#define QE_PF_PROBE_SENT 4u     /* Progress.ProbeSent                        */
#define QE_PF_RECENT_ACTIVE 8u  /* Progress.RecentActive                     */
#define QE_PF_RING_WIDE 16u     /* ABI 4: entries' upper words in infl_hi     */
#define QE_PW_START_SHIFT 8     /* Inflights.start = (word >> 8) & 0xFF       */
#define QE_PW_COUNT_SHIFT 16    /* Inflights.count = (word >> 16) & 0xFF      */
#define QE_PW_RING_MASK 0xFF0000F0u /* ABI 4: WIDE + epoch bits               */
#define QE_RING_EPOCH_MAX 0x7FFu    /* largest epoch held in the word         */
#define QE_PW_EPOCH(w) ((((w) >> 5) & 7u) | (((w) >> 21) & 0x7F8u))
#define QE_PW_EPOCH_BITS(h) ((((uint32_t)(h) & 7u) << 5) | (((uint32_t)(h) & 0x7F8u) << 21))
#define QE_PW_PACK(state, probe_sent, recent_active, start, count)                 \
  ((uint32_t)(state) | ((probe_sent) ? QE_PF_PROBE_SENT : 0u) |                   \
   ((recent_active) ? QE_PF_RECENT_ACTIVE : 0u) |                                 \
   ((uint32_t)(start) << QE_PW_START_SHIFT) | ((uint32_t)(count) << QE_PW_COUNT_SHIFT))
/* ABI 4: words per peer ring in infl_lo / infl_hi (F rounded up to 4, so a
 * ring of F <= 8 is one or two 16-byte accesses, one 32-byte HBM sector) */
#define QE_RING_PITCH(F) (((uint32_t)(F) + 3u) & ~3u)
#define QE_MAX_INFLIGHT 255     /* Inflights capacity (MaxInflightMsgs)      */
#define QE_RING16_MAX_F 8       /* ABI 8: the 16-bit form holds up to 8 entries */
#define QE_RING16_MAX_SLOTS 9   /* ABI 8: ... for up to 9 slots (the pipelined
                                   Progress kernels' shapes) and log_runs <= 4 */
#define QE_MAX_LOG_RUNS 16      /* term runs of the leader-log model          */

/* message kinds of qe_peer_msgs.type (any other value: no message) */
#define QE_MSG_NONE 0
#define QE_MSG_APP_RESP 1             /* MsgAppResp, Reject=false            */
#define QE_MSG_APP_RESP_REJECT 2      /* MsgAppResp, Reject=true             */
#define QE_MSG_HEARTBEAT_RESP 3       /* MsgHeartbeatResp                    */
#define QE_MSG_SNAP_STATUS 4          /* MsgSnapStatus, Reject=false         */
#define QE_MSG_SNAP_STATUS_REJECT 5   /* MsgSnapStatus, Reject=true          */
#define QE_MSG_UNREACHABLE 6          /* MsgUnreachable                      */
#define QE_MSG_TRANSFER_LEADER 7      /* ABI 5: MsgTransferLeader, m.From = the
                                         slot (raft.go:1339-1370)            */

/* ABI 5: ReadIndex requests a leader keeps pending under ReadOnlySafe
 * (readOnly.pendingReadIndex + readIndexQueue, raft/read_only.go:39-63).
 * Each request has a context number (the engine's stand-in for the
 * request's context bytes, unique within the group): queue entry j has
 * context read_head + j; numbers are 32-bit, assigned consecutively by
 * qe_read_index, never 0 (0 = no context).  The first QE_READ_QUEUE entries
 * live in one word per group (read_acks, the fast form every kernel reads
 * with the group); ABI 7: a queue of up to read_cap entries keeps entries
 * QE_READ_QUEUE.. in the overflow ring read_ovf, each at its context number
 * mod read_cap (an entry never moves while it waits there). */
#define QE_READ_QUEUE 4
#define QE_READ_CAP_MAX 255     /* read_count is a byte                      */

/* Leader-side Progress of every peer of G groups (raft/tracker/progress.go:
 * 30-80) plus the leader's log model: term runs r < run_count[g] covering
 * [run_first[r], run_first[r+1]) with run_term[r] (run 0 starts at the
 * snapshot/dummy index = first_index - 1), ending at last_index; the current
 * term's entries are [term_start, last_index].  Entries exist in
 * [first_index, last_index]; max_ents models MaxSizePerMsg for equal-size
 * entries (entries per MsgApp, at least one; 0 = noLimit).  Inflights.start
 * must be < inflight_cap (results are unspecified otherwise; memory stays in
 * bounds). */
typedef struct qe_progress {
  uint64_t num_groups;
  uint64_t group_offset;
  uint32_t num_slots;
  uint32_t inflight_cap;        /* F = MaxInflightMsgs, 1..QE_MAX_INFLIGHT  */
  uint64_t stride;
  uint64_t *match, *next;       /* [S][stride]                               */
  uint64_t *pending_snapshot;   /* [S][stride]; 0 for a peer not in
                                 * StateSnapshot (every reachable Progress:
                                 * ResetState clears it on each state change,
                                 * tracker/progress.go:84-89) -- the kernels
                                 * write it only where its value changes      */
  uint32_t *peer;               /* [S][stride] packed per-peer word (ABI 3):
                                   StateType, ProbeSent, RecentActive,
                                   Inflights.start / count (QE_PW_*)         */
  uint32_t *infl_lo;            /* ABI 4: [S][stride][QE_RING_PITCH(F)]
                                   Inflights.buffer, low 32 bits, lane-major:
                                   entry k of slot s of group g at
                                   (s*stride + g)*QE_RING_PITCH(F) + k       */
  uint32_t *infl_hi;            /* ABI 4: same shape, high 32 bits; read and
                                   written only for QE_PF_RING_WIDE peers    */
  uint64_t *committed;          /* [G] raftLog.committed (rw)                */
  const uint64_t *term_start;   /* [G]                                       */
  const uint64_t *first_index;  /* [G] raftLog.firstIndex()                  */
  const uint64_t *last_index;   /* [G] raftLog.lastIndex()                   */
  uint32_t log_runs;            /* R <= QE_MAX_LOG_RUNS                      */
  uint32_t reserved;
  const uint64_t *run_first;    /* [R][stride]                               */
  const uint64_t *run_term;     /* [R][stride]                               */
  const uint8_t *run_count;     /* [G] valid runs, 1..R                       */
  const void *inc_mask;         /* [G] as in qe_groups (NULL = all slots)    */
  const void *out_mask;         /* [G] or NULL                               */
  /* ABI 2 */
  const void *tracked;          /* [G] slots holding a Progress (ProgressMap
                                   keys); NULL = every slot                  */
  const uint8_t *self_slot;     /* [G] the leader's own slot (bcastAppend
                                   skips it); NULL or >= S = none            */
  uint8_t *lead_transferee;     /* [G] rw (ABI 5): slot of r.leadTransferee;
                                   >= S = no transfer in progress (None).
                                   MsgTransferLeader rewrites it; NULL = no
                                   transfer in progress and the round's
                                   changes are not stored                    */
  const uint64_t *snap_index;   /* [G] index of the snapshot a MsgSnap
                                   carries; NULL = first_index - 1           */
  uint32_t max_ents;            /* entries per MsgApp (0 = noLimit)          */
  uint32_t reserved2;
  /* ABI 5: the ReadIndex queue (r.readOnly, ReadOnlySafe); NULL read_acks =
   * no requests tracked (heartbeat contexts are ignored). */
  void *read_acks;              /* [G][QE_READ_QUEUE] rw mask-typed: acks of
                                   queue entry j (0 = oldest) of group g at
                                   read_acks[g*QE_READ_QUEUE + j] (one 4- or
                                   8-byte word per group)                    */
  uint32_t *read_head;          /* [G] rw: context number of queue entry 0   */
  uint8_t *read_count;          /* [G] rw: pending requests, 0..read_cap     */
  /* ABI 7: a queue longer than the word (readIndexQueue is unbounded in the
   * reference, read_only.go:56-63) and the duplicate-request check */
  uint32_t read_cap;            /* entries a queue holds: 0 (= QE_READ_QUEUE,
                                   ABI 5) or QE_READ_QUEUE..QE_READ_CAP_MAX  */
  uint32_t reserved3;           /* must be 0                                 */
  void *read_ovf;               /* [G][read_cap] rw mask-typed: the acks of
                                   the entry with context c at queue position
                                   >= QE_READ_QUEUE, at read_ovf[g*read_cap +
                                   c % read_cap]; needed when read_cap >
                                   QE_READ_QUEUE                             */
  uint64_t *read_keys;          /* [G][read_cap] rw: the caller's key (e.g. a
                                   hash of the request context bytes) of the
                                   entry with context c, at read_keys[g*
                                   read_cap + c % read_cap]; NULL = keys not
                                   tracked.  Given, it must have been given to
                                   every qe_read_index that queued the pending
                                   entries                                   */
  /* ABI 8 */
  uint16_t *infl16;             /* [S][stride][8] rw or NULL: the 16-bit
                                   Inflights form (see QE_RING16_MAX_F above;
                                   infl_lo / infl_hi then hold the wide peers
                                   only).  Requires inflight_cap <=
                                   QE_RING16_MAX_F, num_slots <=
                                   QE_RING16_MAX_SLOTS, log_runs <= 4        */
} qe_progress;

/* One round of peer responses: message of slot s for group g at
 * [s*stride + g].  Outputs may be NULL. */
typedef struct qe_peer_msgs {
  const uint8_t *type;          /* QE_MSG_*                                  */
  const uint64_t *index;        /* m.Index                                   */
  const uint64_t *reject_hint;  /* m.RejectHint                              */
  const uint64_t *log_term;     /* m.LogTerm                                 */
  void *sent;                   /* [G] out: slots sent >= 1 MsgApp/MsgSnap   */
  uint8_t *bcast;               /* [G] out: bcastAppend calls (commit advances) */
  void *snap;                   /* [G] out: slots sent a MsgSnap             */
  void *timeout_now;            /* [G] out: slots sent MsgTimeoutNow         */
  uint8_t *msg_count;           /* [S][stride] out: MsgApp/MsgSnap sent to the
                                   peer this round (saturates at 255)        */
  uint64_t *msg_index;          /* [S][stride] out: m.Index of the first of
                                   them (MsgSnap: the snapshot index);
                                   written only where msg_count > 0          */
  uint64_t *bytes_requested;    /* measurement aid, normally NULL: when set,
                                   an instrumented kernel adds the bytes the
                                   round reads and writes (field granularity,
                                   the rules of DESIGN.md §3) to
                                   *bytes_requested                          */
  /* ABI 5: ReadIndex under ReadOnlySafe against the queue of p
   * (raft.go:1296-1309, read_only.go:68-112) */
  const uint32_t *read_ctx;     /* [S][stride]: context number a
                                   MsgHeartbeatResp carries (0 = none,
                                   len(m.Context) == 0); NULL = every one
                                   carries the newest context pending when
                                   the round starts (bcastHeartbeat attaches
                                   lastPendingRequestCtx, raft.go:525-532)   */
  uint8_t *read_released;       /* [G] out (may be NULL): requests released
                                   this round, oldest first (readOnly.advance
                                   dequeues through the acked request)      */
  uint8_t *term_commit;         /* [G] out (may be NULL): 1 when this round's
                                   maybeCommit made committedEntryInCurrentTerm
                                   true, i.e. the leader's postponed
                                   MsgReadIndex requests are released now
                                   (raft.go:1259-1262, :1731-1733, :1813-1825) */
  uint64_t *term_commit_index;  /* [G] out (may be NULL): raftLog.committed
                                   right after that maybeCommit -- the index
                                   the released requests are added at
                                   (sendMsgReadIndexResponse, raft.go:1834);
                                   written only where term_commit is 1       */
} qe_peer_msgs;

/* Leader-side handling of one message per peer, slots in ascending order
 * (stepLeader, raft/raft.go:1099-1338), with every send the reference makes
 * while handling the message executed in place (max_ents from p):
 *   MsgAppResp reject: RecentActive; findConflictByTerm (raft/log.go:147-168)
 *     when LogTerm > 0; MaybeDecrTo (progress.go:170-193) -> Replicate ->
 *     BecomeProbe, sendAppend.
 *   MsgAppResp accept: RecentActive; IsPaused; MaybeUpdate -> Probe ->
 *     BecomeReplicate / Snapshot caught up -> BecomeProbe + BecomeReplicate /
 *     Replicate -> Inflights.FreeLE; maybeCommit -> bcastAppend (every tracked
 *     slot but self_slot) or sendAppend if it was paused; then
 *     `for maybeSendAppend(from, false) {}`; MsgTimeoutNow to the lead
 *     transferee once its Match == lastIndex (raft.go:1275-1281).
 *   MsgHeartbeatResp: RecentActive, ProbeSent = false, FreeFirstOne when the
 *     inflights are full, sendAppend if Match < lastIndex; with p->read_acks,
 *     a response carrying a context (ABI 5): recvAck on the queue entry with
 *     that context number (none pending: nothing is recorded), and once
 *     Voters.VoteResult(that entry's acks) == VoteWon, readOnly.advance
 *     releases every entry up to and including it (read_only.go:68-112).
 *   MsgSnapStatus (StateSnapshot only): reject -> PendingSnapshot = 0;
 *     BecomeProbe; ProbeSent = true (raft.go:1310-1331).
 *   MsgUnreachable: Replicate -> BecomeProbe (raft.go:1332-1338).
 *   MsgTransferLeader (ABI 5, raft.go:1339-1370): a learner's is ignored; a
 *     transfer to the slot already in progress is ignored; another transfer
 *     in progress is aborted; a transfer to self_slot is then ignored;
 *     otherwise lead_transferee = the slot, and MsgTimeoutNow goes out at
 *     once when its Match == lastIndex, else sendAppend to it.  (The
 *     reference also resets electionElapsed: tick state stays with the host,
 *     which sees the new lead_transferee.)
 * A send is raft.maybeSendAppend (raft.go:432-492) on the log model; see
 * qe_progress_send.  Messages from untracked slots are dropped.  An accept
 * with index > lastIndex is processed as the reference does and counted as
 * an invariant violation. */
int qe_progress_step(const qe_progress *p, const qe_peer_msgs *m, uint64_t *stats,
                     void *stream);

/* ABI 5: MsgReadIndex on every group's leader whose request[g] is 1
 * (stepLeader, raft/raft.go:1078-1096, sendMsgReadIndexResponse :1827-1843),
 * result[g] (QE_RI_*):
 *   IsSingleton (one voter in Voters[0], Voters[1] empty; tracker.go:158-160)
 *     -> QE_RI_RESPOND at index = committed;
 *   no entry of the leader's term committed yet (committedEntryInCurrentTerm,
 *     :1731-1733: term_start <= committed <= last_index on the log model)
 *     -> QE_RI_POSTPONED (pendingReadIndexMessages; the host keeps the
 *     message and adds it again once qe_progress_step reports term_commit --
 *     its read index is that round's term_commit_index, NOT the index the
 *     re-added qe_read_index call returns: releasePendingReadIndexMessages
 *     runs inside the commit, before later advances of the same round);
 *   lease_based (ReadOnlyLeaseBased) -> QE_RI_RESPOND at committed;
 *   ReadOnlySafe -> readOnly.addRequest(committed) + the leader's own ack
 *     (self_slot; recvAck(r.id)): QE_RI_QUEUED with context number ctx[g]
 *     and index = committed; the host sends the heartbeats carrying ctx and
 *     answers when qe_progress_step releases the entry.  ABI 7: with keys
 *     (key and p->read_keys non-NULL) a request whose key[g] equals a
 *     pending request's is ignored, as addRequest ignores a context already
 *     pending (read_only.go:57-60; etcd's server resends the same request
 *     id, server/etcdserver/v3_server.go:808-824) -> QE_RI_DUPLICATE with
 *     that request's context.  With read_cap (QE_READ_QUEUE when 0)
 *     requests already pending (or the context numbers exhausted: read_head
 *     + read_count would be 0 mod 2^32) -> QE_RI_FULL, nothing changes (a
 *     capacity the host chose; up to QE_READ_CAP_MAX).
 * Needs p->read_acks / read_head / read_count unless every result is
 * RESPOND or POSTPONED (lease_based).  ctx and index may be NULL; they are
 * written only where they apply.  Groups without a request: result 0. */
#define QE_RI_NONE 0
#define QE_RI_RESPOND 1
#define QE_RI_POSTPONED 2
#define QE_RI_QUEUED 3
#define QE_RI_FULL 4
#define QE_RI_DUPLICATE 5  /* ABI 7: key[g] is pending already: addRequest
                              ignores it (read_only.go:57-60); ctx[g] = the
                              pending request's context (the heartbeats the
                              reference sends then carry it), index not set */
int qe_read_index(const qe_progress *p, const uint8_t *request, const uint64_t *key,
                  uint32_t lease_based, uint8_t *result, uint32_t *ctx, uint64_t *index,
                  void *stream);

/* MsgCheckQuorum on every group's leader (stepLeader, raft/raft.go:997-1018):
 * the leader's own Progress (self_slot, when tracked) becomes RecentActive;
 * quorum_active[g] = ProgressTracker.QuorumActive() (raft/tracker/
 * tracker.go:215-225: Voters.VoteResult with each voter's vote = its
 * RecentActive, a voter without a Progress missing) -- 0 means the leader
 * steps down (becomeFollower); then RecentActive = false for every tracked
 * slot but the leader's (prs.Visit, raft.go:1013-1017).  Reads inc_mask /
 * out_mask / tracked / self_slot and the peer words of p.  A slot row in
 * which some group's word changes is rewritten for every tracked slot of
 * the tile, unchanged words included (whole sectors; the values written are
 * the round's result either way), so concurrent writers of other words of
 * p->peer must not overlap the call.  self_slot NULL (or >= S) means the
 * leader has no Progress of its own (the reference then marks nobody
 * active, raft.go:1000-1002): a caller whose leader has a slot must pass
 * it, or the leader is not counted as active.  quorum_active may be NULL.
 * stats: groups, stepdowns (QE_STAT_STEPDOWNS), checksum. */
int qe_check_quorum(const qe_progress *p, uint8_t *quorum_active, uint64_t *stats,
                    void *stream);

/* ABI 6: MsgBeat on every group's leader (stepLeader, raft/raft.go:991-993):
 * bcastHeartbeat (:524-541) -- one MsgHeartbeat to every tracked slot but
 * self_slot, each carrying Commit = min(Progress.Match, raftLog.committed)
 * (sendHeartbeat :494-510: a follower is never told a commit beyond what it
 * matched) and the context of the newest pending ReadIndex request
 * (lastPendingRequestCtx, read_only.go:114-121).  commit[s*stride + g]
 * (DEVICE, [S][stride]) is written for every slot sent to; ctx[g] (may be
 * NULL) = that context number, 0 when nothing is pending or p->read_acks is
 * NULL; sent[g] (mask-typed, may be NULL) = the slots sent to.  Reads
 * match, committed, tracked, self_slot and the ReadIndex queue's head and
 * count; writes nothing of p. */
int qe_heartbeat(const qe_progress *p, uint64_t *commit, uint32_t *ctx, void *sent, void *stream);

/* raft.sendAppend / maybeSendAppend(to, send_if_empty) once for the slots of
 * want[g] (raft.go:432-492; bcastAppend after a proposal is want = every
 * tracked slot but the leader's, send_if_empty = 1): paused peers get
 * nothing; with no entries to send (Next > lastIndex, or Next < firstIndex
 * where entries() fails with ErrCompacted) nothing is sent unless
 * send_if_empty -- this check comes before the snapshot branch; Next >
 * lastIndex sends an empty MsgApp; Next < firstIndex sends a MsgSnap to a
 * recently active peer (BecomeSnapshot(snap_index)); otherwise up to
 * p->max_ents entries (0 = noLimit; ABI 3 takes MaxSizePerMsg from p, as
 * qe_progress_step does): Replicate -> OptimisticUpdate + Inflights.Add,
 * Probe -> ProbeSent.  sent / snap (mask-typed [G], may be NULL) report the
 * outcome. */
int qe_progress_send(const qe_progress *p, const void *want, uint32_t send_if_empty,
                     void *sent, void *snap, void *stream);

/* ---- MsgProp: appendEntry + bcastAppend (ABI 6) ------------------------- */

/* qe_proposals.result */
#define QE_PROP_NONE 0                /* no proposal for the group             */
#define QE_PROP_OK 1                  /* appended and bcastAppend done          */
#define QE_PROP_DROPPED_NOT_MEMBER 2  /* ErrProposalDropped: the leader has no
                                         Progress of its own (raft.go:1023-1028) */
#define QE_PROP_DROPPED_TRANSFER 3    /* ErrProposalDropped: leadership transfer
                                         in progress (raft.go:1029-1032)       */
#define QE_PROP_DROPPED_SIZE 4        /* ErrProposalDropped: the uncommitted
                                         size limit (raft.go:627-633, 1761-1779) */
#define QE_PROP_BAD_CC 5              /* ABI 7: cc_count[g] > max_cc -- refused
                                         whole, nothing changes (an input error
                                         reported per group, never clamped)    */
#define QE_PROP_MAX_CC 8              /* conf-change entries per proposal      */
/* qe_proposals.flags: appendEntry alone, as the reference calls it outside
 * MsgProp (the auto-leave entry of advance, raft.go:555-569; tests'
 * mustAppendEntry): no MsgProp gates except the leader's own Progress, no
 * conf-change checks (max_cc ignored), no bcastAppend */
#define QE_PROP_APPEND_ONLY 1u

/* One MsgProp per group (a launch is one batch of proposals). */
typedef struct qe_proposals {
  const uint32_t *num_entries;   /* [G] len(m.Entries); 0 = no MsgProp         */
  const uint64_t *payload;       /* [G] sum of PayloadSize (len(Data), util.go)
                                    over the entries that are NOT conf
                                    changes; NULL = all of them empty       */
  uint32_t max_cc;               /* conf-change entries per proposal at most,
                                    <= QE_PROP_MAX_CC (0: no conf changes)  */
  uint32_t flags;                /* QE_PROP_APPEND_ONLY or 0                  */
  uint64_t cc_stride;            /* >= num_groups                            */
  const uint8_t *cc_count;       /* [G] conf-change entries of the proposal
                                    (> max_cc: QE_PROP_BAD_CC)              */
  const uint32_t *cc_pos;        /* [max_cc][cc_stride] position in m.Entries,
                                    ascending, < num_entries                */
  const uint8_t *cc_leave;       /* [max_cc][cc_stride] 1: a ConfChangeV2
                                    without Changes (wantsLeaveJoint)        */
  const uint32_t *cc_size;       /* [max_cc][cc_stride] its PayloadSize      */
  const uint64_t *applied;       /* [G] raftLog.applied (read when a group has
                                    conf-change entries)                    */
  uint64_t *pending_conf_index;  /* [G] rw r.pendingConfIndex (ditto)        */
  uint64_t *uncommitted_size;    /* [G] rw r.uncommittedSize; NULL = not
                                    tracked (max_uncommitted must be 0)     */
  uint64_t max_uncommitted;      /* Config.MaxUncommittedEntriesSize; 0 =
                                    noLimit (raft.go:356-358)               */
  uint8_t *result;               /* [G] out QE_PROP_*                         */
  uint8_t *cc_refused;           /* [G] out (may be NULL): bit k = conf-change
                                    entry k was refused and replaced by an
                                    empty EntryNormal (raft.go:1063-1065)   */
  void *sent;                    /* [G] out mask (may be NULL): peers sent a
                                    MsgApp / MsgSnap by the bcastAppend     */
  void *snap;                    /* [G] out mask (may be NULL): a MsgSnap     */
  uint64_t *bytes_requested;     /* measurement aid, normally NULL: adds the
                                    algorithmic bytes (DESIGN.md §3 rules)  */
} qe_proposals;

/* stepLeader's MsgProp arm (raft/raft.go:1019-1076) for every group with
 * num_entries > 0, on the leader-side state p (p->self_slot is required:
 * MsgProp needs the leader's own id, QE_EINVAL without it):
 *   the leader has no Progress of its own (self_slot untracked) -> dropped;
 *   a leadership transfer is in progress (lead_transferee < S) -> dropped;
 *   each conf-change entry in order: refused (replaced by an empty
 *     EntryNormal) when pendingConfIndex > applied, or it enters a change
 *     while Voters[1] is non-empty, or it leaves a joint state that does not
 *     exist; otherwise pendingConfIndex = its index (set even when the
 *     proposal is then dropped for its size, as the reference does);
 *   appendEntry (:621-642): increaseUncommittedSize -> dropped when the
 *     uncommitted tail is non-empty, the proposal's payload is non-zero and
 *     the sum would exceed max_uncommitted; else lastIndex += num_entries
 *     (the entries take the leader's term: the log model's current run,
 *     [term_start, last_index], grows), Progress[self].MaybeUpdate(lastIndex)
 *     and maybeCommit (the term gate of qe_progress_step);
 *   bcastAppend (:515-522): sendAppend (maybeSendAppend(to, true)) to every
 *     tracked slot but self_slot, as qe_progress_send.
 * Writes p->last_index (declared const in qe_progress because the other
 * entry points only read it), p->committed, the leader's Match/Next/word and
 * the peers' Next/word/PendingSnapshot/Inflights.  The reference's
 * reduceUncommittedSize on apply (:544) stays with the host, which owns the
 * applied entries.  stats: groups, commit sum, commit advanced, checksum. */
int qe_propose(const qe_progress *p, const qe_proposals *prop, uint64_t *stats, void *stream);

/* ---- becomeLeader (ABI 7) ----------------------------------------------- */

/* qe_leader.result */
#define QE_BL_NONE 0        /* elected[g] == 0: not part of this call           */
#define QE_BL_LEADER 1      /* becomeLeader done                                */
#define QE_BL_NOT_MEMBER 2  /* self_slot holds no Progress: the reference would
                               panic (a candidate is promotable, so a voter);
                               nothing changes                               */
#define QE_BL_RUNS_FULL 3   /* the new term's run does not fit the log model's
                               log_runs: nothing changes (the host compacts
                               the run table and retries)                    */
#define QE_BL_BCAST 1u      /* qe_leader.flags: then bcastAppend, as
                               stepCandidate does after winning (raft.go:
                               1405-1407)                                     */

typedef struct qe_leader {
  const uint8_t *elected;        /* [G] 1: the group's node won its election
                                    (NULL = every group)                      */
  const uint64_t *term;          /* [G] r.Term of the new leadership           */
  uint32_t flags;                /* QE_BL_BCAST or 0                           */
  uint32_t reserved;             /* must be 0                                  */
  uint64_t *pending_conf_index;  /* [G] out (may be NULL): r.pendingConfIndex =
                                    lastIndex before the empty entry         */
  uint64_t *uncommitted_size;    /* [G] out (may be NULL): 0 (reset; the empty
                                    entry is not counted, raft.go:753-757)   */
  uint8_t *result;               /* [G] out QE_BL_*                            */
  void *sent;                    /* [G] out mask (may be NULL): bcastAppend's  */
  void *snap;                    /* [G] out mask (may be NULL)                 */
} qe_leader;

/* raft.becomeLeader (raft/raft.go:724-759) on every group with elected[g],
 * on the leader-side state p:
 *   reset (:590-613): every tracked slot's Progress becomes Match 0, Next =
 *     lastIndex + 1, StateProbe, not ProbeSent, not RecentActive, no pending
 *     snapshot, empty Inflights; the leader's own (self_slot) Match =
 *     lastIndex, then BecomeReplicate; lead_transferee = none; the ReadIndex
 *     queue emptied (newReadOnly: read_count 0, read_head past the dropped
 *     requests' context numbers, so a late response for one finds nothing);
 *   pendingConfIndex = lastIndex; uncommittedSize = 0;
 *   the log model enters the term: a run [lastIndex + 1, ...) of term[g] is
 *     appended to the run table and term_start = lastIndex + 1;
 *   appendEntry of the empty entry (:621-642): lastIndex + 1, the leader's
 *     MaybeUpdate, maybeCommit (a one-voter config commits it at once);
 *   QE_BL_BCAST: bcastAppend (every tracked slot but the leader's, the
 *     probes of a new term).
 * Writes p's Progress rows, Inflights words, committed, last_index,
 * term_start, the run table (run_first / run_term / run_count) and
 * lead_transferee / the queue when present (declared const in qe_progress
 * because the other entry points only read them).  stats: groups, commit
 * sum, commit advanced, checksum. */
int qe_become_leader(const qe_progress *p, const qe_leader *l, uint64_t *stats, void *stream);

/* ---- switchToConfig: the leader's side of an applied conf change (ABI 7) - */

/* qe_switch.result & QE_SW_OUTCOME */
#define QE_SW_NONE 0       /* switched[g] == 0: not part of this call           */
#define QE_SW_REMOVED 1    /* the leader has no Progress any more, or is a
                              learner: switchToConfig returns at once
                              (raft.go:1663-1674; the leader stays leader)    */
#define QE_SW_NO_VOTERS 2  /* Voters[0] is empty: returns (:1678-1680)         */
#define QE_SW_BCAST 3      /* maybeCommit advanced the commit under the new
                              config: bcastAppend (:1682-1685)                  */
#define QE_SW_PROBE 4      /* it did not: maybeSendAppend(id, false) to every
                              tracked peer (:1686-1692)                         */
#define QE_SW_OUTCOME 0x0Fu
#define QE_SW_TRANSFER_ABORTED 0x10u /* result bit: leadTransferee was not a voter
                                        of the new config, abortLeaderTransfer
                                        (:1694-1697)                            */

typedef struct qe_switch {
  const uint8_t *switched;       /* [G] 1: the group's configuration was just
                                    switched (its conf change applied); NULL =
                                    every group                               */
  uint8_t *result;               /* [G] out QE_SW_* (| QE_SW_TRANSFER_ABORTED) */
  void *sent;                    /* [G] out mask (may be NULL): peers sent a
                                    MsgApp / MsgSnap                          */
  void *snap;                    /* [G] out mask (may be NULL): a MsgSnap      */
  uint64_t *bytes_requested;     /* measurement aid, normally NULL: adds the
                                    algorithmic bytes (DESIGN.md §3 rules)    */
} qe_switch;

/* raft.switchToConfig (raft/raft.go:1651-1700) after the new configuration
 * is in place -- inc_mask / out_mask / tracked of p are the new Voters[0],
 * Voters[1] and ProgressMap keys (e.g. the qe_conf masks qe_confchange just
 * wrote) -- for every group with switched[g]:
 *   the leader (self_slot) has no Progress, or is a learner (tracked but in
 *     neither half: Learners, confchange.go checkInvariants) -> QE_SW_REMOVED;
 *   Voters[0] empty -> QE_SW_NO_VOTERS;
 *   maybeCommit under the new JointConfig (the term gate of qe_progress_step)
 *     advanced -> bcastAppend: sendAppend (sendIfEmpty) to every tracked slot
 *     but the leader's; else maybeSendAppend(id, false) to every tracked slot
 *     (prs.Visit: the leader's own included -- a no-op while its Next is
 *     lastIndex + 1, as appendEntry keeps it);
 *   then a lead_transferee that is not in Voters[0] | Voters[1] is cleared
 *     (abortLeaderTransfer) and QE_SW_TRANSFER_ABORTED set.
 * As in the reference, this maybeCommit does not release postponed ReadIndex
 * requests (only stepLeader's MsgAppResp arm calls
 * releasePendingReadIndexMessages, :1259-1262).  Writes committed, the
 * peers' Next / word / PendingSnapshot / Inflights and lead_transferee.
 * stats: groups, commit sum, commit advanced, checksum. */
int qe_switch_config(const qe_progress *p, const qe_switch *sw, uint64_t *stats, void *stream);

/* ABI 4, HOST pointers: Inflights rings between plain uint64 buffers
 * (Inflights.buffer of each peer, raft/tracker/inflights.go:25-37, peer-major
 * [S][stride][F]: entry k of slot s of group g at (s*stride + g)*F + k) and
 * the device form (infl_lo / infl_hi, pitch QE_RING_PITCH(F)).  qe_ring_pack
 * also writes each peer word's ring representation bits (QE_PW_RING_MASK,
 * canonical form; the other bits are kept: Inflights.start / count must be
 * set).  qe_ring_unpack decodes all F entries of every peer (positions
 * outside the live window decode like live ones; their values are whatever
 * the ring holds there, as in the reference).  Groups [0, num_groups). */
int qe_ring_pack(uint64_t num_groups, uint32_t num_slots, uint32_t inflight_cap,
                 uint64_t stride, const uint64_t *entries, uint32_t *peer,
                 uint32_t *infl_lo, uint32_t *infl_hi);
int qe_ring_unpack(uint64_t num_groups, uint32_t num_slots, uint32_t inflight_cap,
                   uint64_t stride, const uint32_t *infl_lo, const uint32_t *infl_hi,
                   const uint32_t *peer, uint64_t *entries);
/* ABI 8, HOST pointers: the same for the 16-bit form (qe_progress.infl16):
 * Next ([S][stride], next) is the base of each peer's offsets.  Every peer
 * gets the 16-bit form when its live entries fit below its Next, else the
 * wide form (infl_lo / infl_hi, QE_PF_RING_WIDE); infl_lo / infl_hi are
 * written for every peer.  inflight_cap <= QE_RING16_MAX_F. */
int qe_ring_pack16(uint64_t num_groups, uint32_t num_slots, uint32_t inflight_cap,
                   uint64_t stride, const uint64_t *entries, const uint64_t *next,
                   uint32_t *peer, uint16_t *infl16, uint32_t *infl_lo, uint32_t *infl_hi);
int qe_ring_unpack16(uint64_t num_groups, uint32_t num_slots, uint32_t inflight_cap,
                     uint64_t stride, const uint16_t *infl16, const uint32_t *infl_lo,
                     const uint32_t *infl_hi, const uint64_t *next, const uint32_t *peer,
                     uint64_t *entries);

/* ---- sparse MsgAppResp deltas ------------------------------------------ */

/* Apply n MsgAppResp acks in COO form -- ack i: group[i], slot[i] (-1 =
 * skip), index[i] -- with Progress.MaybeUpdate semantics
 * (raft/tracker/progress.go:144-153): match = max(match, index),
 * next = max(next, index + 1), via 64-bit atomic max.  Max is commutative,
 * so duplicated or reordered acks give the same state as applying them one
 * by one in any order.  touched[g] (optional) is set to 1 for every group
 * that received an ack.  All pointers are device pointers. */
int qe_apply_append_resps(uint64_t num_groups, uint32_t num_slots, uint64_t stride,
                          uint64_t *match, uint64_t *next, uint64_t n, const uint64_t *group,
                          const int8_t *slot, const uint64_t *index, uint8_t *touched,
                          void *stream);

/* ---- host-side ConfState packing (wire format -> slot SoA) -------------- */

/* G ConfStates (raft/raftpb/raft.proto:115-130) in CSR form: list k of
 * group g is ids_k[off_k[g] .. off_k[g+1]).  NULL lists are empty.  HOST
 * pointers.  Produced by ProgressTracker.ConfState (tracker.go:146-154). */
typedef struct qe_confstate_csr {
  uint64_t num_groups;
  const uint64_t *voters, *voters_off;
  const uint64_t *voters_outgoing, *outgoing_off;
  const uint64_t *learners, *learners_off;
  const uint64_t *learners_next, *learners_next_off;
  const uint8_t *auto_leave;    /* [G] ConfState.auto_leave (ABI 2; NULL = false) */
  const uint64_t *perm;         /* ABI 3: packed position i takes the caller's
                                   group perm[i] (qe_pack_order); NULL =
                                   identity.  Every packer output is in
                                   packed order. */
} qe_confstate_csr;

/* group_flags bits reported by qe_pack_confstate */
#define QE_PACK_TOO_MANY_PEERS 1u          /* > num_slots peers: group left empty */
#define QE_PACK_LEARNER_IS_VOTER 2u        /* confchange.go:308-318 violated      */
#define QE_PACK_LEARNER_NEXT_NOT_OUTGOING 4u /* confchange.go:299-306 violated   */
#define QE_PACK_ZERO_ID 8u                 /* ID 0 is raft.None                   */

/* Shape bucketing (ABI 3; the order the JointConfig kernels want, DESIGN.md
 * §2): perm[i] = the caller's group placed at packed position i, groups
 * sorted by configuration shape -- (|Voters[0] u Voters[1]|, |Voters[0]|,
 * |Voters[1]|, learners) ascending, caller order within a shape (stable);
 * groups the packer would flag sort last.  With cs->perm = perm the groups
 * of one shape fill consecutive 64-group tiles: every lane of a wave has its
 * voters in the same low slots (voters are placed first), so the joint
 * commit kernel fetches exactly the union's slot rows.  Quorum results are
 * order-free per group; the host maps packed outputs back through perm
 * (qe_collect does it on the device).  *num_shapes (optional) = distinct
 * shapes.  perm is a HOST array of num_groups entries. */
int qe_pack_order(const qe_confstate_csr *cs, uint32_t num_slots, uint64_t *perm,
                  uint64_t *num_shapes);

/* Slot assignment: voters of both halves ascending, then learners ascending.
 * Writes the three masks (mask-typed, may be NULL), slot_ids (ABI 3:
 * ID-major [S][G], slot s of packed group i at slot_ids[s*G + i]; 0 =
 * unused slot) and optional per-group flags; *num_flagged counts flagged
 * groups.  Outputs are in packed order (cs->perm).  Multi-threaded
 * (qe_pack_threads). */
int qe_pack_confstate(const qe_confstate_csr *cs, uint32_t num_slots, void *inc_mask,
                      void *out_mask, void *learner_mask, uint64_t *slot_ids,
                      uint32_t *group_flags, uint64_t *num_flagged);

/* Progress.Match of each peer (CSR prog_ids/prog_match, in the caller's
 * group order) into match[S][stride] (host, packed order); packed group i
 * reads CSR row perm[i] (NULL = identity; ABI 3).  slot_ids as written by
 * qe_pack_confstate ([S][G]).  Peers without a slot are counted in
 * *num_unknown. */
int qe_pack_match(uint64_t num_groups, uint32_t num_slots, const uint64_t *slot_ids,
                  const uint64_t *perm, const uint64_t *prog_off, const uint64_t *prog_ids,
                  const uint64_t *prog_match, uint64_t *match, uint64_t stride,
                  uint64_t *num_unknown);

/* ProgressTracker.Votes (CSR vote_ids / vote_vals 0|1, caller order) into
 * voted/granted bitmaps (packed order, through perm as qe_pack_match); the
 * first vote per peer sticks (tracker.go:258-263). */
int qe_pack_votes(uint64_t num_groups, uint32_t num_slots, const uint64_t *slot_ids,
                  const uint64_t *perm, const uint64_t *vote_off, const uint64_t *vote_ids,
                  const uint8_t *vote_vals, void *voted, void *granted);

/* (packed group, id) -> slot (-1 if the id has no slot) for routing deltas;
 * slot_ids [S][G].  A caller that bucketed maps its group id to the packed
 * position with the inverse of perm. */
int qe_slot_lookup(uint64_t num_groups, uint32_t num_slots, const uint64_t *slot_ids,
                   uint64_t n, const uint64_t *group, const uint64_t *id, int8_t *slot);

/* Host packing threads (0 = min(16, hardware threads)). */
int qe_pack_threads(int n);

/* ---- configuration changes (raft/confchange/confchange.go) ------------- */

/* ConfChangeSingle.Type (raft/raftpb/raft.pb.go:224-227) */
#define QE_CC_ADD_NODE 0
#define QE_CC_REMOVE_NODE 1
#define QE_CC_UPDATE_NODE 2
#define QE_CC_ADD_LEARNER_NODE 3

/* per-group operation */
#define QE_CC_OP_NONE 0
#define QE_CC_OP_SIMPLE 1            /* Changer.Simple          (:130-147) */
#define QE_CC_OP_ENTER_JOINT 2       /* Changer.EnterJoint(false, ...)     */
#define QE_CC_OP_ENTER_JOINT_AUTO 3  /* Changer.EnterJoint(true, ...) (:49-76) */
#define QE_CC_OP_LEAVE_JOINT 4       /* Changer.LeaveJoint      (:92-123) */

/* per-group result (a group with an error keeps its state, as the caller of
 * the reference Changer discards the returned config on error) */
#define QE_CC_OK 0
#define QE_CC_ERR_INVARIANT 1        /* checkInvariants on the input (:186-241) */
#define QE_CC_ERR_ALREADY_JOINT 2    /* "config is already joint"              */
#define QE_CC_ERR_ZERO_VOTER_JOINT 3 /* "can't make a zero-voter config joint" */
#define QE_CC_ERR_NOT_JOINT 4        /* "can't leave a non-joint config"       */
#define QE_CC_ERR_SIMPLE_IN_JOINT 5  /* "can't apply simple config change in joint config" */
#define QE_CC_ERR_BAD_TYPE 6         /* "unexpected conf type %d"              */
#define QE_CC_ERR_REMOVED_ALL 7      /* "removed all voters"                   */
#define QE_CC_ERR_SIMPLE_MULTI 8     /* "more than one voter changed without entering joint config" */
#define QE_CC_ERR_INVARIANT_OUT 9    /* checkInvariants on the result          */
#define QE_CC_ERR_NO_SLOT 10         /* slot model: a new peer found no free slot */

/* tracker.Config + the ProgressMap key set of G groups in slot form.  A slot
 * is tracked when it holds a Progress (ProgressMap key); Voters[0],
 * Voters[1], Learners and LearnersNext are slot masks ([G], u8 for
 * num_slots <= 8, else u16) over tracked slots; is_learner is
 * Progress.IsLearner.  slot_ids is ID-major [S][G] (ABI 3: slot s of group
 * g at slot_ids[s*G + g]) as written by qe_pack_confstate, so a change
 * rewrites only the changed slot's row.  The ids of untracked slots are
 * ignored on input (qe_confchange) and left as they are, except that a slot
 * a change untracks gets 0; the packer writes 0 for every unused slot.
 * qe_pack_match / qe_pack_votes / qe_slot_lookup match ids over all S slots,
 * so a caller that writes slot_ids itself keeps untracked ones 0. */
typedef struct qe_conf {
  uint64_t num_groups;
  uint32_t num_slots;
  uint32_t reserved;
  uint64_t *slot_ids;           /* [S][G]                                   */
  void *inc_mask, *out_mask;    /* Voters[0], Voters[1]                     */
  void *learner_mask;           /* Learners                                 */
  void *learners_next_mask;     /* LearnersNext                             */
  void *is_learner;             /* Progress.IsLearner                       */
  void *tracked;                /* slots holding a Progress                 */
  uint8_t *auto_leave;          /* [G] Config.AutoLeave                     */
} qe_conf;

/* The whole tracker.Config of each group from its ConfState, as
 * ProgressTracker.ConfState / confchange.Restore see it (raft/tracker/
 * tracker.go:146-154, raft/confchange/restore.go:1-155): slot_ids (voters of
 * both halves ascending, then learners), Voters[0], Voters[1], Learners,
 * LearnersNext (outgoing voters only), Progress.IsLearner (= Learners; a
 * LearnersNext peer is still a voter), tracked (every placed peer) and
 * AutoLeave -- the state qe_confchange consumes.  All pointers in `out` are
 * HOST pointers here (copy them to the device for qe_confchange); its
 * num_groups must equal cs->num_groups.  Flagged groups (QE_PACK_*) are left
 * empty. */
int qe_pack_conf(const qe_confstate_csr *cs, const qe_conf *out, uint32_t *group_flags,
                 uint64_t *num_flagged);

/* One operation per group with up to max_changes ConfChangeSingle entries:
 * change c of group g at [c*stride + g]. */
typedef struct qe_conf_changes {
  uint32_t max_changes;
  uint32_t reserved;
  uint64_t stride;              /* >= num_groups                            */
  const uint8_t *op;            /* [G] QE_CC_OP_*                           */
  const uint8_t *count;         /* [G] changes of group g (<= max_changes)  */
  const uint8_t *type;          /* [C][stride] QE_CC_ADD_NODE ...           */
  const uint64_t *node_id;      /* [C][stride] NodeID (0 = ignored, :154-160) */
  const uint64_t *last_index;   /* [G] Changer.LastIndex                    */
  uint8_t *result;              /* [G] out: QE_CC_*                         */
  void *new_progress;           /* [G] out mask (may be NULL): slots whose
                                   Progress initProgress created           */
} qe_conf_changes;

/* Changer.Simple / EnterJoint / LeaveJoint per group (raft/confchange/
 * confchange.go:49-274): makeVoter, makeLearner (LearnersNext while the
 * peer is an outgoing voter), remove (keeps the Progress of an outgoing
 * voter), symdiff over voter ids, checkInvariants before and after.  A new
 * peer takes the lowest untracked slot.  When `p` is non-NULL (same G and S)
 * the Progress of every created slot is initialised as initProgress does
 * (:262-273): Match 0, Next = last_index, StateProbe, RecentActive, empty
 * Inflights, no pending snapshot. */
int qe_confchange(const qe_conf *c, const qe_conf_changes *ch, const qe_progress *p,
                  void *stream);

/* ---- Ready deltas ------------------------------------------------------ */

/* The groups a batch step changed, as a dense list in ascending position
 * order: for every g with flags[g] != 0, out_groups[i] = group_offset + g
 * (ABI 3: group_offset + perm[g] when perm is non-NULL -- the caller's group
 * id of a shape-bucketed batch, qe_pack_order) and (when out_values is
 * non-NULL) out_values[i] = values[g]; *out_count (device) =
 * their number.  raft reports a HardState only when it changed
 * (raft/node.go:571-573 newReady, raft/rawnode.go:152-176 prevHardSt): with
 * flags = qe_replication_round's `adv` and values = `committed` this is the
 * per-round commit delta a host ships instead of all G words.  out_groups /
 * out_values hold up to num_groups entries (NULL: not written).  scratch:
 * qe_collect_scratch_bytes(num_groups) bytes of device memory, 8-B aligned.
 * All pointers are device pointers; stream-ordered. */
size_t qe_collect_scratch_bytes(uint64_t num_groups);
int qe_collect(uint64_t num_groups, uint64_t group_offset, const uint64_t *perm,
               const uint8_t *flags, const uint64_t *values, uint64_t *out_groups,
               uint64_t *out_values, uint64_t *out_count, void *scratch, void *stream);

/* ---- statistics -------------------------------------------------------- */

/* out[QE_STATS_COUNTERS] (device) = sum over shards of stats (device). */
int qe_stats_reduce(const uint64_t *stats, uint64_t *out, void *stream);

/* ---- multi-GPU aggregation (RCCL over xGMI) ---------------------------- */

/* Groups shard across GPUs with no data-path exchange; the one collective is
 * the sum of the statistics vector (the batch form of etcd's per-member
 * Prometheus counters, server/etcdserver/metrics.go:29-85).  Setup: rank 0
 * calls qe_comm_unique_id, the host sends those qe_comm_id_bytes() bytes to
 * every rank over its own transport, every rank calls qe_comm_init with its
 * rank and device.  One communicator per process (one process per GPU). */
size_t qe_comm_id_bytes(void);                 /* size of the id (128) */
int qe_comm_unique_id(void *id);               /* rank 0: new id (host) */
int qe_comm_init(void **comm, uint32_t nranks, uint32_t rank, const void *id,
                 int device);
/* qe_comm_init with a bound (ABI 6): the communicator is created
 * non-blocking and polled; when the other ranks have not joined after
 * timeout_ms (e.g. one of them failed before calling init) it is aborted and
 * QE_ECOMM returned, so no rank waits forever.  timeout_ms == 0: blocking,
 * as qe_comm_init.  Hosts then agree over their own transport on the path
 * every rank takes (bench.py Dist._select_stats_path). */
int qe_comm_init_timeout(void **comm, uint32_t nranks, uint32_t rank, const void *id,
                         int device, uint32_t timeout_ms);
/* ncclCommFinalize (polled, at most 30 s, on a non-blocking communicator;
 * aborted when it does not complete: QE_ECOMM) then ncclCommDestroy. */
int qe_comm_destroy(void *comm);
/* ncclCommAbort (ABI 6): frees the communicator without waiting for its
 * outstanding collectives -- the way out when a peer failed mid-run. */
int qe_comm_abort(void *comm);

/* stats[0..n) (DEVICE, n <= QE_STATS_WORDS; normally the QE_STATS_COUNTERS
 * words qe_stats_reduce produced) = elementwise sum over all ranks of comm,
 * in place, asynchronously on `stream`: ncclAllReduce(ncclUint64, ncclSum).
 * uint64 addition wraps like the counters themselves.  On a non-blocking
 * communicator the enqueue is awaited (sleeping polls, at most 30 s; then
 * QE_ECOMM).  The collective completes only when every rank enqueued it: a
 * host should run it on a stream of its own, agree with its peers over its
 * own transport that every rank enqueued it, and bound its wait for the
 * completion (qe_comm_abort on failure) -- bench.py Dist.sum_stats. */
int qe_allreduce_stats(uint64_t *stats, uint32_t n, void *comm, void *stream);

/* ---- synthetic inputs (counter-based, bit-identical to oracle/) -------- */

typedef struct qe_gen_params {
  uint64_t seed;
  uint64_t group_offset;     /* global id of group 0                         */
  uint32_t dist;             /* 0 clustered, 1 uniform (Int63), 2 small ties */
  uint32_t p_absent_q16;     /* P(slot has no acked index) * 65536           */
  uint32_t p_voted_q16;      /* P(slot voted) * 65536                        */
  uint32_t p_granted_q16;    /* P(granted | voted) * 65536                   */
  uint32_t n_inc;            /* joint: incoming voters (0 = all S slots)     */
  uint32_t n_out;            /* joint: outgoing voters (0 = non-joint)       */
  uint32_t mask_mode;        /* 0 structured + rotated, 1 arbitrary random,
                                2 shape-bucketed (voters in low slots, overlap
                                constant per 2^20 consecutive groups)        */
  uint32_t reserved;
} qe_gen_params;

/* Fill a qe_groups batch (the pointers inside `g` are written through; the
 * const qualifiers of qe_groups are cast away).  Masks pointers that are
 * NULL in `g` are skipped. */
int qe_gen_groups(const qe_groups *g, const qe_gen_params *p, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* ETCD_QUORUM_H */
