/*
 * oracle/quorum_oracle.c — CPU restatement of etcd's raft/quorum +
 * raft/tracker hot path.  TEST INFRASTRUCTURE ONLY: this file is the parity
 * checker and the CPU baseline ("port").  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product (etcd_amd/) never
 * links or calls it.
 *
 * Parity pinning: every scalar function below is checked against the
 * reference's own golden vectors (raft/quorum/testdata/ *.txt files, 127 cases; the
 * TestCommit / TestLeaderElectionInOneRoundRPC / TestProgressUpdate tables),
 * extracted into tests/golden/ by tests/golden/make_golden.py.  The reference
 * itself is Go and cannot be built in this image (no Go toolchain), so those
 * fixtures are the pin.
 *
 * Slot form: a group is S <= 16 slots; bit s of a mask selects slot s.
 * vals[s] is the acked index of slot s, 0 meaning absent (the reference fills
 * unused positions with 0, raft/quorum/majority.go:150-161, so absent == 0).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_INF UINT64_MAX
#define VOTE_PENDING 1
#define VOTE_LOST 2
#define VOTE_WON 3

#define NSTAT 16
enum {
  ST_GROUPS = 0, ST_COMMIT_INF, ST_COMMIT_SUM, ST_COMMIT_ZERO, ST_WON, ST_LOST,
  ST_PENDING, ST_GRANTED, ST_REJECTED, ST_COMMIT_ADVANCED, ST_READ_RELEASED,
  ST_ELECTIONS, ST_LEADERS, ST_STEPDOWNS, ST_VIOLATIONS, ST_CHECKSUM
};

static const uint64_t PHI = 0x9E3779B97F4A7C15ULL;

static inline int popc(uint32_t x) { return __builtin_popcount(x); }

/* ------------------------------------------------------------------------ */
/* Counter-based generator.  Must stay bit-identical with the  */
/* device generator in etcd_amd/csrc/qe_kernels.hip (checked by tests).      */
/* ------------------------------------------------------------------------ */
uint64_t orc_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

uint64_t orc_hash(uint64_t seed, uint64_t gid, uint32_t lane, uint32_t stream) {
  uint64_t k = ((uint64_t)stream << 32) | lane;
  return orc_mix64(orc_mix64(seed + gid * PHI) ^ (k * 0xD6E8FEB86659FD93ULL));
}

static inline uint32_t rotl_s(uint32_t m, uint32_t r, uint32_t S) {
  uint32_t full = (S == 32) ? 0xFFFFFFFFu : ((1u << S) - 1u);
  m &= full;
  if (r == 0) return m;
  return ((m << r) | (m >> (S - r))) & full;
}

/* Generate one group's slot inputs.  Output masks are only meaningful when
 * the caller asked for them (want_masks). */
void orc_gen_group(uint64_t seed, uint64_t gid, uint32_t S, uint32_t dist,
                   uint32_t p_absent, uint32_t p_voted, uint32_t p_granted,
                   uint32_t n_inc, uint32_t n_out, uint32_t mask_mode,
                   uint64_t *vals, uint32_t *inc, uint32_t *out,
                   uint32_t *learner, uint32_t *voted, uint32_t *granted) {
  uint32_t full = (1u << S) - 1u;
  uint64_t hb = orc_hash(seed, gid, 0xFFFFu, 0);
  /* masks */
  uint32_t mi, mo, ml;
  if (mask_mode == 0 || mask_mode == 2) {
    /* 0: structured, rotated per group; 2: shape-bucketed -- voters packed
     * into the low slots (no rotation) and the overlap constant over runs of
     * 2^20 consecutive group ids, the layout a host packer produces when it
     * buckets groups by configuration shape. */
    uint32_t ni = n_inc ? n_inc : S;
    if (ni > S) ni = S;
    uint32_t no = n_out;
    if (no > S) no = S;
    if (no == 0) {
      mi = (ni == 32) ? 0xFFFFFFFFu : ((1u << ni) - 1u);
      mo = 0;
      ml = full & ~mi;
    } else {
      uint32_t omin = (ni + no > S) ? ni + no - S : 0;
      uint32_t omax = ni < no ? ni : no;
      uint64_t okey = mask_mode == 2 ? (gid >> 20) : (hb >> 8);
      uint32_t o = omin + (uint32_t)(okey % (uint64_t)(omax - omin + 1));
      uint32_t uni = ni + no - o;
      mi = (1u << ni) - 1u;
      mo = ((1u << no) - 1u) << (ni - o);
      ml = full & ~((1u << uni) - 1u);
    }
    uint32_t r = mask_mode == 2 ? 0u : (uint32_t)((hb >> 16) % S);
    mi = rotl_s(mi, r, S);
    mo = rotl_s(mo, r, S);
    ml = rotl_s(ml, r, S);
  } else {
    uint64_t hm = orc_hash(seed, gid, 0xFFFEu, 0);
    mi = (uint32_t)hm & full;
    mo = ((hm >> 48) & 3u) == 0 ? 0u : ((uint32_t)(hm >> 16) & full);
    ml = (uint32_t)(hm >> 32) & full;
    if (((hm >> 50) & 7u) != 0) ml &= ~(mi | mo); /* mostly legal configs */
  }
  *inc = mi;
  *out = mo;
  *learner = ml;
  /* acked indexes */
  for (uint32_t s = 0; s < S; s++) {
    uint64_t h = orc_hash(seed, gid, s, 1);
    uint64_t v;
    if ((uint32_t)(h & 0xFFFFu) < p_absent) {
      v = 0;
    } else if (dist == 0) {
      v = (hb >> 2) + ((h >> 40) & 0xFFFFu);
    } else if (dist == 1) {
      v = h >> 1;
    } else {
      v = (h >> 40) & 3u;
    }
    vals[s] = v;
  }
  /* votes */
  uint32_t vd = 0, gr = 0;
  for (uint32_t s = 0; s < S; s++) {
    uint64_t h = orc_hash(seed, gid, s, 2);
    if ((uint32_t)(h & 0xFFFFu) < p_voted) {
      vd |= 1u << s;
      if ((uint32_t)((h >> 16) & 0xFFFFu) < p_granted) gr |= 1u << s;
    }
  }
  *voted = vd;
  *granted = gr;
}

/* ------------------------------------------------------------------------ */
/* Scalar restatements                                                       */
/* ------------------------------------------------------------------------ */

/* raft/quorum/majority.go:115-122 */
static void insertion_sort(uint64_t *sl, int n) {
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0 && sl[j] < sl[j - 1]; j--) {
      uint64_t t = sl[j];
      sl[j] = sl[j - 1];
      sl[j - 1] = t;
    }
}

/* MajorityConfig.CommittedIndex, raft/quorum/majority.go:126-172. */
uint64_t orc_majority_committed(uint32_t S, uint32_t member, const uint64_t *vals) {
  int n = popc(member);
  if (n == 0) return ORC_INF; /* :128-132 */
  uint64_t srt[32];
  memset(srt, 0, sizeof(srt));
  int i = n - 1; /* fill from the right, :150-161 */
  for (uint32_t s = 0; s < S; s++) {
    if (!((member >> s) & 1u)) continue;
    /* AckedIndex(id): absent is represented as 0 which equals an unused
     * (zero) position; the reference only decrements i when found, but the
     * zero it leaves behind is identical. */
    srt[i--] = vals[s];
  }
  insertion_sort(srt, n); /* :165 */
  int pos = n - (n / 2 + 1); /* :170-171 */
  return srt[pos];
}

/* alternativeMajorityCommittedIndex, raft/quorum/quick_test.go:85-122:
 * the largest index acked by >= q voters (counting algorithm). */
uint64_t orc_alt_committed(uint32_t S, uint32_t member, const uint64_t *vals) {
  int n = popc(member);
  if (n == 0) return ORC_INF;
  int q = n / 2 + 1;
  uint64_t best = 0;
  for (uint32_t a = 0; a < S; a++) {
    if (!((member >> a) & 1u) || vals[a] == 0) continue; /* absent => not in idToIdx */
    int cnt = 0;
    for (uint32_t b = 0; b < S; b++)
      if (((member >> b) & 1u) && vals[b] != 0 && vals[b] >= vals[a]) cnt++;
    if (cnt >= q && vals[a] > best) best = vals[a];
  }
  return best;
}

/* MajorityConfig.VoteResult, raft/quorum/majority.go:178-210. */
uint8_t orc_majority_vote(uint32_t member, uint32_t voted, uint32_t granted) {
  int n = popc(member);
  if (n == 0) return VOTE_WON; /* :179-184 */
  int ny[2] = {0, 0}, missing = 0;
  for (int s = 0; s < 32; s++) {
    if (!((member >> s) & 1u)) continue;
    if (!((voted >> s) & 1u)) { missing++; continue; }
    if ((granted >> s) & 1u) ny[1]++; else ny[0]++;
  }
  int q = n / 2 + 1;
  if (ny[1] >= q) return VOTE_WON;
  if (ny[1] + missing >= q) return VOTE_PENDING;
  return VOTE_LOST;
}

/* JointConfig.CommittedIndex, raft/quorum/joint.go:49-56. */
uint64_t orc_joint_committed(uint32_t S, uint32_t inc, uint32_t out, const uint64_t *vals) {
  uint64_t a = orc_majority_committed(S, inc, vals);
  uint64_t b = orc_majority_committed(S, out, vals);
  return a < b ? a : b;
}

/* JointConfig.VoteResult, raft/quorum/joint.go:61-75. */
uint8_t orc_joint_vote(uint32_t inc, uint32_t out, uint32_t voted, uint32_t granted) {
  uint8_t r1 = orc_majority_vote(inc, voted, granted);
  uint8_t r2 = orc_majority_vote(out, voted, granted);
  if (r1 == r2) return r1;
  if (r1 == VOTE_LOST || r2 == VOTE_LOST) return VOTE_LOST;
  return VOTE_PENDING;
}

/* ProgressTracker.TallyVotes, raft/tracker/tracker.go:267-288.  Progress
 * entries are the voters of both halves plus learners; learners skipped. */
uint8_t orc_tally(uint32_t inc, uint32_t out, uint32_t learner, uint32_t voted,
                  uint32_t granted, int *gr, int *rj) {
  uint32_t prog = inc | out | learner;
  int g = 0, r = 0;
  for (int s = 0; s < 32; s++) {
    if (!((prog >> s) & 1u)) continue;
    if ((learner >> s) & 1u) continue; /* :273-275 */
    if (!((voted >> s) & 1u)) continue; /* :276-279 */
    if ((granted >> s) & 1u) g++; else r++;
  }
  *gr = g;
  *rj = r;
  return orc_joint_vote(inc, out, voted, granted); /* :286 */
}

/* ProgressTracker.QuorumActive, raft/tracker/tracker.go:215-225. */
uint8_t orc_quorum_active(uint32_t inc, uint32_t out, uint32_t learner, uint32_t recent) {
  uint32_t prog = inc | out | learner;
  uint32_t votes_present = prog & ~learner; /* votes[id] for non-learners */
  return orc_joint_vote(inc, out, votes_present, recent & votes_present) == VOTE_WON;
}

/* ProgressTracker.RecordVote, raft/tracker/tracker.go:258-263 (first vote
 * sticks), for a set of responders. */
void orc_record_votes(uint32_t *voted, uint32_t *granted, uint32_t resp, uint32_t value) {
  uint32_t fresh = resp & ~*voted;
  *voted |= fresh;
  *granted |= fresh & value;
}

/* Progress.MaybeUpdate, raft/tracker/progress.go:144-153. */
int orc_maybe_update(uint64_t *match, uint64_t *next, uint64_t n) {
  int updated = 0;
  if (*match < n) {
    *match = n;
    updated = 1; /* ProbeAcked: ProbeSent = false (not modelled) */
  }
  if (*next < n + 1) *next = n + 1;
  return updated;
}

/* raft.maybeCommit (raft/raft.go:585-588) -> raftLog.maybeCommit
 * (raft/log.go:325-331) -> commitTo (log.go:233-241) with the synthetic log
 * model: term(i) == Term <=> term_start <= i <= last_index (i > lastIndex has
 * term 0, raft/log.go:265-271).  Returns 1 if committed advanced. */
int orc_maybe_commit(uint64_t mci, uint64_t *committed, uint64_t term_start, uint64_t last_index) {
  if (mci > *committed && mci >= term_start && mci <= last_index) {
    *committed = mci;
    return 1;
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Batch (SoA) runners: the checker and the CPU baseline                     */
/* ------------------------------------------------------------------------ */

static inline uint32_t ld_mask(const void *p, uint32_t mb, uint64_t g) {
  if (!p) return 0;
  return mb == 1 ? ((const uint8_t *)p)[g] : ((const uint16_t *)p)[g];
}
static inline void st_mask(void *p, uint32_t mb, uint64_t g, uint32_t v) {
  if (mb == 1) ((uint8_t *)p)[g] = (uint8_t)v; else ((uint16_t *)p)[g] = (uint16_t)v;
}

uint64_t orc_checksum_cv(uint64_t gid, uint64_t commit, uint32_t vote, uint32_t gc, uint32_t rc) {
  uint64_t tag = (uint64_t)(vote | (gc << 2) | (rc << 7)) << 52;
  return orc_mix64((gid * PHI) ^ commit ^ tag);
}

/* qe_commit_vote restated.  alg: 0 = majority.go insertion sort,
 * 1 = quick_test.go counting alternative. */
void orc_commit_vote_batch(uint64_t G, uint64_t goff, uint32_t S, uint64_t stride,
                           const uint64_t *match, const void *inc, const void *out,
                           const void *learner, const void *voted, const void *granted,
                           uint64_t *commit, uint8_t *vote, uint8_t *gcount, uint8_t *rcount,
                           uint64_t *stats, int alg, int threads) {
  uint32_t mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  uint64_t st[NSTAT];
  memset(st, 0, sizeof(st));
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    uint64_t ls[NSTAT];
    memset(ls, 0, sizeof(ls));
#pragma omp for schedule(static)
    for (int64_t gi = 0; gi < (int64_t)G; gi++) {
      uint64_t g = (uint64_t)gi;
      uint64_t vals[16];
      for (uint32_t s = 0; s < S; s++) vals[s] = match[s * stride + g];
      uint32_t mi = inc ? ld_mask(inc, mb, g) & full : full;
      uint32_t mo = out ? ld_mask(out, mb, g) & full : 0;
      uint32_t ml = ld_mask(learner, mb, g) & full;
      uint32_t vd = ld_mask(voted, mb, g) & full;
      uint32_t gr = voted ? ld_mask(granted, mb, g) & full : 0;
      uint64_t c;
      if (alg == 0) c = orc_joint_committed(S, mi, mo, vals);
      else {
        uint64_t a = orc_alt_committed(S, mi, vals), b = orc_alt_committed(S, mo, vals);
        c = a < b ? a : b;
      }
      int gcn, rcn;
      uint8_t v = orc_tally(mi, mo, ml, vd, gr, &gcn, &rcn);
      if (commit) commit[g] = c;
      if (vote) vote[g] = v;
      if (gcount) gcount[g] = (uint8_t)gcn;
      if (rcount) rcount[g] = (uint8_t)rcn;
      ls[ST_GROUPS] += 1;
      ls[ST_COMMIT_INF] += (c == ORC_INF);
      ls[ST_COMMIT_SUM] += (c == ORC_INF) ? 0 : c;
      ls[ST_COMMIT_ZERO] += (c == 0);
      ls[ST_WON] += (v == VOTE_WON);
      ls[ST_LOST] += (v == VOTE_LOST);
      ls[ST_PENDING] += (v == VOTE_PENDING);
      ls[ST_GRANTED] += (uint64_t)gcn;
      ls[ST_REJECTED] += (uint64_t)rcn;
      ls[ST_VIOLATIONS] += ((ml & (mi | mo)) != 0);
      ls[ST_CHECKSUM] += orc_checksum_cv(goff + g, c, v, (uint32_t)gcn, (uint32_t)rcn);
    }
#pragma omp critical
    for (int k = 0; k < NSTAT; k++) st[k] += ls[k];
  }
  if (stats)
    for (int k = 0; k < NSTAT; k++) stats[k] += st[k];
}

/* Generate a batch on the host (same layout as qe_gen_groups).  Mask
 * pointers may be NULL to skip them. */
void orc_gen_batch(uint64_t G, uint64_t goff, uint32_t S, uint64_t stride, uint64_t seed,
                   uint32_t dist, uint32_t p_absent, uint32_t p_voted, uint32_t p_granted,
                   uint32_t n_inc, uint32_t n_out, uint32_t mask_mode, uint64_t *match,
                   void *inc, void *out, void *learner, void *voted, void *granted,
                   int threads) {
  uint32_t mb = S <= 8 ? 1 : 2;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel for schedule(static)
  for (int64_t gi = 0; gi < (int64_t)G; gi++) {
    uint64_t g = (uint64_t)gi;
    uint64_t vals[16];
    uint32_t mi, mo, ml, vd, gr;
    orc_gen_group(seed, goff + g, S, dist, p_absent, p_voted, p_granted, n_inc, n_out,
                  mask_mode, vals, &mi, &mo, &ml, &vd, &gr);
    if (match)
      for (uint32_t s = 0; s < S; s++) match[s * stride + g] = vals[s];
    if (inc) st_mask(inc, mb, g, mi);
    if (out) st_mask(out, mb, g, mo);
    if (learner) st_mask(learner, mb, g, ml);
    if (voted) st_mask(voted, mb, g, vd);
    if (granted) st_mask(granted, mb, g, gr);
  }
}

void orc_quorum_active_batch(uint64_t G, uint32_t S, const void *inc, const void *out,
                             const void *learner, const void *recent, uint8_t *active) {
  uint32_t mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  for (uint64_t g = 0; g < G; g++) {
    uint32_t mi = inc ? ld_mask(inc, mb, g) & full : full;
    active[g] = orc_quorum_active(mi, ld_mask(out, mb, g) & full, ld_mask(learner, mb, g) & full,
                                  ld_mask(recent, mb, g) & full);
  }
}

void orc_record_votes_batch(uint64_t G, uint32_t S, void *voted, void *granted,
                            const void *resp, const void *value) {
  uint32_t mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  for (uint64_t g = 0; g < G; g++) {
    uint32_t vd = ld_mask(voted, mb, g), gr = ld_mask(granted, mb, g);
    orc_record_votes(&vd, &gr, ld_mask(resp, mb, g) & full, ld_mask(value, mb, g) & full);
    st_mask(voted, mb, g, vd);
    st_mask(granted, mb, g, gr);
  }
}

/* qe_replication_round restated. */
uint64_t orc_checksum_repl(uint64_t gid, uint64_t committed, uint32_t read_ok, uint32_t adv) {
  uint64_t tag = ((uint64_t)read_ok << 62) | ((uint64_t)adv << 61);
  return orc_mix64((gid * PHI) ^ committed ^ tag);
}

void orc_replication_round_batch(uint64_t G, uint64_t goff, uint32_t S, uint64_t stride,
                                 uint64_t *match, uint64_t *next, uint64_t *committed,
                                 const uint64_t *term_start, const uint64_t *last_index,
                                 const void *inc, const void *out, const uint64_t *resp_index,
                                 const void *resp_mask, const void *read_acks, uint8_t *read_ok,
                                 uint8_t *adv_out, uint64_t *stats, int threads) {
  uint32_t mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  uint64_t st[NSTAT];
  memset(st, 0, sizeof(st));
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    uint64_t ls[NSTAT];
    memset(ls, 0, sizeof(ls));
#pragma omp for schedule(static)
    for (int64_t gi = 0; gi < (int64_t)G; gi++) {
      uint64_t g = (uint64_t)gi;
      uint32_t mi = inc ? ld_mask(inc, mb, g) & full : full;
      uint32_t mo = out ? ld_mask(out, mb, g) & full : 0;
      uint32_t rm = ld_mask(resp_mask, mb, g) & full;
      uint64_t vals[16];
      for (uint32_t s = 0; s < S; s++) {
        uint64_t m = match[s * stride + g], n = next[s * stride + g];
        if ((rm >> s) & 1u) orc_maybe_update(&m, &n, resp_index[s * stride + g]);
        match[s * stride + g] = m;
        next[s * stride + g] = n;
        vals[s] = m;
      }
      uint64_t mci = orc_joint_committed(S, mi, mo, vals);
      uint64_t c = committed[g];
      int adv = orc_maybe_commit(mci, &c, term_start[g], last_index[g]);
      committed[g] = c;
      uint32_t ro = 0;
      if (read_acks) {
        uint32_t acks = ld_mask(read_acks, mb, g) & full;
        ro = orc_joint_vote(mi, mo, acks, acks) == VOTE_WON;
        if (read_ok) read_ok[g] = (uint8_t)ro;
      }
      if (adv_out) adv_out[g] = (uint8_t)adv;
      ls[ST_GROUPS] += 1;
      ls[ST_COMMIT_SUM] += c;
      ls[ST_COMMIT_ADVANCED] += (uint64_t)adv;
      ls[ST_READ_RELEASED] += ro;
      ls[ST_VIOLATIONS] += (mci > last_index[g]);
      ls[ST_CHECKSUM] += orc_checksum_repl(goff + g, c, ro, (uint32_t)adv);
    }
#pragma omp critical
    for (int k = 0; k < NSTAT; k++) st[k] += ls[k];
  }
  if (stats)
    for (int k = 0; k < NSTAT; k++) stats[k] += st[k];
}

/* ------------------------------------------------------------------------ */
/* Election simulation (qe_election_steps restated)            */
/* ------------------------------------------------------------------------ */
uint64_t orc_checksum_elec(uint64_t gid, uint64_t term, uint32_t state, uint32_t voted, uint32_t granted) {
  uint64_t tag = ((uint64_t)state << 62) | ((uint64_t)voted << 40) | ((uint64_t)granted << 24);
  return orc_mix64((gid * PHI) ^ term ^ tag);
}

/* One TallyVotes (raft.go:837-845, tracker.go:267-288) with the invariant
 * checks of DESIGN.md §5: the result is symmetric in the halves, VoteWon
 * implies a granted quorum in both halves, and the granted count never
 * falls within a term (gbefore). */
static uint8_t elec_tally(uint32_t mi, uint32_t mo, uint32_t ml, uint32_t vd, uint32_t gr,
                          uint32_t gbefore, uint64_t *ls) {
  int gcn, rcn;
  uint8_t res = orc_tally(mi, mo, ml, vd, gr, &gcn, &rcn);
  uint8_t sym = orc_joint_vote(mo, mi, vd, gr);
  int n0 = popc(mi), n1 = popc(mo);
  int won_ok = (n0 == 0 || popc(gr & vd & mi) >= n0 / 2 + 1) &&
               (n1 == 0 || popc(gr & vd & mo) >= n1 / 2 + 1);
  ls[ST_VIOLATIONS] += (uint64_t)(sym != res) + (uint64_t)(res == VOTE_WON && !won_ok) +
                       (uint64_t)((uint32_t)gcn < gbefore);
  ls[ST_GRANTED] += (uint64_t)gcn;
  ls[ST_REJECTED] += (uint64_t)rcn;
  ls[res == VOTE_WON ? ST_WON : (res == VOTE_LOST ? ST_LOST : ST_PENDING)] += 1;
  return res;
}

/* Counter-based response RNG: per group gkey = mix64(seed +
 * gid*PHI) ^ IV folded to 32 bits (k = lo ^ hi); slot s at step t draws
 * d = fmix32(k + t*C1 + s*C2) (MurmurHash3's 32-bit finalizer), bits 0-15
 * the drop draw and bits 16-31 the grant draw; the CheckQuorum activity
 * draw of a leader's peer is bits 0-15 of fmix32(k + t*C1 + s*C2 + C3). */
static const uint64_t ELEC_IV = 0x6A09E667F3BCC909ULL;
static const uint32_t ELEC_C1 = 0x9E3779B1u, ELEC_C2 = 0x85EBCA77u, ELEC_C3 = 0x27D4EB2Fu;
static inline uint32_t elec_gkey(uint64_t seed, uint64_t gid) {
  uint64_t k = orc_mix64(seed + gid * PHI) ^ ELEC_IV;
  return (uint32_t)k ^ (uint32_t)(k >> 32);
}
static inline uint32_t orc_fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
static inline uint32_t elec_draw(uint32_t gkey, uint64_t step, uint32_t s) {
  return orc_fmix32(gkey + (uint32_t)step * ELEC_C1 + s * ELEC_C2);
}

#define ELEC_PREVOTE 1u
#define ELEC_CHECK_QUORUM 2u
enum { SF = 0, SC = 1, SL = 2, SP = 3 }; /* StateFollower/Candidate/Leader/PreCandidate */

/* raft.campaign (raft.go:785-803) of a promotable node: PreVote ->
 * becomePreCandidate (votes reset, term kept), else becomeCandidate (term+1,
 * votes reset); the self-vote poll; a won (single-voter) pre-vote goes on to
 * campaign(campaignElection) and a won election to becomeLeader. */
static void elec_campaign(int pre, uint32_t mi, uint32_t mo, uint32_t ml, uint32_t self,
                          uint64_t *t, uint32_t *sta, uint32_t *vd, uint32_t *gr, uint64_t *ls) {
  if (pre) {
    *sta = SP;                                   /* becomePreCandidate (:708-722) */
    *vd = 0; *gr = 0;
    orc_record_votes(vd, gr, self, self);
    if (elec_tally(mi, mo, ml, *vd, *gr, 0, ls) != VOTE_WON) return;
  }
  *t += 1;                                       /* becomeCandidate (:695-706) */
  *sta = SC;
  *vd = 0; *gr = 0;
  orc_record_votes(vd, gr, self, self);
  ls[ST_ELECTIONS] += 1;
  if (elec_tally(mi, mo, ml, *vd, *gr, 0, ls) == VOTE_WON) {
    *sta = SL;                                   /* becomeLeader */
    ls[ST_LEADERS] += 1;
  }
}

/* `steps` election steps per group.  Per step:
 *   Leader     CheckQuorum on: one CheckQuorum round (raft.go:997-1018): its
 *              peers' RecentActive from the activity draw (or the script),
 *              self active; !QuorumActive -> becomeFollower (term kept).
 *              CheckQuorum off: the leader is deposed and campaigns (the
 *              simulation keeps elections going).
 *   Follower, or a (pre)candidate whose election timeout fires (script_hup):
 *              hup -> campaign (pre-vote first when PreVote is on).
 *   PreCandidate / Candidate: one round of (pre)vote responses from every
 *              other voter (campaign sends to Voters.IDs(), :813-834):
 *              RecordVote + TallyVotes (stepCandidate, :1399-1414): won ->
 *              campaign(campaignElection) / becomeLeader; lost ->
 *              becomeFollower (term kept); pending -> stay.
 * Non-promotable nodes (no Progress, or a learner, :1618-1623) never step.
 * Script arrays ([steps][sstride]) replace the RNG when sresp != NULL. */
void orc_election_steps_batch(uint64_t G, uint64_t goff, uint32_t S, uint64_t *term,
                              uint8_t *state, void *voted, void *granted, const uint8_t *self_slot,
                              const void *inc, const void *out, const void *learner,
                              uint64_t seed, uint64_t step0, uint32_t steps, uint32_t p_drop,
                              uint32_t p_grant, uint32_t flags, uint32_t p_active,
                              const void *sresp, const void *sgrant, const uint8_t *shup,
                              uint64_t sstride, uint64_t *stats, int threads) {
  uint32_t mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  uint64_t st[NSTAT];
  memset(st, 0, sizeof(st));
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    uint64_t ls[NSTAT];
    memset(ls, 0, sizeof(ls));
#pragma omp for schedule(static)
    for (int64_t gi = 0; gi < (int64_t)G; gi++) {
      uint64_t g = (uint64_t)gi, gid = goff + g;
      uint32_t mi = inc ? ld_mask(inc, mb, g) & full : full;
      uint32_t mo = out ? ld_mask(out, mb, g) & full : 0;
      uint32_t ml = ld_mask(learner, mb, g) & full;
      uint32_t self = 1u << (self_slot[g] % S);
      uint32_t voters = mi | mo;
      /* raft.promotable(): own Progress exists and is not a learner */
      int promotable = (self & voters) != 0 && (self & ml) == 0;
      uint64_t t = term[g];
      uint32_t sta = state[g];
      uint32_t vd = ld_mask(voted, mb, g) & full, gr = ld_mask(granted, mb, g) & full;
      const uint32_t gkey = elec_gkey(seed, gid);
      for (uint32_t k = 0; k < steps && promotable; k++) {
        uint64_t step = step0 + k;
        uint32_t peers = voters & ~self;
        uint32_t resp = 0, val = 0;
        if (sresp) {
          resp = ld_mask(sresp, mb, k * sstride + g) & peers;
          val = ld_mask(sgrant, mb, k * sstride + g) & resp;
        }
        int hup = shup ? shup[k * sstride + g] != 0 : 0;
        if (sta == SL && (flags & ELEC_CHECK_QUORUM)) {
          if (!sresp)
            for (uint32_t s = 0; s < S; s++) {
              if (!((peers >> s) & 1u)) continue;
              uint32_t d = orc_fmix32(gkey + (uint32_t)step * ELEC_C1 + s * ELEC_C2 + ELEC_C3);
              if ((d & 0xFFFFu) < p_active) resp |= 1u << s;
            }
          uint32_t recent = resp | self;  /* the leader always sees itself active */
          uint8_t qa = orc_quorum_active(mi, mo, ml, recent);
          ls[ST_VIOLATIONS] += (uint64_t)(qa != orc_quorum_active(mo, mi, ml, recent));
          if (!qa) {
            sta = SF;                      /* becomeFollower(r.Term, None) */
            ls[ST_STEPDOWNS] += 1;
          }
        } else if (sta == SF || sta == SL || hup) {
          elec_campaign((flags & ELEC_PREVOTE) != 0, mi, mo, ml, self, &t, &sta, &vd, &gr, ls);
        } else {
          if (!sresp)
            for (uint32_t s = 0; s < S; s++) {
              if (!((peers >> s) & 1u)) continue;
              uint32_t d = elec_draw(gkey, step, s);
              if ((d & 0xFFFFu) < p_drop) continue; /* dropped */
              resp |= 1u << s;
              if ((d >> 16) < p_grant) val |= 1u << s;
            }
          uint32_t gbefore = (uint32_t)popc(gr & vd & ~ml & voters);
          orc_record_votes(&vd, &gr, resp, val); /* RecordVote, :844 */
          uint8_t res = elec_tally(mi, mo, ml, vd, gr, gbefore, ls);
          if (res == VOTE_WON) {
            if (sta == SP) {
              elec_campaign(0, mi, mo, ml, self, &t, &sta, &vd, &gr, ls);
            } else {
              sta = SL;
              ls[ST_LEADERS] += 1;
            }
          } else if (res == VOTE_LOST) {
            sta = SF;
            ls[ST_STEPDOWNS] += 1;
          }
        }
        ls[ST_GROUPS] += 1;
      }
      term[g] = t;
      state[g] = (uint8_t)sta;
      st_mask(voted, mb, g, vd);
      st_mask(granted, mb, g, gr);
      ls[ST_CHECKSUM] += orc_checksum_elec(gid, t, sta, vd, gr);
    }
#pragma omp critical
    for (int k = 0; k < NSTAT; k++) st[k] += ls[k];
  }
  if (stats)
    for (int k = 0; k < NSTAT; k++) stats[k] += st[k];
}

/* ------------------------------------------------------------------------ */
/* "Go-faithful" CPU baseline: the reference's per-group loop over maps.     */
/* MajorityConfig/JointConfig are hash sets of voter IDs, the AckedIndexer   */
/* is ProgressTracker.Progress (map id -> *Progress, tracker.go:162-173) and */
/* Votes is a map id -> bool.  CommittedIndex iterates the set, looks each   */
/* id up, fills a stack array and insertion-sorts it (majority.go:126-172).  */
/* ------------------------------------------------------------------------ */
typedef struct gf_progress {          /* raft/tracker/progress.go:30-80 (56 B) */
  uint64_t match, next;
  uint64_t state, pending_snapshot;
  uint8_t recent_active, probe_sent, is_learner, pad[5];
  void *inflights;
  uint64_t pad2;
} gf_progress;

#define GF_BUCKETS 16
typedef struct gf_group {
  uint64_t cfg_ids[2][GF_BUCKETS];    /* open-addressed sets, 0 = empty slot */
  uint64_t prog_ids[GF_BUCKETS];
  gf_progress *prog[GF_BUCKETS];
  uint64_t vote_ids[GF_BUCKETS];
  uint8_t vote_val[GF_BUCKETS];
  int n[2];
} gf_group;

static inline uint32_t gf_slot(uint64_t id) { return (uint32_t)(orc_mix64(id) & (GF_BUCKETS - 1)); }
static void gf_insert(uint64_t *keys, uint64_t id, uint32_t *where) {
  uint32_t b = gf_slot(id);
  while (keys[b] != 0 && keys[b] != id) b = (b + 1) & (GF_BUCKETS - 1);
  keys[b] = id;
  if (where) *where = b;
}
static inline int gf_find(const uint64_t *keys, uint64_t id, uint32_t *where) {
  uint32_t b = gf_slot(id);
  for (int i = 0; i < GF_BUCKETS; i++) {
    if (keys[b] == id) { *where = b; return 1; }
    if (keys[b] == 0) return 0;
    b = (b + 1) & (GF_BUCKETS - 1);
  }
  return 0;
}

typedef struct gf_world {
  uint64_t G;
  gf_group *groups;
  gf_progress *arena;
} gf_world;

/* Build the map-based world from a slot-SoA batch (setup, not timed).  Peer
 * IDs are 1 + slot + 32 * (g % 1024) so they differ across groups. */
void *orc_gf_build(uint64_t G, uint32_t S, uint64_t stride, const uint64_t *match,
                   const void *inc, const void *out, const void *learner, const void *voted,
                   const void *granted) {
  uint32_t mb = S <= 8 ? 1 : 2, full = (1u << S) - 1u;
  gf_world *w = (gf_world *)calloc(1, sizeof(gf_world));
  w->G = G;
  w->groups = (gf_group *)calloc(G, sizeof(gf_group));
  w->arena = (gf_progress *)calloc(G * S, sizeof(gf_progress));
  for (uint64_t g = 0; g < G; g++) {
    gf_group *gp = &w->groups[g];
    uint32_t mi = inc ? ld_mask(inc, mb, g) & full : full;
    uint32_t mo = out ? ld_mask(out, mb, g) & full : 0;
    uint32_t ml = ld_mask(learner, mb, g) & full;
    uint32_t vd = ld_mask(voted, mb, g) & full, gr = ld_mask(granted, mb, g) & full;
    gp->n[0] = popc(mi);
    gp->n[1] = popc(mo);
    for (uint32_t s = 0; s < S; s++) {
      uint64_t id = 1 + s + 32 * (g % 1024);
      if ((mi >> s) & 1u) gf_insert(gp->cfg_ids[0], id, NULL);
      if ((mo >> s) & 1u) gf_insert(gp->cfg_ids[1], id, NULL);
      if (((mi | mo | ml) >> s) & 1u) {
        uint32_t b;
        gf_insert(gp->prog_ids, id, &b);
        /* scatter Progress structs like heap allocations: a bijective
         * multiplicative permutation of the arena (2654435761 is prime). */
        uint64_t n_ar = G * S;
        uint64_t slot = (uint64_t)(((unsigned __int128)(g * S + s) * 2654435761ULL) % n_ar);
        gf_progress *pr = &w->arena[slot];
        pr->match = match[s * stride + g];
        pr->next = pr->match + 1;
        pr->is_learner = (uint8_t)((ml >> s) & 1u);
        gp->prog[b] = pr;
      }
      if ((vd >> s) & 1u) {
        uint32_t b;
        gf_insert(gp->vote_ids, id, &b);
        gp->vote_val[b] = (uint8_t)((gr >> s) & 1u);
      }
    }
  }
  return w;
}

void orc_gf_free(void *p) {
  gf_world *w = (gf_world *)p;
  if (!w) return;
  free(w->groups);
  free(w->arena);
  free(w);
}

static uint64_t gf_majority_committed(const gf_group *gp, int half) {
  int n = gp->n[half];
  if (n == 0) return ORC_INF;
  uint64_t stk[7];
  uint64_t heap[GF_BUCKETS];
  uint64_t *srt = n <= 7 ? stk : heap;
  memset(srt, 0, sizeof(uint64_t) * (size_t)n);
  int i = n - 1;
  for (int b = 0; b < GF_BUCKETS; b++) { /* for id := range c */
    uint64_t id = gp->cfg_ids[half][b];
    if (!id) continue;
    uint32_t w;
    if (gf_find(gp->prog_ids, id, &w)) { /* matchAckIndexer.AckedIndex */
      srt[i--] = gp->prog[w]->match;
    }
  }
  insertion_sort(srt, n);
  return srt[n - (n / 2 + 1)];
}

static uint8_t gf_majority_vote(const gf_group *gp, int half) {
  int n = gp->n[half];
  if (n == 0) return VOTE_WON;
  int ny[2] = {0, 0}, missing = 0;
  for (int b = 0; b < GF_BUCKETS; b++) {
    uint64_t id = gp->cfg_ids[half][b];
    if (!id) continue;
    uint32_t w;
    if (!gf_find(gp->vote_ids, id, &w)) { missing++; continue; }
    ny[gp->vote_val[w]]++;
  }
  int q = n / 2 + 1;
  if (ny[1] >= q) return VOTE_WON;
  if (ny[1] + missing >= q) return VOTE_PENDING;
  return VOTE_LOST;
}

/* Timed loop: JointConfig.CommittedIndex + JointConfig.VoteResult per group,
 * `reps` passes.  Returns elapsed seconds; writes outputs of the last pass. */
double orc_gf_run(void *p, uint64_t *commit, uint8_t *vote, int reps, int threads) {
  gf_world *w = (gf_world *)p;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int r = 0; r < reps; r++) {
#pragma omp parallel for schedule(static)
    for (int64_t gi = 0; gi < (int64_t)w->G; gi++) {
      const gf_group *gp = &w->groups[gi];
      uint64_t a = gf_majority_committed(gp, 0), b = gf_majority_committed(gp, 1);
      uint8_t r1 = gf_majority_vote(gp, 0), r2 = gf_majority_vote(gp, 1);
      uint8_t v = (r1 == r2) ? r1 : ((r1 == VOTE_LOST || r2 == VOTE_LOST) ? VOTE_LOST : VOTE_PENDING);
      commit[gi] = a < b ? a : b;
      vote[gi] = v;
    }
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* Timed SoA restatement (strongest CPU variant): returns elapsed seconds. */
double orc_soa_run(uint64_t G, uint32_t S, uint64_t stride, const uint64_t *match,
                   const void *inc, const void *out, const void *voted, const void *granted,
                   uint64_t *commit, uint8_t *vote, int reps, int threads) {
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int r = 0; r < reps; r++)
    orc_commit_vote_batch(G, 0, S, stride, match, inc, out, NULL, voted, granted, commit, vote,
                          NULL, NULL, NULL, 0, threads);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

int orc_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------------------ */
/* Progress state machine: MsgAppResp accept /   */
/* reject, MsgHeartbeatResp, inflights, and the send side.                  */
/* ------------------------------------------------------------------------ */
enum { PR_PROBE = 0, PR_REPLICATE = 1, PR_SNAPSHOT = 2 };
#define PF_STATE 3u
#define PF_PROBE_SENT 4u
#define PF_RECENT_ACTIVE 8u
/* bits of the device word that describe the ring's representation (ABI 4,
 * QE_PW_RING_MASK), not Progress state: ignored here */
#define PW_RING_MASK 0xFF0000F0u

typedef struct orc_pr {
  uint64_t match, next, pending;
  uint32_t state, probe_sent, recent_active;
  uint32_t start, count, size; /* Inflights (raft/tracker/inflights.go:22-36) */
  uint64_t *buf;               /* strided view: buf[k * bstride] */
  uint64_t bstride;
  uint32_t reset;              /* ResetState ran this round (byte accounting) */
  uint64_t *acct;              /* byte accounting sink, or NULL             */
  uint32_t eb;                 /* bytes of one Inflights entry in the device
                                  form: 4 (32-bit words), 2 (ABI 8 infl16)   */
} orc_pr;

static inline uint64_t *ib(orc_pr *p, uint32_t k) { return &p->buf[(uint64_t)k * p->bstride]; }

/* inflights.go:55-71 Add (accounting: the entry written, 4 B -- the 32-bit
 * entry word of the device representation, ABI 4; 2 B in the 16-bit form,
 * ABI 8; the upper words of a ring straddling a 2^32 boundary, and the
 * 16-bit form's re-based offsets, are representation overhead, not
 * counted) */
static void infl_add(orc_pr *p, uint64_t x) {
  uint32_t nx = p->start + p->count;
  if (nx >= p->size) nx -= p->size;
  *ib(p, nx) = x;
  p->count++;
  if (p->acct) *p->acct += p->eb;
}
/* inflights.go:87-113 FreeLE (accounting: every entry the loop reads,
 * min(count, freed + 1) of them, eb bytes each as in infl_add) */
static void infl_free_le(orc_pr *p, uint64_t to) {
  if (p->count == 0) return;
  if (to < *ib(p, p->start)) {
    if (p->acct) *p->acct += p->eb;
    return;
  }
  uint32_t idx = p->start, i;
  for (i = 0; i < p->count; i++) {
    if (to < *ib(p, idx)) break;
    if (++idx >= p->size) idx -= p->size;
  }
  if (p->acct) *p->acct += p->eb * (uint64_t)(i < p->count ? i + 1 : i);
  p->count -= i;
  p->start = idx;
  if (p->count == 0) p->start = 0;
}
static int infl_full(const orc_pr *p) { return p->count == p->size; }

/* progress.go:84-90 ResetState */
static void pr_reset_state(orc_pr *p, uint32_t st) {
  p->reset = 1;
  p->probe_sent = 0;
  p->pending = 0;
  p->state = st;
  p->count = 0; /* Inflights.reset */
  p->start = 0;
}
/* progress.go:112-125 BecomeProbe */
static void pr_become_probe(orc_pr *p) {
  if (p->state == PR_SNAPSHOT) {
    uint64_t ps = p->pending;
    pr_reset_state(p, PR_PROBE);
    uint64_t a = p->match + 1, b = ps + 1;
    p->next = a > b ? a : b;
  } else {
    pr_reset_state(p, PR_PROBE);
    p->next = p->match + 1;
  }
}
/* progress.go:127-131 BecomeReplicate */
static void pr_become_replicate(orc_pr *p) {
  pr_reset_state(p, PR_REPLICATE);
  p->next = p->match + 1;
}
/* progress.go:135-139 BecomeSnapshot */
static void pr_become_snapshot(orc_pr *p, uint64_t snap) {
  pr_reset_state(p, PR_SNAPSHOT);
  p->pending = snap;
}
/* progress.go:144-153 MaybeUpdate */
static int pr_maybe_update(orc_pr *p, uint64_t n) {
  int updated = 0;
  if (p->match < n) {
    p->match = n;
    updated = 1;
    p->probe_sent = 0; /* ProbeAcked */
  }
  if (p->next < n + 1) p->next = n + 1;
  return updated;
}
/* progress.go:170-193 MaybeDecrTo */
static int pr_maybe_decr_to(orc_pr *p, uint64_t rejected, uint64_t hint) {
  if (p->state == PR_REPLICATE) {
    if (rejected <= p->match) return 0;
    p->next = p->match + 1;
    return 1;
  }
  if (p->next - 1 != rejected) return 0;
  uint64_t m = rejected < hint + 1 ? rejected : hint + 1;
  p->next = m > 1 ? m : 1;
  p->probe_sent = 0;
  return 1;
}
/* progress.go:201-212 IsPaused */
static int pr_is_paused(const orc_pr *p) {
  if (p->state == PR_PROBE) return p->probe_sent;
  if (p->state == PR_REPLICATE) return infl_full(p);
  return 1;
}

/* raftLog.term (raft/log.go:265-285) on the term-run log model: runs r <
 * nruns cover [first[r], first[r+1]) with term[r]; the last run ends at
 * last_index; first[0] is the dummy (snapshot) index.  Out-of-range -> 0. */
uint64_t orc_log_term(uint32_t nruns, const uint64_t *first, const uint64_t *term,
                      uint64_t last_index, uint64_t i) {
  if (nruns == 0 || i < first[0] || i > last_index) return 0;
  uint64_t t = term[0];
  for (uint32_t r = 0; r < nruns; r++)
    if (i >= first[r]) t = term[r];
  return t;
}
/* raftLog.findConflictByTerm (raft/log.go:147-168), linear as written. */
uint64_t orc_find_conflict_by_term(uint32_t nruns, const uint64_t *first, const uint64_t *term,
                                   uint64_t last_index, uint64_t index, uint64_t t) {
  if (index > last_index) return index;
  for (;;) {
    uint64_t lt = orc_log_term(nruns, first, term, last_index, index);
    if (lt <= t) break;
    index--;
  }
  return index;
}

/* The leader-side state of G groups (mirrors qe_progress of
 * include/etcd_quorum.h, except that the Inflights rings are plain uint64
 * as in the reference, entry-major: entry k of slot s of group g at
 * ibuf[(s*F + k)*stride + g]; tests convert through qe_ring_pack /
 * qe_ring_unpack) and one round of peer messages (mirrors qe_peer_msgs).
 * Slot s of group g lives at [s*stride + g].
 * pw is the packed per-peer word: StateType bits 0-1, ProbeSent bit 2,
 * RecentActive bit 3, Inflights.start bits 8-15, Inflights.count 16-23. */
typedef struct orc_prog {
  uint64_t G, goff;
  uint32_t S, F;
  uint64_t stride;
  uint64_t *match, *next, *pending;
  uint32_t *pw;
  uint64_t *ibuf;
  uint64_t *committed;
  const uint64_t *term_start, *first_index, *last_index;
  uint32_t R, reserved;
  const uint64_t *run_first, *run_term;
  const uint8_t *run_count;
  const void *inc, *out;
  const void *tracked;            /* NULL: every slot holds a Progress      */
  const uint8_t *self_slot;       /* NULL / >= S: the leader has no slot    */
  uint8_t *lead_transferee;       /* rw; NULL / >= S: no transfer           */
  const uint64_t *snap_index;     /* NULL: first_index - 1                  */
  uint32_t max_ents, reserved2;   /* entries per MsgApp, 0 = noLimit        */
  /* the ReadIndex queue (qe_progress ABI 5): acks word per group (entry j
   * of mask width at bits [8*mb*j, ...)), context number of entry 0, count */
  void *read_acks;
  uint32_t *read_head;
  uint8_t *read_count;
  /* ABI 7: entries past the word in a ring at context % read_cap (0 = the
   * word alone), the requests' keys likewise (NULL: not tracked) */
  uint32_t read_cap, reserved3;
  void *read_ovf;
  uint64_t *read_keys;
  /* ABI 8: non-NULL = the device keeps the rings in the 16-bit form (the
   * oracle's rings stay uint64; only the byte accounting changes) */
  const void *infl16;
} orc_prog;

typedef struct orc_msgs {
  const uint8_t *type;
  const uint64_t *index, *hint, *logterm;
  void *sent;          /* [G] slots sent >= 1 MsgApp/MsgSnap              */
  uint8_t *bcast;      /* [G] bcastAppend calls (commit advances)         */
  void *snap;          /* [G] slots sent a MsgSnap                        */
  void *timeout_now;   /* [G] slots sent MsgTimeoutNow                    */
  uint8_t *msg_count;  /* [S][stride] messages sent to the peer           */
  uint64_t *msg_index; /* [S][stride] m.Index of the first of them        */
  const uint32_t *read_ctx;   /* [S][stride] context a heartbeat response
                                 carries (0 none); NULL: the newest pending */
  uint8_t *read_released;     /* [G] out: requests released this round    */
  uint8_t *term_commit;       /* [G] out: first commit in the leader's term */
  uint64_t *term_commit_index;/* [G] out: committed right after it          */
  uint64_t *bytes;     /* byte accounting (DESIGN.md §3 rules), or NULL   */
} orc_msgs;

/* message kinds (qe_peer_msgs.type) */
enum { M_NONE = 0, M_APP_RESP, M_APP_RESP_REJECT, M_HEARTBEAT_RESP, M_SNAP_STATUS,
       M_SNAP_STATUS_REJECT, M_UNREACHABLE, M_TRANSFER_LEADER };
#define READ_QUEUE 4 /* QE_READ_QUEUE: the entries of the device form's word */

/* readOnly (raft/read_only.go:39-63) of one group as the reference keeps
 * it: the queue of pending requests in arrival order, each with its
 * context (here its context number) and its acks (a set of slots); at most
 * read_cap (<= 255) of them, the device form's capacity. */
typedef struct orc_ro {
  uint32_t n;                      /* len(readIndexQueue)                  */
  uint32_t ctx[256];               /* readIndexQueue                       */
  uint32_t acks[256];              /* pendingReadIndex[ctx].acks           */
} orc_ro;

static inline uint32_t ro_cap(const orc_prog *a) { return a->read_cap ? a->read_cap : READ_QUEUE; }
static uint32_t ovf_get(const orc_prog *a, uint32_t mb, uint64_t g, uint32_t ctx) {
  uint64_t i = g * ro_cap(a) + ctx % ro_cap(a);
  return mb == 1 ? ((const uint8_t *)a->read_ovf)[i] : ((const uint16_t *)a->read_ovf)[i];
}
static void ovf_set(const orc_prog *a, uint32_t mb, uint64_t g, uint32_t ctx, uint32_t v) {
  uint64_t i = g * ro_cap(a) + ctx % ro_cap(a);
  if (mb == 1) ((uint8_t *)a->read_ovf)[i] = (uint8_t)v;
  else ((uint16_t *)a->read_ovf)[i] = (uint16_t)v;
}

static uint64_t ro_word_get(const void *w, uint32_t mb, uint64_t g) {
  return mb == 1 ? ((const uint32_t *)w)[g] : ((const uint64_t *)w)[g];
}
static void ro_word_set(void *w, uint32_t mb, uint64_t g, uint64_t v) {
  if (mb == 1) ((uint32_t *)w)[g] = (uint32_t)v;
  else ((uint64_t *)w)[g] = v;
}
/* the device form -> the queue: entry j has context head + j; entries
 * j >= READ_QUEUE come from the overflow ring (ABI 7) */
static void ro_load(orc_ro *r, const orc_prog *a, uint64_t g, uint32_t mb) {
  uint64_t word = ro_word_get(a->read_acks, mb, g);
  uint32_t head = a->read_head[g], count = a->read_count[g], cap = ro_cap(a);
  r->n = count < cap ? count : cap;
  for (uint32_t j = 0; j < r->n; j++) {
    r->ctx[j] = head + j;
    r->acks[j] = j < READ_QUEUE ? (uint32_t)(word >> (8 * mb * j)) & ((1u << (8 * mb)) - 1u)
                                : ovf_get(a, mb, g, head + j);
  }
}
/* the queue's entries past the word -> the overflow ring */
static void ro_store_ovf(const orc_ro *r, const orc_prog *a, uint64_t g, uint32_t mb) {
  for (uint32_t j = READ_QUEUE; j < r->n; j++) ovf_set(a, mb, g, r->ctx[j], r->acks[j]);
}
/* the queue -> the device form (entries past the count 0; entries past the
 * word live in the ring only) */
static uint64_t ro_word(const orc_ro *r, uint32_t mb) {
  uint64_t w = 0;
  for (uint32_t j = 0; j < r->n && j < READ_QUEUE; j++) w |= (uint64_t)r->acks[j] << (8 * mb * j);
  return w;
}
/* recvAck (read_only.go:68-76): index of the pending request with context
 * ctx, or -1 (recvAck returns nil: nothing recorded) */
static int ro_find(const orc_ro *r, uint32_t ctx) {
  if (ctx == 0) return -1; /* len(m.Context) == 0 (raft.go:1296) */
  for (uint32_t j = 0; j < r->n; j++)
    if (r->ctx[j] == ctx) return (int)j;
  return -1;
}
/* advance (read_only.go:81-112): dequeue the requests up to and including
 * the one with context ctx; returns how many were released */
static uint32_t ro_advance(orc_ro *r, uint32_t ctx) {
  uint32_t i = 0;
  int found = 0;
  for (uint32_t j = 0; j < r->n; j++) {
    i++;
    if (r->ctx[j] == ctx) {
      found = 1;
      break;
    }
  }
  if (!found) return 0;
  for (uint32_t j = i; j < r->n; j++) {
    r->ctx[j - i] = r->ctx[j];
    r->acks[j - i] = r->acks[j];
  }
  r->n -= i;
  return i;
}

static uint32_t pr_word(const orc_pr *p) {
  return p->state | (p->probe_sent ? PF_PROBE_SENT : 0) | (p->recent_active ? PF_RECENT_ACTIVE : 0) |
         (p->start << 8) | (p->count << 16);
}
static void pr_load2(orc_pr *p, const orc_prog *a, uint32_t s, uint64_t g) {
  uint64_t off = s * a->stride + g;
  uint32_t w = a->pw[off];
  p->match = a->match[off];
  p->next = a->next[off];
  p->pending = a->pending[off];
  p->state = w & PF_STATE;
  p->probe_sent = (w & PF_PROBE_SENT) != 0;
  p->recent_active = (w & PF_RECENT_ACTIVE) != 0;
  p->start = (w >> 8) & 0xFFu;
  p->count = (w >> 16) & 0xFFu;
  p->size = a->F;
  p->buf = a->ibuf + (uint64_t)s * a->F * a->stride + g; /* entry k at buf[k*stride] */
  p->bstride = a->stride;
  p->reset = 0;
  p->acct = NULL;
  p->eb = a->infl16 ? 2 : 4;
}
static void pr_store2(const orc_pr *p, const orc_prog *a, uint32_t s, uint64_t g) {
  uint64_t off = s * a->stride + g;
  a->match[off] = p->match;
  a->next[off] = p->next;
  a->pending[off] = p->pending;
  a->pw[off] = pr_word(p);
}

/* Per-group context of one round: the log model and the message record. */
typedef struct orc_gctx {
  const orc_prog *a;
  const orc_msgs *m;
  uint64_t g, fi, li, snap;
  uint32_t me, sent, snapm;
} orc_gctx;

static void rec_msg(orc_gctx *c, uint32_t s, uint64_t index) {
  uint64_t off = s * c->a->stride + c->g;
  if (c->m && c->m->msg_count) {
    if (c->m->msg_count[off] == 0 && c->m->msg_index) c->m->msg_index[off] = index;
    if (c->m->msg_count[off] < 255) c->m->msg_count[off]++;
  }
  c->sent |= 1u << s;
}

/* raft.maybeSendAppend (raft/raft.go:432-492) on the log model: entries
 * exist in [first_index, last_index]; term(i) never fails (log.go:265-271
 * returns 0, nil outside [dummy, last]), entries(Next) is (nil, nil) for
 * Next > lastIndex (:287-291) and ErrCompacted for Next < firstIndex
 * (:381-388).  The `len(ents) == 0 && !sendIfEmpty` return (:442-444) comes
 * BEFORE the snapshot branch (:446-469).  max_ents models MaxSizePerMsg for
 * equal-size entries (limitSize keeps at least one entry); 0 = noLimit. */
static int send_append(orc_gctx *c, orc_pr *p, uint32_t s, int send_if_empty) {
  if (pr_is_paused(p)) return 0;                       /* :434-436 */
  if (p->next > c->li) {                               /* no entries */
    if (!send_if_empty) return 0;
    rec_msg(c, s, p->next - 1);                        /* empty MsgApp (commit) */
    return 1;
  }
  if (p->next < c->fi) {                               /* ErrCompacted */
    if (!send_if_empty) return 0;                      /* :442-444 */
    if (!p->recent_active) return 0;                   /* :447-450 */
    pr_become_snapshot(p, c->snap);                    /* :468 */
    rec_msg(c, s, c->snap);
    c->snapm |= 1u << s;
    return 1;
  }
  uint64_t last = c->li;
  if (c->me) {
    uint64_t l = p->next + (c->me - 1);
    if (l >= p->next && l < last) last = l;
  }
  rec_msg(c, s, p->next - 1);                          /* MsgApp Index = Next-1 */
  if (p->state == PR_REPLICATE) {                      /* :478-482 */
    p->next = last + 1;                                /* OptimisticUpdate */
    infl_add(p, last);
  } else if (p->state == PR_PROBE) {                   /* :483-484 */
    p->probe_sent = 1;
  }
  return 1;
}

/* Per-group parts: (commit, bcast count), the sent mask, the ReadIndex
 * requests released, the first commit in the leader's term and a changed
 * lead transferee. */
uint64_t orc_checksum_step(uint64_t gid, uint64_t committed, uint32_t send, uint32_t bcast,
                           uint32_t released, int term_commit, uint64_t term_commit_index,
                           int lt_changed, uint32_t lt) {
  uint64_t h = gid * PHI;
  return orc_mix64(h ^ committed ^ ((uint64_t)bcast << 62)) +
         orc_mix64(h ^ ((uint64_t)send << 40) ^ 0xD1B54A32D192ED03ull) +
         (released ? orc_mix64(h ^ 0x8CB92BA72F3D8DD7ull ^ ((uint64_t)released << 56)) : 0) +
         (term_commit ? orc_mix64(h ^ 0x589965CC75374CC3ull ^ term_commit_index) : 0) +
         (lt_changed ? orc_mix64(h ^ 0x1D8E4E27C47D124Full ^ lt) : 0);
}

/* One round of leader-side message handling per group, messages taken in
 * slot order (stepLeader, raft/raft.go:1099-1338), sends executed inline
 * exactly where the reference executes them:
 *   MsgAppResp reject  RecentActive; findConflictByTerm (log.go:147-168)
 *                      when LogTerm > 0; MaybeDecrTo -> (Replicate ->
 *                      BecomeProbe), sendAppend                 :1107-1236
 *   MsgAppResp accept  RecentActive; oldPaused; MaybeUpdate -> Probe ->
 *                      BecomeReplicate / Snapshot caught up -> BecomeProbe
 *                      + BecomeReplicate / Replicate -> FreeLE; maybeCommit
 *                      -> bcastAppend (every other peer, sendIfEmpty), else
 *                      sendAppend if oldPaused; then
 *                      `for maybeSendAppend(from, false) {}`; MsgTimeoutNow
 *                      to the lead transferee once Match == lastIndex
 *                                                               :1237-1282
 *   MsgHeartbeatResp   RecentActive, ProbeSent = false, FreeFirstOne when
 *                      the inflights are full, sendAppend if Match <
 *                      lastIndex                                :1284-1294
 *   MsgSnapStatus      in StateSnapshot only: (reject -> PendingSnapshot =
 *                      0), BecomeProbe, ProbeSent = true        :1310-1331
 *   MsgUnreachable     Replicate -> BecomeProbe                 :1332-1338
 *   MsgTransferLeader  learner: ignored; same transferee: ignored; another
 *                      in progress: aborted; to self: ignored; else
 *                      leadTransferee = from, MsgTimeoutNow if its Match ==
 *                      lastIndex, else sendAppend             :1339-1370
 * MsgHeartbeatResp under ReadOnlySafe with a context: recvAck, and
 * VoteResult(acks) == VoteWon -> readOnly.advance (:1296-1309).  Every
 * maybeCommit that returns true calls releasePendingReadIndexMessages
 * (:1259-1262), which answers the postponed MsgReadIndex requests once
 * committedEntryInCurrentTerm holds (:1813-1825): reported as term_commit
 * with the committed index at that moment.
 * A message from a slot without a Progress is dropped (:1100-1104).  The
 * commit gate is raftLog.maybeCommit on the log model (term(i) == Term <=>
 * term_start <= i <= last_index, log.go:325-331).  An accept beyond
 * lastIndex is processed as the reference does and also counted as an
 * invariant violation (a follower cannot ack entries the leader lacks). */
void orc_progress_step_batch(const orc_prog *a, const orc_msgs *m, uint64_t *stats, int threads) {
  uint32_t S = a->S, mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  uint64_t st[NSTAT];
  uint64_t bytes = 0;
  memset(st, 0, sizeof(st));
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    uint64_t ls[NSTAT];
    uint64_t lbytes = 0;
    memset(ls, 0, sizeof(ls));
#pragma omp for schedule(static)
    for (int64_t gi = 0; gi < (int64_t)a->G; gi++) {
      uint64_t g = (uint64_t)gi;
      orc_gctx c;
      c.a = a;
      c.m = m;
      c.g = g;
      c.fi = a->first_index[g];
      c.li = a->last_index[g];
      c.snap = a->snap_index ? a->snap_index[g] : c.fi - 1;
      c.me = a->max_ents;
      c.sent = c.snapm = 0;
      uint32_t mi = a->inc ? ld_mask(a->inc, mb, g) & full : full;
      uint32_t mo = a->out ? ld_mask(a->out, mb, g) & full : 0;
      uint32_t trk = a->tracked ? ld_mask(a->tracked, mb, g) & full : full;
      uint32_t self = a->self_slot ? a->self_slot[g] : 0xFFu;
      uint32_t lt = a->lead_transferee ? a->lead_transferee[g] : 0xFFu, lt0 = lt;
      uint64_t ts = a->term_start[g], li = c.li, cm = a->committed[g], c0 = cm;
      uint32_t nr = a->run_count[g] < a->R ? a->run_count[g] : a->R;
      uint64_t rf[16], rt[16];
      for (uint32_t r = 0; r < nr; r++) {
        rf[r] = a->run_first[r * a->stride + g];
        rt[r] = a->run_term[r * a->stride + g];
      }
      /* ReadOnlySafe: the leader's readOnly queue (read_only.go:39-63) */
      int rd = a->read_acks != NULL;
      orc_ro ro;
      uint64_t rword0 = 0;
      uint32_t rhead0 = 0, rn0 = 0, released = 0, dctx = 0;
      int rtouch = 0;
      ro.n = 0;
      uint64_t ovfB = 0; /* overflow-ring bytes (ABI 7) */
      if (rd) {
        rword0 = ro_word_get(a->read_acks, mb, g);
        rhead0 = a->read_head[g];
        ro_load(&ro, a, g, mb);
        rn0 = ro.n;
        /* lastPendingRequestCtx (raft.go:525-532) */
        dctx = ro.n ? ro.ctx[ro.n - 1] : 0;
      }
      int first_commit = 1;
      uint64_t tci = 0;
      /* byte accounting (only when m->bytes): everything the round needs,
       * field granularity, each once */
      uint64_t B = 0;
      orc_pr prs[16];
      uint64_t vals[16], match0[16], next0[16], pend0[16];
      uint32_t word0[16], state0[16];
      for (uint32_t s = 0; s < S; s++) {
        pr_load2(&prs[s], a, s, g);
        if (m->bytes) prs[s].acct = &B;
        match0[s] = prs[s].match;
        next0[s] = prs[s].next;
        pend0[s] = prs[s].pending;
        word0[s] = a->pw[s * a->stride + g] & ~PW_RING_MASK;
        state0[s] = prs[s].state;
        if (m->msg_count) m->msg_count[s * a->stride + g] = 0;
      }
      uint32_t bc = 0, tnow = 0, runs_read = 0;
      for (uint32_t s = 0; s < S; s++) {
        if (!((trk >> s) & 1u)) continue; /* no Progress: dropped */
        uint64_t off = s * a->stride + g;
        uint32_t ty = m->type[off];
        orc_pr *p = &prs[s];
        if (ty == M_APP_RESP_REJECT) {
          p->recent_active = 1;
          uint64_t probe = m->hint[off];
          if (m->logterm[off] > 0) {
            probe = orc_find_conflict_by_term(nr, rf, rt, li, m->hint[off], m->logterm[off]);
            runs_read = 1;
          }
          if (pr_maybe_decr_to(p, m->index[off], probe)) {
            if (p->state == PR_REPLICATE) pr_become_probe(p);
            send_append(&c, p, s, 1);
          }
        } else if (ty == M_APP_RESP) {
          p->recent_active = 1;
          uint64_t idx = m->index[off];
          if (idx > li) ls[ST_VIOLATIONS] += 1;
          int old_paused = pr_is_paused(p);
          if (pr_maybe_update(p, idx)) {
            if (p->state == PR_PROBE) {
              pr_become_replicate(p);
            } else if (p->state == PR_SNAPSHOT && p->match >= p->pending) {
              pr_become_probe(p);
              pr_become_replicate(p);
            } else if (p->state == PR_REPLICATE) {
              infl_free_le(p, idx);
            }
            for (uint32_t q = 0; q < S; q++) vals[q] = prs[q].match;
            uint64_t mci = orc_joint_committed(S, mi, mo, vals);
            if (orc_maybe_commit(mci, &cm, ts, li)) {
              /* releasePendingReadIndexMessages: the reads postponed while no
               * entry of this term was committed are answered at the commit
               * of this moment (the first such call of the round) */
              if (first_commit) tci = cm;
              first_commit = 0;
              if (bc < 255) bc++;
              /* bcastAppend: every Progress but the leader's own (:515-522) */
              for (uint32_t q = 0; q < S; q++)
                if (((trk >> q) & 1u) && q != self) send_append(&c, &prs[q], q, 1);
            } else if (old_paused) {
              send_append(&c, p, s, 1);
            }
            while (send_append(&c, p, s, 0)) {
            }
            if (s == lt && p->match == li) tnow |= 1u << s; /* sendTimeoutNow */
          }
        } else if (ty == M_HEARTBEAT_RESP) {
          p->recent_active = 1;
          p->probe_sent = 0;
          if (p->state == PR_REPLICATE && infl_full(p)) infl_free_le(p, *ib(p, p->start));
          if (p->match < li) send_append(&c, p, s, 1);
          /* :1296-1309: ReadOnlySafe with a context -> recvAck; a won vote
           * -> advance releases the queue through that request (a later
           * response carrying a released context records nothing) */
          if (rd) {
            uint32_t cx = m->read_ctx ? m->read_ctx[off] : dctx;
            int j = ro_find(&ro, cx);
            if (j >= 0) {
              uint32_t n_old = ro.n;
              ro.acks[j] |= 1u << s;
              rtouch = 1;
              int won = orc_joint_vote(mi, mo, ro.acks[j], ro.acks[j]) == VOTE_WON;
              /* an entry past the word: read from the ring, written back
               * unless released (device-form accounting, ABI 7) */
              if (j >= READ_QUEUE) ovfB += won ? mb : 2 * mb;
              /* the ack of an entry past the word is written to its ring slot
               * at once, as the device form does; an entry released later in
               * the round keeps the ack in its (then dead) slot */
              if (j >= READ_QUEUE && !won) ovf_set(a, mb, g, ro.ctx[j], ro.acks[j]);
              if (won) {
                uint32_t r = ro_advance(&ro, cx);
                released += r;
                /* the entries that move into the word are read from the ring */
                if (n_old > READ_QUEUE)
                  for (uint32_t q = 0; q < READ_QUEUE; q++)
                    if (q < ro.n && q + r >= READ_QUEUE) ovfB += mb;
              }
            }
          }
        } else if (ty == M_SNAP_STATUS || ty == M_SNAP_STATUS_REJECT) {
          if (p->state == PR_SNAPSHOT) {
            if (ty == M_SNAP_STATUS_REJECT) p->pending = 0;
            pr_become_probe(p);
            p->probe_sent = 1;
          }
        } else if (ty == M_UNREACHABLE) {
          if (p->state == PR_REPLICATE) pr_become_probe(p);
        } else if (ty == M_TRANSFER_LEADER) {
          int is_learner = !(((mi | mo) >> s) & 1u); /* tracked, not a voter */
          if (!is_learner) {
            int go = 1;
            if (lt < S) {              /* lastLeadTransferee != None */
              if (lt == s) go = 0;     /* same node: ignored */
              else lt = 0xFFu;         /* abortLeaderTransfer */
            }
            if (go && s == self) go = 0; /* already leader */
            if (go) {
              lt = s;
              if (p->match == li) tnow |= 1u << s; /* sendTimeoutNow */
              else send_append(&c, p, s, 1);
            }
          }
        }
      }
      int tc = cm != c0 && !(c0 >= ts && c0 <= li); /* committedEntryInCurrentTerm became true */
      uint64_t rword = rd ? ro_word(&ro, mb) : 0;
      int wq = rd && rtouch && rword != rword0;
      if (m->bytes) {
        /* per group: masks, log model, commit, ReadIndex masks */
        B += (a->inc ? mb : 0) + (a->out ? mb : 0) + (a->tracked ? mb : 0) + (a->self_slot ? 1 : 0) +
             (a->lead_transferee ? 1 : 0) + 32 + (a->snap_index ? 8 : 0);
        /* the queue: head and count, the acks word when requests pend */
        B += rd ? 5 + (rn0 ? READ_QUEUE * mb : 0) : 0;
        for (uint32_t s = 0; s < S; s++) {
          uint64_t off = s * a->stride + g;
          int tr = (trk >> s) & 1u;
          uint32_t ty = tr ? m->type[off] : 0;
          int msg = ty >= M_APP_RESP && ty <= M_TRANSFER_LEADER;
          int touched = tr && (msg || (bc > 0 && s != self));
          const orc_pr *p = &prs[s];
          B += 8;                                             /* Match (the commit pass) */
          B += tr ? 1 : 0;                                    /* message kind            */
          B += (ty == M_APP_RESP || ty == M_APP_RESP_REJECT) ? 8 : 0; /* m.Index         */
          if (touched) {
            B += 12;                                          /* Next + the packed word  */
            B += ty == M_APP_RESP_REJECT ? 16 : 0;            /* RejectHint, LogTerm     */
            B += (rd && m->read_ctx && ty == M_HEARTBEAT_RESP) ? 4 : 0; /* its context   */
            B += state0[s] == PR_SNAPSHOT ? 8 : 0;            /* PendingSnapshot         */
            B += p->match != match0[s] ? 8 : 0;
            B += p->next != next0[s] ? 8 : 0;
            B += p->pending != pend0[s] ? 8 : 0;              /* (0 outside StateSnapshot) */
            B += pr_word(p) != word0[s] ? 4 : 0;
          }
          B += m->msg_count ? 1 : 0;
          B += (m->msg_index && m->msg_count && m->msg_count[off]) ? 8 : 0;
        }
        B += runs_read ? 1 + 16 * (uint64_t)nr : 0;           /* the term-run table      */
        B += cm != c0 ? 8 : 0;
        B += (m->sent ? mb : 0) + (m->snap ? mb : 0) + (m->timeout_now ? mb : 0) +
             (m->bcast ? 1 : 0) + (m->read_released ? 1 : 0) + (m->term_commit ? 1 : 0);
        B += wq ? READ_QUEUE * mb : 0;
        B += released ? 5 : 0;
        B += (tc && m->term_commit_index) ? 8 : 0;
        B += (a->lead_transferee && lt != lt0) ? 1 : 0;
        B += ovfB;
        lbytes += B;
      }
      for (uint32_t s = 0; s < S; s++) pr_store2(&prs[s], a, s, g);
      a->committed[g] = cm;
      if (m->sent) st_mask(m->sent, mb, g, c.sent);
      if (m->snap) st_mask(m->snap, mb, g, c.snapm);
      if (m->timeout_now) st_mask(m->timeout_now, mb, g, tnow);
      if (m->bcast) m->bcast[g] = (uint8_t)bc;
      if (wq) ro_word_set(a->read_acks, mb, g, rword);
      if (rd && released) {
        a->read_head[g] = rhead0 + released;
        a->read_count[g] = (uint8_t)ro.n;
      }
      if (m->read_released) m->read_released[g] = (uint8_t)released;
      if (m->term_commit) m->term_commit[g] = (uint8_t)tc;
      if (m->term_commit_index && tc) m->term_commit_index[g] = tci;
      if (a->lead_transferee && lt != lt0) a->lead_transferee[g] = (uint8_t)lt;
      ls[ST_GROUPS] += 1;
      ls[ST_COMMIT_SUM] += cm;
      ls[ST_COMMIT_ADVANCED] += (cm != c0);
      ls[ST_READ_RELEASED] += released;
      ls[ST_CHECKSUM] += orc_checksum_step(a->goff + g, cm, c.sent, bc, released, tc, tci,
                                           lt != lt0, lt);
    }
#pragma omp critical
    {
      for (int k = 0; k < NSTAT; k++) st[k] += ls[k];
      bytes += lbytes;
    }
  }
  if (stats)
    for (int k = 0; k < NSTAT; k++) stats[k] += st[k];
  if (m->bytes) *m->bytes += bytes;
}

/* MsgCheckQuorum on each group's leader (stepLeader, raft/raft.go:997-1018):
 * `if pr := r.prs.Progress[r.id]; pr != nil { pr.RecentActive = true }`;
 * `!r.prs.QuorumActive()` -> becomeFollower (qa[g] = 0); then
 * `r.prs.Visit(... if id != r.id { pr.RecentActive = false })`.
 * QuorumActive (raft/tracker/tracker.go:215-225) over the Progress map:
 * votes[id] = RecentActive for every Progress that is not a learner (a
 * learner is never a voter, confchange.go:308-318, so the voters' Progress
 * entries are the votes), VoteResult over Voters -- a voter without a
 * Progress is missing. */
void orc_check_quorum_batch(const orc_prog *a, uint8_t *qa, uint64_t *stats) {
  uint32_t S = a->S, mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  uint64_t st[NSTAT];
  memset(st, 0, sizeof(st));
  for (uint64_t g = 0; g < a->G; g++) {
    uint32_t mi = a->inc ? ld_mask(a->inc, mb, g) & full : full;
    uint32_t mo = a->out ? ld_mask(a->out, mb, g) & full : 0;
    uint32_t trk = a->tracked ? ld_mask(a->tracked, mb, g) & full : full;
    uint32_t self = a->self_slot ? a->self_slot[g] : 0xFFu;
    if (self < S && ((trk >> self) & 1u)) a->pw[self * a->stride + g] |= PF_RECENT_ACTIVE;
    uint32_t votes = 0, yes = 0;
    for (uint32_t s = 0; s < S; s++) {
      if (!((trk >> s) & 1u)) continue;
      votes |= 1u << s;
      if (a->pw[s * a->stride + g] & PF_RECENT_ACTIVE) yes |= 1u << s;
    }
    int active = orc_joint_vote(mi, mo, votes, yes) == VOTE_WON;
    for (uint32_t s = 0; s < S; s++)
      if (((trk >> s) & 1u) && s != self) a->pw[s * a->stride + g] &= ~PF_RECENT_ACTIVE;
    if (qa) qa[g] = (uint8_t)active;
    st[ST_GROUPS] += 1;
    st[ST_STEPDOWNS] += !active;
    st[ST_CHECKSUM] += orc_mix64(((a->goff + g) * PHI) ^ ((uint64_t)yes << 32) ^
                                 (active ? 0xA0761D6478BD642Full : 0));
  }
  if (stats)
    for (int k = 0; k < NSTAT; k++) stats[k] += st[k];
}

/* MsgReadIndex on each group's leader with request[g] != 0 (stepLeader,
 * raft/raft.go:1078-1096; sendMsgReadIndexResponse :1827-1843):
 *   r.prs.IsSingleton() (tracker.go:158-160) -> respond at committed;
 *   !committedEntryInCurrentTerm() (:1731-1733) -> postponed;
 *   ReadOnlyLeaseBased -> respond at committed;
 *   ReadOnlySafe -> addRequest(committed, m) + recvAck(r.id) (read_only.go:
 *   56-76), the request's context number being the next in the queue; a
 *   queue of READ_QUEUE requests (or exhausted numbers) -> full (the
 *   engine's limit, nothing changes).
 * result: 1 respond, 2 postponed, 3 queued, 4 full (QE_RI_*). */
void orc_read_index_batch(const orc_prog *a, const uint8_t *request, const uint64_t *key,
                          uint32_t lease_based, uint8_t *result, uint32_t *ctx, uint64_t *index) {
  uint32_t S = a->S, mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  for (uint64_t g = 0; g < a->G; g++) {
    result[g] = 0;
    if (!request[g]) continue;
    uint32_t mi = a->inc ? ld_mask(a->inc, mb, g) & full : full;
    uint32_t mo = a->out ? ld_mask(a->out, mb, g) & full : 0;
    uint64_t c = a->committed[g], ts = a->term_start[g], li = a->last_index[g];
    if (popc(mi) == 1 && mo == 0) { /* only one voting member: the leader */
      result[g] = 1;
      if (index) index[g] = c;
      continue;
    }
    if (!(c >= ts && c <= li)) { /* no entry of this term committed yet */
      result[g] = 2;
      continue;
    }
    if (lease_based) {
      result[g] = 1;
      if (index) index[g] = c;
      continue;
    }
    orc_ro ro;
    uint32_t head = a->read_head[g], cap = ro_cap(a);
    ro_load(&ro, a, g, mb);
    if (ro.n == 0 && head == 0) head = 1; /* context numbers start at 1 */
    /* addRequest ignores a request already pending (read_only.go:57-60):
     * the keys stand for the context bytes (ABI 7) */
    uint64_t *keys = (key && a->read_keys) ? a->read_keys + g * cap : NULL;
    int dup = -1;
    for (uint32_t j = 0; keys && j < ro.n && dup < 0; j++)
      if (keys[(head + j) % cap] == key[g]) dup = (int)j;
    if (dup >= 0) {
      result[g] = 5; /* QE_RI_DUPLICATE */
      if (ctx) ctx[g] = head + (uint32_t)dup;
      continue;
    }
    if (ro.n >= cap || head + ro.n == 0u) {
      result[g] = 4;
      continue;
    }
    uint32_t self = a->self_slot ? a->self_slot[g] : 0xFFu;
    ro.ctx[ro.n] = head + ro.n;                              /* addRequest */
    ro.acks[ro.n] = self < S ? 1u << self : 0u;              /* recvAck(r.id) */
    if (keys) keys[(head + ro.n) % cap] = key[g];
    ro.n++;
    ro_word_set(a->read_acks, mb, g, ro_word(&ro, mb));
    if (a->read_ovf) ro_store_ovf(&ro, a, g, mb);
    a->read_head[g] = head;
    a->read_count[g] = (uint8_t)ro.n;
    result[g] = 3;
    if (ctx) ctx[g] = head + ro.n - 1;
    if (index) index[g] = c;
  }
}

/* raft.sendAppend / maybeSendAppend(to, send_if_empty) once for every slot
 * of want[g] (bcastAppend after a proposal, raft.go:515-522, or a single
 * sendAppend), see send_append above.  sent / snap report the outcome. */
void orc_progress_send_batch(const orc_prog *a, const void *want, uint32_t send_if_empty,
                             uint32_t max_ents, void *sent, void *snap) {
  uint32_t S = a->S, mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  for (uint64_t g = 0; g < a->G; g++) {
    orc_gctx c;
    c.a = a;
    c.m = NULL;
    c.g = g;
    c.fi = a->first_index[g];
    c.li = a->last_index[g];
    c.snap = a->snap_index ? a->snap_index[g] : c.fi - 1;
    c.me = max_ents;
    c.sent = c.snapm = 0;
    uint32_t w = ld_mask(want, mb, g) & full;
    for (uint32_t s = 0; s < S; s++) {
      if (!((w >> s) & 1u)) continue;
      orc_pr p;
      pr_load2(&p, a, s, g);
      send_append(&c, &p, s, (int)send_if_empty);
      pr_store2(&p, a, s, g);
    }
    if (sent) st_mask(sent, mb, g, c.sent);
    if (snap) st_mask(snap, mb, g, c.snapm);
  }
}

/* MsgProp on each group's leader (stepLeader, raft/raft.go:1019-1076), its
 * appendEntry (:621-642) and the bcastAppend that follows (:515-522).  The
 * proposal of group g is num_entries[g] entries; payload[g] = the sum of
 * PayloadSize (len(Data), util.go) over the entries that are not conf
 * changes; its conf-change entries are listed (position in m.Entries, a
 * ConfChangeV2 without Changes = wantsLeaveJoint, PayloadSize).
 * result: 0 no proposal, 1 appended + bcastAppend, 2 dropped (no Progress
 * of its own, :1023-1028), 3 dropped (leadership transfer, :1029-1032),
 * 4 dropped (increaseUncommittedSize, :627-633 / :1761-1779), 5 more
 * conf-change entries than max_cc (QE_PROP_BAD_CC, ABI 7: refused whole, no
 * state changes -- an input error, reported per group). */
typedef struct orc_props {
  const uint32_t *num_entries;
  const uint64_t *payload;
  uint32_t max_cc, flags;       /* flags 1: appendEntry alone (QE_PROP_APPEND_ONLY) */
  uint64_t cc_stride;
  const uint8_t *cc_count;
  const uint32_t *cc_pos;
  const uint8_t *cc_leave;
  const uint32_t *cc_size;
  const uint64_t *applied;
  uint64_t *pending_conf_index;
  uint64_t *uncommitted_size;
  uint64_t max_uncommitted;     /* 0 = noLimit (raft.go:356-358) */
  uint8_t *result;
  uint8_t *cc_refused;
  void *sent, *snap;
  uint64_t *bytes;              /* byte accounting (DESIGN.md §3 rules), or NULL */
} orc_props;

uint64_t orc_checksum_prop(uint64_t gid, uint32_t result, uint64_t last_index, uint64_t committed,
                           uint32_t sent) {
  uint64_t h = gid * PHI;
  return orc_mix64(h ^ 0x9E6C63D0676A9A99ull ^ ((uint64_t)result << 60) ^ last_index) +
         orc_mix64(h ^ committed ^ ((uint64_t)sent << 40));
}

void orc_propose_batch(const orc_prog *a, const orc_props *q, uint64_t *stats) {
  uint32_t S = a->S, mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  uint64_t *last_index = (uint64_t *)a->last_index; /* appendEntry advances it */
  uint64_t maxu = q->max_uncommitted ? q->max_uncommitted : UINT64_MAX;
  uint64_t st[NSTAT];
  memset(st, 0, sizeof(st));
  uint64_t bytes = 0;
  for (uint64_t g = 0; g < a->G; g++) {
    uint32_t n = q->num_entries[g];
    uint32_t res = 0, refused = 0, sentm = 0, snapm = 0;
    uint64_t li = last_index[g], cm = a->committed[g], c0 = cm;
    uint64_t B = 4;                                          /* num_entries */
    int out_counted = 0;
    if (n) {
      uint32_t trk = a->tracked ? ld_mask(a->tracked, mb, g) & full : full;
      uint32_t self = a->self_slot ? a->self_slot[g] : 0xFFu;
      uint32_t lt = a->lead_transferee ? a->lead_transferee[g] : 0xFFu;
      B += (a->self_slot ? 1 : 0) + (a->tracked ? mb : 0) + (a->lead_transferee ? 1 : 0);
      int app_only = (q->flags & 1u) != 0;                  /* appendEntry alone: no MsgProp gates, no bcast */
      if (!(self < S && ((trk >> self) & 1u))) res = 2;      /* Progress[r.id] == nil */
      else if (!app_only && lt < S) res = 3;                 /* leadTransferee != None */
      else {
        uint32_t mi = a->inc ? ld_mask(a->inc, mb, g) & full : full;
        uint32_t mo = a->out ? ld_mask(a->out, mb, g) & full : 0;
        uint64_t s = q->payload ? q->payload[g] : 0;
        uint32_t mcc = app_only ? 0 : q->max_cc;
        B += (q->payload ? 8 : 0) + (mcc ? 1 : 0);
        uint32_t ncc = mcc ? q->cc_count[g] : 0;
        if (ncc > mcc) {                                     /* QE_PROP_BAD_CC: refused whole */
          res = 5;
        } else if (ncc) {
          uint64_t pci = q->pending_conf_index[g], pci0 = pci, applied = q->applied[g];
          int joint = mo != 0;                               /* len(Voters[1]) > 0 */
          B += (a->out ? mb : 0) + 16;                       /* out mask, applied, pendingConfIndex */
          out_counted = a->out != NULL;
          for (uint32_t k = 0; k < ncc; k++) {
            uint64_t o = (uint64_t)k * q->cc_stride + g;
            int leave = q->cc_leave[o] != 0;
            B += 9;                                          /* position, kind, size */
            int already_pending = pci > applied;
            if (already_pending || (joint && !leave) || (!joint && leave)) {
              refused |= 1u << k;                            /* -> pb.Entry{Type: EntryNormal} */
            } else {
              pci = li + q->cc_pos[o] + 1;
              s += q->cc_size[o];
            }
          }
          q->pending_conf_index[g] = pci;
          B += pci != pci0 ? 8 : 0;
        }
        /* appendEntry -> increaseUncommittedSize (:1761-1779) */
        uint64_t us = (res != 5 && q->uncommitted_size) ? q->uncommitted_size[g] : 0;
        B += (res != 5 && q->uncommitted_size) ? 8 : 0;
        if (res == 5) {
          /* nothing appended */
        } else if (us > 0 && s > 0 && us + s > maxu) {
          res = 4;
        } else {
          res = 1;
          if (q->uncommitted_size) {
            q->uncommitted_size[g] = us + s;
            B += s ? 8 : 0;
          }
          li += n;                                           /* raftLog.append */
          last_index[g] = li;
          B += 16 + 8 + 8 + (app_only ? 0 : 8 + (a->snap_index ? 8 : 0)); /* lastIndex rw, term_start, committed, firstIndex */
          B += (a->inc ? mb : 0) + (a->out && !out_counted ? mb : 0);
          orc_gctx c;
          c.a = a;
          c.m = NULL;
          c.g = g;
          c.fi = a->first_index[g];
          c.li = li;
          c.snap = a->snap_index ? a->snap_index[g] : c.fi - 1;
          c.me = a->max_ents;
          c.sent = c.snapm = 0;
          orc_pr prs[16];
          uint64_t vals[16];
          for (uint32_t t = 0; t < S; t++) {
            pr_load2(&prs[t], a, t, g);
            B += 8;                                          /* Match (Committed) */
          }
          /* Progress[r.id].MaybeUpdate(li) */
          orc_pr *me = &prs[self];
          uint64_t m0 = me->match, n0 = me->next;
          uint32_t w0 = pr_word(me);
          pr_maybe_update(me, li);
          B += 12 + (me->match != m0 ? 8 : 0) + (me->next != n0 ? 8 : 0) + (pr_word(me) != w0 ? 4 : 0);
          for (uint32_t t = 0; t < S; t++) vals[t] = prs[t].match;
          uint64_t mci = orc_joint_committed(S, mi, mo, vals);
          orc_maybe_commit(mci, &cm, a->term_start[g], li);
          B += cm != c0 ? 8 : 0;
          /* bcastAppend: sendAppend to every Progress but the leader's */
          for (uint32_t t = 0; t < S; t++) {
            if (app_only || !((trk >> t) & 1u) || t == self) continue;
            orc_pr *p = &prs[t];
            uint64_t nx0 = p->next;
            uint32_t pw0 = pr_word(p);
            if (q->bytes) p->acct = &B;                      /* appended entries: 4 B each */
            send_append(&c, p, t, 1);
            p->acct = NULL;
            B += 12 + (p->next != nx0 ? 8 : 0) + (pr_word(p) != pw0 ? 4 : 0) +
                 (p->reset ? 8 : 0);                         /* Next + word; PendingSnapshot written */
          }
          for (uint32_t t = 0; t < S; t++) pr_store2(&prs[t], a, t, g);
          a->committed[g] = cm;
          sentm = c.sent;
          snapm = c.snapm;
        }
      }
    }
    q->result[g] = (uint8_t)res;
    if (q->cc_refused) q->cc_refused[g] = (uint8_t)refused;
    if (q->sent) st_mask(q->sent, mb, g, sentm);
    if (q->snap) st_mask(q->snap, mb, g, snapm);
    B += 1 + (q->cc_refused ? 1 : 0) + (q->sent ? mb : 0) + (q->snap ? mb : 0);
    bytes += B;
    st[ST_GROUPS] += 1;
    st[ST_COMMIT_ADVANCED] += cm != c0;
    st[ST_COMMIT_SUM] += cm;
    st[ST_CHECKSUM] += orc_checksum_prop(a->goff + g, res, li, cm, sentm);
  }
  if (stats)
    for (int k = 0; k < NSTAT; k++) stats[k] += st[k];
  if (q->bytes) *q->bytes += bytes;
}

/* raft.becomeLeader (raft/raft.go:724-759) on every group with elected[g]
 * (NULL = every group): reset (:590-613) -- every Progress of the
 * ProgressMap becomes {Match 0, Next lastIndex + 1, new Inflights, the
 * same IsLearner}, the leader's own Match = lastIndex; abortLeaderTransfer;
 * pendingConfIndex = uncommittedSize = 0; newReadOnly (the queue emptied;
 * the device form's context numbers move past the dropped requests) -- then
 * Progress[r.id].BecomeReplicate, pendingConfIndex = lastIndex, the log
 * enters term[g] (a term run from lastIndex + 1; term_start), appendEntry of
 * the empty entry (lastIndex + 1, the leader's MaybeUpdate, maybeCommit) and,
 * with flags & 1, stepCandidate's bcastAppend (:1405-1407).  result: 0 not
 * elected, 1 leader, 2 no Progress for the leader (the reference panics), 3
 * the run table is full (nothing changes). */
uint64_t orc_checksum_leader(uint64_t gid, uint32_t result, uint64_t committed, uint32_t sent,
                             uint32_t snap) {
  uint64_t h = gid * PHI;
  return orc_mix64(h ^ 0x6A09E667BB67AE85ull ^ ((uint64_t)result << 56) ^ committed) +
         orc_mix64(h ^ 0xD1B54A32D192ED03ull ^ ((uint64_t)sent << 40) ^ ((uint64_t)snap << 20));
}

void orc_become_leader_batch(const orc_prog *a, const uint8_t *elected, const uint64_t *term,
                             uint32_t flags, uint64_t *pci, uint64_t *unc, uint8_t *result,
                             void *sent, void *snap, uint64_t *stats) {
  uint32_t S = a->S, mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  uint64_t *last_index = (uint64_t *)a->last_index, *term_start = (uint64_t *)a->term_start;
  uint64_t *run_first = (uint64_t *)a->run_first, *run_term = (uint64_t *)a->run_term;
  uint8_t *run_count = (uint8_t *)a->run_count;
  uint64_t st[NSTAT];
  memset(st, 0, sizeof(st));
  for (uint64_t g = 0; g < a->G; g++) {
    uint64_t cm = a->committed[g], c0 = cm;
    uint32_t res = 0, sentm = 0, snapm = 0;
    if (!elected || elected[g]) {
      uint32_t trk = a->tracked ? ld_mask(a->tracked, mb, g) & full : full;
      uint32_t self = a->self_slot ? a->self_slot[g] : 0xFFu;
      uint32_t mi = a->inc ? ld_mask(a->inc, mb, g) & full : full;
      uint32_t mo = a->out ? ld_mask(a->out, mb, g) & full : 0;
      uint32_t rc = (a->R && run_count) ? run_count[g] : 0;
      if (!(self < S && ((trk >> self) & 1u))) res = 2;
      else if (a->R && rc >= a->R) res = 3;
      else {
        res = 1;
        uint64_t li = last_index[g];
        /* reset: every Progress; the leader's own Match = lastIndex */
        orc_pr prs[16];
        for (uint32_t t = 0; t < S; t++) {
          if (!((trk >> t) & 1u)) continue;
          pr_load2(&prs[t], a, t, g);
          prs[t].match = t == self ? li : 0;
          prs[t].next = li + 1;
          prs[t].pending = 0;
          prs[t].state = PR_PROBE;
          prs[t].probe_sent = prs[t].recent_active = 0;
          prs[t].start = prs[t].count = 0; /* tracker.NewInflights */
        }
        if (a->lead_transferee) a->lead_transferee[g] = 0xFF; /* abortLeaderTransfer */
        if (a->read_acks) {                                   /* newReadOnly */
          uint32_t cap = a->read_cap ? a->read_cap : READ_QUEUE;
          uint32_t qn = a->read_count[g] < cap ? a->read_count[g] : cap;
          a->read_head[g] += qn;
          a->read_count[g] = 0;
        }
        pr_become_replicate(&prs[self]);                      /* Next = Match + 1 */
        if (pci) pci[g] = li;
        if (unc) unc[g] = 0;
        /* the log enters the new term: a run from lastIndex + 1, unless the
         * last run already has that term (the bootstrap snapshot of the new
         * leader's own term), where the term then starts */
        uint64_t ts2 = li + 1;
        if (a->R) {
          if (rc > 0 && run_term[(rc - 1) * a->stride + g] == term[g]) {
            ts2 = run_first[(rc - 1) * a->stride + g];
          } else {
            run_first[rc * a->stride + g] = li + 1;
            run_term[rc * a->stride + g] = term[g];
            run_count[g] = (uint8_t)(rc + 1);
          }
        }
        term_start[g] = ts2;
        /* appendEntry(empty) */
        li += 1;
        last_index[g] = li;
        pr_maybe_update(&prs[self], li);
        uint64_t vals[16];
        for (uint32_t t = 0; t < S; t++) vals[t] = ((trk >> t) & 1u) ? prs[t].match : 0;
        orc_maybe_commit(orc_joint_committed(S, mi, mo, vals), &cm, term_start[g], li);
        if (flags & 1u) { /* bcastAppend */
          orc_gctx c;
          c.a = a;
          c.m = NULL;
          c.g = g;
          c.fi = a->first_index[g];
          c.li = li;
          c.snap = a->snap_index ? a->snap_index[g] : c.fi - 1;
          c.me = a->max_ents;
          c.sent = c.snapm = 0;
          for (uint32_t t = 0; t < S; t++)
            if (((trk >> t) & 1u) && t != self) send_append(&c, &prs[t], t, 1);
          sentm = c.sent;
          snapm = c.snapm;
        }
        for (uint32_t t = 0; t < S; t++)
          if ((trk >> t) & 1u) pr_store2(&prs[t], a, t, g);
        a->committed[g] = cm;
      }
    }
    result[g] = (uint8_t)res;
    if (sent) st_mask(sent, mb, g, sentm);
    if (snap) st_mask(snap, mb, g, snapm);
    st[ST_GROUPS] += 1;
    st[ST_COMMIT_ADVANCED] += cm != c0;
    st[ST_COMMIT_SUM] += cm;
    st[ST_CHECKSUM] += orc_checksum_leader(a->goff + g, res, cm, sentm, snapm);
  }
  if (stats)
    for (int k = 0; k < NSTAT; k++) stats[k] += st[k];
}

/* raft.switchToConfig (raft/raft.go:1651-1700) on every group with
 * switched[g] (NULL = every group), after the new configuration -- inc /
 * out / tracked of `a` -- is in place.  result: 0 not switched, 1 the leader
 * has no Progress or is a learner (r.isLearner, :1660; a learner is a
 * tracked peer in neither half) -> return (:1663-1674), 2 len(cs.Voters) ==
 * 0 -> return (:1678-1680), 3 maybeCommit -> bcastAppend (:1682-1685), 4
 * else maybeSendAppend(id, false) for every Progress (prs.Visit, the
 * leader's own included, :1686-1692); | 0x10 when leadTransferee is not in
 * Voters.IDs() and abortLeaderTransfer runs (:1694-1697).  Byte accounting
 * as orc_propose_batch's rules. */
uint64_t orc_checksum_switch(uint64_t gid, uint32_t result, uint64_t committed, uint32_t sent,
                             uint32_t snap) {
  uint64_t h = gid * PHI;
  return orc_mix64(h ^ 0x2545F4914F6CDD1Dull ^ ((uint64_t)result << 56) ^ committed) +
         orc_mix64(h ^ 0xD1B54A32D192ED03ull ^ ((uint64_t)sent << 40) ^ ((uint64_t)snap << 20));
}

void orc_switch_config_batch(const orc_prog *a, const uint8_t *switched, uint8_t *result,
                             void *sent, void *snap, uint64_t *stats, uint64_t *bytes) {
  uint32_t S = a->S, mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  uint64_t st[NSTAT];
  memset(st, 0, sizeof(st));
  uint64_t total = 0;
  for (uint64_t g = 0; g < a->G; g++) {
    uint64_t B = (switched ? 1 : 0) + 8;                     /* switched, committed */
    uint64_t cm = a->committed[g], c0 = cm;
    uint32_t res = 0, sentm = 0, snapm = 0;
    if (!switched || switched[g]) {
      uint32_t trk = a->tracked ? ld_mask(a->tracked, mb, g) & full : full;
      uint32_t self = a->self_slot ? a->self_slot[g] : 0xFFu;
      uint32_t mi = a->inc ? ld_mask(a->inc, mb, g) & full : full;
      uint32_t mo = a->out ? ld_mask(a->out, mb, g) & full : 0;
      uint32_t lt = a->lead_transferee ? a->lead_transferee[g] : 0xFFu;
      B += (a->self_slot ? 1 : 0) + (a->tracked ? mb : 0) + (a->inc ? mb : 0) + (a->out ? mb : 0) +
           (a->lead_transferee ? 1 : 0);
      int ok = self < S && ((trk >> self) & 1u);             /* pr, ok := Progress[r.id] */
      int is_learner = ok && !(((mi | mo) >> self) & 1u);    /* pr.IsLearner */
      if (!ok || is_learner) {
        res = 1;
      } else if (mi == 0) {
        res = 2;
      } else {
        orc_gctx c;
        c.a = a;
        c.m = NULL;
        c.g = g;
        c.fi = a->first_index[g];
        c.li = a->last_index[g];
        c.snap = a->snap_index ? a->snap_index[g] : c.fi - 1;
        c.me = a->max_ents;
        c.sent = c.snapm = 0;
        B += 24 + (a->snap_index ? 8 : 0) + 8 * (uint64_t)popc(mi | mo); /* log model, Match */
        uint64_t vals[16];
        for (uint32_t t = 0; t < S; t++) vals[t] = a->match[t * a->stride + g];
        uint64_t mci = orc_joint_committed(S, mi, mo, vals);
        int adv = orc_maybe_commit(mci, &cm, a->term_start[g], c.li);
        res = adv ? 3 : 4;
        for (uint32_t t = 0; t < S; t++) {
          if (!((trk >> t) & 1u)) continue;
          if (adv && t == self) continue;                    /* bcastAppend skips r.id */
          orc_pr p;
          pr_load2(&p, a, t, g);
          uint64_t nx0 = p.next;
          uint32_t pw0 = pr_word(&p);
          if (bytes) p.acct = &B;
          send_append(&c, &p, t, adv);                       /* sendAppend / maybeSendAppend(id, false) */
          p.acct = NULL;
          B += 12 + (p.next != nx0 ? 8 : 0) + (pr_word(&p) != pw0 ? 4 : 0) + (p.reset ? 8 : 0);
          pr_store2(&p, a, t, g);
        }
        a->committed[g] = cm;
        B += cm != c0 ? 8 : 0;
        sentm = c.sent;
        snapm = c.snapm;
        if (lt < S && !(((mi | mo) >> lt) & 1u)) {           /* leadTransferee not a voter */
          a->lead_transferee[g] = 0xFF;                      /* abortLeaderTransfer */
          res |= 0x10;
          B += 1;
        }
      }
    }
    result[g] = (uint8_t)res;
    if (sent) st_mask(sent, mb, g, sentm);
    if (snap) st_mask(snap, mb, g, snapm);
    B += 1 + (sent ? mb : 0) + (snap ? mb : 0);
    total += B;
    st[ST_GROUPS] += 1;
    st[ST_COMMIT_ADVANCED] += cm != c0;
    st[ST_COMMIT_SUM] += cm;
    st[ST_CHECKSUM] += orc_checksum_switch(a->goff + g, res, cm, sentm, snapm);
  }
  if (stats)
    for (int k = 0; k < NSTAT; k++) stats[k] += st[k];
  if (bytes) *bytes += total;
}

/* MsgBeat on each group's leader (stepLeader, raft/raft.go:991-993):
 * bcastHeartbeat (:524-541) -> sendHeartbeat (:494-510) to every Progress
 * but the leader's, Commit = min(Match, committed), Context =
 * lastPendingRequestCtx (read_only.go:114-121; here the context number of
 * the newest pending request, 0 = none).  commit [S][stride] is written
 * for the slots sent to. */
void orc_heartbeat_batch(const orc_prog *a, uint64_t *commit, uint32_t *ctx, void *sent) {
  uint32_t S = a->S, mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  for (uint64_t g = 0; g < a->G; g++) {
    uint32_t trk = a->tracked ? ld_mask(a->tracked, mb, g) & full : full;
    uint32_t self = a->self_slot ? a->self_slot[g] : 0xFFu;
    uint32_t to = 0;
    uint64_t c = a->committed[g];
    for (uint32_t s = 0; s < S; s++) {
      if (!((trk >> s) & 1u) || s == self) continue;
      uint64_t m = a->match[s * a->stride + g];
      commit[s * a->stride + g] = m < c ? m : c;
      to |= 1u << s;
    }
    if (ctx) {
      uint32_t cx = 0;
      if (a->read_acks) {
        orc_ro ro;
        ro_load(&ro, a, g, mb);
        cx = ro.n ? ro.ctx[ro.n - 1] : 0;
      }
      ctx[g] = cx;
    }
    if (sent) st_mask(sent, mb, g, to);
  }
}

/* Scalar helpers for the golden tables (tests only). */
int orc_pr_maybe_decr_to(uint32_t state, uint64_t *match, uint64_t *next, uint64_t rejected,
                         uint64_t hint) {
  orc_pr p;
  memset(&p, 0, sizeof(p));
  p.state = state;
  p.match = *match;
  p.next = *next;
  int r = pr_maybe_decr_to(&p, rejected, hint);
  *match = p.match;
  *next = p.next;
  return r;
}

int orc_pr_is_paused(uint32_t state, uint32_t probe_sent, uint32_t count, uint32_t size) {
  orc_pr p;
  memset(&p, 0, sizeof(p));
  p.state = state;
  p.probe_sent = probe_sent;
  p.count = count;
  p.size = size;
  return pr_is_paused(&p);
}

uint64_t orc_pr_become_probe(uint32_t state, uint64_t match, uint64_t next, uint64_t pending) {
  orc_pr p;
  memset(&p, 0, sizeof(p));
  p.state = state;
  p.match = match;
  p.next = next;
  p.pending = pending;
  pr_become_probe(&p);
  return p.next;
}

/* Inflights op sequence on a contiguous buffer: ops[i] >= 0 -> Add(ops[i]),
 * ops[i] == -1 -> FreeFirstOne, ops[i] <= -2 -> FreeLE(-ops[i] - 2). */
void orc_inflights_ops(uint32_t size, uint32_t *start, uint32_t *count, uint64_t *buf,
                       const int64_t *ops, uint32_t nops) {
  orc_pr p;
  memset(&p, 0, sizeof(p));
  p.size = size;
  p.start = *start;
  p.count = *count;
  p.buf = buf;
  p.bstride = 1;
  for (uint32_t i = 0; i < nops; i++) {
    if (ops[i] >= 0) infl_add(&p, (uint64_t)ops[i]);
    else if (ops[i] == -1) infl_free_le(&p, *ib(&p, p.start));
    else infl_free_le(&p, (uint64_t)(-ops[i] - 2));
  }
  *start = p.start;
  *count = p.count;
}
