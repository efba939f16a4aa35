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

/* One TallyVotes + transition with the invariant checks of DESIGN.md §5. */
static void elec_tally(uint32_t mi, uint32_t mo, uint32_t ml, uint32_t vd, uint32_t gr,
                       uint32_t gbefore, uint32_t *sta, uint64_t *ls) {
  int gcn, rcn;
  uint8_t res = orc_tally(mi, mo, ml, vd, gr, &gcn, &rcn); /* raft.go:845 */
  uint8_t sym = orc_joint_vote(mo, mi, vd, gr);           /* symmetry */
  int n0 = popc(mi), n1 = popc(mo);
  int won_ok = (n0 == 0 || popc(gr & vd & mi) >= n0 / 2 + 1) &&
               (n1 == 0 || popc(gr & vd & mo) >= n1 / 2 + 1);
  ls[ST_VIOLATIONS] += (uint64_t)(sym != res) + (uint64_t)(res == VOTE_WON && !won_ok) +
                       (uint64_t)((uint32_t)gcn < gbefore);
  ls[ST_GRANTED] += (uint64_t)gcn;
  ls[ST_REJECTED] += (uint64_t)rcn;
  if (res == VOTE_WON) {            /* becomeLeader, raft.go:1402-1409 */
    *sta = 2; ls[ST_LEADERS] += 1; ls[ST_WON] += 1;
  } else if (res == VOTE_LOST) {    /* becomeFollower, raft.go:1410-1413 */
    *sta = 0; ls[ST_STEPDOWNS] += 1; ls[ST_LOST] += 1;
  } else {
    ls[ST_PENDING] += 1;
  }
}

/* Counter-based response RNG: per group gkey = mix64(seed +
 * gid*PHI) ^ IV folded to 32 bits (k = lo ^ hi); slot s at step t draws
 * d = fmix32(k + t*C1 + s*C2) (MurmurHash3's 32-bit finalizer), bits 0-15
 * the drop draw and bits 16-31 the grant draw. */
static const uint64_t ELEC_IV = 0x6A09E667F3BCC909ULL;
static const uint32_t ELEC_C1 = 0x9E3779B1u, ELEC_C2 = 0x85EBCA77u;
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

void orc_election_steps_batch(uint64_t G, uint64_t goff, uint32_t S, uint64_t *term,
                              uint8_t *state, void *voted, void *granted, const uint8_t *self_slot,
                              const void *inc, const void *out, const void *learner,
                              uint64_t seed, uint64_t step0, uint32_t steps, uint32_t p_drop,
                              uint32_t p_grant, uint64_t *stats, int threads) {
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
      uint32_t prog = mi | mo | ml;
      /* raft.promotable(): own Progress exists and is not a learner */
      int promotable = (self & (mi | mo)) != 0 && (self & ml) == 0;
      uint64_t t = term[g];
      uint32_t sta = state[g];
      uint32_t vd = ld_mask(voted, mb, g) & full, gr = ld_mask(granted, mb, g) & full;
      const uint32_t gkey = elec_gkey(seed, gid);
      for (uint32_t k = 0; k < steps && promotable; k++) {
        uint64_t step = step0 + k;
        if (sta != 1) {
          /* hup -> campaign(campaignElection), raft.go:785-803 */
          t += 1;                                  /* becomeCandidate */
          vd = 0; gr = 0;                          /* ResetVotes */
          orc_record_votes(&vd, &gr, self, self);  /* poll(r.id, ..., true) */
          sta = 1;
          ls[ST_ELECTIONS] += 1;
          elec_tally(mi, mo, ml, vd, gr, 0, &sta, ls);
        } else {
          /* one round of MsgVoteResp from every other Progress peer */
          uint32_t resp = 0, val = 0;
          for (uint32_t s = 0; s < S; s++) {
            if (!((prog >> s) & 1u) || ((self >> s) & 1u)) continue;
            uint32_t d = elec_draw(gkey, step, s);
            if ((d & 0xFFFFu) < p_drop) continue; /* dropped */
            resp |= 1u << s;
            if ((d >> 16) < p_grant) val |= 1u << s;
          }
          uint32_t gbefore = (uint32_t)popc(gr & vd & ~ml & (mi | mo));
          orc_record_votes(&vd, &gr, resp, val);   /* RecordVote, :844 */
          elec_tally(mi, mo, ml, vd, gr, gbefore, &sta, ls);
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

typedef struct orc_pr {
  uint64_t match, next, pending;
  uint32_t state, probe_sent, recent_active;
  uint32_t start, count, size; /* Inflights (raft/tracker/inflights.go:22-36) */
  uint64_t *buf;               /* strided view: buf[k * bstride] */
  uint64_t bstride;
} orc_pr;

static inline uint64_t *ib(orc_pr *p, uint32_t k) { return &p->buf[(uint64_t)k * p->bstride]; }

/* inflights.go:55-71 Add */
static void infl_add(orc_pr *p, uint64_t x) {
  uint32_t nx = p->start + p->count;
  if (nx >= p->size) nx -= p->size;
  *ib(p, nx) = x;
  p->count++;
}
/* inflights.go:87-113 FreeLE */
static void infl_free_le(orc_pr *p, uint64_t to) {
  if (p->count == 0 || to < *ib(p, p->start)) return;
  uint32_t idx = p->start, i;
  for (i = 0; i < p->count; i++) {
    if (to < *ib(p, idx)) break;
    if (++idx >= p->size) idx -= p->size;
  }
  p->count -= i;
  p->start = idx;
  if (p->count == 0) p->start = 0;
}
static int infl_full(const orc_pr *p) { return p->count == p->size; }

/* progress.go:84-90 ResetState */
static void pr_reset_state(orc_pr *p, uint32_t st) {
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

static void pr_load(orc_pr *p, uint64_t off, uint64_t stride, uint32_t F, uint64_t *match,
                    uint64_t *next, uint64_t *pending, uint8_t *pflags, uint8_t *istart,
                    uint8_t *icount, uint64_t *ibuf, uint32_t s, uint64_t g) {
  p->match = match[off];
  p->next = next[off];
  p->pending = pending[off];
  p->state = pflags[off] & PF_STATE;
  p->probe_sent = (pflags[off] & PF_PROBE_SENT) != 0;
  p->recent_active = (pflags[off] & PF_RECENT_ACTIVE) != 0;
  p->start = istart[off];
  p->count = icount[off];
  p->size = F;
  p->buf = ibuf + ((uint64_t)s * stride + g) * F; /* ring row [S][stride][F] */
  p->bstride = 1;
}
static void pr_store(const orc_pr *p, uint64_t off, uint64_t *match, uint64_t *next,
                     uint64_t *pending, uint8_t *pflags, uint8_t *istart, uint8_t *icount) {
  match[off] = p->match;
  next[off] = p->next;
  pending[off] = p->pending;
  pflags[off] = (uint8_t)(p->state | (p->probe_sent ? PF_PROBE_SENT : 0) |
                          (p->recent_active ? PF_RECENT_ACTIVE : 0));
  istart[off] = (uint8_t)p->start;
  icount[off] = (uint8_t)p->count;
}

uint64_t orc_checksum_step(uint64_t gid, uint64_t committed, uint32_t send, uint32_t bcast) {
  uint64_t tag = ((uint64_t)send << 40) | ((uint64_t)bcast << 62);
  return orc_mix64((gid * PHI) ^ committed ^ tag);
}

/* One round of leader-side message handling per group (raft/raft.go:
 * 1106-1296), messages taken in slot order.  type: 0 none, 1 MsgAppResp,
 * 2 MsgAppResp reject, 3 MsgHeartbeatResp.  Accepts with index > lastIndex
 * are invalid input: counted as invariant violations and ignored. */
void orc_progress_step_batch(uint64_t G, uint64_t goff, uint32_t S, uint32_t F, uint64_t stride,
                             uint64_t *match, uint64_t *next, uint64_t *pending, uint8_t *pflags,
                             uint8_t *istart, uint8_t *icount, uint64_t *ibuf, uint64_t *committed,
                             const uint64_t *term_start, const uint64_t *last_index, uint32_t R,
                             const uint64_t *run_first, const uint64_t *run_term,
                             const uint8_t *run_count, const void *inc, const void *out,
                             const uint8_t *mtype, const uint64_t *mindex, const uint64_t *mhint,
                             const uint64_t *mlogterm, void *send_mask, uint8_t *bcast,
                             uint64_t *stats, int threads) {
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
      uint64_t li = last_index[g], ts = term_start[g], c = committed[g];
      uint32_t nr = run_count[g] < R ? run_count[g] : R;
      uint64_t rf[16], rt[16];
      for (uint32_t r = 0; r < nr; r++) {
        rf[r] = run_first[r * stride + g];
        rt[r] = run_term[r * stride + g];
      }
      uint64_t vals[16];
      for (uint32_t s = 0; s < S; s++) vals[s] = match[s * stride + g];
      uint32_t send = 0, bc = 0;
      for (uint32_t s = 0; s < S; s++) {
        uint64_t off = s * stride + g;
        uint32_t ty = mtype[off];
        if (ty == 0 || ty > 3) continue; /* no message / unknown kind: ignored */
        orc_pr p;
        pr_load(&p, off, stride, F, match, next, pending, pflags, istart, icount, ibuf, s, g);
        p.recent_active = 1;
        if (ty == 2) { /* MsgAppResp reject, raft.go:1109-1236 */
          uint64_t probe = mhint[off];
          if (mlogterm[off] > 0)
            probe = orc_find_conflict_by_term(nr, rf, rt, li, mhint[off], mlogterm[off]);
          if (pr_maybe_decr_to(&p, mindex[off], probe)) {
            if (p.state == PR_REPLICATE) pr_become_probe(&p);
            send |= 1u << s; /* sendAppend(m.From) */
          }
        } else if (ty == 1) { /* MsgAppResp accept, raft.go:1237-1282 */
          if (mindex[off] > li) {
            ls[ST_VIOLATIONS] += 1;
          } else {
            int old_paused = pr_is_paused(&p);
            if (pr_maybe_update(&p, mindex[off])) {
              if (p.state == PR_PROBE) {
                pr_become_replicate(&p);
              } else if (p.state == PR_SNAPSHOT && p.match >= p.pending) {
                pr_become_probe(&p);
                pr_become_replicate(&p);
              } else if (p.state == PR_REPLICATE) {
                infl_free_le(&p, mindex[off]);
              }
              vals[s] = p.match;
              uint64_t mci = orc_joint_committed(S, mi, mo, vals);
              if (orc_maybe_commit(mci, &c, ts, li)) {
                bc = 1; /* releasePendingReadIndexMessages + bcastAppend */
              } else if (old_paused) {
                send |= 1u << s;
              }
            }
          }
        } else if (ty == 3) { /* MsgHeartbeatResp, raft.go:1284-1296 */
          p.probe_sent = 0;
          if (p.state == PR_REPLICATE && infl_full(&p)) infl_free_le(&p, *ib(&p, p.start));
          if (p.match < li) send |= 1u << s;
        }
        pr_store(&p, off, match, next, pending, pflags, istart, icount);
      }
      uint64_t c0 = committed[g];
      committed[g] = c;
      if (send_mask) st_mask(send_mask, mb, g, send);
      if (bcast) bcast[g] = (uint8_t)bc;
      ls[ST_GROUPS] += 1;
      ls[ST_COMMIT_SUM] += c;
      ls[ST_COMMIT_ADVANCED] += (c != c0);
      ls[ST_CHECKSUM] += orc_checksum_step(goff + g, c, send, bc);
    }
#pragma omp critical
    for (int k = 0; k < NSTAT; k++) st[k] += ls[k];
  }
  if (stats)
    for (int k = 0; k < NSTAT; k++) stats[k] += st[k];
}

/* raft.maybeSendAppend (raft/raft.go:432-492) for the slots in want[g]:
 * entries exist in [first_index, last_index] (first_index - 1 is the
 * snapshot index); at most max_ents entries per MsgApp. */
void orc_progress_send_batch(uint64_t G, uint32_t S, uint32_t F, uint64_t stride, uint64_t *match,
                             uint64_t *next, uint64_t *pending, uint8_t *pflags, uint8_t *istart,
                             uint8_t *icount, uint64_t *ibuf, const uint64_t *first_index,
                             const uint64_t *last_index, const void *want, uint32_t send_if_empty,
                             uint32_t max_ents, void *sent, void *snap) {
  uint32_t mb = S <= 8 ? 1 : 2;
  uint32_t full = (1u << S) - 1u;
  for (uint64_t g = 0; g < G; g++) {
    uint32_t w = ld_mask(want, mb, g) & full, sm = 0, sn = 0;
    uint64_t fi = first_index[g], li = last_index[g];
    for (uint32_t s = 0; s < S; s++) {
      if (!((w >> s) & 1u)) continue;
      uint64_t off = s * stride + g;
      orc_pr p;
      pr_load(&p, off, stride, F, match, next, pending, pflags, istart, icount, ibuf, s, g);
      if (pr_is_paused(&p)) continue;
      if (p.next > li) { /* no entries */
        if (!send_if_empty) continue;
        sm |= 1u << s;
      } else if (p.next < fi) { /* entries compacted -> snapshot */
        if (!p.recent_active) continue;
        pr_become_snapshot(&p, fi - 1);
        sm |= 1u << s;
        sn |= 1u << s;
      } else {
        uint64_t last = p.next + (max_ents ? max_ents : 1) - 1;
        if (last > li || last < p.next) last = li;
        if (p.state == PR_REPLICATE) {
          p.next = last + 1; /* OptimisticUpdate */
          infl_add(&p, last);
        } else if (p.state == PR_PROBE) {
          p.probe_sent = 1;
        }
        sm |= 1u << s;
      }
      pr_store(&p, off, match, next, pending, pflags, istart, icount);
    }
    if (sent) st_mask(sent, mb, g, sm);
    if (snap) st_mask(snap, mb, g, sn);
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
