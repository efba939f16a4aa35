// qe_api.hip — C ABI of include/etcd_quorum.h: argument checks, alignment
// selection of the vectorised path and launch of the MI355X kernels.
#include <stdio.h>
#include <string.h>

#include "qe_dispatch.hpp"
#include "qe_conf.hpp"
#include "qe_collect.hpp"

namespace qe {

int g_blocks_per_cu = 0;  // 0 = kernel occupancy
int g_nontemporal = 3;  // nt loads + nt stores (measured best)
int g_tiles_per_wave = -1;  // -1 = per-kernel default, 0 = persistent grid
int g_cv_kernel = -1;  // qe_commit_vote kernel: 0 pair, 1 stream, -1 per-mode default
int g_repl_kernel = -1;  // qe_replication_round kernel: 0 pair, 1 stream, -1 default

static thread_local char g_errbuf[256];

void set_error(const char *msg) { snprintf(g_errbuf, sizeof(g_errbuf), "%s", msg); }

int hip_status(hipError_t e) {
  if (e == hipSuccess) return QE_OK;
  snprintf(g_errbuf, sizeof(g_errbuf), "HIP error %d: %s", static_cast<int>(e),
           hipGetErrorString(e));
  return QE_EHIP;
}

static inline bool al(const void *p, size_t a) {
  return (reinterpret_cast<uintptr_t>(p) % a) == 0;
}

static unsigned simple_grid(uint64_t G) {
  const uint64_t cap = static_cast<uint64_t>(num_cus()) * 8;
  const uint64_t need = (G + kBlock - 1) / kBlock;
  return static_cast<unsigned>(need < cap ? (need ? need : 1) : cap);
}

// Sparse MsgAppResp acks: Progress.MaybeUpdate with 64-bit atomic max.
__global__ __launch_bounds__(kBlock) void k_apply_acks(uint64_t G, uint32_t S, uint64_t stride,
                                                       uint64_t *match, uint64_t *next,
                                                       uint64_t n, const uint64_t *group,
                                                       const int8_t *slot,
                                                       const uint64_t *index,
                                                       uint8_t *touched) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint64_t g = group[i];
    const int s = slot[i];
    if (g >= G || s < 0 || s >= static_cast<int>(S)) continue;
    const uint64_t x = index[i];
    const uint64_t off = static_cast<uint64_t>(s) * stride + g;
    atomicMax(reinterpret_cast<unsigned long long *>(match + off),
              static_cast<unsigned long long>(x));
    if (x != ~0ull)  // next = max(next, x+1); x+1 wraps only for x = max
      atomicMax(reinterpret_cast<unsigned long long *>(next + off),
                static_cast<unsigned long long>(x + 1));
    if (touched) touched[g] = 1;
  }
}

__global__ void k_stats_reduce(const uint64_t *stats, uint64_t *out) {
  const int c = threadIdx.x;
  if (c < QE_STATS_COUNTERS) {
    uint64_t s = 0;
    for (int k = 0; k < QE_STATS_SHARDS; k++) s += stats[k * QE_STATS_COUNTERS + c];
    out[c] = s;
  }
}


#define QE_SWITCH(S, CALL)                                                              \
  switch (S) {                                                                          \
    case 1: return CALL(1); case 2: return CALL(2); case 3: return CALL(3);             \
    case 4: return CALL(4); case 5: return CALL(5); case 6: return CALL(6);             \
    case 7: return CALL(7); case 8: return CALL(8); case 9: return CALL(9);             \
    case 10: return CALL(10); case 11: return CALL(11); case 12: return CALL(12);       \
    case 13: return CALL(13); case 14: return CALL(14); case 15: return CALL(15);       \
    case 16: return CALL(16);                                                           \
    default: return QE_EINVAL;                                                          \
  }

static int dispatch_cv(uint32_t S, const CVArgs &a, int mode, bool vec, hipStream_t st) {
#define QE_C(n) dispatch_cv_##n(a, mode, vec, st)
  QE_SWITCH(S, QE_C)
#undef QE_C
}

static int dispatch_repl(uint32_t S, const RArgs &a, bool masked, bool joint, bool vec,
                         hipStream_t st) {
#define QE_C(n) dispatch_repl_##n(a, masked, joint, vec, st)
  QE_SWITCH(S, QE_C)
#undef QE_C
}

static int dispatch_elec(uint32_t S, const EArgs &a, hipStream_t st) {
#define QE_C(n) dispatch_elec_##n(a, st)
  QE_SWITCH(S, QE_C)
#undef QE_C
}

static int dispatch_progress(uint32_t S, const PArgs &a, int kind, bool masked, bool joint,
                             hipStream_t st) {
#define QE_C(n) dispatch_progress_##n(a, kind, masked, joint, st)
  QE_SWITCH(S, QE_C)
#undef QE_C
}

}  // namespace qe

// ===========================================================================
// C ABI
// ===========================================================================
using namespace qe;

extern "C" {

int qe_abi_version(void) { return QE_ABI_VERSION; }

const char *qe_strerror(int status) {
  switch (status) {
    case QE_OK: return "ok";
    case QE_EINVAL: return "invalid argument";
    case QE_ERANGE: return "out of range";
    case QE_EHIP: return g_errbuf[0] ? g_errbuf : "HIP error";
    case QE_ECOMM: return g_errbuf[0] ? g_errbuf : "RCCL error";
    default: return "unknown status";
  }
}

size_t qe_mask_bytes(uint32_t num_slots) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return 0;
  return num_slots <= 8 ? 1 : 2;
}

// Optional tuning knobs (not part of the reference semantics):
//   "blocks_per_cu"  cap on persistent-grid workgroups per CU (0 = occupancy)
//   "tiles_per_wave" -1 = per-kernel default, 0 = persistent grid,
//                    T > 0 = each wave walks T tiles
//   "nontemporal"    bit 0: non-temporal loads, bit 1: non-temporal stores
//   "cv_kernel", "repl_kernel"  0 = pair kernel, 1 = stream kernel, -1 = default
int qe_tune(const char *key, int value) {
  if (!key) return QE_EINVAL;
  if (!strcmp(key, "blocks_per_cu")) {
    if (value < 0 || value > 32) return QE_ERANGE;
    g_blocks_per_cu = value;
    return QE_OK;
  }
  if (!strcmp(key, "tiles_per_wave")) {
    if (value < -1 || value > 4096) return QE_ERANGE;
    g_tiles_per_wave = value;
    return QE_OK;
  }
  if (!strcmp(key, "cv_kernel")) {
    if (value < -1 || value > 1) return QE_ERANGE;
    g_cv_kernel = value;
    return QE_OK;
  }
  if (!strcmp(key, "repl_kernel")) {
    if (value < -1 || value > 1) return QE_ERANGE;
    g_repl_kernel = value;
    return QE_OK;
  }
  if (!strcmp(key, "nontemporal")) {
    if (value < 0 || value > 3) return QE_ERANGE;
    g_nontemporal = value;
    return QE_OK;
  }
  return QE_EINVAL;
}

static int check_groups(const qe_groups *g) {
  if (!g) return QE_EINVAL;
  if (g->num_slots == 0 || g->num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (g->reserved != 0) return QE_EINVAL;
  if (g->num_groups && g->stride < g->num_groups) return QE_EINVAL;
  if (g->out_mask && !g->inc_mask) return QE_EINVAL;
  return QE_OK;
}

int qe_commit_vote(const qe_groups *g, const qe_outputs *out, void *stream) {
  int rc = check_groups(g);
  if (rc) return rc;
  if (!out) return QE_EINVAL;
  if (g->num_groups == 0) return QE_OK;
  if (!g->match) return QE_EINVAL;
  CVArgs a{};
  a.G = g->num_groups;
  a.goff = g->group_offset;
  a.stride = g->stride;
  a.match = g->match;
  a.inc = g->inc_mask;
  a.out = g->out_mask;
  a.learner = g->learner_mask;
  a.voted = g->voted;
  a.granted = g->granted;
  a.commit = out->commit;
  a.vote = out->vote;
  a.gcount = out->granted_count;
  a.rcount = out->rejected_count;
  a.stats = out->stats;
  const int mode = g->out_mask ? 2 : (g->inc_mask ? 1 : 0);
  const size_t mb = qe_mask_bytes(g->num_slots);
  bool vec = al(g->match, 16) && (g->stride % 2 == 0) && al(out->commit, 16);
  const void *masks[] = {g->inc_mask, g->out_mask, g->learner_mask, g->voted, g->granted};
  for (const void *m : masks) vec = vec && al(m, 2 * mb);
  const uint8_t *bytes[] = {out->vote, out->granted_count, out->rejected_count};
  for (const uint8_t *b : bytes) vec = vec && al(b, 2);
  return dispatch_cv(g->num_slots, a, mode, vec, static_cast<hipStream_t>(stream));
}

int qe_committed_index(const qe_groups *g, uint64_t *commit, void *stream) {
  if (!g || !commit) return QE_EINVAL;
  qe_groups gg = *g;
  gg.voted = nullptr;
  gg.granted = nullptr;
  qe_outputs o{};
  o.commit = commit;
  return qe_commit_vote(&gg, &o, stream);
}

int qe_vote_result(const qe_groups *g, uint8_t *vote, void *stream) {
  int rc = check_groups(g);
  if (rc) return rc;
  if (!vote) return QE_EINVAL;
  if (g->num_groups == 0) return QE_OK;
  const uint32_t full = (1u << g->num_slots) - 1u;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned grid = simple_grid(g->num_groups);
  if (g->num_slots <= 8)
    hipLaunchKernelGGL(k_vote_result<uint8_t>, dim3(grid), dim3(kBlock), 0, st, g->num_groups,
                       full, g->inc_mask, g->out_mask, g->voted, g->granted, vote);
  else
    hipLaunchKernelGGL(k_vote_result<uint16_t>, dim3(grid), dim3(kBlock), 0, st,
                       g->num_groups, full, g->inc_mask, g->out_mask, g->voted, g->granted,
                       vote);
  return hip_status(hipGetLastError());
}

int qe_quorum_active(const qe_groups *g, const void *recent_active, uint8_t *active,
                     void *stream) {
  int rc = check_groups(g);
  if (rc) return rc;
  if (!recent_active || !active) return QE_EINVAL;
  if (g->num_groups == 0) return QE_OK;
  const uint32_t full = (1u << g->num_slots) - 1u;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned grid = simple_grid(g->num_groups);
  if (g->num_slots <= 8)
    hipLaunchKernelGGL(k_quorum_active<uint8_t>, dim3(grid), dim3(kBlock), 0, st,
                       g->num_groups, full, g->inc_mask, g->out_mask, g->learner_mask,
                       recent_active, active);
  else
    hipLaunchKernelGGL(k_quorum_active<uint16_t>, dim3(grid), dim3(kBlock), 0, st,
                       g->num_groups, full, g->inc_mask, g->out_mask, g->learner_mask,
                       recent_active, active);
  return hip_status(hipGetLastError());
}

int qe_record_votes(uint64_t num_groups, uint32_t num_slots, void *voted, void *granted,
                    const void *resp_mask, const void *resp_value, void *stream) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (num_groups == 0) return QE_OK;
  if (!voted || !granted || !resp_mask || !resp_value) return QE_EINVAL;
  const uint32_t full = (1u << num_slots) - 1u;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned grid = simple_grid(num_groups);
  if (num_slots <= 8)
    hipLaunchKernelGGL(k_record_votes<uint8_t>, dim3(grid), dim3(kBlock), 0, st, num_groups,
                       full, voted, granted, resp_mask, resp_value);
  else
    hipLaunchKernelGGL(k_record_votes<uint16_t>, dim3(grid), dim3(kBlock), 0, st, num_groups,
                       full, voted, granted, resp_mask, resp_value);
  return hip_status(hipGetLastError());
}

int qe_replication_round(const qe_repl_state *s, const qe_repl_msgs *m, uint64_t *stats,
                         void *stream) {
  if (!s || !m) return QE_EINVAL;
  if (s->num_slots == 0 || s->num_slots > QE_MAX_SLOTS || s->reserved) return QE_EINVAL;
  if (s->num_groups == 0) return QE_OK;
  if (s->stride < s->num_groups) return QE_EINVAL;
  if (!s->match || !s->next || !s->committed || !s->term_start || !s->last_index ||
      !m->resp_index)
    return QE_EINVAL;
  if (s->out_mask && !s->inc_mask) return QE_EINVAL;
  RArgs a{};
  a.G = s->num_groups;
  a.goff = s->group_offset;
  a.stride = s->stride;
  a.match = s->match;
  a.next = s->next;
  a.committed = s->committed;
  a.term_start = s->term_start;
  a.last_index = s->last_index;
  a.resp = m->resp_index;
  a.inc = s->inc_mask;
  a.out = s->out_mask;
  a.resp_mask = m->resp_mask;
  a.read_acks = m->read_acks;
  a.read_ok = m->read_ok;
  a.adv = m->commit_advanced;
  a.stats = stats;
  const size_t mb = qe_mask_bytes(s->num_slots);
  bool vec = (s->stride % 2 == 0);
  const void *p16[] = {s->match, s->next, s->committed, s->term_start, s->last_index,
                       m->resp_index};
  for (const void *p : p16) vec = vec && al(p, 16);
  const void *pm[] = {s->inc_mask, s->out_mask, m->resp_mask, m->read_acks};
  for (const void *p : pm) vec = vec && al(p, 2 * mb);
  vec = vec && al(m->read_ok, 2) && al(m->commit_advanced, 2);
  return dispatch_repl(s->num_slots, a, s->inc_mask != nullptr, s->out_mask != nullptr, vec,
                       static_cast<hipStream_t>(stream));
}

int qe_election_steps(const qe_election_state *s, const qe_election_params *p, uint64_t *stats,
                      void *stream) {
  if (!s || !p) return QE_EINVAL;
  if (s->num_slots == 0 || s->num_slots > QE_MAX_SLOTS || s->reserved) return QE_EINVAL;
  if (s->num_groups == 0) return QE_OK;
  if (!s->term || !s->state || !s->voted || !s->granted || !s->self_slot) return QE_EINVAL;
  if (s->out_mask && !s->inc_mask) return QE_EINVAL;
  if (p->p_drop_q16 > 65536 || p->p_grant_q16 > 65536 || p->p_active_q16 > 65536)
    return QE_ERANGE;
  if (p->flags & ~(QE_ELEC_PREVOTE | QE_ELEC_CHECK_QUORUM)) return QE_EINVAL;
  if (p->reserved) return QE_EINVAL;
  if (p->script_resp && (!p->script_grant || p->script_stride < s->num_groups)) return QE_EINVAL;
  EArgs a{};
  a.G = s->num_groups;
  a.goff = s->group_offset;
  a.term = s->term;
  a.state = s->state;
  a.voted = s->voted;
  a.granted = s->granted;
  a.self_slot = s->self_slot;
  a.inc = s->inc_mask;
  a.out = s->out_mask;
  a.learner = s->learner_mask;
  a.seed = p->seed;
  a.step0 = p->step0;
  a.steps = p->steps;
  a.p_drop = p->p_drop_q16;
  a.p_grant = p->p_grant_q16;
  a.flags = p->flags;
  a.p_active = p->p_active_q16;
  a.sresp = p->script_resp;
  a.sgrant = p->script_grant;
  a.shup = p->script_resp ? p->script_hup : nullptr;
  a.sstride = p->script_stride;
  a.stats = stats;
  return dispatch_elec(s->num_slots, a, static_cast<hipStream_t>(stream));
}

int qe_apply_append_resps(uint64_t num_groups, uint32_t num_slots, uint64_t stride,
                          uint64_t *match, uint64_t *next, uint64_t n, const uint64_t *group,
                          const int8_t *slot, const uint64_t *index, uint8_t *touched,
                          void *stream) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (n == 0 || num_groups == 0) return QE_OK;
  if (stride < num_groups || !match || !next || !group || !slot || !index) return QE_EINVAL;
  hipLaunchKernelGGL(k_apply_acks, dim3(simple_grid(n)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), num_groups, num_slots, stride, match,
                     next, n, group, slot, index, touched);
  return hip_status(hipGetLastError());
}

// The ReadIndex queue's ABI 7 fields: a capacity of 0 is QE_READ_QUEUE (the
// ABI 5 queue); a longer queue needs the overflow ring.
static int read_queue_args(const qe_progress *p, PArgs &a) {
  if (p->reserved3) return QE_EINVAL;
  if (p->read_cap != 0 && (p->read_cap < QE_READ_QUEUE || p->read_cap > QE_READ_CAP_MAX))
    return QE_ERANGE;
  a.read_cap = p->read_cap ? p->read_cap : QE_READ_QUEUE;
  if (p->read_acks && a.read_cap > QE_READ_QUEUE && !p->read_ovf) return QE_EINVAL;
  a.read_ovf = p->read_ovf;
  a.read_keys = p->read_keys;
  return QE_OK;
}

static int progress_args(const qe_progress *p, PArgs &a) {
  if (!p) return QE_EINVAL;
  if (p->num_slots == 0 || p->num_slots > QE_MAX_SLOTS || p->reserved || p->reserved2)
    return QE_EINVAL;
  if (p->inflight_cap == 0 || p->inflight_cap > QE_MAX_INFLIGHT) return QE_ERANGE;
  if (p->log_runs > QE_MAX_LOG_RUNS) return QE_ERANGE;
  if (p->num_groups && p->stride < p->num_groups) return QE_EINVAL;
  if (p->out_mask && !p->inc_mask) return QE_EINVAL;
  if (p->num_groups &&
      (!p->match || !p->next || !p->pending_snapshot || !p->peer || !p->infl_lo || !p->infl_hi ||
       !p->committed || !p->term_start || !p->first_index || !p->last_index))
    return QE_EINVAL;
  if (p->num_groups && p->log_runs && (!p->run_first || !p->run_term || !p->run_count))
    return QE_EINVAL;
  // a slot's ring block of a 64-group tile is addressed with 32-bit offsets
  if (static_cast<uint64_t>(QE_RING_PITCH(p->inflight_cap)) * 4 * 64 > 0x7FFFFFFFull)
    return QE_ERANGE;
  // ABI 8: the 16-bit Inflights form exists for the pipelined kernels' shapes
  if (p->infl16 && (p->inflight_cap > QE_RING16_MAX_F || p->num_slots > QE_RING16_MAX_SLOTS ||
                    p->log_runs > 4))
    return QE_ERANGE;
  a = PArgs{};
  a.G = p->num_groups;
  a.goff = p->group_offset;
  a.stride = p->stride;
  a.F = p->inflight_cap;
  a.R = p->log_runs;
  a.match = p->match;
  a.next = p->next;
  a.pending = p->pending_snapshot;
  a.pw = p->peer;
  a.ilo = p->infl_lo;
  a.ihi = p->infl_hi;
  a.infl16 = p->infl16;
  a.FP = QE_RING_PITCH(p->inflight_cap);
  a.committed = p->committed;
  a.term_start = p->term_start;
  a.first_index = p->first_index;
  a.last_index = p->last_index;
  a.snap_index = p->snap_index;
  a.run_first = p->run_first;
  a.run_term = p->run_term;
  a.run_count = p->run_count;
  a.inc = p->inc_mask;
  a.out = p->out_mask;
  a.tracked = p->tracked;
  a.self_slot = p->self_slot;
  a.transferee = p->lead_transferee;
  a.max_ents = p->max_ents;
  a.read_acks = p->read_acks;
  a.read_head = p->read_head;
  a.read_count = p->read_count;
  return read_queue_args(p, a);
}

int qe_progress_step(const qe_progress *p, const qe_peer_msgs *m, uint64_t *stats,
                     void *stream) {
  PArgs a;
  int rc = progress_args(p, a);
  if (rc) return rc;
  if (!m) return QE_EINVAL;
  if (p->num_groups == 0) return QE_OK;
  if (!m->type || !m->index || !m->reject_hint || !m->log_term) return QE_EINVAL;
  if (p->log_runs == 0) return QE_EINVAL;  // findConflictByTerm needs the log model
  a.mtype = m->type;
  a.mindex = m->index;
  a.mhint = m->reject_hint;
  a.mlogterm = m->log_term;
  a.sent = m->sent;
  a.bcast = m->bcast;
  a.snap = m->snap;
  a.tnow = m->timeout_now;
  a.msg_count = m->msg_count;
  a.msg_index = m->msg_index;
  a.acct = m->bytes_requested;
  // ABI 5: the ReadIndex queue comes whole or not at all
  if (p->read_acks && (!p->read_head || !p->read_count)) return QE_EINVAL;
  a.read_ctx = p->read_acks ? m->read_ctx : nullptr;
  a.read_released = m->read_released;
  a.term_commit = m->term_commit;
  a.term_commit_index = m->term_commit_index;
  a.stats = stats;
  const int kind = m->bytes_requested ? 2 : 0;
  return dispatch_progress(p->num_slots, a, kind, p->inc_mask != nullptr, p->out_mask != nullptr,
                           static_cast<hipStream_t>(stream));
}

int qe_progress_send(const qe_progress *p, const void *want, uint32_t send_if_empty,
                     void *sent, void *snap, void *stream) {
  PArgs a;
  int rc = progress_args(p, a);
  if (rc) return rc;
  if (p->num_groups == 0) return QE_OK;
  if (!want) return QE_EINVAL;
  a.want = want;
  a.send_if_empty = send_if_empty;
  a.sent = sent;
  a.snap = snap;
  return dispatch_progress(p->num_slots, a, 1, false, false, static_cast<hipStream_t>(stream));
}

int qe_propose(const qe_progress *p, const qe_proposals *prop, uint64_t *stats, void *stream) {
  PArgs a;
  int rc = progress_args(p, a);
  if (rc) return rc;
  if (!prop || (prop->flags & ~QE_PROP_APPEND_ONLY)) return QE_EINVAL;
  if (prop->max_cc > QE_PROP_MAX_CC) return QE_ERANGE;
  if (p->num_groups == 0) return QE_OK;
  if (!prop->num_entries || !prop->result) return QE_EINVAL;
  if (!p->self_slot) return QE_EINVAL;  // MsgProp is handled by the leader: its slot is needed
  if (prop->max_cc && (!prop->cc_count || !prop->cc_pos || !prop->cc_leave || !prop->cc_size ||
                       !prop->applied || !prop->pending_conf_index ||
                       prop->cc_stride < p->num_groups))
    return QE_EINVAL;
  if (!prop->uncommitted_size && prop->max_uncommitted) return QE_EINVAL;
  a.prop_n = prop->num_entries;
  a.prop_payload = prop->payload;
  const bool append_only = (prop->flags & QE_PROP_APPEND_ONLY) != 0;
  a.max_cc = append_only ? 0u : prop->max_cc;
  a.prop_flags = prop->flags;
  a.cc_stride = prop->cc_stride;
  a.cc_count = prop->cc_count;
  a.cc_pos = prop->cc_pos;
  a.cc_leave = prop->cc_leave;
  a.cc_size = prop->cc_size;
  a.applied = prop->applied;
  a.pci = prop->pending_conf_index;
  a.unc = prop->uncommitted_size;
  a.max_unc = prop->max_uncommitted;
  a.prop_result = prop->result;
  a.cc_refused = prop->cc_refused;
  a.sent = prop->sent;
  a.snap = prop->snap;
  a.acct = prop->bytes_requested;
  a.last_index_rw = const_cast<uint64_t *>(p->last_index);
  a.stats = stats;
  return dispatch_progress(p->num_slots, a, prop->bytes_requested ? 6 : 5, p->inc_mask != nullptr,
                           p->out_mask != nullptr, static_cast<hipStream_t>(stream));
}

int qe_switch_config(const qe_progress *p, const qe_switch *sw, uint64_t *stats, void *stream) {
  PArgs a;
  int rc = progress_args(p, a);
  if (rc) return rc;
  if (!sw) return QE_EINVAL;
  if (p->num_groups == 0) return QE_OK;
  if (!sw->result) return QE_EINVAL;
  a.sw_switched = sw->switched;
  a.sw_result = sw->result;
  a.sent = sw->sent;
  a.snap = sw->snap;
  a.acct = sw->bytes_requested;
  a.stats = stats;
  return dispatch_progress(p->num_slots, a, sw->bytes_requested ? 9 : 8, p->inc_mask != nullptr,
                           p->out_mask != nullptr, static_cast<hipStream_t>(stream));
}

int qe_become_leader(const qe_progress *p, const qe_leader *l, uint64_t *stats, void *stream) {
  PArgs a;
  int rc = progress_args(p, a);
  if (rc) return rc;
  if (!l || l->reserved || (l->flags & ~QE_BL_BCAST)) return QE_EINVAL;
  if (p->num_groups == 0) return QE_OK;
  if (!l->term || !l->result || !p->self_slot) return QE_EINVAL;
  if (p->log_runs && !p->run_count) return QE_EINVAL;
  a.bl_elected = l->elected;
  a.bl_term = l->term;
  a.bl_flags = l->flags;
  a.bl_pci = l->pending_conf_index;
  a.bl_unc = l->uncommitted_size;
  a.bl_result = l->result;
  a.sent = l->sent;
  a.snap = l->snap;
  a.stats = stats;
  return dispatch_progress(p->num_slots, a, 10, p->inc_mask != nullptr, p->out_mask != nullptr,
                           static_cast<hipStream_t>(stream));
}

int qe_heartbeat(const qe_progress *p, uint64_t *commit, uint32_t *ctx, void *sent, void *stream) {
  if (!p) return QE_EINVAL;
  if (p->num_slots == 0 || p->num_slots > QE_MAX_SLOTS || p->reserved || p->reserved2)
    return QE_EINVAL;
  if (p->num_groups == 0) return QE_OK;
  if (p->stride < p->num_groups || !p->match || !p->committed || !commit) return QE_EINVAL;
  if (p->read_acks && (!p->read_head || !p->read_count)) return QE_EINVAL;
  PArgs a{};
  a.G = p->num_groups;
  a.stride = p->stride;
  a.match = p->match;
  a.committed = p->committed;
  a.tracked = p->tracked;
  a.self_slot = p->self_slot;
  a.read_acks = p->read_acks;
  a.read_head = p->read_head;
  a.read_count = p->read_count;
  const int rq = read_queue_args(p, a);
  if (rq) return rq;
  a.hb_commit = commit;
  a.hb_ctx = ctx;
  a.sent = sent;
  return dispatch_progress(p->num_slots, a, 7, false, false, static_cast<hipStream_t>(stream));
}

int qe_read_index(const qe_progress *p, const uint8_t *request, const uint64_t *key,
                  uint32_t lease_based, uint8_t *result, uint32_t *ctx, uint64_t *index,
                  void *stream) {
  if (!p) return QE_EINVAL;
  if (p->num_slots == 0 || p->num_slots > QE_MAX_SLOTS || p->reserved || p->reserved2)
    return QE_EINVAL;
  if (p->num_groups == 0) return QE_OK;
  if (p->stride < p->num_groups || !request || !result) return QE_EINVAL;
  if (!p->committed || !p->term_start || !p->last_index) return QE_EINVAL;
  if (p->out_mask && !p->inc_mask) return QE_EINVAL;
  // ReadOnlySafe queues: the queue must be there
  if (!lease_based && (!p->read_acks || !p->read_head || !p->read_count)) return QE_EINVAL;
  PArgs a{};
  a.G = p->num_groups;
  a.goff = p->group_offset;
  a.stride = p->stride;
  a.committed = p->committed;
  a.term_start = p->term_start;
  a.last_index = p->last_index;
  a.inc = p->inc_mask;
  a.out = p->out_mask;
  a.self_slot = p->self_slot;
  a.read_acks = p->read_acks;
  a.read_head = p->read_head;
  a.read_count = p->read_count;
  const int rq = read_queue_args(p, a);
  if (rq) return rq;
  a.ri_key = p->read_keys ? key : nullptr;  // keys are checked only when the state keeps them
  a.ri_request = request;
  a.ri_result = result;
  a.ri_ctx = ctx;
  a.ri_index = index;
  a.lease_based = lease_based ? 1u : 0u;
  return dispatch_progress(p->num_slots, a, 4, p->inc_mask != nullptr, p->out_mask != nullptr,
                           static_cast<hipStream_t>(stream));
}

int qe_check_quorum(const qe_progress *p, uint8_t *quorum_active, uint64_t *stats,
                    void *stream) {
  if (!p) return QE_EINVAL;
  if (p->num_slots == 0 || p->num_slots > QE_MAX_SLOTS || p->reserved || p->reserved2)
    return QE_EINVAL;
  if (p->num_groups == 0) return QE_OK;
  if (p->stride < p->num_groups || !p->peer) return QE_EINVAL;
  if (p->out_mask && !p->inc_mask) return QE_EINVAL;
  PArgs a{};
  a.G = p->num_groups;
  a.goff = p->group_offset;
  a.stride = p->stride;
  a.pw = p->peer;
  a.inc = p->inc_mask;
  a.out = p->out_mask;
  a.tracked = p->tracked;
  a.self_slot = p->self_slot;
  a.qactive = quorum_active;
  a.stats = stats;
  return dispatch_progress(p->num_slots, a, 3, p->inc_mask != nullptr, p->out_mask != nullptr,
                           static_cast<hipStream_t>(stream));
}

int qe_confchange(const qe_conf *c, const qe_conf_changes *ch, const qe_progress *p,
                  void *stream) {
  if (!c || !ch) return QE_EINVAL;
  if (c->num_slots == 0 || c->num_slots > QE_MAX_SLOTS || c->reserved) return QE_EINVAL;
  if (c->num_groups == 0) return QE_OK;
  if (!c->slot_ids || !c->inc_mask || !c->out_mask || !c->learner_mask ||
      !c->learners_next_mask || !c->is_learner || !c->tracked || !c->auto_leave)
    return QE_EINVAL;
  if (!ch->op || !ch->count || !ch->last_index || !ch->result) return QE_EINVAL;
  if (ch->max_changes > 255) return QE_EINVAL;  // count is a u8 per group
  if (ch->max_changes > 0 && (!ch->type || !ch->node_id || ch->stride < c->num_groups))
    return QE_EINVAL;
  CCArgs a{};
  a.G = c->num_groups;
  a.C = ch->max_changes;
  a.stride = ch->stride;
  a.ids = c->slot_ids;
  a.inc = c->inc_mask;
  a.out = c->out_mask;
  a.lrn = c->learner_mask;
  a.lnx = c->learners_next_mask;
  a.isl = c->is_learner;
  a.trk = c->tracked;
  a.auto_leave = c->auto_leave;
  a.op = ch->op;
  a.count = ch->count;
  a.type = ch->type;
  a.node = ch->node_id;
  a.last_index = ch->last_index;
  a.result = ch->result;
  a.new_progress = ch->new_progress;
  if (p) {
    if (p->num_groups != c->num_groups || p->num_slots != c->num_slots ||
        p->stride < p->num_groups)
      return QE_EINVAL;
    if (!p->match || !p->next || !p->pending_snapshot || !p->peer) return QE_EINVAL;
    a.pstride = p->stride;
    a.p_match = p->match;
    a.p_next = p->next;
    a.p_pending = p->pending_snapshot;
    a.p_pw = p->peer;
  }
  // chunks of up to kCCTPW tiles per wave, >= 2 so the two register sets
  // overlap; shorter chunks when the batch cannot give every CU 32 waves
  const uint64_t tiles = (a.G + 63) / 64;
  const uint64_t waves = static_cast<uint64_t>(num_cus()) * 32;
  uint64_t chunk = g_tiles_per_wave > 0 ? static_cast<uint64_t>(g_tiles_per_wave)
                                        : (tiles + waves - 1) / waves;
  if (chunk < 2) chunk = 2;
  if (chunk > static_cast<uint64_t>(kCCTPW)) chunk = kCCTPW;
  a.chunk = static_cast<uint32_t>(chunk);
  const uint64_t per_block = (kBlock / 64) * chunk;
  const uint64_t blocks = (tiles + per_block - 1) / per_block;
  if (blocks > 0x7FFFFFFFull) return QE_ERANGE;
  const dim3 grid(static_cast<unsigned>(blocks));
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (c->num_slots) {
#define QE_CC_CASE(n) \
  case n: hipLaunchKernelGGL(k_confchange<n>, grid, dim3(kBlock), 0, st, a); break;
    QE_CC_CASE(1) QE_CC_CASE(2) QE_CC_CASE(3) QE_CC_CASE(4) QE_CC_CASE(5) QE_CC_CASE(6)
    QE_CC_CASE(7) QE_CC_CASE(8) QE_CC_CASE(9) QE_CC_CASE(10) QE_CC_CASE(11) QE_CC_CASE(12)
    QE_CC_CASE(13) QE_CC_CASE(14) QE_CC_CASE(15) QE_CC_CASE(16)
#undef QE_CC_CASE
  }
  return hip_status(hipGetLastError());
}

size_t qe_collect_scratch_bytes(uint64_t num_groups) {
  const uint64_t nb = (num_groups + kCollectChunk - 1) / kCollectChunk;
  return static_cast<size_t>(nb * (sizeof(uint32_t) + sizeof(uint64_t)) + 64);
}

int qe_collect(uint64_t num_groups, uint64_t group_offset, const uint64_t *perm,
               const uint8_t *flags, const uint64_t *values, uint64_t *out_groups,
               uint64_t *out_values, uint64_t *out_count, void *scratch, void *stream) {
  if (!out_count || (num_groups && (!flags || !scratch))) return QE_EINVAL;
  if (out_values && !values) return QE_EINVAL;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (num_groups == 0)
    return hip_status(hipMemsetAsync(out_count, 0, sizeof(uint64_t), st));
  const uint64_t nb = (num_groups + kCollectChunk - 1) / kCollectChunk;
  if (nb > 0x7FFFFFFFull) return QE_ERANGE;
  // scratch: offsets (u64, 8-B aligned at the start), then counts (u32)
  if (reinterpret_cast<uintptr_t>(scratch) % 8) return QE_EINVAL;
  uint64_t *offsets = static_cast<uint64_t *>(scratch);
  uint32_t *counts = reinterpret_cast<uint32_t *>(offsets + nb);
  const bool vec = (reinterpret_cast<uintptr_t>(flags) % 16) == 0;
  hipLaunchKernelGGL(k_collect_count, dim3(static_cast<unsigned>((nb + kCountWaves - 1) / kCountWaves)),
                     dim3(kBlock), 0, st, flags, num_groups, vec, nb, counts);
  hipLaunchKernelGGL(k_collect_scan, dim3(1), dim3(1024), 0, st, counts, nb, offsets, out_count);
  hipLaunchKernelGGL(k_collect_scatter, dim3(static_cast<unsigned>(nb)), dim3(kBlock), 0, st, flags,
                     num_groups, vec, group_offset, perm, values, offsets, out_groups, out_values);
  return hip_status(hipGetLastError());
}

int qe_stats_reduce(const uint64_t *stats, uint64_t *out, void *stream) {
  if (!stats || !out) return QE_EINVAL;
  hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                     stats, out);
  return hip_status(hipGetLastError());
}

int qe_gen_groups(const qe_groups *g, const qe_gen_params *p, void *stream) {
  int rc = check_groups(g);
  if (rc) return rc;
  if (!p) return QE_EINVAL;
  if (g->num_groups == 0) return QE_OK;
  if (p->p_absent_q16 > 65536 || p->p_voted_q16 > 65536 || p->p_granted_q16 > 65536)
    return QE_ERANGE;
  GArgs a{};
  a.G = g->num_groups;
  a.goff = g->group_offset;
  a.stride = g->stride;
  a.S = g->num_slots;
  a.match = const_cast<uint64_t *>(g->match);
  a.inc = const_cast<void *>(g->inc_mask);
  a.out = const_cast<void *>(g->out_mask);
  a.learner = const_cast<void *>(g->learner_mask);
  a.voted = const_cast<void *>(g->voted);
  a.granted = const_cast<void *>(g->granted);
  a.p = *p;
  // qe_gen_params.group_offset adds to qe_groups.group_offset.
  a.goff = g->group_offset + p->group_offset;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned grid = simple_grid(g->num_groups);
  if (g->num_slots <= 8)
    hipLaunchKernelGGL(k_gen<uint8_t>, dim3(grid), dim3(kBlock), 0, st, a);
  else
    hipLaunchKernelGGL(k_gen<uint16_t>, dim3(grid), dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

}  // extern "C"
