// qe_host.cpp — C++ host mirror of raft/quorum + raft/tracker
// (include/etcd_quorum.hpp).  Groups are packed into the slot-SoA layout
// (voters of both halves ascending, then learners: etcd_amd/packing.py uses
// the same order), copied to a grow-only device arena and evaluated by the
// C ABI kernels; results are copied back.  Decisions never run on the CPU.
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <sstream>

#include "../../include/etcd_quorum.hpp"

namespace etcd_amd {

EngineError::EngineError(const std::string &fn, int st)
    : std::runtime_error(fn + " failed: " + std::to_string(st) + " (" + qe_strerror(st) + ")"),
      status(st) {}

namespace {

void check(const char *fn, int st) {
  if (st != QE_OK) throw EngineError(fn, st);
}
void hip_check(const char *fn, hipError_t e) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string(fn) + ": " + hipGetErrorString(e));
}

// Grow-only device arena, one per process (calls are serialised).
struct Arena {
  std::mutex mu;
  void *ptr = nullptr;
  size_t cap = 0;
  void *get(size_t bytes) {
    if (bytes > cap) {
      if (ptr) hip_check("hipFree", hipFree(ptr));
      size_t n = std::max<size_t>(bytes, 1 << 20);
      hip_check("hipMalloc", hipMalloc(&ptr, n));
      cap = n;
    }
    return ptr;
  }
};
Arena g_arena;

struct Group {
  const std::set<uint64_t> *c0, *c1;
  std::vector<uint64_t> learners;
  const quorum::AckedIndexer *acked = nullptr;
  const std::map<uint64_t, uint64_t> *match = nullptr;
  const quorum::Votes *votes = nullptr;
  std::vector<uint64_t> recent;
};

// Slot-SoA host image of a batch; offsets of each array inside one buffer.
struct Packed {
  uint64_t G = 0, stride = 0;
  uint32_t S = 1, mb = 1;
  std::vector<uint8_t> buf;
  size_t off_match = 0, off_inc = 0, off_out = 0, off_lrn = 0, off_vd = 0, off_gr = 0,
         off_rec = 0, off_commit = 0, off_vote = 0, off_gc = 0, off_rc = 0, off_act = 0, size = 0;
  void put_mask(size_t off, uint64_t g, uint32_t v) {
    if (mb == 1) buf[off + g] = static_cast<uint8_t>(v);
    else memcpy(&buf[off + 2 * g], &v, 2);
  }
};

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

Packed pack(const std::vector<Group> &gs) {
  Packed p;
  p.G = gs.size();
  std::vector<std::vector<uint64_t>> orders(gs.size());
  uint32_t need = 1;
  for (size_t i = 0; i < gs.size(); i++) {
    std::vector<uint64_t> v(gs[i].c0->begin(), gs[i].c0->end());
    v.insert(v.end(), gs[i].c1->begin(), gs[i].c1->end());
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    std::vector<uint64_t> l;
    for (uint64_t id : gs[i].learners)
      if (!std::binary_search(v.begin(), v.end(), id)) l.push_back(id);
    std::sort(l.begin(), l.end());
    l.erase(std::unique(l.begin(), l.end()), l.end());
    v.insert(v.end(), l.begin(), l.end());
    need = std::max<uint32_t>(need, static_cast<uint32_t>(v.size()));
    orders[i] = std::move(v);
  }
  if (need > QE_MAX_SLOTS) throw EngineError("pack", QE_ERANGE);
  p.S = need;
  p.mb = static_cast<uint32_t>(qe_mask_bytes(p.S));
  p.stride = std::max<uint64_t>(64, (p.G + 63) / 64 * 64);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    size_t r = o;
    o = align256(o + bytes);
    return r;
  };
  p.off_match = take(8 * p.S * p.stride);
  p.off_inc = take(p.mb * p.G);
  p.off_out = take(p.mb * p.G);
  p.off_lrn = take(p.mb * p.G);
  p.off_vd = take(p.mb * p.G);
  p.off_gr = take(p.mb * p.G);
  p.off_rec = take(p.mb * p.G);
  p.off_commit = take(8 * p.G);
  p.off_vote = take(p.G);
  p.off_gc = take(p.G);
  p.off_rc = take(p.G);
  p.off_act = take(p.G);
  p.size = o;
  p.buf.assign(p.off_commit, 0);  // inputs only; outputs come back separately
  uint64_t *match = reinterpret_cast<uint64_t *>(&p.buf[p.off_match]);
  for (size_t g = 0; g < gs.size(); g++) {
    const Group &gr = gs[g];
    uint32_t mi = 0, mo = 0, ml = 0, vd = 0, gv = 0, ra = 0;
    const auto &ord = orders[g];
    for (uint32_t s = 0; s < ord.size(); s++) {
      const uint64_t id = ord[s], bit = 1u << s;
      if (gr.c0->count(id)) mi |= bit;
      if (gr.c1->count(id)) mo |= bit;
      if (std::find(gr.learners.begin(), gr.learners.end(), id) != gr.learners.end() &&
          !(mi & bit) && !(mo & bit))
        ml |= bit;
      uint64_t idx = 0;
      if (gr.acked) {
        quorum::Index x = 0;
        if (gr.acked->AckedIndex(id, &x)) idx = x;  // absent == 0 (majority.go:150-161)
      } else if (gr.match) {
        auto it = gr.match->find(id);
        if (it != gr.match->end()) idx = it->second;
      }
      match[s * p.stride + g] = idx;
      if (gr.votes) {
        auto it = gr.votes->find(id);
        if (it != gr.votes->end()) {
          vd |= bit;
          if (it->second) gv |= bit;
        }
      }
      if (std::find(gr.recent.begin(), gr.recent.end(), id) != gr.recent.end()) ra |= bit;
    }
    p.put_mask(p.off_inc, g, mi);
    p.put_mask(p.off_out, g, mo);
    p.put_mask(p.off_lrn, g, ml);
    p.put_mask(p.off_vd, g, vd);
    p.put_mask(p.off_gr, g, gv);
    p.put_mask(p.off_rec, g, ra);
  }
  return p;
}

struct Results {
  std::vector<uint64_t> commit;
  std::vector<uint8_t> vote, gc, rc, active;
};

Results run(const Packed &p, bool quorum_active) {
  Results r;
  if (p.G == 0) return r;
  std::lock_guard<std::mutex> lk(g_arena.mu);
  uint8_t *d = static_cast<uint8_t *>(g_arena.get(p.size));
  hip_check("hipMemcpy", hipMemcpy(d, p.buf.data(), p.buf.size(), hipMemcpyHostToDevice));
  qe_groups g{};
  g.num_groups = p.G;
  g.num_slots = p.S;
  g.stride = p.stride;
  g.match = reinterpret_cast<const uint64_t *>(d + p.off_match);
  g.inc_mask = d + p.off_inc;
  g.out_mask = d + p.off_out;
  g.learner_mask = d + p.off_lrn;
  g.voted = d + p.off_vd;
  g.granted = d + p.off_gr;
  qe_outputs o{};
  o.commit = reinterpret_cast<uint64_t *>(d + p.off_commit);
  o.vote = d + p.off_vote;
  o.granted_count = d + p.off_gc;
  o.rejected_count = d + p.off_rc;
  check("qe_commit_vote", qe_commit_vote(&g, &o, nullptr));
  if (quorum_active)
    check("qe_quorum_active", qe_quorum_active(&g, d + p.off_rec, d + p.off_act, nullptr));
  r.commit.resize(p.G);
  r.vote.resize(p.G);
  r.gc.resize(p.G);
  r.rc.resize(p.G);
  hip_check("hipMemcpy", hipMemcpy(r.commit.data(), o.commit, 8 * p.G, hipMemcpyDeviceToHost));
  hip_check("hipMemcpy", hipMemcpy(r.vote.data(), o.vote, p.G, hipMemcpyDeviceToHost));
  hip_check("hipMemcpy", hipMemcpy(r.gc.data(), o.granted_count, p.G, hipMemcpyDeviceToHost));
  hip_check("hipMemcpy", hipMemcpy(r.rc.data(), o.rejected_count, p.G, hipMemcpyDeviceToHost));
  if (quorum_active) {
    r.active.resize(p.G);
    hip_check("hipMemcpy", hipMemcpy(r.active.data(), d + p.off_act, p.G, hipMemcpyDeviceToHost));
  }
  return r;
}

}  // namespace

namespace quorum {

std::string IndexString(Index i) { return i == kIndexInf ? "∞" : std::to_string(i); }

const char *VoteResultString(VoteResult r) {
  switch (r) {
    case VoteResult::VotePending: return "VotePending";
    case VoteResult::VoteLost: return "VoteLost";
    case VoteResult::VoteWon: return "VoteWon";
  }
  return "VoteResult(?)";
}

bool MapAckIndexer::AckedIndex(uint64_t voter_id, Index *idx) const {
  auto it = m.find(voter_id);
  if (it == m.end()) return false;
  *idx = it->second;
  return true;
}

std::string MajorityConfig::String() const {
  std::ostringstream os;
  os << '(';
  bool first = true;
  for (uint64_t id : ids) {
    if (!first) os << ' ';
    os << id;
    first = false;
  }
  os << ')';
  return os.str();
}

std::vector<uint64_t> MajorityConfig::Slice() const { return {ids.begin(), ids.end()}; }

// majority.go:45-101: sort by (index, id), the i-th gets bar i when its
// index is above its predecessor's (else 0), print sorted by id.
std::string MajorityConfig::Describe(const AckedIndexer &l) const {
  if (ids.empty()) return "<empty majority quorum>";
  struct Tup {
    uint64_t id;
    Index idx;
    bool ok;
    size_t bar;
  };
  const size_t n = ids.size();
  std::vector<Tup> info;
  info.reserve(n);
  for (uint64_t id : ids) {
    Index idx = 0;
    const bool ok = l.AckedIndex(id, &idx);
    info.push_back({id, ok ? idx : 0, ok, 0});
  }
  std::sort(info.begin(), info.end(), [](const Tup &a, const Tup &b) {
    return a.idx == b.idx ? a.id < b.id : a.idx < b.idx;
  });
  for (size_t i = 1; i < n; i++)
    if (info[i - 1].idx < info[i].idx) info[i].bar = i;
  std::sort(info.begin(), info.end(), [](const Tup &a, const Tup &b) { return a.id < b.id; });
  std::ostringstream os;
  os << std::string(n, ' ') << "    idx\n";
  for (const Tup &t : info) {
    if (!t.ok) os << '?' << std::string(n, ' ');
    else os << std::string(t.bar, 'x') << '>' << std::string(n - t.bar, ' ');
    char buf[64];
    snprintf(buf, sizeof(buf), " %5llu    (id=%llu)\n", static_cast<unsigned long long>(t.idx),
             static_cast<unsigned long long>(t.id));
    os << buf;
  }
  return os.str();
}

Index MajorityConfig::CommittedIndex(const AckedIndexer &l) const {
  return JointConfig(*this).CommittedIndex(l);
}

VoteResult MajorityConfig::VoteResult(const Votes &votes) const {
  return JointConfig(*this).VoteResult(votes);
}

std::string JointConfig::String() const {
  if (c[1].size() > 0) return c[0].String() + "&&" + c[1].String();
  return c[0].String();
}

std::set<uint64_t> JointConfig::IDs() const {
  std::set<uint64_t> s(c[0].ids);
  s.insert(c[1].ids.begin(), c[1].ids.end());
  return s;
}

std::string JointConfig::Describe(const AckedIndexer &l) const {
  return MajorityConfig(IDs()).Describe(l);
}

Index JointConfig::CommittedIndex(const AckedIndexer &l) const {
  return CommittedIndexBatch({*this}, {&l})[0];
}

VoteResult JointConfig::VoteResult(const Votes &votes) const {
  return VoteResultBatch({*this}, {&votes})[0];
}

std::vector<Index> CommittedIndexBatch(const std::vector<JointConfig> &cfgs,
                                       const std::vector<const AckedIndexer *> &acked) {
  if (cfgs.size() != acked.size()) throw EngineError("CommittedIndexBatch", QE_EINVAL);
  std::vector<Group> gs(cfgs.size());
  for (size_t i = 0; i < cfgs.size(); i++) {
    gs[i].c0 = &cfgs[i].c[0].ids;
    gs[i].c1 = &cfgs[i].c[1].ids;
    gs[i].acked = acked[i];
  }
  return run(pack(gs), false).commit;
}

std::vector<VoteResult> VoteResultBatch(const std::vector<JointConfig> &cfgs,
                                        const std::vector<const Votes *> &votes) {
  if (cfgs.size() != votes.size()) throw EngineError("VoteResultBatch", QE_EINVAL);
  std::vector<Group> gs(cfgs.size());
  for (size_t i = 0; i < cfgs.size(); i++) {
    gs[i].c0 = &cfgs[i].c[0].ids;
    gs[i].c1 = &cfgs[i].c[1].ids;
    gs[i].votes = votes[i];
  }
  Results r = run(pack(gs), false);
  std::vector<VoteResult> out(r.vote.size());
  for (size_t i = 0; i < out.size(); i++) out[i] = static_cast<VoteResult>(r.vote[i]);
  return out;
}

}  // namespace quorum

namespace tracker {

std::string Progress::String() const {
  static const char *kState[] = {"StateProbe", "StateReplicate", "StateSnapshot"};
  std::string s = std::string(kState[State <= StateSnapshot ? State : 0]) +
                  " match=" + std::to_string(Match) + " next=" + std::to_string(Next);
  if (IsLearner) s += " learner";
  if (State == StateProbe && ProbeSent) s += " paused";
  if (PendingSnapshot > 0) s += " pendingSnap=" + std::to_string(PendingSnapshot);
  if (!RecentActive) s += " inactive";
  return s;
}

std::string Config::String() const {
  std::string s = "voters=" + Voters.String();
  if (!Learners.empty()) s += " learners=" + quorum::MajorityConfig(Learners).String();
  if (!LearnersNext.empty()) s += " learners_next=" + quorum::MajorityConfig(LearnersNext).String();
  if (AutoLeave) s += " autoleave";
  return s;
}

bool ProgressTracker::IsSingleton() const {
  return Voters.c[0].size() == 1 && Voters.c[1].size() == 0;
}

std::vector<uint64_t> ProgressTracker::VoterNodes() const {
  auto s = Voters.IDs();
  return {s.begin(), s.end()};
}

std::vector<uint64_t> ProgressTracker::LearnerNodes() const {
  return {Learners.begin(), Learners.end()};
}

void ProgressTracker::RecordVote(uint64_t id, bool v) { Votes.emplace(id, v); }

ProgressTracker MakeProgressTracker(int max_inflight) { return ProgressTracker(max_inflight); }

namespace {
struct TrackerPack {
  std::vector<std::map<uint64_t, uint64_t>> match;
  std::vector<Group> gs;
};

TrackerPack tracker_groups(const std::vector<const ProgressTracker *> &pts) {
  TrackerPack tp;
  tp.match.resize(pts.size());
  tp.gs.resize(pts.size());
  for (size_t i = 0; i < pts.size(); i++) {
    const ProgressTracker &pt = *pts[i];
    Group &g = tp.gs[i];
    g.c0 = &pt.Voters.c[0].ids;
    g.c1 = &pt.Voters.c[1].ids;
    for (const auto &kv : pt.Progress) {
      tp.match[i][kv.first] = kv.second.Match;  // matchAckIndexer, tracker.go:162-173
      if (kv.second.IsLearner) g.learners.push_back(kv.first);
      if (kv.second.RecentActive) g.recent.push_back(kv.first);
    }
    g.match = &tp.match[i];
    g.votes = &pt.Votes;
  }
  return tp;
}
}  // namespace

uint64_t ProgressTracker::Committed() const { return CommittedBatch({this})[0]; }
TallyResult ProgressTracker::TallyVotes() const { return TallyVotesBatch({this})[0]; }
bool ProgressTracker::QuorumActive() const { return QuorumActiveBatch({this})[0]; }

std::vector<uint64_t> CommittedBatch(const std::vector<const ProgressTracker *> &pts) {
  TrackerPack tp = tracker_groups(pts);
  return run(pack(tp.gs), false).commit;
}

std::vector<TallyResult> TallyVotesBatch(const std::vector<const ProgressTracker *> &pts) {
  TrackerPack tp = tracker_groups(pts);
  Results r = run(pack(tp.gs), false);
  std::vector<TallyResult> out(pts.size());
  for (size_t i = 0; i < out.size(); i++) {
    out[i].granted = r.gc[i];
    out[i].rejected = r.rc[i];
    out[i].result = static_cast<quorum::VoteResult>(r.vote[i]);
  }
  return out;
}

std::vector<bool> QuorumActiveBatch(const std::vector<const ProgressTracker *> &pts) {
  TrackerPack tp = tracker_groups(pts);
  Results r = run(pack(tp.gs), true);
  std::vector<bool> out(pts.size());
  for (size_t i = 0; i < out.size(); i++) out[i] = r.active[i] != 0;
  return out;
}

}  // namespace tracker

namespace confchange {

namespace {

const char *cc_error_text(int rc) {
  switch (rc) {
    case QE_CC_ERR_INVARIANT: return "invalid input configuration (checkInvariants)";
    case QE_CC_ERR_ALREADY_JOINT: return "config is already joint";
    case QE_CC_ERR_ZERO_VOTER_JOINT: return "can't make a zero-voter config joint";
    case QE_CC_ERR_NOT_JOINT: return "can't leave a non-joint config";
    case QE_CC_ERR_SIMPLE_IN_JOINT: return "can't apply simple config change in joint config";
    case QE_CC_ERR_BAD_TYPE: return "unexpected conf type";
    case QE_CC_ERR_REMOVED_ALL: return "removed all voters";
    case QE_CC_ERR_SIMPLE_MULTI:
      return "more than one voter changed without entering joint config";
    case QE_CC_ERR_INVARIANT_OUT: return "invalid resulting configuration (checkInvariants)";
    case QE_CC_ERR_NO_SLOT: return "more than 16 peers";
  }
  return "unknown confchange result";
}

}  // namespace

// Packs every tracker into slots (its Progress ids ascending), runs
// qe_confchange once for the batch and unpacks the results.  All groups
// share S = the largest (peers + changes) of the batch, capped at 16.
std::vector<Result> ChangeBatch(const std::vector<const Changer *> &changers,
                                const std::vector<Op> &ops,
                                const std::vector<std::vector<ConfChangeSingle>> &ccs) {
  const uint64_t G = changers.size();
  if (ops.size() != G || ccs.size() != G)
    throw std::invalid_argument("ChangeBatch: ops/ccs size mismatch");
  std::vector<Result> out(G);
  if (G == 0) return out;
  size_t need = 1, C = 0;
  for (uint64_t g = 0; g < G; g++) {
    // qe_conf_changes.count is a u8 per group: a longer change list cannot be
    // represented (the reference Changer has no such limit), so refuse it
    // instead of silently applying a truncated list
    if (ccs[g].size() > 255)
      throw std::invalid_argument("ChangeBatch: more than 255 changes in one group");
    need = std::max(need, changers[g]->Tracker.Progress.size() + ccs[g].size());
    C = std::max(C, ccs[g].size());
  }
  const uint32_t S = static_cast<uint32_t>(std::min<size_t>(need, QE_MAX_SLOTS));
  const size_t mb = qe_mask_bytes(S), Cs = std::max<size_t>(C, 1);
  // one host image: ids | 6 masks | auto_leave | op | count | last_index |
  // type | node | result | new_progress
  const size_t o_ids = 0, o_m = o_ids + 8 * G * S, o_al = o_m + 6 * mb * G, o_op = o_al + G,
               o_cnt = o_op + G, o_li = (o_cnt + G + 7) / 8 * 8, o_node = o_li + 8 * G,
               o_type = o_node + 8 * Cs * G, o_res = o_type + Cs * G, o_np = o_res + G,
               size = o_np + mb * G;
  std::vector<uint8_t> h(size, 0);
  auto put_mask = [&](int k, uint64_t g, uint32_t v) {
    memcpy(&h[o_m + (k * G + g) * mb], &v, mb);  // little endian
  };
  std::vector<std::vector<uint64_t>> slot_of(G);
  std::vector<bool> too_many(G, false);
  for (uint64_t g = 0; g < G; g++) {
    const tracker::ProgressTracker &t = changers[g]->Tracker;
    if (t.Progress.size() > S) {
      too_many[g] = true;
      continue;
    }
    uint32_t m[6] = {0, 0, 0, 0, 0, 0};  // inc out lrn lnx isl trk
    uint32_t s = 0;
    for (const auto &kv : t.Progress) {
      const uint64_t id = kv.first, b = 1u << s;
      memcpy(&h[o_ids + 8 * (s * G + g)], &id, 8);  // ID-major [S][G]
      m[0] |= t.Voters.c[0].ids.count(id) ? b : 0;
      m[1] |= t.Voters.c[1].ids.count(id) ? b : 0;
      m[2] |= t.Learners.count(id) ? b : 0;
      m[3] |= t.LearnersNext.count(id) ? b : 0;
      m[4] |= kv.second.IsLearner ? b : 0;
      m[5] |= b;
      s++;
    }
    // set members without a Progress cannot be placed: an invalid input
    bool orphan = false;
    for (const auto *set : {&t.Voters.c[0].ids, &t.Voters.c[1].ids, &t.Learners, &t.LearnersNext})
      for (uint64_t id : *set) orphan |= t.Progress.count(id) == 0;
    for (int k = 0; k < 6; k++) put_mask(k, g, m[k]);
    h[o_al + g] = t.AutoLeave ? 1 : 0;
    h[o_op + g] = orphan ? 0 : static_cast<uint8_t>(ops[g]);
    if (orphan) too_many[g] = true;  // reported below as an invariant error
    h[o_cnt + g] = static_cast<uint8_t>(ccs[g].size());
    memcpy(&h[o_li + 8 * g], &changers[g]->LastIndex, 8);
    for (size_t k = 0; k < ccs[g].size(); k++) {
      memcpy(&h[o_node + 8 * (k * G + g)], &ccs[g][k].NodeID, 8);
      h[o_type + k * G + g] = ccs[g][k].Type;
    }
  }
  {
    std::lock_guard<std::mutex> lk(g_arena.mu);
    uint8_t *d = static_cast<uint8_t *>(g_arena.get(size));
    hip_check("hipMemcpy", hipMemcpy(d, h.data(), size, hipMemcpyHostToDevice));
    qe_conf c{};
    c.num_groups = G;
    c.num_slots = S;
    c.slot_ids = reinterpret_cast<uint64_t *>(d + o_ids);
    c.inc_mask = d + o_m;
    c.out_mask = d + o_m + mb * G;
    c.learner_mask = d + o_m + 2 * mb * G;
    c.learners_next_mask = d + o_m + 3 * mb * G;
    c.is_learner = d + o_m + 4 * mb * G;
    c.tracked = d + o_m + 5 * mb * G;
    c.auto_leave = d + o_al;
    qe_conf_changes x{};
    x.max_changes = static_cast<uint32_t>(C);
    x.stride = G;
    x.op = d + o_op;
    x.count = d + o_cnt;
    x.type = d + o_type;
    x.node_id = reinterpret_cast<const uint64_t *>(d + o_node);
    x.last_index = reinterpret_cast<const uint64_t *>(d + o_li);
    x.result = d + o_res;
    x.new_progress = d + o_np;
    check("qe_confchange", qe_confchange(&c, &x, nullptr, nullptr));
    hip_check("hipMemcpy", hipMemcpy(h.data(), d, size, hipMemcpyDeviceToHost));
  }
  auto get_mask = [&](size_t off, uint64_t g) {
    uint32_t v = 0;
    memcpy(&v, &h[off + g * mb], mb);
    return v;
  };
  for (uint64_t g = 0; g < G; g++) {
    Result &r = out[g];
    const Changer &ch = *changers[g];
    const int rc = too_many[g] ? (ch.Tracker.Progress.size() > S ? QE_CC_ERR_NO_SLOT
                                                                 : QE_CC_ERR_INVARIANT)
                               : h[o_res + g];
    if (rc != QE_CC_OK) {
      r.Err = cc_error_text(rc);
      continue;
    }
    const uint32_t inc = get_mask(o_m, g), outm = get_mask(o_m + mb * G, g),
                   lrn = get_mask(o_m + 2 * mb * G, g), lnx = get_mask(o_m + 3 * mb * G, g),
                   isl = get_mask(o_m + 4 * mb * G, g), trk = get_mask(o_m + 5 * mb * G, g),
                   np = get_mask(o_np, g);
    r.Config.AutoLeave = h[o_al + g] != 0;
    for (uint32_t s = 0; s < S; s++) {
      if (((trk >> s) & 1u) == 0) continue;
      uint64_t id;
      memcpy(&id, &h[o_ids + 8 * (s * G + g)], 8);
      if ((inc >> s) & 1u) r.Config.Voters.c[0].ids.insert(id);
      if ((outm >> s) & 1u) r.Config.Voters.c[1].ids.insert(id);
      if ((lrn >> s) & 1u) r.Config.Learners.insert(id);
      if ((lnx >> s) & 1u) r.Config.LearnersNext.insert(id);
      tracker::Progress pr;
      auto it = ch.Tracker.Progress.find(id);
      if (((np >> s) & 1u) || it == ch.Tracker.Progress.end()) {
        pr.Match = 0;  // initProgress (:262-273)
        pr.Next = ch.LastIndex;
        pr.State = tracker::StateProbe;
        pr.RecentActive = true;
      } else {
        pr = it->second;
      }
      pr.IsLearner = (isl >> s) & 1u;
      r.Progress[id] = pr;
    }
  }
  return out;
}

Result Changer::EnterJoint(bool autoLeave, const std::vector<ConfChangeSingle> &ccs) const {
  return ChangeBatch({this}, {autoLeave ? Op::EnterJointAutoLeave : Op::EnterJoint}, {ccs})[0];
}

Result Changer::LeaveJoint() const { return ChangeBatch({this}, {Op::LeaveJoint}, {{}})[0]; }

Result Changer::Simple(const std::vector<ConfChangeSingle> &ccs) const {
  return ChangeBatch({this}, {Op::Simple}, {ccs})[0];
}

}  // namespace confchange
}  // namespace etcd_amd
