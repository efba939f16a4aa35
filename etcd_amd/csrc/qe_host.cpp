// qe_host.cpp — C++ host mirror of raft/quorum + raft/tracker
// (include/etcd_quorum.hpp).  Groups are packed into the slot-SoA layout
// (voters of both halves ascending, then learners: etcd_amd/packing.py uses
// the same order), copied to a grow-only device arena and evaluated by the
// C ABI kernels; results are copied back.  Decisions never run on the CPU.
#include <hip/hip_runtime_api.h>
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
}  // namespace etcd_amd
