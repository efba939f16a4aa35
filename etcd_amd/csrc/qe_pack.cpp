// qe_pack.cpp — host-side ConfState -> slot-SoA packing (C ABI in
// include/etcd_quorum.h).  This is the wire-format side of the boundary:
// raft/raftpb/raft.proto:115-130 ConfState {voters, learners,
// voters_outgoing, learners_next, auto_leave}, as produced by
// ProgressTracker.ConfState (raft/tracker/tracker.go:146-154).
//
// Slot order per group: JointConfig.IDs() (raft/quorum/joint.go:30-38) in
// ascending ID order, then learners in ascending ID order.  Every quorum
// function is order-free, so this choice is free; ascending order makes the
// packing deterministic.  Work is split over std::threads by group range.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/etcd_quorum.h"

namespace {

int g_pack_threads = 0;  // 0 = hardware_concurrency (capped at 16)

template <typename F>
void parallel_for(uint64_t n, F f) {
  unsigned nt = g_pack_threads > 0 ? static_cast<unsigned>(g_pack_threads)
                                   : std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  if (n < 4096 || nt <= 1) {
    f(0, n);
    return;
  }
  if (nt > n / 1024) nt = static_cast<unsigned>(std::max<uint64_t>(1, n / 1024));
  std::vector<std::thread> th;
  const uint64_t chunk = (n + nt - 1) / nt;
  for (unsigned t = 0; t < nt; t++) {
    const uint64_t b = t * chunk, e = std::min(n, b + chunk);
    if (b >= e) break;
    th.emplace_back([=] { f(b, e); });
  }
  for (auto &x : th) x.join();
}

inline void put_mask(void *p, uint32_t mb, uint64_t g, uint32_t v) {
  if (!p) return;
  if (mb == 1) static_cast<uint8_t *>(p)[g] = static_cast<uint8_t>(v);
  else static_cast<uint16_t *>(p)[g] = static_cast<uint16_t>(v);
}

inline int slot_of(const uint64_t *ids, uint32_t S, uint64_t id) {
  for (uint32_t s = 0; s < S; s++)
    if (ids[s] == id) return static_cast<int>(s);
  return -1;
}

struct List {
  const uint64_t *ids;
  const uint64_t *off;
  bool has(uint64_t) const { return ids && off; }
  const uint64_t *begin(uint64_t g) const { return ids + off[g]; }
  const uint64_t *end(uint64_t g) const { return ids + off[g + 1]; }
};

}  // namespace

extern "C" {

int qe_pack_threads(int n) {
  if (n < 0 || n > 256) return QE_ERANGE;
  g_pack_threads = n;
  return QE_OK;
}

}  // extern "C"

namespace {

// One group of a ConfState CSR batch in slot form: ids[S] (0 = unused), the
// masks of Voters[0], Voters[1], Learners, LearnersNext, and QE_PACK_* flags.
// A flagged group (too many peers, zero ID) is left empty.
struct PackedGroup {
  uint32_t mi, mo, ml, mlnx, flags;
};

PackedGroup pack_group(const List &voters, const List &outgoing, const List &learners,
                       const List &lnext, uint64_t g, uint32_t S, uint64_t *ids) {
  PackedGroup r{0, 0, 0, 0, 0};
  uint64_t vbuf[2 * QE_MAX_SLOTS + 2], lbuf[QE_MAX_SLOTS + 1];
  memset(ids, 0, sizeof(uint64_t) * S);
  // voters of both halves, ascending + deduplicated (JointConfig.IDs)
  uint32_t nv = 0;
  auto add_voters = [&](const List &l) {
    if (!l.has(g)) return;
    for (const uint64_t *p = l.begin(g); p != l.end(g); ++p) {
      if (nv >= 2 * QE_MAX_SLOTS + 1) { r.flags |= QE_PACK_TOO_MANY_PEERS; return; }
      vbuf[nv++] = *p;
    }
  };
  add_voters(voters);
  add_voters(outgoing);
  std::sort(vbuf, vbuf + nv);
  nv = static_cast<uint32_t>(std::unique(vbuf, vbuf + nv) - vbuf);
  uint32_t nl = 0;
  if (learners.has(g)) {
    for (const uint64_t *p = learners.begin(g); p != learners.end(g); ++p) {
      if (std::binary_search(vbuf, vbuf + nv, *p)) {
        r.flags |= QE_PACK_LEARNER_IS_VOTER;  // confchange.go:308-318 invariant
        continue;
      }
      if (nl >= QE_MAX_SLOTS) { r.flags |= QE_PACK_TOO_MANY_PEERS; break; }
      lbuf[nl++] = *p;
    }
  }
  std::sort(lbuf, lbuf + nl);
  nl = static_cast<uint32_t>(std::unique(lbuf, lbuf + nl) - lbuf);
  if (nv + nl > S) r.flags |= QE_PACK_TOO_MANY_PEERS;
  // LearnersNext must be outgoing voters (confchange.go:299-306)
  if (lnext.has(g)) {
    for (const uint64_t *p = lnext.begin(g); p != lnext.end(g); ++p) {
      bool in_out = false;
      if (outgoing.has(g))
        for (const uint64_t *q = outgoing.begin(g); q != outgoing.end(g); ++q)
          in_out |= (*q == *p);
      if (!in_out) r.flags |= QE_PACK_LEARNER_NEXT_NOT_OUTGOING;
    }
  }
  // ID 0 is raft.None, and slot id 0 marks an unused slot: a voter or a
  // learner with ID 0 cannot be placed
  for (uint32_t i = 0; i < nv; i++)
    if (vbuf[i] == 0) r.flags |= QE_PACK_ZERO_ID;
  for (uint32_t i = 0; i < nl; i++)
    if (lbuf[i] == 0) r.flags |= QE_PACK_ZERO_ID;
  if (!(r.flags & QE_PACK_TOO_MANY_PEERS) && !(r.flags & QE_PACK_ZERO_ID)) {
    for (uint32_t i = 0; i < nv; i++) ids[i] = vbuf[i];
    for (uint32_t i = 0; i < nl; i++) ids[nv + i] = lbuf[i];
    auto mark = [&](const List &l, uint32_t &m) {
      if (!l.has(g)) return;
      for (const uint64_t *p = l.begin(g); p != l.end(g); ++p) {
        const int s = slot_of(ids, S, *p);
        if (s >= 0) m |= 1u << s;
      }
    };
    mark(voters, r.mi);
    mark(outgoing, r.mo);
    mark(lnext, r.mlnx);
    r.mlnx &= r.mo;  // only outgoing voters can be LearnersNext
    for (uint32_t i = 0; i < nl; i++) r.ml |= 1u << (nv + i);
  }
  return r;
}

}  // namespace

extern "C" {

int qe_pack_confstate(const qe_confstate_csr *cs, uint32_t num_slots, void *inc_mask,
                      void *out_mask, void *learner_mask, uint64_t *slot_ids,
                      uint32_t *group_flags, uint64_t *num_flagged) {
  if (!cs || !slot_ids) return QE_EINVAL;
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  const uint64_t G = cs->num_groups;
  if (num_flagged) *num_flagged = 0;
  if (G == 0) return QE_OK;
  if (!cs->voters || !cs->voters_off) return QE_EINVAL;
  const uint32_t S = num_slots, mb = S <= 8 ? 1 : 2;
  const List voters{cs->voters, cs->voters_off}, outgoing{cs->voters_outgoing, cs->outgoing_off};
  const List learners{cs->learners, cs->learners_off};
  const List lnext{cs->learners_next, cs->learners_next_off};
  std::atomic<uint64_t> flagged{0};
  parallel_for(G, [&](uint64_t b, uint64_t e) {
    uint64_t local_flagged = 0;
    for (uint64_t g = b; g < e; g++) {
      const PackedGroup r = pack_group(voters, outgoing, learners, lnext, g, S, slot_ids + g * S);
      put_mask(inc_mask, mb, g, r.mi);
      put_mask(out_mask, mb, g, r.mo);
      put_mask(learner_mask, mb, g, r.ml);
      if (group_flags) group_flags[g] = r.flags;
      local_flagged += r.flags != 0;
    }
    flagged += local_flagged;
  });
  if (num_flagged) *num_flagged = flagged.load();
  return QE_OK;
}

int qe_pack_conf(const qe_confstate_csr *cs, const qe_conf *out, uint32_t *group_flags,
                 uint64_t *num_flagged) {
  if (!cs || !out) return QE_EINVAL;
  if (out->num_slots == 0 || out->num_slots > QE_MAX_SLOTS || out->reserved) return QE_EINVAL;
  if (out->num_groups != cs->num_groups) return QE_EINVAL;
  const uint64_t G = cs->num_groups;
  if (num_flagged) *num_flagged = 0;
  if (G == 0) return QE_OK;
  if (!cs->voters || !cs->voters_off) return QE_EINVAL;
  if (!out->slot_ids || !out->inc_mask || !out->out_mask || !out->learner_mask ||
      !out->learners_next_mask || !out->is_learner || !out->tracked || !out->auto_leave)
    return QE_EINVAL;
  const uint32_t S = out->num_slots, mb = S <= 8 ? 1 : 2;
  const List voters{cs->voters, cs->voters_off}, outgoing{cs->voters_outgoing, cs->outgoing_off};
  const List learners{cs->learners, cs->learners_off};
  const List lnext{cs->learners_next, cs->learners_next_off};
  std::atomic<uint64_t> flagged{0};
  parallel_for(G, [&](uint64_t b, uint64_t e) {
    uint64_t local_flagged = 0;
    for (uint64_t g = b; g < e; g++) {
      uint64_t *ids = out->slot_ids + g * S;
      const PackedGroup r = pack_group(voters, outgoing, learners, lnext, g, S, ids);
      uint32_t trk = 0;
      for (uint32_t s = 0; s < S; s++) trk |= ids[s] ? (1u << s) : 0u;
      put_mask(out->inc_mask, mb, g, r.mi);
      put_mask(out->out_mask, mb, g, r.mo);
      put_mask(out->learner_mask, mb, g, r.ml);
      put_mask(out->learners_next_mask, mb, g, r.mlnx);
      put_mask(out->is_learner, mb, g, r.ml);  // LearnersNext stay !IsLearner (confchange.go:299-306)
      put_mask(out->tracked, mb, g, trk);
      out->auto_leave[g] = (cs->auto_leave && r.flags == 0) ? (cs->auto_leave[g] != 0) : 0;
      if (group_flags) group_flags[g] = r.flags;
      local_flagged += r.flags != 0;
    }
    flagged += local_flagged;
  });
  if (num_flagged) *num_flagged = flagged.load();
  return QE_OK;
}

int qe_pack_match(uint64_t num_groups, uint32_t num_slots, const uint64_t *slot_ids,
                  const uint64_t *prog_off, const uint64_t *prog_ids, const uint64_t *prog_match,
                  uint64_t *match, uint64_t stride, uint64_t *num_unknown) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (num_unknown) *num_unknown = 0;
  if (num_groups == 0) return QE_OK;
  if (!slot_ids || !prog_off || !prog_ids || !prog_match || !match) return QE_EINVAL;
  if (stride < num_groups) return QE_EINVAL;
  const uint32_t S = num_slots;
  std::atomic<uint64_t> unknown{0};
  parallel_for(num_groups, [&](uint64_t b, uint64_t e) {
    uint64_t u = 0;
    for (uint64_t g = b; g < e; g++) {
      const uint64_t *ids = slot_ids + g * S;
      for (uint32_t s = 0; s < S; s++) match[s * stride + g] = 0;  // absent
      for (uint64_t k = prog_off[g]; k < prog_off[g + 1]; k++) {
        const int s = slot_of(ids, S, prog_ids[k]);
        if (s < 0 || prog_ids[k] == 0) { u++; continue; }
        match[static_cast<uint64_t>(s) * stride + g] = prog_match[k];
      }
    }
    unknown += u;
  });
  if (num_unknown) *num_unknown = unknown.load();
  return QE_OK;
}

int qe_pack_votes(uint64_t num_groups, uint32_t num_slots, const uint64_t *slot_ids,
                  const uint64_t *vote_off, const uint64_t *vote_ids, const uint8_t *vote_vals,
                  void *voted, void *granted) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (num_groups == 0) return QE_OK;
  if (!slot_ids || !vote_off || !vote_ids || !vote_vals || !voted || !granted) return QE_EINVAL;
  const uint32_t S = num_slots, mb = S <= 8 ? 1 : 2;
  parallel_for(num_groups, [&](uint64_t b, uint64_t e) {
    for (uint64_t g = b; g < e; g++) {
      const uint64_t *ids = slot_ids + g * S;
      uint32_t vd = 0, gr = 0;
      for (uint64_t k = vote_off[g]; k < vote_off[g + 1]; k++) {
        const int s = slot_of(ids, S, vote_ids[k]);
        if (s < 0 || vote_ids[k] == 0) continue;  // votes from non-peers never count
        const uint32_t bit = 1u << s;
        if (vd & bit) continue;  // RecordVote: the first vote sticks
        vd |= bit;
        if (vote_vals[k]) gr |= bit;
      }
      put_mask(voted, mb, g, vd);
      put_mask(granted, mb, g, gr);
    }
  });
  return QE_OK;
}

int qe_slot_lookup(uint64_t num_groups, uint32_t num_slots, const uint64_t *slot_ids,
                   uint64_t n, const uint64_t *group, const uint64_t *id, int8_t *slot) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (n == 0) return QE_OK;
  if (!slot_ids || !group || !id || !slot) return QE_EINVAL;
  const uint32_t S = num_slots;
  parallel_for(n, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; i++) {
      const uint64_t g = group[i];
      slot[i] = (g < num_groups && id[i] != 0) ? static_cast<int8_t>(slot_of(slot_ids + g * S, S, id[i]))
                                                : static_cast<int8_t>(-1);
    }
  });
  return QE_OK;
}

}  // extern "C"
