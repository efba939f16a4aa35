// qe_pack.cpp — host-side ConfState -> slot-SoA packing (C ABI in
// include/etcd_quorum.h).  This is the wire-format side of the boundary:
// raft/raftpb/raft.proto:115-130 ConfState {voters, learners,
// voters_outgoing, learners_next, auto_leave}, as produced by
// ProgressTracker.ConfState (raft/tracker/tracker.go:146-154).
//
// Slot order per group: JointConfig.IDs() (raft/quorum/joint.go:30-38) in
// ascending ID order, then learners in ascending ID order.  Every quorum
// function is order-free, so this choice is free; ascending order makes the
// packing deterministic.  Slot IDs are stored ID-major, [S][G] (slot s of
// packed group i at slot_ids[s*G + i]), so a kernel that rewrites one slot's
// ID touches one row.
//
// Group order (ABI 3): packed position i holds the caller's group perm[i]
// (identity when cs->perm is NULL).  qe_pack_order computes the
// shape-bucketed order -- groups sorted by configuration shape, so the 64
// groups of a wave have their voters in the same low slots and the joint
// commit kernel fetches only those slot rows.  Work is split
// over std::threads by group range.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/etcd_quorum.h"

namespace {

int g_pack_threads = 0;  // 0 = hardware_concurrency (capped at 16)

// Contiguous ranges of [0, n), one per worker thread (deterministic for a
// given n and thread setting, so two passes see the same split).
std::vector<std::pair<uint64_t, uint64_t>> ranges_of(uint64_t n) {
  unsigned nt = g_pack_threads > 0 ? static_cast<unsigned>(g_pack_threads)
                                   : std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  if (n < 4096) nt = 1;
  if (nt > n / 1024) nt = static_cast<unsigned>(std::max<uint64_t>(1, n / 1024));
  std::vector<std::pair<uint64_t, uint64_t>> r;
  const uint64_t chunk = (n + nt - 1) / nt;
  for (unsigned t = 0; t < nt; t++) {
    const uint64_t b = t * chunk, e = std::min(n, b + chunk);
    if (b >= e) break;
    r.emplace_back(b, e);
  }
  if (r.empty()) r.emplace_back(0, n);
  return r;
}

// f(thread_index, begin, end) over the ranges of ranges_of(n)
template <typename F>
void parallel_ranges(const std::vector<std::pair<uint64_t, uint64_t>> &r, F f) {
  if (r.size() == 1) {
    f(0u, r[0].first, r[0].second);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < r.size(); t++) th.emplace_back([&, t] { f(t, r[t].first, r[t].second); });
  for (auto &x : th) x.join();
}

template <typename F>
void parallel_for(uint64_t n, F f) {
  parallel_ranges(ranges_of(n), [&](unsigned, uint64_t b, uint64_t e) { f(b, e); });
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

// The S slot IDs of packed group i from the ID-major block.
inline void gather_ids(const uint64_t *slot_ids, uint64_t G, uint32_t S, uint64_t i,
                       uint64_t *ids) {
  for (uint32_t s = 0; s < S; s++) ids[s] = slot_ids[s * G + i];
}

struct List {
  const uint64_t *ids;
  const uint64_t *off;
  bool has(uint64_t) const { return ids && off; }
  const uint64_t *begin(uint64_t g) const { return ids + off[g]; }
  const uint64_t *end(uint64_t g) const { return ids + off[g + 1]; }
};

struct Lists {
  List voters, outgoing, learners, lnext;
  explicit Lists(const qe_confstate_csr *cs)
      : voters{cs->voters, cs->voters_off},
        outgoing{cs->voters_outgoing, cs->outgoing_off},
        learners{cs->learners, cs->learners_off},
        lnext{cs->learners_next, cs->learners_next_off} {}
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
// A flagged group (too many peers, zero ID) is left empty.  nv / nl: the
// number of distinct voters (union of both halves) and learners placed;
// ni / no: distinct voters of each half.
struct PackedGroup {
  uint32_t mi, mo, ml, mlnx, flags;
  uint32_t nv, nl, ni, no;
};

uint32_t count_unique(const List &l, uint64_t g, uint64_t *buf, bool &over) {
  if (!l.has(g)) return 0;
  uint32_t n = 0;
  for (const uint64_t *p = l.begin(g); p != l.end(g); ++p) {
    if (n >= 2 * QE_MAX_SLOTS + 1) {
      over = true;
      break;
    }
    buf[n++] = *p;
  }
  std::sort(buf, buf + n);
  return static_cast<uint32_t>(std::unique(buf, buf + n) - buf);
}

PackedGroup pack_group(const Lists &L, uint64_t g, uint32_t S, uint64_t *ids) {
  PackedGroup r{0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t vbuf[2 * QE_MAX_SLOTS + 2], lbuf[QE_MAX_SLOTS + 1], tmp[2 * QE_MAX_SLOTS + 2];
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
  add_voters(L.voters);
  add_voters(L.outgoing);
  std::sort(vbuf, vbuf + nv);
  nv = static_cast<uint32_t>(std::unique(vbuf, vbuf + nv) - vbuf);
  bool over = false;
  r.ni = count_unique(L.voters, g, tmp, over);
  r.no = count_unique(L.outgoing, g, tmp, over);
  if (over) r.flags |= QE_PACK_TOO_MANY_PEERS;
  uint32_t nl = 0;
  if (L.learners.has(g)) {
    for (const uint64_t *p = L.learners.begin(g); p != L.learners.end(g); ++p) {
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
  if (L.lnext.has(g)) {
    for (const uint64_t *p = L.lnext.begin(g); p != L.lnext.end(g); ++p) {
      bool in_out = false;
      if (L.outgoing.has(g))
        for (const uint64_t *q = L.outgoing.begin(g); q != L.outgoing.end(g); ++q)
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
  r.nv = nv;
  r.nl = nl;
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
    mark(L.voters, r.mi);
    mark(L.outgoing, r.mo);
    mark(L.lnext, r.mlnx);
    r.mlnx &= r.mo;  // only outgoing voters can be LearnersNext
    for (uint32_t i = 0; i < nl; i++) r.ml |= 1u << (nv + i);
  }
  return r;
}

// Shape key of a group: (union size, |Voters[0]|, |Voters[1]|, learners),
// each 0..16 for a placeable group; flagged groups (left empty) sort last.
constexpr uint32_t kShapeDim = QE_MAX_SLOTS + 1;
constexpr uint32_t kShapes = kShapeDim * kShapeDim * kShapeDim * kShapeDim + 1;

uint32_t shape_key(const Lists &L, uint64_t g, uint32_t S) {
  uint64_t ids[QE_MAX_SLOTS];
  const PackedGroup r = pack_group(L, g, S, ids);
  if (r.flags & (QE_PACK_TOO_MANY_PEERS | QE_PACK_ZERO_ID)) return kShapes - 1;
  return ((r.nv * kShapeDim + r.ni) * kShapeDim + r.no) * kShapeDim + r.nl;
}

bool perm_ok(const uint64_t *perm, uint64_t G) {
  if (!perm) return true;
  std::atomic<bool> ok{true};
  parallel_for(G, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; i++)
      if (perm[i] >= G) { ok = false; return; }
  });
  return ok.load();
}

}  // namespace

extern "C" {

int qe_pack_order(const qe_confstate_csr *cs, uint32_t num_slots, uint64_t *perm,
                  uint64_t *num_shapes) {
  if (!cs || !perm) return QE_EINVAL;
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  const uint64_t G = cs->num_groups;
  if (num_shapes) *num_shapes = 0;
  if (G == 0) return QE_OK;
  if (!cs->voters || !cs->voters_off) return QE_EINVAL;
  const Lists L(cs);
  const uint32_t S = num_slots;
  // stable counting sort by shape: per-thread histograms over the thread's
  // contiguous range, bucket-major / thread-minor offsets, then each thread
  // scatters its range in order
  const auto rg = ranges_of(G);
  const size_t nt = rg.size();
  std::vector<uint32_t> key(G);
  std::vector<uint64_t> hist(nt * kShapes, 0);
  parallel_ranges(rg, [&](unsigned t, uint64_t b, uint64_t e) {
    uint64_t *h = &hist[t * kShapes];
    for (uint64_t g = b; g < e; g++) {
      key[g] = shape_key(L, g, S);
      h[key[g]]++;
    }
  });
  uint64_t run = 0, shapes = 0;
  for (uint32_t k = 0; k < kShapes; k++) {
    uint64_t tot = 0;
    for (size_t t = 0; t < nt; t++) {
      const uint64_t c = hist[t * kShapes + k];
      hist[t * kShapes + k] = run;
      run += c;
      tot += c;
    }
    shapes += tot != 0;
  }
  parallel_ranges(rg, [&](unsigned t, uint64_t b, uint64_t e) {
    uint64_t *h = &hist[t * kShapes];
    for (uint64_t g = b; g < e; g++) perm[h[key[g]]++] = g;
  });
  if (num_shapes) *num_shapes = shapes;
  return QE_OK;
}

int qe_pack_confstate(const qe_confstate_csr *cs, uint32_t num_slots, void *inc_mask,
                      void *out_mask, void *learner_mask, uint64_t *slot_ids,
                      uint32_t *group_flags, uint64_t *num_flagged) {
  if (!cs || !slot_ids) return QE_EINVAL;
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  const uint64_t G = cs->num_groups;
  if (num_flagged) *num_flagged = 0;
  if (G == 0) return QE_OK;
  if (!cs->voters || !cs->voters_off) return QE_EINVAL;
  if (!perm_ok(cs->perm, G)) return QE_EINVAL;
  const uint32_t S = num_slots, mb = S <= 8 ? 1 : 2;
  const Lists L(cs);
  std::atomic<uint64_t> flagged{0};
  parallel_for(G, [&](uint64_t b, uint64_t e) {
    uint64_t local_flagged = 0;
    uint64_t ids[QE_MAX_SLOTS];
    for (uint64_t i = b; i < e; i++) {
      const uint64_t g = cs->perm ? cs->perm[i] : i;
      const PackedGroup r = pack_group(L, g, S, ids);
      for (uint32_t s = 0; s < S; s++) slot_ids[s * G + i] = ids[s];
      put_mask(inc_mask, mb, i, r.mi);
      put_mask(out_mask, mb, i, r.mo);
      put_mask(learner_mask, mb, i, r.ml);
      if (group_flags) group_flags[i] = r.flags;
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
  if (!perm_ok(cs->perm, G)) return QE_EINVAL;
  const uint32_t S = out->num_slots, mb = S <= 8 ? 1 : 2;
  const Lists L(cs);
  std::atomic<uint64_t> flagged{0};
  parallel_for(G, [&](uint64_t b, uint64_t e) {
    uint64_t local_flagged = 0;
    uint64_t ids[QE_MAX_SLOTS];
    for (uint64_t i = b; i < e; i++) {
      const uint64_t g = cs->perm ? cs->perm[i] : i;
      const PackedGroup r = pack_group(L, g, S, ids);
      uint32_t trk = 0;
      for (uint32_t s = 0; s < S; s++) {
        out->slot_ids[s * G + i] = ids[s];
        trk |= ids[s] ? (1u << s) : 0u;
      }
      put_mask(out->inc_mask, mb, i, r.mi);
      put_mask(out->out_mask, mb, i, r.mo);
      put_mask(out->learner_mask, mb, i, r.ml);
      put_mask(out->learners_next_mask, mb, i, r.mlnx);
      put_mask(out->is_learner, mb, i, r.ml);  // LearnersNext stay !IsLearner (confchange.go:299-306)
      put_mask(out->tracked, mb, i, trk);
      // restore.go:118-155: AutoLeave takes effect only through EnterJoint,
      // i.e. in a joint config; a non-joint ConfState restores AutoLeave =
      // false (checkInvariants rejects AutoLeave without Voters[1])
      out->auto_leave[i] = (cs->auto_leave && r.flags == 0 && r.mo != 0) ? (cs->auto_leave[g] != 0) : 0;
      if (group_flags) group_flags[i] = r.flags;
      local_flagged += r.flags != 0;
    }
    flagged += local_flagged;
  });
  if (num_flagged) *num_flagged = flagged.load();
  return QE_OK;
}

int qe_pack_match(uint64_t num_groups, uint32_t num_slots, const uint64_t *slot_ids,
                  const uint64_t *perm, const uint64_t *prog_off, const uint64_t *prog_ids,
                  const uint64_t *prog_match, uint64_t *match, uint64_t stride,
                  uint64_t *num_unknown) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (num_unknown) *num_unknown = 0;
  if (num_groups == 0) return QE_OK;
  if (!slot_ids || !prog_off || !prog_ids || !prog_match || !match) return QE_EINVAL;
  if (stride < num_groups) return QE_EINVAL;
  if (!perm_ok(perm, num_groups)) return QE_EINVAL;
  const uint32_t S = num_slots;
  const uint64_t G = num_groups;
  std::atomic<uint64_t> unknown{0};
  parallel_for(G, [&](uint64_t b, uint64_t e) {
    uint64_t u = 0;
    uint64_t ids[QE_MAX_SLOTS];
    for (uint64_t i = b; i < e; i++) {
      const uint64_t g = perm ? perm[i] : i;
      gather_ids(slot_ids, G, S, i, ids);
      for (uint32_t s = 0; s < S; s++) match[s * stride + i] = 0;  // absent
      for (uint64_t k = prog_off[g]; k < prog_off[g + 1]; k++) {
        const int s = slot_of(ids, S, prog_ids[k]);
        if (s < 0 || prog_ids[k] == 0) { u++; continue; }
        match[static_cast<uint64_t>(s) * stride + i] = prog_match[k];
      }
    }
    unknown += u;
  });
  if (num_unknown) *num_unknown = unknown.load();
  return QE_OK;
}

int qe_pack_votes(uint64_t num_groups, uint32_t num_slots, const uint64_t *slot_ids,
                  const uint64_t *perm, const uint64_t *vote_off, const uint64_t *vote_ids,
                  const uint8_t *vote_vals, void *voted, void *granted) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (num_groups == 0) return QE_OK;
  if (!slot_ids || !vote_off || !vote_ids || !vote_vals || !voted || !granted) return QE_EINVAL;
  if (!perm_ok(perm, num_groups)) return QE_EINVAL;
  const uint32_t S = num_slots, mb = S <= 8 ? 1 : 2;
  const uint64_t G = num_groups;
  parallel_for(G, [&](uint64_t b, uint64_t e) {
    uint64_t ids[QE_MAX_SLOTS];
    for (uint64_t i = b; i < e; i++) {
      const uint64_t g = perm ? perm[i] : i;
      gather_ids(slot_ids, G, S, i, ids);
      uint32_t vd = 0, gr = 0;
      for (uint64_t k = vote_off[g]; k < vote_off[g + 1]; k++) {
        const int s = slot_of(ids, S, vote_ids[k]);
        if (s < 0 || vote_ids[k] == 0) continue;  // votes from non-peers never count
        const uint32_t bit = 1u << s;
        if (vd & bit) continue;  // RecordVote: the first vote sticks
        vd |= bit;
        if (vote_vals[k]) gr |= bit;
      }
      put_mask(voted, mb, i, vd);
      put_mask(granted, mb, i, gr);
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
    uint64_t ids[QE_MAX_SLOTS];
    for (uint64_t i = b; i < e; i++) {
      const uint64_t g = group[i];
      if (g >= num_groups || id[i] == 0) {
        slot[i] = -1;
        continue;
      }
      gather_ids(slot_ids, num_groups, S, g, ids);
      slot[i] = static_cast<int8_t>(slot_of(ids, S, id[i]));
    }
  });
  return QE_OK;
}

// ---- Inflights rings: plain uint64 <-> infl_lo / infl_hi (ABI 4) ----------
// The canonical representation (include/etcd_quorum.h): a peer with no live
// entry has epoch 0 and is not wide; otherwise it is not wide iff every live
// entry (positions start .. start+count-1 mod F, inflights.go:25-37) has the
// same upper word h <= QE_RING_EPOCH_MAX, and then its epoch is h.  Both
// words of every position are stored (infl_hi too), so unpacking a wide peer
// returns every position exactly.
int qe_ring_pack(uint64_t num_groups, uint32_t num_slots, uint32_t inflight_cap,
                 uint64_t stride, const uint64_t *entries, uint32_t *peer,
                 uint32_t *infl_lo, uint32_t *infl_hi) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (inflight_cap == 0 || inflight_cap > QE_MAX_INFLIGHT) return QE_ERANGE;
  if (num_groups == 0) return QE_OK;
  if (stride < num_groups || !entries || !peer || !infl_lo || !infl_hi) return QE_EINVAL;
  const uint32_t F = inflight_cap, FP = QE_RING_PITCH(F);
  for (uint32_t s = 0; s < num_slots; s++) {
    parallel_for(num_groups, [&](uint64_t b, uint64_t e) {
      for (uint64_t g = b; g < e; g++) {
        const uint64_t row = s * stride + g;
        const uint64_t *src = entries + row * F;
        uint32_t *lo = infl_lo + row * FP, *hi = infl_hi + row * FP;
        for (uint32_t k = 0; k < FP; k++) {
          const uint64_t v = k < F ? src[k] : 0;
          lo[k] = static_cast<uint32_t>(v);
          hi[k] = static_cast<uint32_t>(v >> 32);
        }
        uint32_t w = peer[row] & ~QE_PW_RING_MASK;
        const uint32_t start = (w >> QE_PW_START_SHIFT) & 0xFFu;
        const uint32_t count = (w >> QE_PW_COUNT_SHIFT) & 0xFFu;
        if (count > 0) {
          const uint32_t st = start < F ? start : 0;  // as the kernels read an invalid start
          const uint32_t h = hi[st];
          bool wide = h > QE_RING_EPOCH_MAX;
          for (uint32_t j = 0; j < count && j < F && !wide; j++) {
            uint32_t pos = st + j;
            if (pos >= F) pos -= F;
            wide = hi[pos] != h;
          }
          w |= wide ? QE_PF_RING_WIDE : QE_PW_EPOCH_BITS(h);
        }
        peer[row] = w;
      }
    });
  }
  return QE_OK;
}

int qe_ring_unpack(uint64_t num_groups, uint32_t num_slots, uint32_t inflight_cap,
                   uint64_t stride, const uint32_t *infl_lo, const uint32_t *infl_hi,
                   const uint32_t *peer, uint64_t *entries) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (inflight_cap == 0 || inflight_cap > QE_MAX_INFLIGHT) return QE_ERANGE;
  if (num_groups == 0) return QE_OK;
  if (stride < num_groups || !entries || !peer || !infl_lo || !infl_hi) return QE_EINVAL;
  const uint32_t F = inflight_cap, FP = QE_RING_PITCH(F);
  for (uint32_t s = 0; s < num_slots; s++) {
    parallel_for(num_groups, [&](uint64_t b, uint64_t e) {
      for (uint64_t g = b; g < e; g++) {
        const uint64_t row = s * stride + g;
        const uint32_t w = peer[row];
        const bool wide = (w & QE_PF_RING_WIDE) != 0;
        const uint64_t h = QE_PW_EPOCH(w);
        for (uint32_t k = 0; k < F; k++)
          entries[row * F + k] = ((wide ? infl_hi[row * FP + k] : h) << 32) | infl_lo[row * FP + k];
      }
    });
  }
  return QE_OK;
}

// ---- ABI 8: the 16-bit form (infl16, offsets below Next) ------------------
// A peer is in the 16-bit form iff every live entry v satisfies
// Next - 65536 <= v <= Next - 1; else it is wide.  Every position is encoded
// both ways (the 16-bit offset of a dead or out-of-range position is the low
// half of Next - 1 - v), so unpacking returns every position exactly.
int qe_ring_pack16(uint64_t num_groups, uint32_t num_slots, uint32_t inflight_cap,
                   uint64_t stride, const uint64_t *entries, const uint64_t *next,
                   uint32_t *peer, uint16_t *infl16, uint32_t *infl_lo, uint32_t *infl_hi) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (inflight_cap == 0 || inflight_cap > QE_RING16_MAX_F) return QE_ERANGE;
  if (num_groups == 0) return QE_OK;
  if (stride < num_groups || !entries || !next || !peer || !infl16 || !infl_lo || !infl_hi)
    return QE_EINVAL;
  const uint32_t F = inflight_cap, FP = QE_RING_PITCH(F);
  for (uint32_t s = 0; s < num_slots; s++) {
    parallel_for(num_groups, [&](uint64_t b, uint64_t e) {
      for (uint64_t g = b; g < e; g++) {
        const uint64_t row = s * stride + g;
        const uint64_t *src = entries + row * F;
        const uint64_t top = next[row] - 1;
        uint32_t *lo = infl_lo + row * FP, *hi = infl_hi + row * FP;
        uint16_t *o = infl16 + row * QE_RING16_MAX_F;
        for (uint32_t k = 0; k < QE_RING16_MAX_F; k++) {
          const uint64_t v = k < F ? src[k] : top;
          o[k] = static_cast<uint16_t>(top - v);
          if (k < FP) {
            lo[k] = static_cast<uint32_t>(v);
            hi[k] = static_cast<uint32_t>(v >> 32);
          }
        }
        uint32_t w = peer[row] & ~QE_PW_RING_MASK;
        const uint32_t start = (w >> QE_PW_START_SHIFT) & 0xFFu;
        const uint32_t count = (w >> QE_PW_COUNT_SHIFT) & 0xFFu;
        const uint32_t st = start < F ? start : 0;  // as the kernels read an invalid start
        bool fits = true;
        for (uint32_t j = 0; j < count && j < F && fits; j++) {
          uint32_t pos = st + j;
          if (pos >= F) pos -= F;
          fits = src[pos] <= top && top - src[pos] <= 0xFFFFu;
        }
        peer[row] = w | (fits ? 0u : QE_PF_RING_WIDE);
      }
    });
  }
  return QE_OK;
}

int qe_ring_unpack16(uint64_t num_groups, uint32_t num_slots, uint32_t inflight_cap,
                     uint64_t stride, const uint16_t *infl16, const uint32_t *infl_lo,
                     const uint32_t *infl_hi, const uint64_t *next, const uint32_t *peer,
                     uint64_t *entries) {
  if (num_slots == 0 || num_slots > QE_MAX_SLOTS) return QE_EINVAL;
  if (inflight_cap == 0 || inflight_cap > QE_RING16_MAX_F) return QE_ERANGE;
  if (num_groups == 0) return QE_OK;
  if (stride < num_groups || !entries || !next || !peer || !infl16 || !infl_lo || !infl_hi)
    return QE_EINVAL;
  const uint32_t F = inflight_cap, FP = QE_RING_PITCH(F);
  for (uint32_t s = 0; s < num_slots; s++) {
    parallel_for(num_groups, [&](uint64_t b, uint64_t e) {
      for (uint64_t g = b; g < e; g++) {
        const uint64_t row = s * stride + g;
        const bool wide = (peer[row] & QE_PF_RING_WIDE) != 0;
        const uint64_t top = next[row] - 1;
        for (uint32_t k = 0; k < F; k++)
          entries[row * F + k] =
              wide ? (static_cast<uint64_t>(infl_hi[row * FP + k]) << 32) | infl_lo[row * FP + k]
                   : top - infl16[row * QE_RING16_MAX_F + k];
      }
    });
  }
  return QE_OK;
}

}  // extern "C"
