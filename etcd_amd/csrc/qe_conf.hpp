// qe_conf.hpp — qe_confchange: raft/confchange's Changer (Simple,
// EnterJoint, LeaveJoint) over slot masks, one group per lane.
//
// The reference works on ID-keyed maps (tracker.Config, ProgressMap).  Here a
// group's peers sit in up to 16 slots; every set is a slot mask, and a change
// names a peer by ID, found by comparing the ID against the tracked slots
// (an unrolled compare over at most 16 registers, no dynamic indexing).  All
// set operations are then single bit operations.  The kernel is not on the
// hot path (one launch per configuration change of a batch of groups); it
// keeps membership changes on the device next to the quorum state instead of
// round-tripping the masks through the host packer.
#pragma once
#include "qe_kernels.hpp"

namespace qe {

constexpr int kCCMax = 16;  // QE_MAX_SLOTS

struct CCArgs {
  uint64_t G, stride, pstride;
  uint32_t C;
  uint64_t *ids;
  void *inc, *out, *lrn, *lnx, *isl, *trk;
  uint8_t *auto_leave;
  const uint8_t *op, *count, *type;
  const uint64_t *node, *last_index;
  uint8_t *result;
  void *new_progress;
  // optional Progress rows to initialise ([S][pstride])
  uint64_t *p_match, *p_next, *p_pending;
  uint32_t *p_pw;
};

struct CCState {
  uint32_t inc, out, lrn, lnx, isl, trk, al, newp;
};

// checkInvariants (raft/confchange/confchange.go:186-241) on slot masks,
// plus what the map model guarantees by construction: tracked ids are
// distinct and nonzero (raft.None is never a peer).
template <int S>
__device__ __forceinline__ bool cc_invariants(const CCState &c, const uint64_t (&id)[kCCMax]) {
  bool ok = ((c.inc | c.out | c.lrn | c.lnx) & ~c.trk) == 0;  // "no progress for %d"
  ok &= (c.lnx & ~c.out) == 0;                                  // LearnersNext ⊆ Voters[1]
  ok &= (c.lnx & c.isl) == 0;                                   // staged, not yet learner
  ok &= (c.lrn & (c.out | c.inc)) == 0;                         // Learners ∩ Voters = ∅
  ok &= (c.lrn & ~c.isl) == 0;                                  // learners marked IsLearner
  ok &= c.out != 0 || (c.lnx == 0 && c.al == 0);                // non-joint: nil / false
#pragma unroll
  for (int s = 0; s < S; s++) {
    const bool ts = (c.trk >> s) & 1u;
    ok &= !ts || id[s] != 0;
#pragma unroll
    for (int t = s + 1; t < S; t++) {
      const bool tt = (c.trk >> t) & 1u;
      ok &= !(ts && tt && id[s] == id[t]);
    }
  }
  return ok;
}

// Slot bit of tracked peer `node`, 0 if it has no Progress.
template <int S>
__device__ __forceinline__ uint32_t cc_find(const uint64_t (&id)[kCCMax], uint32_t trk,
                                            uint64_t node) {
  uint32_t m = 0;
#pragma unroll
  for (int s = 0; s < S; s++) m |= (((trk >> s) & 1u) && id[s] == node) ? (1u << s) : 0u;
  return m & (0u - m);
}

// initProgress (:251-274): the lowest untracked slot gets the peer.
template <int S>
__device__ __forceinline__ int cc_init(CCState &c, uint64_t (&id)[kCCMax], uint64_t node,
                                       bool learner) {
  const uint32_t free = ~c.trk & ((1u << S) - 1u);
  if (free == 0) return QE_CC_ERR_NO_SLOT;
  const uint32_t b = free & (0u - free);
#pragma unroll
  for (int s = 0; s < S; s++) id[s] = b == (1u << s) ? node : id[s];
  c.trk |= b;
  c.newp |= b;
  if (learner) {
    c.lrn |= b;
    c.isl |= b;
  } else {
    c.inc |= b;
    c.isl &= ~b;
  }
  return QE_CC_OK;
}

// remove (:234-248): drop the peer from Voters[0] / Learners / LearnersNext;
// its Progress survives only while it is an outgoing voter.
__device__ __forceinline__ void cc_remove(CCState &c, uint32_t b) {
  c.inc &= ~b;
  c.lrn &= ~b;
  c.lnx &= ~b;
  if ((c.out & b) == 0) {
    c.trk &= ~b;
    c.newp &= ~b;
    c.isl &= ~b;
  }
}

// apply (:152-177).
template <int S>
__device__ __forceinline__ int cc_apply(const CCArgs &a, uint64_t g, CCState &c,
                                        uint64_t (&id)[kCCMax]) {
  const uint32_t n = a.count[g] < a.C ? a.count[g] : a.C;
  for (uint32_t k = 0; k < n; k++) {
    const uint64_t node = a.node[k * a.stride + g];
    const uint32_t typ = a.type[k * a.stride + g];
    if (node == 0) continue;  // etcd's "do not apply" marker (:154-160)
    const uint32_t b = cc_find<S>(id, c.trk, node);
    if (typ == QE_CC_ADD_NODE) {  // makeVoter (:181-193)
      if (b == 0) {
        const int rc = cc_init<S>(c, id, node, false);
        if (rc) return rc;
      } else {
        c.isl &= ~b;
        c.lrn &= ~b;
        c.lnx &= ~b;
        c.inc |= b;
      }
    } else if (typ == QE_CC_ADD_LEARNER_NODE) {  // makeLearner (:207-231)
      if (b == 0) {
        const int rc = cc_init<S>(c, id, node, true);
        if (rc) return rc;
      } else if ((c.isl & b) == 0) {
        // remove(), but the Progress is put back (prs[id] = pr)
        c.inc &= ~b;
        c.lrn &= ~b;
        c.lnx &= ~b;
        if (c.out & b) {
          c.lnx |= b;
        } else {
          c.isl |= b;
          c.lrn |= b;
        }
      }
    } else if (typ == QE_CC_REMOVE_NODE) {
      if (b) cc_remove(c, b);
    } else if (typ != QE_CC_UPDATE_NODE) {
      return QE_CC_ERR_BAD_TYPE;
    }
  }
  return c.inc == 0 ? QE_CC_ERR_REMOVED_ALL : QE_CC_OK;
}

// One group's change (one lane).  Slot IDs are ID-major, [S][G]: the
// group's tracked IDs are loaded row by row (consecutive lanes, consecutive
// addresses), and only the IDs the change rewrites are stored -- a created
// slot's new ID, a removed slot's 0 -- so a change touches one ID row, not
// the group's whole ID block.
template <int S>
__device__ __forceinline__ void cc_group(const CCArgs &a, uint64_t g) {
  using MT = typename std::conditional<(S <= 8), uint8_t, uint16_t>::type;
  constexpr uint32_t full = (1u << S) - 1u;
  const uint32_t op = a.op[g];
  if (op == QE_CC_OP_NONE) {
    a.result[g] = QE_CC_OK;
    if (a.new_progress) static_cast<MT *>(a.new_progress)[g] = 0;
    return;
  }
  // raw words as loaded: a field whose new value equals them is not stored
  const uint32_t r_inc = static_cast<const MT *>(a.inc)[g], r_out = static_cast<const MT *>(a.out)[g];
  const uint32_t r_lrn = static_cast<const MT *>(a.lrn)[g], r_lnx = static_cast<const MT *>(a.lnx)[g];
  const uint32_t r_isl = static_cast<const MT *>(a.isl)[g], r_trk = static_cast<const MT *>(a.trk)[g];
  const uint32_t r_al = a.auto_leave[g];
  CCState c{r_inc & full, r_out & full, r_lrn & full, r_lnx & full, r_isl & full, r_trk & full,
            r_al != 0 ? 1u : 0u, 0u};
  // the tracked slots' IDs (an untracked slot's ID is ignored)
  uint64_t id[kCCMax];
#pragma unroll
  for (int s = 0; s < kCCMax; s++)
    id[s] = (s < S && ((c.trk >> s) & 1u)) ? a.ids[static_cast<uint64_t>(s) * a.G + g] : 0ull;
  uint64_t id0[kCCMax];
#pragma unroll
  for (int s = 0; s < kCCMax; s++) id0[s] = id[s];
  const uint32_t inc0 = c.inc, trk0 = c.trk;
  int rc = cc_invariants<S>(c, id) ? QE_CC_OK : QE_CC_ERR_INVARIANT;  // checkAndCopy
  if (rc == QE_CC_OK) {
    if (op == QE_CC_OP_SIMPLE) {  // :130-147
      if (c.out) rc = QE_CC_ERR_SIMPLE_IN_JOINT;
      if (rc == QE_CC_OK) rc = cc_apply<S>(a, g, c, id);
      if (rc == QE_CC_OK) {
        // symdiff of the incoming voter ids (:384-401)
        uint32_t diff = 0;
#pragma unroll
        for (int s = 0; s < S; s++) {
          bool in_new = false, in_old = false;
#pragma unroll
          for (int t = 0; t < S; t++) {
            in_new |= ((c.inc >> t) & 1u) && id[t] == id0[s];
            in_old |= ((inc0 >> t) & 1u) && id0[t] == id[s];
          }
          diff += (((inc0 >> s) & 1u) && !in_new) ? 1u : 0u;
          diff += (((c.inc >> s) & 1u) && !in_old) ? 1u : 0u;
        }
        if (diff > 1) rc = QE_CC_ERR_SIMPLE_MULTI;
      }
    } else if (op == QE_CC_OP_ENTER_JOINT || op == QE_CC_OP_ENTER_JOINT_AUTO) {  // :49-76
      if (c.out) rc = QE_CC_ERR_ALREADY_JOINT;
      else if (c.inc == 0) rc = QE_CC_ERR_ZERO_VOTER_JOINT;
      if (rc == QE_CC_OK) {
        c.out = c.inc;
        rc = cc_apply<S>(a, g, c, id);
        c.al = op == QE_CC_OP_ENTER_JOINT_AUTO ? 1u : 0u;
      }
    } else if (op == QE_CC_OP_LEAVE_JOINT) {  // :92-123
      if (c.out == 0) {
        rc = QE_CC_ERR_NOT_JOINT;
      } else {
        c.lrn |= c.lnx;
        c.isl |= c.lnx;
        c.lnx = 0;
        const uint32_t dead = c.out & ~c.inc & ~c.lrn;
        c.trk &= ~dead;
        c.isl &= ~dead;
        c.out = 0;
        c.al = 0;
      }
    } else {
      rc = QE_CC_ERR_BAD_TYPE;
    }
    if (rc == QE_CC_OK && !cc_invariants<S>(c, id)) rc = QE_CC_ERR_INVARIANT_OUT;
  }
  a.result[g] = static_cast<uint8_t>(rc);
  const uint32_t created = rc == QE_CC_OK ? (c.newp & c.trk) : 0u;
  if (a.new_progress) static_cast<MT *>(a.new_progress)[g] = static_cast<MT>(created);
  if (rc != QE_CC_OK) return;  // a failed change keeps the group's state
  // only the words the change rewrote (a wave none of whose lanes changes a
  // field issues no store for it; in a Simple change out, LearnersNext and
  // AutoLeave never change)
  auto st = [&](void *p, uint32_t v, uint32_t raw) {
    if (v != raw) static_cast<MT *>(p)[g] = static_cast<MT>(v);
  };
  st(a.inc, c.inc, r_inc);
  st(a.out, c.out, r_out);
  st(a.lrn, c.lrn, r_lrn);
  st(a.lnx, c.lnx, r_lnx);
  st(a.isl, c.isl & c.trk, r_isl);
  st(a.trk, c.trk, r_trk);
  if (c.al != r_al) a.auto_leave[g] = static_cast<uint8_t>(c.al);
  // a slot the change untracks: 0; a slot tracked afterwards whose ID is
  // new (created, or freed and reused within the change list): the new ID
#pragma unroll
  for (int s = 0; s < S; s++) {
    const bool was = (trk0 >> s) & 1u, now = (c.trk >> s) & 1u;
    if ((was && !now) || (now && (!was || id[s] != id0[s])))
      a.ids[static_cast<uint64_t>(s) * a.G + g] = now ? id[s] : 0ull;
  }
  if (a.p_match && created) {
    const uint64_t li = a.last_index[g];
    for (int s = 0; s < S; s++) {
      if (((created >> s) & 1u) == 0) continue;
      const uint64_t r = s * a.pstride + g;
      a.p_match[r] = 0;
      a.p_next[r] = li;
      a.p_pending[r] = 0;
      a.p_pw[r] = QE_PR_PROBE | QE_PF_RECENT_ACTIVE;  // empty Inflights
    }
  }
}

template <int S>
__global__ __launch_bounds__(kBlock) void k_confchange(CCArgs a) {
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (g < a.G) cc_group<S>(a, g);
}

}  // namespace qe
