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
#include "qe_progress.hpp"

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
  uint32_t chunk;  // tiles per wave (<= kCCTPW)
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

// Per tile of 64 groups (one per lane), what the change reads besides the
// header word staged in LDS: the masks, the tracked slots' IDs, the first
// kCCPre changes and lastIndex.
constexpr int kCCTPW = 8;  // tiles per wave chunk (LDS: 256 B per tile per wave)
constexpr int kCCPre = 2;  // changes per group loaded with its tile; later ones on demand

template <int S>
struct CCTile {
  uint32_t inc, out, lrn, lnx, isl;
  uint64_t id[S];
  uint64_t node[kCCPre];
  uint32_t typ[kCCPre];
  uint64_t li;
};

// header word: op (bits 0-2), AutoLeave (3), count (8-15), tracked (16-31)
__device__ __forceinline__ uint32_t cc_op(uint32_t h) { return h & 7u; }
__device__ __forceinline__ uint32_t cc_count(uint32_t h) { return (h >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t cc_trk(uint32_t h) { return h >> 16; }

template <typename MT>
__device__ __forceinline__ uint32_t cc_ldm(const void *p, uint64_t g0, uint32_t n, uint32_t off) {
  const rsrc_t r = mk_rsrc(static_cast<const MT *>(p) + g0, n * sizeof(MT));
  if constexpr (sizeof(MT) == 1)
    return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
  else
    return __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
}

template <typename MT>
__device__ __forceinline__ void cc_stm(void *p, uint64_t g0, uint32_t n, uint32_t v, bool on,
                                       uint32_t lane) {
  if (!__builtin_amdgcn_ballot_w64(on)) return;  // no lane of the wave rewrites it
  bst_mask<MT>(v, mk_rsrc(static_cast<MT *>(p) + g0, n * sizeof(MT)), lane, on);
}

// One tile's loads.  A group with op None loads nothing but its header; an
// untracked slot's ID and a change past the group's count are dropped
// accesses (out-of-range offsets), so only what the change uses is fetched.
template <int S, typename MT>
__device__ __forceinline__ void cc_issue(const CCArgs &a, uint64_t t, uint32_t lane, uint32_t h,
                                         CCTile<S> &x) {
  const uint64_t g0 = t * 64;
  const uint32_t n = tile_n(a.G, t);
  const bool act = cc_op(h) != QE_CC_OP_NONE;
  const uint32_t mo = act ? lane * static_cast<uint32_t>(sizeof(MT)) : kOOB;
  x.inc = cc_ldm<MT>(a.inc, g0, n, mo);
  x.out = cc_ldm<MT>(a.out, g0, n, mo);
  x.lrn = cc_ldm<MT>(a.lrn, g0, n, mo);
  x.lnx = cc_ldm<MT>(a.lnx, g0, n, mo);
  x.isl = cc_ldm<MT>(a.isl, g0, n, mo);
  const uint32_t trk = act ? cc_trk(h) : 0u;
#pragma unroll
  for (int s = 0; s < S; s++)
    x.id[s] = bld64(mk_rsrc(a.ids + static_cast<uint64_t>(s) * a.G + g0, n * 8),
                    bit_off(trk, s, lane * 8));
  const uint32_t cnt = act ? cc_count(h) : 0u;
#pragma unroll
  for (int j = 0; j < kCCPre; j++) {
    const bool on = static_cast<uint32_t>(j) < cnt && static_cast<uint32_t>(j) < a.C;
    const uint32_t nj = static_cast<uint32_t>(j) < a.C ? n : 0u;
    const uint64_t r0 = static_cast<uint64_t>(j) * a.stride + g0;
    x.node[j] = bld64(mk_rsrc(a.node + (nj ? r0 : 0), nj * 8), on ? lane * 8 : kOOB);
    x.typ[j] = bld8(mk_rsrc(a.type + (nj ? r0 : 0), nj), on ? lane : kOOB);
  }
  x.li = bld64(mk_rsrc(a.last_index + g0, a.p_match ? n * 8 : 0u), act ? lane * 8 : kOOB);
}

// apply (:152-177): change k is (node[k], type[k]); the first kCCPre come
// from the tile's registers, later ones are loaded here.
template <int S>
__device__ __forceinline__ int cc_apply(const CCArgs &a, uint64_t g, uint32_t count,
                                        const CCTile<S> &x, CCState &c, uint64_t (&id)[kCCMax]) {
  const uint32_t n = count < a.C ? count : a.C;
  auto one = [&](uint64_t node, uint32_t typ) -> int {
    if (node == 0) return QE_CC_OK;  // etcd's "do not apply" marker (:154-160)
    const uint32_t b = cc_find<S>(id, c.trk, node);
    if (typ == QE_CC_ADD_NODE) {  // makeVoter (:181-193)
      if (b == 0) return cc_init<S>(c, id, node, false);
      c.isl &= ~b;
      c.lrn &= ~b;
      c.lnx &= ~b;
      c.inc |= b;
    } else if (typ == QE_CC_ADD_LEARNER_NODE) {  // makeLearner (:207-231)
      if (b == 0) return cc_init<S>(c, id, node, true);
      if ((c.isl & b) == 0) {
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
    return QE_CC_OK;
  };
#pragma unroll
  for (int j = 0; j < kCCPre; j++) {
    if (static_cast<uint32_t>(j) >= n) break;
    const int rc = one(x.node[j], x.typ[j]);
    if (rc) return rc;
  }
  for (uint32_t k = kCCPre; k < n; k++) {
    const int rc = one(a.node[k * a.stride + g], a.type[k * a.stride + g]);
    if (rc) return rc;
  }
  return c.inc == 0 ? QE_CC_ERR_REMOVED_ALL : QE_CC_OK;
}

// One tile's change (a group per lane) and its stores: the result and
// new_progress of every group; of a successful change only the words it
// rewrote.  Slot IDs are ID-major, [S][G]: a created slot's new ID and a
// removed slot's 0 are stored, so a change touches one ID row, not the
// group's whole ID block.  A wave none of whose lanes changes
// a field issues no store for it.
template <int S, typename MT>
__device__ __forceinline__ void cc_finish(const CCArgs &a, uint64_t t, uint32_t lane, uint32_t h,
                                          const CCTile<S> &x) {
  constexpr uint32_t full = (1u << S) - 1u;
  const uint64_t g0 = t * 64;
  const uint32_t n = tile_n(a.G, t);
  const uint32_t op = cc_op(h);
  const uint32_t r_trk = cc_trk(h), r_al = (h >> 3) & 1u;
  CCState c{x.inc & full, x.out & full, x.lrn & full, x.lnx & full, x.isl & full, r_trk & full,
            r_al, 0u};
  // the tracked slots' IDs (an untracked slot's ID is ignored)
  uint64_t id[kCCMax];
#pragma unroll
  for (int s = 0; s < kCCMax; s++) id[s] = s < S ? x.id[s] : 0ull;
  uint64_t id0[kCCMax];
#pragma unroll
  for (int s = 0; s < kCCMax; s++) id0[s] = id[s];
  const uint32_t inc0 = c.inc, trk0 = c.trk;
  int rc = QE_CC_OK;
  if (op != QE_CC_OP_NONE) {
    rc = cc_invariants<S>(c, id) ? QE_CC_OK : QE_CC_ERR_INVARIANT;  // checkAndCopy
    if (rc == QE_CC_OK) {
      if (op == QE_CC_OP_SIMPLE) {  // :130-147
        if (c.out) rc = QE_CC_ERR_SIMPLE_IN_JOINT;
        if (rc == QE_CC_OK) rc = cc_apply<S>(a, g0 + lane, cc_count(h), x, c, id);
        if (rc == QE_CC_OK) {
          // symdiff of the incoming voter ids (:384-401)
          uint32_t diff = 0;
#pragma unroll
          for (int s = 0; s < S; s++) {
            bool in_new = false, in_old = false;
#pragma unroll
            for (int u = 0; u < S; u++) {
              in_new |= ((c.inc >> u) & 1u) && id[u] == id0[s];
              in_old |= ((inc0 >> u) & 1u) && id0[u] == id[s];
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
          rc = cc_apply<S>(a, g0 + lane, cc_count(h), x, c, id);
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
  }
  bst8(static_cast<uint32_t>(rc), mk_rsrc(a.result + g0, n), lane);
  const bool ok = rc == QE_CC_OK && op != QE_CC_OP_NONE;  // a failed change keeps the state
  const uint32_t created = ok ? (c.newp & c.trk) : 0u;
  if (a.new_progress) bst_mask<MT>(created, mk_rsrc(static_cast<MT *>(a.new_progress) + g0,
                                                     n * sizeof(MT)), lane);
  // (compared with the words as loaded; in a Simple change out,
  // LearnersNext and AutoLeave never change)
  cc_stm<MT>(a.inc, g0, n, c.inc, ok && c.inc != x.inc, lane);
  cc_stm<MT>(a.out, g0, n, c.out, ok && c.out != x.out, lane);
  cc_stm<MT>(a.lrn, g0, n, c.lrn, ok && c.lrn != x.lrn, lane);
  cc_stm<MT>(a.lnx, g0, n, c.lnx, ok && c.lnx != x.lnx, lane);
  cc_stm<MT>(a.isl, g0, n, c.isl & c.trk, ok && (c.isl & c.trk) != x.isl, lane);
  cc_stm<MT>(a.trk, g0, n, c.trk, ok && c.trk != r_trk, lane);
  {
    const bool on = ok && c.al != r_al;
    if (__builtin_amdgcn_ballot_w64(on)) bst8(c.al, mk_rsrc(a.auto_leave + g0, n), on ? lane : kOOB);
  }
  // a slot the change untracks: 0; a slot tracked afterwards whose ID is
  // new (created, or freed and reused within the change list): the new ID
#pragma unroll
  for (int s = 0; s < S; s++) {
    const bool was = (trk0 >> s) & 1u, now = (c.trk >> s) & 1u;
    const bool wr = ok && ((was && !now) || (now && (!was || id[s] != id0[s])));
    if (__builtin_amdgcn_ballot_w64(wr))
      bst64(now ? id[s] : 0ull, mk_rsrc(a.ids + static_cast<uint64_t>(s) * a.G + g0, n * 8),
            wr ? lane * 8 : kOOB);
  }
  // initProgress (:251-274): Match 0, Next = lastIndex, Probe, RecentActive,
  // empty Inflights
  if (a.p_match) {
#pragma unroll
    for (int s = 0; s < S; s++) {
      const bool wr = (created >> s) & 1u;
      if (!__builtin_amdgcn_ballot_w64(wr)) continue;
      const uint64_t r0 = static_cast<uint64_t>(s) * a.pstride + g0;
      const uint32_t o8 = wr ? lane * 8 : kOOB;
      bst64(0, mk_rsrc(a.p_match + r0, n * 8), o8);
      bst64(x.li, mk_rsrc(a.p_next + r0, n * 8), o8);
      bst64(0, mk_rsrc(a.p_pending + r0, n * 8), o8);
      bst32(QE_PR_PROBE | QE_PF_RECENT_ACTIVE, mk_rsrc(a.p_pw + r0, n * 4), wr ? lane * 4 : kOOB);
    }
  }
}

// qe_confchange: each wave owns a chunk of up to kCCTPW tiles.  The chunk's
// header words (op, count, AutoLeave, tracked) are staged in LDS first, so a
// tile's ID and change loads depend on an LDS read, not on a vector load;
// two register sets keep tile k+1's loads in flight while tile k computes
// and stores (the stream kernels' pipeline, qe_stream.hpp).
template <int S>
__global__ __launch_bounds__(kBlock) void k_confchange(CCArgs a) {
  using MT = typename std::conditional<(S <= 8), uint8_t, uint16_t>::type;
  __shared__ uint32_t lds_h[kBlock / 64][kCCTPW][64];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t ntiles = (a.G + 63) / 64;
  const uint64_t t0 = (static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + wv) * a.chunk;
  if (t0 >= ntiles) return;
  const uint32_t nt = static_cast<uint32_t>(ntiles - t0 < a.chunk ? ntiles - t0 : a.chunk);
  uint32_t hv[kCCTPW];
#pragma unroll
  for (int k = 0; k < kCCTPW; k++) {
    const uint64_t g0 = (t0 + k) * 64;
    const uint32_t n = static_cast<uint32_t>(k) < nt ? tile_n(a.G, t0 + k) : 0u;
    const uint32_t op = bld8(mk_rsrc(a.op + g0, n), lane);
    const uint32_t cnt = bld8(mk_rsrc(a.count + g0, n), lane);
    const uint32_t al = bld8(mk_rsrc(a.auto_leave + g0, n), lane);
    const uint32_t trk = cc_ldm<MT>(a.trk, g0, n, lane * static_cast<uint32_t>(sizeof(MT)));
    hv[k] = (op > 7u ? 7u : op) | (al != 0 ? 8u : 0u) | (cnt << 8) | (trk << 16);
  }
#pragma unroll
  for (int k = 0; k < kCCTPW; k++) lds_h[wv][k][lane] = hv[k];
  // tile k of the chunk, or past the end (n = 0: no loads, no stores)
  auto tix = [&](uint32_t k) -> uint64_t { return k < nt ? t0 + k : ntiles; };
  auto hdr = [&](uint32_t k) -> uint32_t { return k < nt ? lds_h[wv][k][lane] : 0u; };
  CCTile<S> xa, xb;
  cc_issue<S, MT>(a, tix(0), lane, hdr(0), xa);
  for (uint32_t k = 0; k < nt; k += 2) {
    cc_issue<S, MT>(a, tix(k + 1), lane, hdr(k + 1), xb);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the change
    cc_finish<S, MT>(a, tix(k), lane, hdr(k), xa);
    cc_issue<S, MT>(a, tix(k + 2), lane, hdr(k + 2), xa);
    __builtin_amdgcn_sched_barrier(0);
    cc_finish<S, MT>(a, tix(k + 1), lane, hdr(k + 1), xb);
  }
}

}  // namespace qe
