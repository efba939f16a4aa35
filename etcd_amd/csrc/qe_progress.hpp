// qe_progress.hpp — qe_progress_step: the leader-side Progress state machine
// (stepLeader, raft/raft.go:1099-1338) with the sends it triggers executed
// where the reference executes them, and qe_progress_send.
//
// Decomposition (exact).  In the reference a message from
// peer s can call bcastAppend, which sends to EVERY peer, so the order of
// events matters.  But the only state a send changes is the receiving
// peer's own Progress, and the commit decisions depend on Match alone,
// which only the peer's own MsgAppResp changes.  So:
//   phase 1  (per group, registers only) replays MaybeUpdate + maybeCommit
//            over the slots in message order -> B = the set of slots whose
//            accept advanced the commit (each one bcastAppend);
//   phase 2  (per peer, slots in order) replays that peer's event sequence:
//            one sendAppend per bcast from a slot before it, its own
//            message (with the bcast of its own accept, the oldPaused
//            sendAppend, the `for maybeSendAppend(from, false)` loop and the
//            MsgTimeoutNow check), then one sendAppend per later bcast.
// One lane per group, a wave per 64-group tile; the next slot's loads are
// issued before this slot's work.  (A two-pass variant -- commit pass, then
// one lane per peer -- was measured slower: DESIGN.md §6.)
//
// Sends have a closed form (send_burst): consecutive maybeSendAppend calls
// on one peer append an arithmetic run of Inflights entries.  A peer's round
// appends at most two runs (before and after its own message, whose handler
// may reset the ring), so for F <= kRingChunk the ring is written once at
// the end, entry row by entry row, from the two runs.
//
// Inflights rings are entry-major, [S][F][stride] (entry k of slot s of
// group g at (s*F + k)*stride + g): entry k of a tile is one coalesced
// 512-B access, where a peer-major row per lane touched 32-64 cache lines.
//
// Accesses go through per-tile buffer descriptors (wave-uniform base, 32-bit
// lane offset, num_records clipping the ragged last tile), as in the stream
// commit/vote kernel (qe_stream.hpp): a conditional access is an
// unconditional load or store whose offset is pushed out of range when its
// condition is false (no traffic, no branch, loads return 0).  Accesses that
// are rare for a whole wave sit behind real (wave-uniform) branches.
#pragma once
#include "qe_stream.hpp"

namespace qe {

constexpr int kRingChunk = 8;  // F <= kRingChunk: the ring lives in registers (row form)

// Cache policy of the Progress kernels' accesses (the helpers' AUX: 0 =
// default, 2 = non-temporal).  The Progress step re-touches the lines it
// loads (non-temporal loads: +15 %) and so does CheckQuorum (+17 %); the send
// kernel's appends and Progress rows go non-temporal, kNT: -9 %
// (profiles/r04/pstep_ab.txt, send_cq_nt_ab.txt).
// QE_LD_AUX / QE_ST_AUX: A/B knobs for the default.
#ifndef QE_LD_AUX
#define QE_LD_AUX 0
#endif
#ifndef QE_ST_AUX
#define QE_ST_AUX 0
#endif
#ifndef QE_SEND_AUX  // A/B knob: the send kernel's policy
#define QE_SEND_AUX 2
#endif
constexpr int kNT = QE_SEND_AUX;
template <int AUX = QE_LD_AUX>
__device__ __forceinline__ uint64_t bld64(rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX));
}
template <int AUX = QE_LD_AUX>
__device__ __forceinline__ uint32_t bld8(rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, AUX);
}
template <int AUX = QE_ST_AUX>
__device__ __forceinline__ void bst64(uint64_t v, rsrc_t r, uint32_t off) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, AUX);
}
template <int AUX = QE_ST_AUX>
__device__ __forceinline__ void bst8(uint32_t v, rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(v), r, off, 0, AUX);
}
template <int AUX = QE_LD_AUX>
__device__ __forceinline__ uint32_t bld32(rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, AUX);
}
template <int AUX = QE_ST_AUX>
__device__ __forceinline__ void bst32(uint32_t v, rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, AUX);
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 bld128(rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, QE_LD_AUX));
}
__device__ __forceinline__ void bst128(u32x4 v, rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, QE_ST_AUX);
}
template <typename MT>
__device__ __forceinline__ void bst_mask(uint32_t v, rsrc_t r, uint32_t lane, bool on = true) {
  const uint32_t off = on ? lane * static_cast<uint32_t>(sizeof(MT)) : kOOB;
  if constexpr (sizeof(MT) == 1)
    __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(v), r, off, 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(v), r, off, 0, 0);
}

// Byte accounting of the instrumented variant (ACCT): the bytes of every
// access the reference logic needs (field granularity, each once), i.e. the
// algorithmic bytes of the round.  Re-reads (Match, m.Index in phase 2)
// are not counted.  The rules are restated independently by
// the oracle (orc_progress_step_batch's byte count), and the GPU tests
// require the two counts to be equal.
template <bool ACCT>
struct Acct {
  uint64_t b = 0;
  __device__ __forceinline__ void add(bool on, uint32_t bytes) {
    if constexpr (ACCT) b += on ? bytes : 0u;
  }
};
template <bool ACCT>
__device__ __forceinline__ void acct_flush(const Acct<ACCT> &ac, uint64_t *acct) {
  if constexpr (ACCT) {
    uint64_t b = ac.b;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) b += __shfl_xor(b, d, 64);
    if ((threadIdx.x & 63) == 0 && acct)
      atomicAdd(reinterpret_cast<unsigned long long *>(acct), static_cast<unsigned long long>(b));
  }
}

// Checksum of the round: a per-group part from the commit pass and a
// per-group part from the peer pass (oracle/quorum_oracle.c orc_checksum_step).
constexpr uint64_t kSentSalt = 0xD1B54A32D192ED03ull;
constexpr uint64_t kReadSalt = 0x8CB92BA72F3D8DD7ull;   // released ReadIndex requests
constexpr uint64_t kTermSalt = 0x589965CC75374CC3ull;   // first commit in the leader's term
constexpr uint64_t kTransferSalt = 0x1D8E4E27C47D124Full; // lead_transferee changed
constexpr uint64_t kQuorumSalt = 0xA0761D6478BD642Full; // CheckQuorum: quorum active

// ---------------------------------------------------------------------------
// Inflights rings (ABI 4, include/etcd_quorum.h): 32-bit entry words,
// lane-major [S][stride][FP], the upper words given by the peer word's epoch
// (or, for a "wide" peer, by infl_hi).  A tile's ring block for one slot is
// 64 x FP words; lane l's ring starts at byte l*FP*4 of it, so a ring of
// F <= 8 entries is one or two 16-byte accesses and one 32-byte HBM sector.
// The partial-sector write of a single appended entry is what an Inflights.
// Add costs the memory system (scripts/append_probe.hip: ~990 cycles per
// wave for an 8-byte entry, ~505 for a 4-byte one, ~460 for rewriting the
// whole 32-byte ring), hence 32-bit words and whole-ring writes where the
// ring is in registers anyway.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool rep_wide(uint32_t rep) { return (rep & QE_PF_RING_WIDE) != 0; }
__device__ __forceinline__ uint32_t rep_epoch(uint32_t rep) { return QE_PW_EPOCH(rep); }
__device__ __forceinline__ uint64_t ent64(uint32_t hi, uint32_t lo) {
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// ---------------------------------------------------------------------------
// Sends: raft.maybeSendAppend (raft/raft.go:432-492) in closed form.
// ---------------------------------------------------------------------------
// A run of Inflights entries appended by consecutive sends: n entries from
// ring position p, the first MsgApp starting at Next = b; entry j is the
// last index of MsgApp j: b + min(lastIndex - b, (j+1)*max_ents - 1)
// (OptimisticUpdate moves Next past it, the next MsgApp starts there), or
// lastIndex when max_ents = 0 (noLimit: one MsgApp carries every entry).
struct PRun {
  uint32_t p, n;
  uint64_t b;
};

struct PSend {
  rsrc_t rlo, rhi;  // this slot's ring block of the tile (infl_lo / infl_hi)
  rsrc_t r16;       // ABI 8: the block in the 16-bit form (infl16; lane * 16)
  uint32_t lb;      // lane * FP * 4: the lane's ring in the block
  uint32_t eb = 4;  // bytes of one entry in the device form (accounting): 4, 2
  bool row;         // F <= kRingChunk: the runs are written by ring_store_row
  uint32_t F, me;
  uint64_t fi, li, snap;
  uint32_t count_msgs;   // messages sent to this peer this round (saturating)
  uint64_t first_index;  // m.Index of the first of them
  bool snapped;
};

__device__ __forceinline__ uint64_t run_val(const PRun &r, uint32_t j, uint32_t me, uint64_t li) {
  if (me == 0) return li;
  const uint64_t step = static_cast<uint64_t>(j + 1) * me - 1;
  const uint64_t d = li - r.b;
  return r.b + (step < d ? step : d);
}

// Ring position of the next append (Inflights.Add, inflights.go:55-71); an
// invalid Inflights.start (>= F) stays inside the ring.
__device__ __forceinline__ uint32_t ring_pos(uint32_t start, uint32_t count, uint32_t F) {
  uint32_t pos = start + count;
  if (pos >= F) pos -= F;
  if (pos >= F) pos = 0;
  return pos;
}

// Inflights.Add(v) at ring position pos, memory form (F > kRingChunk, and
// the single appends of qe_progress_send): the entry's low word always; the
// first entry of an empty ring sets the epoch (or, above QE_RING_EPOCH_MAX,
// makes the ring wide); an entry whose upper word differs from the epoch of
// a non-empty ring turns it wide -- every live entry's upper word (the
// epoch) is written first, a rare path; a wide ring also gets the entry's
// upper word.
template <int AUX = QE_ST_AUX>
__device__ __forceinline__ void ring_add_mem(PR &p, const PSend &x, bool on, uint32_t pos,
                                             uint64_t v) {
  const uint32_t h = static_cast<uint32_t>(v >> 32);
  bst32<AUX>(static_cast<uint32_t>(v), x.rlo, on ? x.lb + pos * 4 : kOOB);
  const bool first = p.count == 0;
  const bool conv = on && !first && !rep_wide(p.rep) && h != rep_epoch(p.rep);
  if (__builtin_amdgcn_ballot_w64(conv)) {
    const uint32_t ep = rep_epoch(p.rep);
    uint32_t q = p.start;
    while (q >= x.F) q -= x.F;
    for (uint32_t j = 0; __builtin_amdgcn_ballot_w64(conv && j < p.count); j++) {
      bst32<AUX>(ep, x.rhi, (conv && j < p.count) ? x.lb + q * 4 : kOOB);
      if (++q >= x.F) q = 0;
    }
  }
  if (on) {
    if (first)
      p.rep = h <= QE_RING_EPOCH_MAX ? QE_PW_EPOCH_BITS(h) : QE_PF_RING_WIDE;
    else if (conv)
      p.rep = QE_PF_RING_WIDE;
  }
  const bool whi = on && rep_wide(p.rep);
  if (__builtin_amdgcn_ballot_w64(whi)) bst32<AUX>(h, x.rhi, whi ? x.lb + pos * 4 : kOOB);
}

// Entry at ring position pos, memory form, decoded with the representation
// `rep` the ring had when the round began.
__device__ __forceinline__ uint64_t ring_get_mem(const PSend &x, uint32_t rep, bool on, uint32_t pos) {
  const uint32_t off = on ? x.lb + pos * 4 : kOOB;
  const uint32_t lo = bld32(x.rlo, off);
  const uint32_t hi = rep_wide(rep) ? bld32(x.rhi, off) : rep_epoch(rep);
  return ent64(hi, lo);
}

constexpr uint32_t kLoop = 0xFFFFFFFFu;

// `k` consecutive raft.maybeSendAppend(to, sei) calls on one peer, or with
// k = kLoop one call with `sei` followed by `for maybeSendAppend(to, false)
// {}`.  A paused peer gets nothing; with no entries (Next > lastIndex) every
// call with sendIfEmpty sends an empty MsgApp; Next < firstIndex: nothing
// unless sendIfEmpty (raft.go:442-444 come first), then one MsgSnap to a
// recently active peer (BecomeSnapshot pauses it); Probe: one MsgApp,
// ProbeSent pauses it; Replicate: one MsgApp per max_ents entries
// (OptimisticUpdate + Inflights.Add) until the ring is full or Next passes
// lastIndex, then empty MsgApps for the remaining calls with sendIfEmpty.
// The appended entries extend `run`.
template <bool ACCT, int AUX = QE_ST_AUX>
__device__ __forceinline__ void send_burst(PR &p, bool sei, uint32_t k, PSend &x, PRun &run,
                                           Acct<ACCT> &ac) {
  const bool loop = k == kLoop;
  const bool go = k > 0 && !pr_paused(p, x.F);
  const bool empty = p.next > x.li;
  const bool comp = !empty && p.next < x.fi;  // entries() fails with ErrCompacted
  uint64_t idx0 = p.next - 1;
  uint32_t nmsg = (go && empty && sei) ? (loop ? 1u : k) : 0u;
  if (go && comp && sei && p.recent_active) {  // the sendIfEmpty check comes first (:442-444)
    pr_reset(p, QE_PR_SNAPSHOT);                // BecomeSnapshot(snapshot index) (:468)
    p.pending = x.snap;
    x.snapped = true;
    idx0 = x.snap;
    nmsg = 1;
  }
  const bool ents = go && !empty && !comp;
  if (ents && p.state == QE_PR_PROBE) {
    p.probe_sent = 1;
    nmsg = 1;
  }
  const bool repl = ents && p.state == QE_PR_REPLICATE;
  const uint32_t room = x.F > p.count ? x.F - p.count : 0u;
  const uint32_t lim = repl ? ((loop || room < k) ? room : k) : 0u;
  const uint64_t d = x.li - p.next;  // valid when repl
  uint32_t added = 0;
  if (x.row) {  // lim <= F <= kRingChunk: count the appends directly
    // MsgApps whose first entry is <= lastIndex: 1 + min(7, d / max_ents),
    // by a 3-step binary search on the quotient (the multiples are uniform)
    uint32_t fit = 1;
    if (x.me) {
      const uint64_t me = x.me;
      uint32_t q = d >= 4 * me ? 4u : 0u;
      q += d >= (q + 2) * me ? 2u : 0u;
      q += d >= (q + 1) * me ? 1u : 0u;
      fit += q;
    }
    added = x.me ? (lim < fit ? lim : fit) : (lim ? 1u : 0u);
    if (added) {
      if (run.n == 0) {
        run.p = ring_pos(p.start, p.count, x.F);
        run.b = p.next;
      }
      run.n += added;
      const PRun here{0, 0, p.next};
      p.next = run_val(here, added - 1, x.me, x.li) + 1;
      p.count += added;
      ac.add(true, x.eb * added);
    }
  } else {  // memory form: append entry by entry, straight to memory
    while (__builtin_amdgcn_ballot_w64(added < lim && p.next <= x.li)) {
      const bool on = added < lim && p.next <= x.li;
      const PRun here{0, 0, p.next};
      const uint64_t last = run_val(here, 0, x.me, x.li);
      const uint32_t pos = ring_pos(p.start, p.count, x.F);
      ring_add_mem<AUX>(p, x, on, pos, last);
      if (on) {
        if (run.n == 0) {
          run.p = pos;
          run.b = p.next;
        }
        run.n += 1;
        p.next = last + 1;
        p.count += 1;
        added += 1;
      }
      ac.add(on, x.eb);
    }
  }
  if (repl) {
    nmsg = added;
    if (!loop && sei && added < k && p.count < x.F && p.next > x.li) nmsg += k - added;  // empties
  }
  if (nmsg) {
    if (x.count_msgs == 0) x.first_index = idx0;
    const uint32_t c = x.count_msgs + (nmsg < 255u ? nmsg : 255u);
    x.count_msgs = c < 255u ? c : 255u;
  }
}

// Row form (F <= kRingChunk): the whole ring of a peer whose ring may be
// read or rewritten (`ld`: touched, with live entries) in registers, one or
// two 16-byte loads per lane; hi[] holds every position's upper word (the
// epoch unless the peer is wide).
// ABI 8, the 16-bit form: entry k = Next - 1 - off[k] (eight u16 offsets in
// 16 bytes per lane), decoded with the peer's Next as the round found it; a
// wide peer's entries from infl_lo / infl_hi (rare).
template <bool P>
__device__ __forceinline__ void ring_load_n16(const PSend &x, bool ld, uint32_t rep, uint32_t FP,
                                              uint32_t (&lo)[kRingChunk],
                                              uint32_t (&hi)[kRingChunk], const uint32_t *pre,
                                              uint64_t nx_old) {
  u32x4 a = {0, 0, 0, 0};
  if (pre) {
    a = u32x4{pre[0], pre[1], pre[2], pre[3]};
  } else if (__builtin_amdgcn_ballot_w64(ld)) {
    a = bld128(x.r16, ld ? (threadIdx.x & 63) * 16 : kOOB);
  }
  const uint64_t top = nx_old - 1;
  const uint32_t w4[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int k = 0; k < kRingChunk; k++) {
    const uint64_t e = top - ((w4[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
    lo[k] = static_cast<uint32_t>(e);
    hi[k] = static_cast<uint32_t>(e >> 32);
  }
  const bool w = ld && rep_wide(rep);
  if (__builtin_amdgcn_ballot_w64(w)) {  // rare: a window past 65535 indices
    const u32x4 l0 = bld128(x.rlo, w ? x.lb : kOOB);
    const u32x4 h0 = bld128(x.rhi, w ? x.lb : kOOB);
    u32x4 l1 = {0, 0, 0, 0}, h1 = {0, 0, 0, 0};
    if (FP > 4) {
      l1 = bld128(x.rlo, w ? x.lb + 16 : kOOB);
      h1 = bld128(x.rhi, w ? x.lb + 16 : kOOB);
    }
    if constexpr (P)  // waited here, on this (rare) path only
      asm volatile("" ::"v"(l0.x), "v"(l0.y), "v"(l0.z), "v"(l0.w), "v"(h0.x), "v"(h0.y),
                   "v"(h0.z), "v"(h0.w), "v"(l1.x), "v"(l1.y), "v"(l1.z), "v"(l1.w), "v"(h1.x),
                   "v"(h1.y), "v"(h1.z), "v"(h1.w));
    if (w) {
      lo[0] = l0.x, lo[1] = l0.y, lo[2] = l0.z, lo[3] = l0.w;
      lo[4] = l1.x, lo[5] = l1.y, lo[6] = l1.z, lo[7] = l1.w;
      hi[0] = h0.x, hi[1] = h0.y, hi[2] = h0.z, hi[3] = h0.w;
      hi[4] = h1.x, hi[5] = h1.y, hi[6] = h1.z, hi[7] = h1.w;
    }
  }
}

template <bool P>
__device__ __forceinline__ void ring_load_row(const PSend &x, bool ld, uint32_t rep, uint32_t FP,
                                              uint32_t (&lo)[kRingChunk],
                                              uint32_t (&hi)[kRingChunk],
                                              const uint32_t *pre = nullptr) {
#pragma unroll
  for (int k = 0; k < kRingChunk; k++) lo[k] = (pre && ld) ? pre[k] : 0u;
  if (!pre && __builtin_amdgcn_ballot_w64(ld)) {
    const u32x4 a = bld128(x.rlo, ld ? x.lb : kOOB);
    lo[0] = a.x, lo[1] = a.y, lo[2] = a.z, lo[3] = a.w;
    if (FP > 4) {
      const u32x4 b = bld128(x.rlo, ld ? x.lb + 16 : kOOB);
      lo[4] = b.x, lo[5] = b.y, lo[6] = b.z, lo[7] = b.w;
    }
  }
  const uint32_t ep = rep_epoch(rep);
#pragma unroll
  for (int k = 0; k < kRingChunk; k++) hi[k] = ep;
  const bool w = ld && rep_wide(rep);
  if (__builtin_amdgcn_ballot_w64(w)) {  // rare: entries straddling epochs
    const u32x4 a = bld128(x.rhi, w ? x.lb : kOOB);
    u32x4 b = {0, 0, 0, 0};
    if (FP > 4) b = bld128(x.rhi, w ? x.lb + 16 : kOOB);
    if constexpr (P)  // waited here, on this (rare) path only
      asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z),
                   "v"(b.w));
    if (w) hi[0] = a.x, hi[1] = a.y, hi[2] = a.z, hi[3] = a.w;
    if (w) hi[4] = b.x, hi[5] = b.y, hi[6] = b.z, hi[7] = b.w;
  }
}

// Row form: the peer's ring after the round, where a run appended.
// Positions a run covers take the run's entry (the later run wins: it was
// appended after the earlier one), the others keep what was loaded; the ring
// is written back whole (full 32-byte sectors, no partial-sector writes) and
// its representation recomputed canonically from the live entries (the
// upper words written only when the peer is wide).  A ring nothing appended
// to keeps its representation: FreeLE and ResetState keep it valid.
// Low words of a run's entries in 32-bit arithmetic: entry j is
// b + min(d, (j+1)*me - 1) with d = lastIndex - b (run_val), so its low word
// is lo(b) + lo(min) mod 2^32, and the min is the step for j < jcap =
// min(8, floor(d / me)) (0 for noLimit: every entry is lastIndex), else d.
struct RunLo {
  uint32_t lob, lod, jcap;
};
__device__ __forceinline__ RunLo run_lo(const PRun &r, uint32_t me, uint64_t li) {
  const uint64_t d = li - r.b;
  uint32_t q = 0;
  if (me) {  // wave-uniform
    const uint64_t m = me;
    q = d >= 4 * m ? 4u : 0u;
    q += d >= (q + 2) * m ? 2u : 0u;
    q += d >= (q + 1) * m ? 1u : 0u;
    q = d >= 8 * m ? 8u : q;
  }
  return RunLo{static_cast<uint32_t>(r.b), static_cast<uint32_t>(d), q};
}
__device__ __forceinline__ uint32_t run_lo_at(const RunLo &L, uint32_t j, uint32_t me) {
  return L.lob + (j < L.jcap ? (j + 1) * me - 1u : L.lod);
}

template <bool P>
__device__ __forceinline__ void ring_store_row(PR &p, const PSend &x, const PRun &r1,
                                               const PRun &r2, bool touched, uint32_t rep_in,
                                               uint32_t c_old, uint32_t FP,
                                               uint32_t (&lo)[kRingChunk],
                                               uint32_t (&hi)[kRingChunk]) {
  const bool any = (r1.n | r2.n) != 0;
  if (!P && !__builtin_amdgcn_ballot_w64(touched && any))
    return;  // the ring stands as loaded
  const bool wl = touched && any;
  {
    // Common case: every appended entry and every old one share one upper
    // word h <= QE_RING_EPOCH_MAX (runs are monotonic: their first and last
    // entries decide), so the ring stays narrow and only low words change.
    const uint32_t hb1 = static_cast<uint32_t>(r1.b >> 32), hb2 = static_cast<uint32_t>(r2.b >> 32);
    const uint32_t h = r2.n ? hb2 : hb1;
    const uint32_t hl1 =
        static_cast<uint32_t>(run_val(r1, r1.n ? r1.n - 1 : 0, x.me, x.li) >> 32);
    const uint32_t hl2 =
        static_cast<uint32_t>(run_val(r2, r2.n ? r2.n - 1 : 0, x.me, x.li) >> 32);
    const bool ok = h <= QE_RING_EPOCH_MAX && (r1.n == 0 || (hb1 == h && hl1 == h)) &&
                    (r2.n == 0 || (hb2 == h && hl2 == h)) &&
                    (c_old == 0 || (!rep_wide(rep_in) && rep_epoch(rep_in) == h));
    if (!__builtin_amdgcn_ballot_w64(wl && !ok)) {
      const RunLo L1 = run_lo(r1, x.me, x.li), L2 = run_lo(r2, x.me, x.li);
#pragma unroll
      for (int k = 0; k < kRingChunk; k++) {
        if (static_cast<uint32_t>(k) >= x.F) break;
        const uint32_t j1 = static_cast<uint32_t>(k) >= r1.p ? k - r1.p : k + x.F - r1.p;
        const uint32_t j2 = static_cast<uint32_t>(k) >= r2.p ? k - r2.p : k + x.F - r2.p;
        lo[k] = j2 < r2.n ? run_lo_at(L2, j2, x.me) : (j1 < r1.n ? run_lo_at(L1, j1, x.me) : lo[k]);
      }
      if (wl) p.rep = p.count ? QE_PW_EPOCH_BITS(h) : 0u;
      if (P || __builtin_amdgcn_ballot_w64(wl)) {
        bst128(u32x4{lo[0], lo[1], lo[2], lo[3]}, x.rlo, wl ? x.lb : kOOB);
        if (FP > 4) bst128(u32x4{lo[4], lo[5], lo[6], lo[7]}, x.rlo, wl ? x.lb + 16 : kOOB);
      }
      return;
    }
  }
  // General case (some lane's ring straddles upper words): every position's
  // full value, the representation recomputed from the live entries.
  uint32_t h0 = 0;
  bool seen = false, uni = true;
  const uint32_t st = p.start;
#pragma unroll
  for (int k = 0; k < kRingChunk; k++) {
    if (static_cast<uint32_t>(k) >= x.F) break;
    const uint32_t j1 = static_cast<uint32_t>(k) >= r1.p ? k - r1.p : k + x.F - r1.p;
    const uint32_t j2 = static_cast<uint32_t>(k) >= r2.p ? k - r2.p : k + x.F - r2.p;
    const bool on1 = j1 < r1.n, on2 = j2 < r2.n;
    if (on1 || on2) {
      const uint64_t v = on2 ? run_val(r2, j2, x.me, x.li) : run_val(r1, j1, x.me, x.li);
      lo[k] = static_cast<uint32_t>(v);
      hi[k] = static_cast<uint32_t>(v >> 32);
    }
    const uint32_t rel = static_cast<uint32_t>(k) >= st ? k - st : k + x.F - st;
    if (rel < p.count) {
      uni = uni && (!seen || hi[k] == h0);
      h0 = seen ? h0 : hi[k];
      seen = true;
    }
  }
  const bool wide = seen && (!uni || h0 > QE_RING_EPOCH_MAX);
  if (wl) p.rep = !seen ? 0u : (wide ? QE_PF_RING_WIDE : QE_PW_EPOCH_BITS(h0));
  if (__builtin_amdgcn_ballot_w64(wl)) {
    bst128(u32x4{lo[0], lo[1], lo[2], lo[3]}, x.rlo, wl ? x.lb : kOOB);
    if (FP > 4) bst128(u32x4{lo[4], lo[5], lo[6], lo[7]}, x.rlo, wl ? x.lb + 16 : kOOB);
  }
  const bool wh = wl && wide;
  if (__builtin_amdgcn_ballot_w64(wh)) {
    bst128(u32x4{hi[0], hi[1], hi[2], hi[3]}, x.rhi, wh ? x.lb : kOOB);
    if (FP > 4) bst128(u32x4{hi[4], hi[5], hi[6], hi[7]}, x.rhi, wh ? x.lb + 16 : kOOB);
  }
}

// ABI 8, the 16-bit form: the peer's ring after the round, re-based on its
// final Next, wherever the round appended or moved Next while entries are
// live (both only on appends in reachable states: OptimisticUpdate, while
// MaybeUpdate past every sent index empties the ring).  Positions a run
// covers take the run's entry (the later run wins), the others keep what
// was loaded.  A ring whose live entries all lie in [Next - 65536, Next - 1]
// is written as eight offsets, 16 bytes (two lanes per 32-byte sector);
// otherwise (rare) it turns wide: both words of every position in infl_lo /
// infl_hi.
template <bool P>
__device__ __forceinline__ void ring_store_n16(PR &p, const PSend &x, const PRun &r1,
                                               const PRun &r2, bool touched, uint64_t nx_old,
                                               uint32_t FP, uint32_t (&lo)[kRingChunk],
                                               uint32_t (&hi)[kRingChunk]) {
  const bool any = (r1.n | r2.n) != 0;
  const bool wl = touched && p.count > 0 && (any || p.next != nx_old);
  if (!P && !__builtin_amdgcn_ballot_w64(wl)) return;  // the ring stands as loaded
  const uint64_t top = p.next - 1;
  const uint32_t st = p.start;
  bool fits = true;
  uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < kRingChunk; k++) {
    const uint32_t j1 = static_cast<uint32_t>(k) >= r1.p ? k - r1.p : k + x.F - r1.p;
    const uint32_t j2 = static_cast<uint32_t>(k) >= r2.p ? k - r2.p : k + x.F - r2.p;
    const bool on1 = j1 < r1.n, on2 = j2 < r2.n;
    const uint64_t v = on2 ? run_val(r2, j2, x.me, x.li)
                           : (on1 ? run_val(r1, j1, x.me, x.li) : ent64(hi[k], lo[k]));
    lo[k] = static_cast<uint32_t>(v);
    hi[k] = static_cast<uint32_t>(v >> 32);
    const uint32_t rel = static_cast<uint32_t>(k) >= st ? k - st : k + x.F - st;
    const bool live = static_cast<uint32_t>(k) < x.F && rel < p.count;
    fits = fits && (!live || (v <= top && top - v <= 0xFFFFull));
    o[k >> 1] |= (static_cast<uint32_t>(top - v) & 0xFFFFu) << (16 * (k & 1));
  }
  if (wl) p.rep = fits ? 0u : QE_PF_RING_WIDE;
  if (P || __builtin_amdgcn_ballot_w64(wl))
    bst128(u32x4{o[0], o[1], o[2], o[3]}, x.r16, (wl && fits) ? (threadIdx.x & 63) * 16 : kOOB);
  const bool ww = wl && !fits;
  if (__builtin_amdgcn_ballot_w64(ww)) {
    bst128(u32x4{lo[0], lo[1], lo[2], lo[3]}, x.rlo, ww ? x.lb : kOOB);
    bst128(u32x4{hi[0], hi[1], hi[2], hi[3]}, x.rhi, ww ? x.lb : kOOB);
    if (FP > 4) {
      bst128(u32x4{lo[4], lo[5], lo[6], lo[7]}, x.rlo, ww ? x.lb + 16 : kOOB);
      bst128(u32x4{hi[4], hi[5], hi[6], hi[7]}, x.rhi, ww ? x.lb + 16 : kOOB);
    }
  }
}

// ABI 8, the appends of the send-only kernels (qe_progress_send, qe_propose,
// qe_switch_config: one maybeSendAppend per peer, so at most ONE appended
// entry) in the 16-bit form, on the offsets themselves: an append moves Next
// by delta, so every old offset grows by delta and the new entry v takes
// Next - 1 - v -- 32-bit arithmetic, no decoding of the ring.  `raw` is the
// ring as loaded (16 bytes).  Rare: a wide ring stays wide (the new entry's
// two words written); a ring whose entries no longer fit turns wide (every
// position's two words written, rolled, few registers).
__device__ __forceinline__ void ring_append_n16(PR &p, const PSend &x, const PRun &run, bool on,
                                                uint64_t nx_old, uint32_t rep_old, u32x4 raw,
                                                uint32_t FP) {
  const bool wl = on && p.count > 0 && (run.n != 0 || p.next != nx_old);
  if (!__builtin_amdgcn_ballot_w64(wl)) return;
  const uint64_t d64 = p.next - nx_old;
  const uint32_t delta = d64 > 0xFFFFull ? 0x10000u : static_cast<uint32_t>(d64);
  const uint32_t w4[4] = {raw.x, raw.y, raw.z, raw.w};
  const uint32_t st = p.start;
  bool fits = !rep_wide(rep_old);
  uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < kRingChunk; k++) {
    const uint32_t j = static_cast<uint32_t>(k) >= run.p ? k - run.p : k + x.F - run.p;
    const uint32_t rel = static_cast<uint32_t>(k) >= st ? k - st : k + x.F - st;
    const bool live = static_cast<uint32_t>(k) < x.F && rel < p.count;
    uint32_t off;
    if (j < run.n) {  // appended this call: Next - 1 - v, v <= Next - 1
      const uint64_t d = p.next - 1 - run_val(run, j, x.me, x.li);
      off = d > 0xFFFFull ? 0x10000u : static_cast<uint32_t>(d);
    } else {
      off = ((w4[k >> 1] >> (16 * (k & 1))) & 0xFFFFu) + delta;
    }
    fits = fits && (!live || off <= 0xFFFFu);
    o[k >> 1] |= (off & 0xFFFFu) << (16 * (k & 1));
  }
  if (wl && fits) p.rep = 0u;
  bst128(u32x4{o[0], o[1], o[2], o[3]}, x.r16, (wl && fits) ? (threadIdx.x & 63) * 16 : kOOB);
  const bool slow = wl && !fits;
  if (__builtin_amdgcn_ballot_w64(slow)) {  // a wide ring, or a window past 65535 indices
    const bool was_wide = rep_wide(rep_old);
    const uint64_t top_old = nx_old - 1;
    const uint64_t vnew = run.n ? run_val(run, 0, x.me, x.li) : 0;
#pragma unroll 1
    for (uint32_t k = 0; k < x.F; k++) {
      const bool isnew = run.n != 0 && k == run.p;
      const bool wr = slow && (isnew || !was_wide);  // a wide ring keeps its old words
      const uint32_t h = k >> 1;
      const uint32_t wd = h == 0 ? raw.x : (h == 1 ? raw.y : (h == 2 ? raw.z : raw.w));
      const uint64_t v = isnew ? vnew : top_old - ((wd >> (16 * (k & 1))) & 0xFFFFu);
      bst32(static_cast<uint32_t>(v), x.rlo, wr ? x.lb + k * 4 : kOOB);
      bst32(static_cast<uint32_t>(v >> 32), x.rhi, wr ? x.lb + k * 4 : kOOB);
    }
    if (slow) p.rep = QE_PF_RING_WIDE;
  }
}

// Inflights.FreeLE(to) (raft/tracker/inflights.go:87-113) given fr_old, the
// number of this round's c_old initial entries (from start) that are <= to,
// stopping at the first that is not; the entries this round appended before
// it (run r1) follow them.  Exactly min(count, freed + 1) entries are
// examined, as the reference's loop does.
template <bool ACCT>
__device__ __forceinline__ void free_le(PR &p, uint64_t to, uint32_t c_old, uint32_t fr_old,
                                        const PRun &r1, const PSend &x, Acct<ACCT> &ac) {
  uint32_t fr = fr_old;
  if (fr == c_old) {
    for (uint32_t j = 0; j < r1.n && run_val(r1, j, x.me, x.li) <= to; j++) fr++;
  }
  ac.add(p.count > 0, x.eb * (fr + 1 < p.count ? fr + 1 : p.count));
  if (fr > 0) {
    p.count -= fr;
    uint32_t st2 = p.start + fr;
    while (st2 >= x.F) st2 -= x.F;
    p.start = p.count == 0 ? 0 : st2;
    if (p.count == 0) p.rep = 0;  // empty ring: canonical representation
  }
}

// Initial ring entries <= to, from start: row form (F <= kRingChunk).
__device__ __forceinline__ uint32_t row_prefix_le(const uint32_t (&lo)[kRingChunk],
                                                  const uint32_t (&hi)[kRingChunk], uint32_t F,
                                                  uint32_t start, uint32_t c_old, uint64_t to) {
  // every position compared, the ones past F masked off after (a per-k
  // "k < F" test in the loop is a wave-uniform lane mask per k that hipcc
  // keeps in SGPR pairs -- spilled, and reloaded with v_readlane)
  uint32_t pm = 0;
#pragma unroll
  for (int k = 0; k < kRingChunk; k++) pm |= ent64(hi[k], lo[k]) <= to ? (1u << k) : 0u;
  const uint32_t full = (1u << F) - 1u;
  pm &= full;
  const uint32_t st = start < F ? start : 0u;
  const uint32_t rk = ((pm >> st) | (pm << (F - st))) & full;  // bit k: entry of rank k
  const uint32_t run = __builtin_ctz(~rk);                     // <= F
  return run < c_old ? run : c_old;
}
// The entry at pos as masked ORs: a select chain here is turned into an
// indexed load by the compiler, which would move the whole ring to scratch
__device__ __forceinline__ uint64_t row_at(const uint32_t (&lo)[kRingChunk],
                                           const uint32_t (&hi)[kRingChunk], uint32_t pos) {
  uint32_t l = 0, h = 0;
#pragma unroll
  for (int k = 0; k < kRingChunk; k++) {
    const uint32_t m = 0u - static_cast<uint32_t>(pos == static_cast<uint32_t>(k));
    l |= lo[k] & m;
    h |= hi[k] & m;
  }
  return ent64(h, l);
}
// The same from memory (F > kRingChunk): lo/hi hold the first min(CH,
// c_old) entries from start, decoded with the round's initial
// representation rep.
__device__ __forceinline__ uint32_t mem_prefix_le(const uint32_t (&lo)[kRingChunk],
                                                  const uint32_t (&hi)[kRingChunk], uint32_t npre,
                                                  uint32_t start, uint32_t c_old, uint64_t to,
                                                  uint32_t rep, const PSend &x) {
  uint32_t fr = 0;
  bool go = true;
#pragma unroll
  for (int k = 0; k < kRingChunk; k++) {
    go = go && static_cast<uint32_t>(k) < npre && ent64(hi[k], lo[k]) <= to;
    fr += go ? 1u : 0u;
  }
  if (fr == npre && fr < c_old) {
    uint32_t pos = start + fr;
    while (pos >= x.F) pos -= x.F;
    while (fr < c_old && ring_get_mem(x, rep, true, pos) <= to) {
      fr++;
      if (++pos >= x.F) pos -= x.F;
    }
  }
  return fr;
}

// ---------------------------------------------------------------------------
// k_progress_step: one lane per group, a wave per 64-group tile.  Phase 1
// (MaybeUpdate + maybeCommit over the slots in message order -> the bcast
// set) runs in registers; phase 2 walks the slots, each peer's whole event
// sequence at once, with the next slot's loads issued before this slot's
// work.
//
// Two forms of the slot loop (template P):
// - rolled (P = false; any F, the memory form of the rings): one copy of
//   the per-peer code, loads and stores skipped by wave ballots where no lane
//   needs them, and the next slot's loads retired before the slot's first
//   store (pb_ready);
// - pipelined (P = true; rings in row form, F <= kRingChunk, S <= 9): the
//   loop spelled out over the slots, with a FIXED memory-instruction count
//   per slot -- every load and store issued, lanes that do not need one
//   dropped by an out-of-range offset -- and the ring's low words loaded with
//   the slot's other Progress loads one slot ahead.  hipcc's s_waitcnt
//   bookkeeping then sees the same instruction sequence on every path and
//   waits, at each slot's first use, for exactly that slot's prefetch
//   (vmcnt(N), N = the instructions issued after it: the previous slot's
//   stores and the next slot's loads), where the rolled form's merged paths
//   wait vmcnt(0) at the ring load: S = 5 3.30 -> 2.80 ms, joint 4.14 ->
//   3.68, S = 7 4.74 -> 4.45 ms (profiles/r05/pstep_pipe_ab*.txt); at S = 7
//   the loads run two slots ahead (PF2 below).
// ---------------------------------------------------------------------------
// The ReadIndex queue beyond its word (ABI 7): entry j >= QE_READ_QUEUE of
// group g, context c, at read_ovf[g*cap + c % cap] -- lane `lane` of a tile's
// block [64][cap] (mask-typed); keys likewise in read_keys.  Offsets for the
// tile's descriptors.
template <typename MT>
__device__ __forceinline__ rsrc_t ovf_rsrc(const PArgs &a, uint64_t g0, uint32_t n) {
  return mk_rsrc(static_cast<const MT *>(a.read_ovf) + g0 * a.read_cap, n * a.read_cap * sizeof(MT));
}
__device__ __forceinline__ uint32_t ovf_off(const PArgs &a, uint32_t lane, uint32_t ctx, uint32_t mb) {
  return (lane * a.read_cap + ctx % a.read_cap) * mb;
}
template <typename MT>
__device__ __forceinline__ uint32_t ovf_ld(rsrc_t r, uint32_t off) {
  if constexpr (sizeof(MT) == 1) return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
  else return __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
}
template <typename MT>
__device__ __forceinline__ void ovf_st(uint32_t v, rsrc_t r, uint32_t off) {
  if constexpr (sizeof(MT) == 1) __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(v), r, off, 0, 0);
  else __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(v), r, off, 0, 0);
}
// A lane's own earlier store to the overflow ring must have landed before it
// reads the same entry again (rare paths only: the ring is touched by groups
// with more than QE_READ_QUEUE pending requests).
__device__ __forceinline__ void ovf_fence() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct PB {  // per-peer loads of one slot (the ring is loaded at the slot's turn)
  uint64_t mt, ix, nx, hn, lt;  // mt, ix: from the wave's LDS copy of phase 1's rows
  uint32_t w;                   // the packed per-peer word (QE_PW_*)
  uint32_t rc;                  // the context number a MsgHeartbeatResp carries
  uint32_t rl[kRingChunk];      // pipelined loop: the ring's low words, prefetched
};

// Loads of slot row `row` (= s*stride + tile0): Next and the packed word of
// a peer that may be touched (`ld`, a superset of the lanes the round
// touches), RejectHint/LogTerm of a reject and the context number of a
// heartbeat response (`rcl`).  The byte accounting is done
// by the caller, on the lanes the round actually touches.
// The rolled loop skips each group of loads no lane needs with a wave-level
// branch; the pipelined one issues them all (fixed wait counts).
// The arguments the slot loop reads (a PArgs subset with the same names).
struct SlotArgs {
  uint64_t stride;
  uint32_t F, FP;
  uint64_t *match, *next, *pending;
  uint32_t *pw, *ilo, *ihi;
  uint16_t *infl16;
  const uint64_t *mhint, *mlogterm;
  const uint32_t *read_ctx;
  uint8_t *msg_count;
  uint64_t *msg_index;
};

// The pipelined loop reads the slot's arguments again from the kernarg
// segment in every slot (scalar loads behind an opaque copy of the segment
// pointer, so they are not hoisted): the kernel's ~40 argument pointers and
// the per-slot descriptors exceed the 102 SGPRs, and hipcc otherwise keeps
// the arguments in VGPR lanes and reloads them with v_readlane (VALU, half
// rate) -- 1173 of them in the S = 5 code object, 751 with the reloads.
// joint 5+5 over 6 slots 3.57 -> 3.33 ms, S = 7 4.13 -> 4.08, S = 5 equal
// (profiles/r05/pstep_karg_ab.txt).  The rolled loop keeps the arguments
// (re-reading them there was 12 % slower in round 4).
template <bool P>
__device__ __forceinline__ SlotArgs slot_args(const PArgs &a) {
  if constexpr (P) {
    typedef const PArgs __attribute__((address_space(4))) KA;
    KA *ka = (KA *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    return SlotArgs{ka->stride, ka->F, ka->FP, ka->match, ka->next, ka->pending, ka->pw,
                    ka->ilo, ka->ihi, ka->infl16, ka->mhint, ka->mlogterm, ka->read_ctx,
                    ka->msg_count, ka->msg_index};
  } else {
    return SlotArgs{a.stride, a.F, a.FP, a.match, a.next, a.pending, a.pw, a.ilo, a.ihi,
                    a.infl16, a.mhint, a.mlogterm, a.read_ctx, a.msg_count, a.msg_index};
  }
}

template <bool P, bool RD, bool N16, class A>
__device__ __forceinline__ void pb_load(const A &a, uint64_t row, const uint64_t *l_mix,
                                        uint32_t n, uint32_t lane, bool ld, bool rej,
                                        bool has_ix, bool rcl, PB &b) {
  b.mt = l_mix[lane];
  b.ix = has_ix ? l_mix[64 + lane] : 0;
  if constexpr (P) {  // fixed count: every load issued, unused lanes dropped
    const bool rl = ld;  // (P: row form only)
    if constexpr (N16) {  // ABI 8: the 16-bit form, one 16-byte load
      const u32x4 x0 = bld128(mk_rsrc(a.infl16 + row * QE_RING16_MAX_F, n * 16), rl ? lane * 16 : kOOB);
      b.rl[0] = x0.x, b.rl[1] = x0.y, b.rl[2] = x0.z, b.rl[3] = x0.w;
      b.rl[4] = b.rl[5] = b.rl[6] = b.rl[7] = 0u;
    } else {
      const rsrc_t rr = mk_rsrc(a.ilo + row * a.FP, n * a.FP * 4);
      const uint32_t lb = lane * a.FP * 4;
      const u32x4 x0 = bld128(rr, rl ? lb : kOOB);
      const u32x4 x1 = bld128(rr, (rl && a.FP > 4) ? lb + 16 : kOOB);
      b.rl[0] = x0.x, b.rl[1] = x0.y, b.rl[2] = x0.z, b.rl[3] = x0.w;
      b.rl[4] = x1.x, b.rl[5] = x1.y, b.rl[6] = x1.z, b.rl[7] = x1.w;
    }
    b.nx = bld64(mk_rsrc(a.next + row, n * 8), ld ? lane * 8 : kOOB);
    b.w = bld32(mk_rsrc(a.pw + row, n * 4), ld ? lane * 4 : kOOB);
    b.hn = bld64(mk_rsrc(a.mhint + row, n * 8), rej ? lane * 8 : kOOB);
    b.lt = bld64(mk_rsrc(a.mlogterm + row, n * 8), rej ? lane * 8 : kOOB);
    // (the heartbeat contexts: only in the variant that tracks ReadIndex --
    // elsewhere the value is unused and the load was dead code already)
    if constexpr (RD) b.rc = bld32(opt_rsrc(a.read_ctx, row, n), rcl ? lane * 4 : kOOB);
    else b.rc = 0;
    return;
  }
  if (__builtin_amdgcn_ballot_w64(ld)) {
    b.nx = bld64(mk_rsrc(a.next + row, n * 8), ld ? lane * 8 : kOOB);
    b.w = bld32(mk_rsrc(a.pw + row, n * 4), ld ? lane * 4 : kOOB);
  } else {
    b.nx = 0;
    b.w = 0;
  }
  if (__builtin_amdgcn_ballot_w64(rej)) {
    b.hn = bld64(mk_rsrc(a.mhint + row, n * 8), rej ? lane * 8 : kOOB);
    b.lt = bld64(mk_rsrc(a.mlogterm + row, n * 8), rej ? lane * 8 : kOOB);
  } else {
    b.hn = b.lt = 0;
  }
  if (__builtin_amdgcn_ballot_w64(rcl)) b.rc = bld32(mk_rsrc(a.read_ctx + row, n * 4), rcl ? lane * 4 : kOOB);
  else b.rc = 0;
}

// The next slot's loads have arrived (an empty asm using them: hipcc waits
// for them here).  Called before a slot's first store, on every path: with
// the loads retired there, `cur = nxt` at the loop latch and the first use of
// cur at the loop head need no wait, where hipcc's path-merged bookkeeping
// would otherwise wait vmcnt(0) -- draining the slot's own stores before the
// next slot starts (vmcnt counts stores, in issue order).  S = 7 4.89 ->
// 4.68 ms, joint 4.26 -> 4.07 ms (profiles/r04/pstep_ab.txt).
template <bool P>
__device__ __forceinline__ void pb_ready(const PB &b) {
  if constexpr (P) return;  // pipelined: consumed one slot later, waited exactly
  asm volatile("" ::"v"(b.nx), "v"(b.w), "v"(b.hn), "v"(b.lt), "v"(b.rc));
}

#ifndef QE_PSTEP_WAVES
#define QE_PSTEP_WAVES 3  // min waves per SIMD requested (VGPR budget)
#endif

// WPB waves per block: 4, or 1 for the 16-run table, whose per-wave LDS
// (21 KB at S = 5) would allow one 4-wave block per CU.  P: the pipelined
// slot loop (above; the launcher picks it for row-form rings).  The 16-bit
// form's pipelined loop up to S = 5 without ReadIndex gets 4 waves (128
// VGPRs, 28 spilled at S = 5): 2.485 -> 2.392 ms (profiles/r06/pstep_w4_ab.txt;
// from S = 6 hipcc cannot meet 4 waves, and the 32-bit form spills 143)
template <int S, typename MT, bool MASKED, bool JOINT, int RM, bool ACCT, bool RD,
          int WPB = kBlock / 64, bool P = false, bool N16 = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 64 * WPB),
                          amdgpu_waves_per_eu(S <= 9 ? ((N16 && P && !RD && S <= 5) ? 4 : QE_PSTEP_WAVES)
                                                     : 2))) void
k_progress_step(PArgs a) {
  constexpr int CH = kRingChunk;
  constexpr uint32_t kFull = (1u << S) - 1u;
  // the ReadIndex queue's acks, one word per group: entry j in bits
  // [EW*j, EW*j + EW) (QE_READ_QUEUE entries of the mask type)
  using QT = typename std::conditional<sizeof(MT) == 1, uint32_t, uint64_t>::type;
  constexpr uint32_t EW = 8 * sizeof(MT);
  constexpr uint32_t kRQ = QE_READ_QUEUE;
#ifdef QE_NO_READ_OVF  // A/B knob: without the overflow-ring paths (ABI 5 queue only)
  constexpr bool OVF = false;
#else
  constexpr bool OVF = RD;  // queue entries past the word (ABI 7)
#endif
  // statistics: per-lane counts in 32 bits (a lane sees at most one group
  // per tile), the sums in 64
  uint32_t n_groups = 0, n_adv = 0, n_viol = 0, n_read = 0;
  uint64_t sum_c = 0, csum = 0;
  Acct<ACCT> ac;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave =
      static_cast<uint64_t>(blockIdx.x) * WPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * WPB;
  const uint64_t ntiles = (a.G + 63) / 64;
  const uint32_t F = a.F;
  static_assert(!P || (S <= 9 && !ACCT), "pipelined form: S <= 9, no accounting");
  const bool row_ring = P || F <= CH;  // wave-uniform (P: the launcher checked F <= CH)
  // P: the term-run table of every group comes with round trip 1 (bit 1;
  // not behind a ballot of the rejecting lanes after it, whose merged paths
  // wait for everything issued); m.Index of every tracked slot with it too
  // (bit 0) was slower (profiles/r05/pstep_head_ab.txt: S = 5 2.80 -> 2.86 ms)
  constexpr int HD = P ? 2 : 0;
  const uint32_t o8 = lane * 8;
  // per wave: Match and m.Index of every slot (phase 1's rows, read again in
  // phase 2) and the group's term runs once a slot needs them
  __shared__ uint64_t l_mix[WPB][S][2][64];
  __shared__ uint64_t l_run[WPB][RM][2][64];
  const uint32_t wv = threadIdx.x >> 6;
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    const uint64_t g0 = t * 64;
    const uint32_t n = tile_n(a.G, t);
    const bool live = lane < n;
    uint32_t nr = 0;
    // ---- round trip 1: per group; message type and Match per slot ----
    const uint32_t mi =
        MASKED ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.inc) + g0, n * sizeof(MT)), lane) &
                  kFull)
               : kFull;
    const uint32_t mo =
        JOINT ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.out) + g0, n * sizeof(MT)), lane) &
                 kFull)
              : 0u;
    const uint32_t trk =
        a.tracked ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.tracked) + g0,
                                           n * sizeof(MT)), lane) & kFull)
                  : kFull;
    const uint32_t self = a.self_slot ? bld8(mk_rsrc(a.self_slot + g0, n), lane) : 0xFFu;
    const uint32_t ltr0 = a.transferee ? bld8(mk_rsrc(a.transferee + g0, n), lane) : 0xFFu;
    uint32_t ltr = ltr0;  // r.leadTransferee (MsgTransferLeader rewrites it)
    const uint64_t li = bld64(mk_rsrc(a.last_index + g0, n * 8), o8);
    const uint64_t fi = bld64(mk_rsrc(a.first_index + g0, n * 8), o8);
    const uint64_t ts = bld64(mk_rsrc(a.term_start + g0, n * 8), o8);
    const rsrc_t r_commit = mk_rsrc(a.committed + g0, n * 8);
    const uint64_t c0 = bld64(r_commit, o8);
    const uint64_t snap_ld = a.snap_index ? bld64(mk_rsrc(a.snap_index + g0, n * 8), o8) : 0;
    // ReadIndex queue (ABI 5): entry 0's context number, the pending count
    // (clamped: a count above the capacity is invalid input) and the first
    // QE_READ_QUEUE entries' acks in one word; entries beyond it (ABI 7) in
    // the overflow ring, read only when a response carries their context
    const bool rd = RD && a.read_acks != nullptr;  // RD: the variant that tracks ReadIndex
    uint32_t qh = 0, qn = 0;
    QT q0 = 0;
    if (rd) {
      qn = bld8(mk_rsrc(a.read_count + g0, n), lane);
      qn = qn < a.read_cap ? qn : a.read_cap;
      qh = bld32(mk_rsrc(a.read_head + g0, n * 4), o8 >> 1);
      if constexpr (sizeof(QT) == 4)
        q0 = bld32(mk_rsrc(static_cast<const QT *>(a.read_acks) + g0, n * 4), o8 >> 1);
      else
        q0 = bld64(mk_rsrc(static_cast<const QT *>(a.read_acks) + g0, n * 8), o8);
    }
    // the context of a response when read_ctx is NULL: the newest request
    // pending when the round starts (lastPendingRequestCtx)
    const uint32_t dctx = qn ? qh + qn - 1u : 0u;
    const uint32_t qn0 = qn;
    QT q = q0;
    bool qtouch = false;
    uint32_t nrel = 0;
    ac.add(live, (MASKED ? sizeof(MT) : 0) + (JOINT ? sizeof(MT) : 0) +
                     (a.tracked ? sizeof(MT) : 0) + (a.self_slot ? 1 : 0) +
                     (a.transferee ? 1 : 0) + 32 + (a.snap_index ? 8 : 0) + (rd ? 5 : 0) +
                     ((rd && qn0) ? sizeof(QT) : 0));
    uint64_t m0[S];
    uint32_t ty[S];
    uint64_t ix[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const bool tr = (trk >> s) & 1u;
      m0[s] = bld64(mk_rsrc(a.match + row, n * 8), o8);
      ty[s] = bld8(mk_rsrc(a.mtype + row, n), tr ? lane : kOOB);
      // HEAD1: m.Index of every tracked slot now (used only where the type
      // says MsgAppResp; counted below where it is)
      if constexpr ((HD & 1) != 0) ix[s] = bld64(mk_rsrc(a.mindex + row, n * 8), tr ? o8 : kOOB);
      ac.add(live, 8);
      ac.add(live && tr, 1);
    }
    uint64_t rr0[RM], rr1[RM];  // HEAD1: the term-run table of every group, with round trip 1
    uint32_t rc_all = 0;
    if constexpr ((HD & 2) != 0) {
      rc_all = bld8(opt_rsrc(a.run_count, g0, n), lane);  // (NULL with no log runs)
#pragma unroll
      for (int r = 0; r < RM; r++) {
        const uint64_t rrow = static_cast<uint64_t>(r) * a.stride + g0;
        const uint32_t off = static_cast<uint32_t>(r) < a.R ? o8 : kOOB;
        rr0[r] = bld64(mk_rsrc(a.run_first + rrow, n * 8), off);
        rr1[r] = bld64(mk_rsrc(a.run_term + rrow, n * 8), off);
      }
    }
    // message kinds, 4 bits per slot, for the rolled phase-2 loop (kinds
    // above QE_MSG_UNREACHABLE are "no message")
    uint64_t tys = 0;
    // per-lane slot masks (bit s = slot s), so per-slot conditions below are
    // bit tests, not short-circuit logic the compiler turns into branches
    uint32_t msgm = 0, rejm = 0, appm = 0, hbm = 0;
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint32_t t = ty[s];
      tys |= static_cast<uint64_t>(t <= QE_MSG_TRANSFER_LEADER ? t : 15u) << (4 * s);
      msgm |= (t - 1u <= QE_MSG_TRANSFER_LEADER - 1u ? 1u : 0u) << s;
      rejm |= (t == QE_MSG_APP_RESP_REJECT ? 1u : 0u) << s;
      appm |= (t == QE_MSG_APP_RESP ? 1u : 0u) << s;
      hbm |= (t == QE_MSG_HEARTBEAT_RESP ? 1u : 0u) << s;
    }
    const uint32_t ixm = appm | rejm;  // slots whose message carries m.Index
    // heartbeat responses whose context number is loaded
    const uint32_t rcm = (rd && a.read_ctx) ? (hbm & trk) : 0u;
    // ---- round trip 2: m.Index of every MsgAppResp and slot 0's peer loads ----
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const bool has_ix = ty[s] == QE_MSG_APP_RESP || ty[s] == QE_MSG_APP_RESP_REJECT;
      if constexpr ((HD & 1) == 0) ix[s] = bld64(mk_rsrc(a.mindex + row, n * 8), has_ix ? o8 : kOOB);
      ac.add(has_ix, 8);
      l_mix[wv][s][0][lane] = m0[s];
      l_mix[wv][s][1][lane] = ix[s];
    }
    // the term-run table of every group with a tracked peer's rejection (the
    // only user: findConflictByTerm in phase 2), loaded with round trip 2
    // and staged into LDS at once -- not a round trip of its own
    const bool need_runs = (rejm & trk) != 0;
    if constexpr ((HD & 2) != 0) {
      nr = need_runs ? (rc_all < a.R ? rc_all : a.R) : 0u;
#pragma unroll
      for (int r = 0; r < RM; r++) {
        l_run[wv][r][0][lane] = rr0[r];
        l_run[wv][r][1][lane] = rr1[r];
      }
    } else if (__builtin_amdgcn_ballot_w64(need_runs)) {
      const uint32_t rc = bld8(mk_rsrc(a.run_count + g0, n), need_runs ? lane : kOOB);
      nr = rc < a.R ? rc : a.R;
#pragma unroll
      for (int r = 0; r < RM; r++) {
        const uint64_t rrow = static_cast<uint64_t>(r) * a.stride + g0;
        const uint32_t off = (need_runs && static_cast<uint32_t>(r) < a.R) ? o8 : kOOB;
        l_run[wv][r][0][lane] = bld64(mk_rsrc(a.run_first + rrow, n * 8), off);
        l_run[wv][r][1][lane] = bld64(mk_rsrc(a.run_term + rrow, n * 8), off);
      }
    }
    bool runs_counted = false;  // ACCT: the run table counts once, when first used
    auto ty_of = [&](uint32_t s) -> uint32_t { return static_cast<uint32_t>(tys >> (4 * s)) & 15u; };
    PB cur;
    // PF2: the pipelined loop's loads two slots ahead (Match / m.Index then
    // come from LDS at use).  Measured (profiles/r05/pstep_pf2_ab.txt): S = 7
    // 4.26 -> 4.07 ms; S = 5 and the joint 6 slots unchanged; at S = 8, 9 it
    // spills (16-120 B of scratch at the 168-VGPR budget), so S = 7 only
    constexpr bool PF2 = P && S == 7;
    PB nx1{};  // PF2: slot s+1's loads while slot s runs
    // SKIP: the pipelined loop walks S - 1 slots when one slot is untouched
    // in every group of the tile whatever phase 1 decides (no tracked
    // peer's message, not a bcast target: untracked or the leader's own) --
    // its only output is MsgCount = 0.  The walked slots keep slot order.
    // (the leader's slot in a steady round: profiles/r05/pstep_skip_ab.txt,
    // S = 5 2.54 -> 2.49 ms, S = 7 3.64 -> 3.62, joint 3.22 -> 3.17)
    constexpr bool SKIP = P && S >= 2;
    uint32_t skip = S;  // wave-uniform: the slot not walked (S: none)
    if constexpr (SKIP) {
      uint32_t um = 0;
#pragma unroll
      for (int s = 0; s < S; s++) {
        const bool may = live && ((((trk & msgm) >> s) & 1u) != 0 ||
                                  (((trk >> s) & 1u) != 0 && self != static_cast<uint32_t>(s)));
        um |= __builtin_amdgcn_ballot_w64(may) ? 0u : (1u << s);
      }
      skip = um ? static_cast<uint32_t>(__builtin_ctz(um)) : static_cast<uint32_t>(S);
    }
    // the walked slot after slot s (S and above: none)
    auto after = [&](uint32_t s) -> uint32_t { return s + 1 + (s + 1 == skip ? 1u : 0u); };
    const uint32_t p0 = skip == 0 ? 1u : 0u;
    {  // the first walked slot, before phase 1: every possible event
      const bool ld = (((trk & (msgm | (self != p0 ? (1u << p0) : 0u))) >> p0) & 1u) != 0;
      pb_load<P, RD, N16>(a, static_cast<uint64_t>(p0) * a.stride + g0, &l_mix[wv][p0][0][0], n, lane, ld,
                 ((rejm >> p0) & 1u) != 0, ((ixm >> p0) & 1u) != 0, ((rcm >> p0) & 1u) != 0, cur);
    }
    if constexpr (PF2 && S > 2) {  // and the second
      const uint32_t p1 = after(p0);
      const bool ld = (((trk & (msgm | (self != p1 ? (1u << p1) : 0u))) >> p1) & 1u) != 0;
      pb_load<P, RD, N16>(a, static_cast<uint64_t>(p1) * a.stride + g0, &l_mix[wv][p1][0][0], n, lane, ld,
                 ((rejm >> p1) & 1u) != 0, ((ixm >> p1) & 1u) != 0, ((rcm >> p1) & 1u) != 0, nx1);
    }
    // ---- phase 1: MaybeUpdate + maybeCommit in message order -> bcasts ----
    uint64_t c = c0;
    uint64_t cfirst = 0;  // the commit after the round's first advance
    uint32_t bset = 0, upd = 0;
    {
      uint64_t vals[S];
#pragma unroll
      for (int s = 0; s < S; s++) vals[s] = m0[s];
#pragma unroll
      for (int s = 0; s < S; s++) {
        if (ty[s] == QE_MSG_APP_RESP && vals[s] < ix[s]) {
          vals[s] = ix[s];
          upd |= 1u << s;
          const uint64_t mci = mci_of<S, MASKED, JOINT>(vals, mi, mo);
          if (mci > c && mci >= ts && mci <= li) {
            cfirst = bset ? cfirst : mci;
            c = mci;
            bset |= 1u << s;
          }
        }
      }
    }
    pb_ready<P>(cur);  // (so no wait at the slot loop's head merges in the stores)
    // ---- phase 2: every peer's event sequence ----
    PSend x;
    x.F = F;
    x.me = a.max_ents;
    x.fi = fi;
    x.li = li;
    x.snap = a.snap_index ? snap_ld : fi - 1;
    x.lb = lane * a.FP * 4;
    x.eb = N16 ? 2u : 4u;  // (the accounting's entry width)
    x.row = row_ring;
    uint32_t sent = 0, snapm = 0, tnow = 0;
    // touched: a tracked peer with a message, or a bcast target (every
    // tracked slot but the leader's when some accept advanced the commit);
    // ringm: FreeLE may run for this peer
    const uint32_t selfb = self < static_cast<uint32_t>(S) ? (1u << self) : 0u;
    const uint32_t tchm = trk & (msgm | (bset != 0 ? (kFull & ~selfb) : 0u));
    const uint32_t ringm = tchm & ((appm & upd) | hbm);
    // rolled over the slots (one copy of the per-peer code; the next slot's
    // loads are issued before this slot's work)
    if constexpr (SKIP) {
      if (skip < static_cast<uint32_t>(S)) {
        const SlotArgs sa = slot_args<P>(a);
        bst8(0u, opt_rsrc(sa.msg_count, static_cast<uint64_t>(skip) * sa.stride + g0, n), lane);
      }
    }
    constexpr int kSlotUnroll = P ? S : 1;
#pragma unroll kSlotUnroll
    for (uint32_t s = 0; s < static_cast<uint32_t>(S); s++) {
      if (SKIP && s == skip) continue;  // (wave-uniform)
      const uint32_t s1 = SKIP ? after(s) : s + 1;  // the next walked slots
      const uint32_t s2 = SKIP ? after(s1) : s + 2;
      const SlotArgs sa = slot_args<P>(a);
      const uint64_t row = static_cast<uint64_t>(s) * sa.stride + g0;
      const uint32_t tt = ty_of(s);
      const bool touched = ((tchm >> s) & 1u) != 0;
      PB nxt{};  // (the last slot has no next: zeros)
      if constexpr (PF2) {
        if (s2 < static_cast<uint32_t>(S)) {
          pb_load<P, RD, N16>(sa, static_cast<uint64_t>(s2) * sa.stride + g0, &l_mix[wv][s2][0][0], n, lane,
                     ((tchm >> s2) & 1u) != 0, ((rejm >> s2) & 1u) != 0, ((ixm >> s2) & 1u) != 0,
                     ((rcm >> s2) & 1u) != 0, nxt);
        }
        // Match / m.Index from the wave's LDS rows at use (not held two slots)
        cur.mt = l_mix[wv][s][0][lane];
        cur.ix = ((ixm >> s) & 1u) ? l_mix[wv][s][1][lane] : 0;
      } else if (s1 < static_cast<uint32_t>(S)) {
        pb_load<P, RD, N16>(sa, static_cast<uint64_t>(s1) * sa.stride + g0, &l_mix[wv][s1][0][0], n, lane,
                   ((tchm >> s1) & 1u) != 0, ((rejm >> s1) & 1u) != 0, ((ixm >> s1) & 1u) != 0,
                   ((rcm >> s1) & 1u) != 0, nxt);
      }
      if (!P && !__builtin_amdgcn_ballot_w64(touched)) {
        // no event for this slot in any group of the tile (e.g. the leader's
        // own slot): only the per-peer output
        pb_ready<P>(nxt);
        if (sa.msg_count) bst8(0u, mk_rsrc(sa.msg_count + row, n), lane);
        ac.add(live && sa.msg_count, 1);
        if (s1 < static_cast<uint32_t>(S)) cur = nxt;
        continue;
      }
      ac.add(touched, 12);  // Next + the packed word
      ac.add(touched && tt == QE_MSG_APP_RESP_REJECT, 16);  // RejectHint + LogTerm
      ac.add(touched && ((rcm >> s) & 1u), 4);               // the heartbeat's context
      PR p;
      p.match = cur.mt;
      p.next = cur.nx;
      pr_unpack(p, cur.w);
      p.reset = 0;
      const uint32_t rep0 = p.rep;
      const uint64_t nx_old = cur.nx;  // (the 16-bit form's base as loaded)
      // PendingSnapshot is read only in StateSnapshot (every other state only
      // ever overwrites it)
      const bool need_pd = touched && p.state == QE_PR_SNAPSHOT;
      uint64_t pd0 = 0;
      if (__builtin_amdgcn_ballot_w64(need_pd)) {
        pd0 = bld64(mk_rsrc(sa.pending + row, n * 8), need_pd ? o8 : kOOB);
        if constexpr (P) asm volatile("" ::"v"(pd0));  // (rare path's wait)
        ac.add(need_pd, 8);
      }
      p.pending = pd0;
      {
        const uint64_t rb = (static_cast<uint64_t>(s) * sa.stride + g0) * sa.FP;
        x.rlo = mk_rsrc(sa.ilo + rb, n * sa.FP * 4);
        x.rhi = mk_rsrc(sa.ihi + rb, n * sa.FP * 4);
        if constexpr (N16) x.r16 = mk_rsrc(sa.infl16 + row * QE_RING16_MAX_F, n * 16);
      }
      const bool up = (upd >> s) & 1u;
      const uint32_t c_old = p.count;
      // the peer's ring: row form, the whole ring of a touched peer with live
      // entries (its appends rewrite it whole); memory form, the first
      // entries from start when FreeLE may run (loaded after the Progress
      // arrived, FreeLE continues from memory)
      uint32_t rlo[kRingChunk], rhi[kRingChunk];
      uint32_t npre = 0;
      if (N16) {  // (row form: F <= kRingChunk, host-checked)
        ring_load_n16<P>(x, touched && c_old > 0, rep0, sa.FP, rlo, rhi, P ? cur.rl : nullptr,
                         nx_old);
      } else if (row_ring) {
        ring_load_row<P>(x, touched && c_old > 0, rep0, sa.FP, rlo, rhi, P ? cur.rl : nullptr);
      } else {
#pragma unroll
        for (int k = 0; k < CH; k++) rlo[k] = rhi[k] = 0;
        const bool scan = ((ringm >> s) & 1u) != 0 && p.state == QE_PR_REPLICATE;
        npre = scan ? (c_old < CH ? c_old : CH) : 0u;
        if (__builtin_amdgcn_ballot_w64(npre > 0)) {
#pragma unroll
          for (int k = 0; k < CH; k++) {
            uint32_t pos = p.start + k;
            if (pos >= F) pos -= F;
            if (pos >= F) pos = 0;  // invalid Inflights.start: stay inside the ring
            const uint64_t v = ring_get_mem(x, rep0, static_cast<uint32_t>(k) < npre, pos);
            rlo[k] = static_cast<uint32_t>(v);
            rhi[k] = static_cast<uint32_t>(v >> 32);
          }
        }
      }
      x.count_msgs = 0;
      x.first_index = 0;
      x.snapped = false;
      PRun r1{0, 0, 0}, r2{0, 0, 0};
      // The peer's events in order: k1 bcast sends (from accepts of earlier
      // slots), its own message, that message's sendAppend (k2), the
      // `for maybeSendAppend(from, false) {}` loop (lp), k3 bcast sends (from
      // later slots).
      const bool bcast_target = touched && s != self;
      const uint32_t below = (1u << s) - 1u;
      const uint32_t k1 = bcast_target ? popc(bset & below) : 0u;
      const uint32_t k3 = bcast_target ? popc(bset & ~below & ~(1u << s)) : 0u;
      uint32_t k2 = 0;
      bool lp = false;
      pb_ready<P>(nxt);  // (before the sends: in memory form they append in memory)
      if (__builtin_amdgcn_ballot_w64(k1 > 0)) send_burst<ACCT>(p, true, k1, x, r1, ac);
      // ReadIndex: the entries this slot's heartbeat response releases
      // (readOnly.advance through the acked one); a response for an entry
      // in the overflow ring (ABI 7) is resolved after the handlers
      uint32_t rel = 0;
      bool ovf_hit = false;
      if (touched) {
        if (tt == QE_MSG_APP_RESP_REJECT) {  // raft.go:1109-1236
          p.recent_active = 1;
          uint64_t probe = cur.hn;
          if (cur.lt > 0) {  // the group's term runs (read at most once per tile)
            uint64_t rf[RM], rt[RM];
#pragma unroll
            for (int r = 0; r < RM; r++) {
              rf[r] = l_run[wv][r][0][lane];
              rt[r] = l_run[wv][r][1][lane];
            }
            probe = find_conflict_by_term<RM>(rf, rt, nr, li, probe, cur.lt);
            ac.add(!runs_counted, 1 + 16 * nr);
            runs_counted = true;
          }
          bool decr;  // MaybeDecrTo(m.Index, probe), progress.go:170-193
          if (p.state == QE_PR_REPLICATE) {
            decr = cur.ix > p.match;
            if (decr) p.next = p.match + 1;
          } else {
            decr = (p.next - 1 == cur.ix);
            if (decr) {
              const uint64_t m = cur.ix < probe + 1 ? cur.ix : probe + 1;
              p.next = m > 1 ? m : 1;
              p.probe_sent = 0;
            }
          }
          if (decr && p.state == QE_PR_REPLICATE) pr_become_probe(p);
          k2 = decr ? 1u : 0u;
        } else if (tt == QE_MSG_APP_RESP) {  // raft.go:1237-1282
          p.recent_active = 1;
          const uint64_t idx = cur.ix;
          n_viol += (idx > li);
          const bool old_paused = pr_paused(p, F);
          if (up) {  // MaybeUpdate (progress.go:144-153)
            p.match = idx;
            p.probe_sent = 0;
          }
          if (p.next < idx + 1) p.next = idx + 1;
          if (up) {
            if (p.state == QE_PR_PROBE) {
              pr_become_replicate(p);
            } else if (p.state == QE_PR_SNAPSHOT && p.match >= p.pending) {
              pr_become_probe(p);
              pr_become_replicate(p);
            } else if (p.state == QE_PR_REPLICATE) {
              const uint32_t fo = row_ring ? row_prefix_le(rlo, rhi, F, p.start, c_old, idx)
                                           : mem_prefix_le(rlo, rhi, npre, p.start, c_old, idx, rep0, x);
              free_le<ACCT>(p, idx, c_old, fo, r1, x, ac);
            }
            // bcastAppend of this accept (skips the leader) / sendAppend if
            // it was paused; then the send loop
            k2 = ((bset >> s) & 1u) ? (s != self ? 1u : 0u) : (old_paused ? 1u : 0u);
            lp = true;
            if (s == ltr && p.match == li) tnow |= 1u << s;
          }
        } else if (tt == QE_MSG_HEARTBEAT_RESP) {  // raft.go:1284-1294
          p.recent_active = 1;
          p.probe_sent = 0;
          if (p.state == QE_PR_REPLICATE && p.count == F) {
            // FreeFirstOne = FreeLE(buffer[start])
            uint64_t first;
            if (c_old == 0) first = run_val(r1, 0, x.me, li);
            else if (row_ring) first = row_at(rlo, rhi, p.start < F ? p.start : 0u);
            else first = ent64(rhi[0], rlo[0]);
            const uint32_t fo = row_ring ? row_prefix_le(rlo, rhi, F, p.start, c_old, first)
                                         : mem_prefix_le(rlo, rhi, npre, p.start, c_old, first, rep0, x);
            free_le<ACCT>(p, first, c_old, fo, r1, x, ac);
          }
          k2 = p.match < li ? 1u : 0u;
          // ReadOnlySafe (raft.go:1296-1309): recvAck on the pending request
          // with the response's context (none pending: recvAck returns nil,
          // nothing recorded); once its acks win the vote, readOnly.advance
          // dequeues every request through it (read_only.go:81-112)
          if (rd) {
            const uint32_t cx = sa.read_ctx ? cur.rc : dctx;
            const uint32_t j = cx - qh;
            if (cx != 0 && j < kRQ && j < qn) {
              q |= static_cast<QT>(1u << s) << (EW * j);
              qtouch = true;
              const uint32_t e = static_cast<uint32_t>(q >> (EW * j)) & kFull;
              if (joint_vote(mi, mo, e, e) == kVoteWon) rel = j + 1;
            }
            ovf_hit = OVF && cx != 0 && j >= kRQ && j < qn;  // an entry beyond the word
          }
        } else if (tt == QE_MSG_SNAP_STATUS || tt == QE_MSG_SNAP_STATUS_REJECT) {  // :1310-1331
          if (p.state == QE_PR_SNAPSHOT) {
            if (tt == QE_MSG_SNAP_STATUS_REJECT) p.pending = 0;
            pr_become_probe(p);
            p.probe_sent = 1;
          }
        } else if (tt == QE_MSG_UNREACHABLE) {  // :1332-1338
          if (p.state == QE_PR_REPLICATE) pr_become_probe(p);
        } else if (tt == QE_MSG_TRANSFER_LEADER) {  // :1339-1370
          if ((((mi | mo) >> s) & 1u) != 0) {  // a learner's request is ignored (:1340-1343)
            bool go = true;
            if (ltr < static_cast<uint32_t>(S)) {  // a transfer is in progress
              if (ltr == s) go = false;  // to the same node: ignored (:1347-1350)
              else ltr = 0xFFu;          // abortLeaderTransfer (:1352)
            }
            if (s == self) go = false;  // to the leader itself: ignored (:1355-1358)
            if (go) {
              ltr = s;
              if (p.match == li) tnow |= 1u << s;  // sendTimeoutNow (:1364-1366)
              else k2 = 1;                         // sendAppend (:1368)
            }
          }
        }
      }
      if constexpr (RD) {
        // an ack for an entry past the word: its acks from the overflow ring
        // (a rare, wave-uniform path; the fence orders this lane's earlier
        // ring stores of the round before the load)
        if (OVF && __builtin_amdgcn_ballot_w64(ovf_hit)) {
          ovf_fence();
          const uint32_t ovf_ctx = sa.read_ctx ? cur.rc : dctx;  // (the context of the response)
          const rsrc_t r_ovf = ovf_rsrc<MT>(a, g0, n);
          const uint32_t off = ovf_hit ? ovf_off(a, lane, ovf_ctx, sizeof(MT)) : kOOB;
          const uint32_t e = ovf_ld<MT>(r_ovf, off) | (1u << s);
          const bool won = ovf_hit && joint_vote(mi, mo, e & kFull, e & kFull) == kVoteWon;
          ovf_st<MT>(e, r_ovf, (ovf_hit && !won) ? off : kOOB);
          rel = won ? ovf_ctx - qh + 1u : rel;
          ac.add(ovf_hit, sizeof(MT));
          ac.add(ovf_hit && !won, sizeof(MT));
        }
        if (__builtin_amdgcn_ballot_w64(rel != 0)) {  // readOnly.advance (read_only.go:81-112)
          const uint32_t qn_old = qn;
          if (rel != 0) {
            q = rel >= kRQ ? static_cast<QT>(0) : static_cast<QT>(q >> (EW * rel));
            qh += rel;
            qn -= rel;
            nrel += rel;
            qtouch = true;
          }
          // the entries that move into the word come from the overflow ring
          if (OVF && __builtin_amdgcn_ballot_w64(rel != 0 && qn_old > kRQ)) {
            ovf_fence();
            const rsrc_t r_ovf = ovf_rsrc<MT>(a, g0, n);
#pragma unroll 1
            for (uint32_t pp = 0; pp < kRQ; pp++) {  // (rolled: a rare path, few registers)
              const bool on = rel != 0 && qn_old > kRQ && pp < qn && pp + rel >= kRQ;
              const uint32_t e = ovf_ld<MT>(r_ovf, on ? ovf_off(a, lane, qh + pp, sizeof(MT)) : kOOB);
              if (on) q |= static_cast<QT>(e) << (EW * pp);
              ac.add(on, sizeof(MT));
            }
          }
        }
      }
      // After an accept: its sendAppend (sendIfEmpty), then the loop; the
      // later bcasts follow the loop.  Otherwise the message's sendAppend
      // and the later bcasts are consecutive sendIfEmpty sends: one burst.
      const uint32_t km = lp ? kLoop : k2 + k3;
      if (__builtin_amdgcn_ballot_w64(km > 0)) send_burst<ACCT>(p, lp ? k2 != 0 : true, km, x, r2, ac);
      if (__builtin_amdgcn_ballot_w64(lp && k3 > 0)) send_burst<ACCT>(p, true, lp ? k3 : 0u, x, r2, ac);
      if constexpr (N16) ring_store_n16<P>(p, x, r1, r2, touched, nx_old, sa.FP, rlo, rhi);
      else if (row_ring) ring_store_row<P>(p, x, r1, r2, touched, rep0, c_old, sa.FP, rlo, rhi);
      // ---- stores: the peer's new Progress (unchanged words skipped) ----
      const uint32_t nw = pr_pack(p);
      const bool tw = touched;
      const bool wm = tw && up, wn = tw && p.next != cur.nx;
      // PendingSnapshot is 0 outside StateSnapshot in every reachable state
      // (ResetState clears it on each state change, progress.go:84-89, and
      // only BecomeSnapshot sets it; the ABI requires it of the input): it is
      // written only where its value changes -- a rare path, so the store
      // stays behind its ballot in both loop forms
      const bool wp = tw && p.pending != pd0;
      const bool ww = tw && nw != cur.w;
      // (storing a changed row for every touched lane, whole sectors, made
      // no difference here: profiles/r03/cq_fullrow_ab.txt; in the pipelined
      // loop too, profiles/r05/pstep_full_ab.txt)
      const bool fm = wm, fn = wn, fw = ww;
      // the ring representation bits are not Progress state (not counted)
      const bool wc = touched && ((nw ^ cur.w) & ~QE_PW_RING_MASK) != 0;
      constexpr bool PIPE = P;  // a fixed store count per slot
      if (PIPE || __builtin_amdgcn_ballot_w64(wm))
        bst64(p.match, mk_rsrc(sa.match + row, n * 8), fm ? o8 : kOOB);
      if (PIPE || __builtin_amdgcn_ballot_w64(wn))
        bst64(p.next, mk_rsrc(sa.next + row, n * 8), fn ? o8 : kOOB);
      if (__builtin_amdgcn_ballot_w64(wp))
        bst64(p.pending, mk_rsrc(sa.pending + row, n * 8), wp ? o8 : kOOB);
      if (PIPE || __builtin_amdgcn_ballot_w64(ww))
        bst32(nw, mk_rsrc(sa.pw + row, n * 4), fw ? lane * 4 : kOOB);
      if (PIPE) {  // optional outputs through a descriptor with no records when NULL
        bst8(x.count_msgs, opt_rsrc(sa.msg_count, row, n), lane);
        bst64(x.first_index, opt_rsrc(sa.msg_index, row, n), x.count_msgs ? o8 : kOOB);
      } else {
        if (sa.msg_count) bst8(x.count_msgs, mk_rsrc(sa.msg_count + row, n), lane);  // optional outputs
        if (sa.msg_index && __builtin_amdgcn_ballot_w64(x.count_msgs != 0))
          bst64(x.first_index, mk_rsrc(sa.msg_index + row, n * 8), x.count_msgs ? o8 : kOOB);
      }
      ac.add(wm, 8);
      ac.add(wn, 8);
      ac.add(wp, 8);
      ac.add(wc, 4);
      ac.add(live && sa.msg_count, 1);
      ac.add(x.count_msgs && sa.msg_index, 8);
      sent |= x.count_msgs ? (1u << s) : 0u;
      snapm |= x.snapped ? (1u << s) : 0u;
      if (s1 < static_cast<uint32_t>(S)) {  // a walked slot follows
        if constexpr (PF2) {
          cur = nx1;
          nx1 = nxt;
        } else {
          cur = nxt;
        }
      }
    }
    const uint32_t bc = popc(bset);
    bst64(c, r_commit, c != c0 ? o8 : kOOB);
    // optional outputs: no instruction at all for a NULL one
    if (a.sent) bst_mask<MT>(sent, opt_rsrc(static_cast<const MT *>(a.sent), g0, n), lane);
    if (a.snap) bst_mask<MT>(snapm, opt_rsrc(static_cast<const MT *>(a.snap), g0, n), lane);
    if (a.tnow) bst_mask<MT>(tnow, opt_rsrc(static_cast<const MT *>(a.tnow), g0, n), lane);
    if (a.bcast) bst8(bc, opt_rsrc(static_cast<const uint8_t *>(a.bcast), g0, n), lane);
    if (rd) {
      // the queue word in canonical form (entries past the count 0), stored
      // when a response was recorded on it and it changed; head and count
      // when requests were released
      const QT canon = qn >= kRQ ? q : static_cast<QT>(q & ((static_cast<QT>(1) << (EW * qn)) - 1u));
      const bool wq = qtouch && canon != q0, wr = nrel != 0;
      if (__builtin_amdgcn_ballot_w64(wq)) {
        if constexpr (sizeof(QT) == 4)
          bst32(canon, mk_rsrc(static_cast<QT *>(a.read_acks) + g0, n * 4), wq ? o8 >> 1 : kOOB);
        else
          bst64(canon, mk_rsrc(static_cast<QT *>(a.read_acks) + g0, n * 8), wq ? o8 : kOOB);
      }
      if (__builtin_amdgcn_ballot_w64(wr)) {
        bst32(qh, mk_rsrc(a.read_head + g0, n * 4), wr ? o8 >> 1 : kOOB);
        bst8(qn, mk_rsrc(a.read_count + g0, n), wr ? lane : kOOB);
      }
      ac.add(wq, sizeof(QT));
      ac.add(wr, 5);
    }
    if (a.read_released) bst8(nrel, opt_rsrc(a.read_released, g0, n), lane);
    ac.add(live && a.read_released, 1);
    // committedEntryInCurrentTerm became true: the postponed reads go out
    const bool tc = c != c0 && !(c0 >= ts && c0 <= li);
    if (a.term_commit) bst8(tc ? 1u : 0u, opt_rsrc(a.term_commit, g0, n), lane);
    if (a.term_commit_index && __builtin_amdgcn_ballot_w64(tc))
      bst64(cfirst, mk_rsrc(a.term_commit_index + g0, n * 8), tc ? o8 : kOOB);
    ac.add(live && a.term_commit, 1);
    ac.add(tc && a.term_commit_index, 8);
    const bool wt = a.transferee && ltr != ltr0;
    if (__builtin_amdgcn_ballot_w64(wt)) bst8(ltr, mk_rsrc(a.transferee + g0, n), wt ? lane : kOOB);
    ac.add(wt, 1);
    ac.add(live && c != c0, 8);
    ac.add(live && a.sent, sizeof(MT));
    ac.add(live && a.snap, sizeof(MT));
    ac.add(live && a.tnow, sizeof(MT));
    ac.add(live && a.bcast, 1);
    if (live) {
      const uint64_t gh = (a.goff + g0 + lane) * kPhi;
      n_groups += 1;
      sum_c += c;
      n_adv += (c != c0);
      n_read += nrel;
      csum += mix64(gh ^ c ^ (static_cast<uint64_t>(bc) << 62)) +
                     mix64(gh ^ (static_cast<uint64_t>(sent) << 40) ^ kSentSalt) +
                     (nrel ? mix64(gh ^ kReadSalt ^ (static_cast<uint64_t>(nrel) << 56)) : 0ull) +
                     (tc ? mix64(gh ^ kTermSalt ^ cfirst) : 0ull) +
                     (ltr != ltr0 ? mix64(gh ^ kTransferSalt ^ ltr) : 0ull);
    }
  }
  if (a.stats) {
    const int idx[P_N] = {QE_STAT_GROUPS, QE_STAT_COMMIT_SUM, QE_STAT_COMMIT_ADVANCED,
                          QE_STAT_INVARIANT_VIOLATIONS, QE_STAT_READ_RELEASED,
                          QE_STAT_CHECKSUM};
    uint64_t cnt[P_N];
    cnt[P_GROUPS] = n_groups;
    cnt[P_SUM] = sum_c;
    cnt[P_ADV] = n_adv;
    cnt[P_VIOL] = n_viol;
    cnt[P_READ] = n_read;
    cnt[P_CSUM] = csum;
    block_stats_add<P_N, 64 * WPB>(cnt, idx, a.stats);
  }
  acct_flush<ACCT>(ac, a.acct);
}

// qe_progress_send: raft.sendAppend / maybeSendAppend(to, send_if_empty)
// once for every slot of want[g] (bcastAppend after a proposal,
// raft/raft.go:515-522).  PendingSnapshot is never read (BecomeSnapshot
// only writes it).
//
// Software-pipelined like the stream commit kernel (qe_stream.hpp): a wave
// owns a chunk of up to kSendTPW tiles, the chunk's want masks are staged in
// LDS first (so a tile's Progress loads depend on an LDS read, not on a
// vector load queued behind the previous tile's traffic), and two register
// sets keep tile t+1's Progress loads in flight while tile t sends.
constexpr int kSendTPW = 8;

#ifndef QE_SEND16_ISSUE  // A/B knob: 1 = the 16-bit rings prefetched with the tile
#define QE_SEND16_ISSUE 0
#endif
template <int S, bool N16>
struct SendSet {
  uint64_t fi, li, sn;
  uint64_t nx[S];
  uint32_t pw[S];
  // ABI 8: each wanted peer's 16-bit ring, prefetched with the tile
  // (QE_SEND16_ISSUE; the default loads it one peer ahead in ps_finish)
  u32x4 rg[(N16 && QE_SEND16_ISSUE) ? S : 1];
};

template <int S, bool N16>
__device__ __forceinline__ void ps_issue(const PArgs &a, uint64_t t, uint32_t lane, uint32_t w,
                                         SendSet<S, N16> &x) {
  const uint64_t g0 = t * 64;
  const uint32_t n = tile_n(a.G, t);
  const uint32_t o8 = lane * 8, o4 = lane * 4;
  x.fi = bld64<kNT>(mk_rsrc(a.first_index + g0, n * 8), w ? o8 : kOOB);
  x.li = bld64<kNT>(mk_rsrc(a.last_index + g0, n * 8), w ? o8 : kOOB);
  x.sn = a.snap_index ? bld64<kNT>(mk_rsrc(a.snap_index + g0, n * 8), w ? o8 : kOOB) : 0;
#pragma unroll
  for (int s = 0; s < S; s++) {
    const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
    x.nx[s] = bld64<kNT>(mk_rsrc(a.next + row, n * 8), bit_off(w, s, o8));
    x.pw[s] = bld32<kNT>(mk_rsrc(a.pw + row, n * 4), bit_off(w, s, o4));
    if constexpr (N16 && QE_SEND16_ISSUE)
      x.rg[s] = bld128(mk_rsrc(a.infl16 + row * QE_RING16_MAX_F, n * 16), bit_off(w, s, lane * 16));
  }
}

template <int S, typename MT, bool N16>
__device__ __forceinline__ void ps_finish(const PArgs &a, uint64_t t, uint32_t lane, uint32_t w,
                                          const SendSet<S, N16> &x) {
  const uint64_t g0 = t * 64;
  const uint32_t n = tile_n(a.G, t);
  Acct<false> ac;
  PSend xs;
  xs.F = a.F;
  xs.me = a.max_ents;
  xs.fi = x.fi;
  xs.li = x.li;
  xs.snap = a.snap_index ? x.sn : x.fi - 1;
  xs.lb = lane * a.FP * 4;
  // one maybeSendAppend appends at most one entry: its 32-bit word stored
  // directly at its ring position (one instruction, memory form); in the
  // 16-bit form (ABI 8) the peer's 16-byte ring is rewritten whole, re-based
  // on the new Next (row form)
  xs.row = N16;
  uint32_t sent = 0, snapm = 0;
  // (the default: each wanted peer's ring loaded one peer ahead of its turn)
  auto ring16_ld = [&](int s) -> u32x4 {
    const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
    const bool on = ((w >> s) & 1u) && ((x.pw[s] >> QE_PW_COUNT_SHIFT) & 0xFFu) != 0;
    return bld128(mk_rsrc(a.infl16 + row * QE_RING16_MAX_F, n * 16), on ? lane * 16 : kOOB);
  };
  u32x4 raw_nx = {0, 0, 0, 0};
  if constexpr (N16 && !QE_SEND16_ISSUE) raw_nx = ring16_ld(0);
#pragma unroll
  for (int s = 0; s < S; s++) {
    const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
    const bool on = (w >> s) & 1u;
    u32x4 raw = raw_nx;
    if constexpr (N16 && !QE_SEND16_ISSUE) {
      if (s + 1 < S) raw_nx = ring16_ld(s + 1);
    }
    if constexpr (N16 && QE_SEND16_ISSUE) raw = x.rg[s];
    PR p;
    p.match = 0;
    p.next = x.nx[s];
    pr_unpack(p, x.pw[s]);
    p.pending = 0;
    p.reset = 0;
    {
      const uint64_t rb = (static_cast<uint64_t>(s) * a.stride + g0) * a.FP;
      xs.rlo = mk_rsrc(a.ilo + rb, n * a.FP * 4);
      xs.rhi = mk_rsrc(a.ihi + rb, n * a.FP * 4);
      if constexpr (N16) xs.r16 = mk_rsrc(a.infl16 + (static_cast<uint64_t>(s) * a.stride + g0) * QE_RING16_MAX_F, n * 16);
    }
    xs.count_msgs = 0;
    xs.first_index = 0;
    xs.snapped = false;
    PRun run{0, 0, 0};
    const uint32_t rep_old = p.rep;
    send_burst<false, kNT>(p, a.send_if_empty != 0, on ? 1u : 0u, xs, run, ac);
    if constexpr (N16) ring_append_n16(p, xs, run, on, x.nx[s], rep_old, raw, a.FP);
    const uint32_t nw = pr_pack(p);
    const bool wn = on && p.next != x.nx[s], wp = on && xs.snapped, ww = on && nw != x.pw[s];
    if (__builtin_amdgcn_ballot_w64(wn)) bst64<kNT>(p.next, mk_rsrc(a.next + row, n * 8), wn ? lane * 8 : kOOB);
    if (__builtin_amdgcn_ballot_w64(wp))
      bst64<kNT>(p.pending, mk_rsrc(a.pending + row, n * 8), wp ? lane * 8 : kOOB);
    if (__builtin_amdgcn_ballot_w64(ww)) bst32<kNT>(nw, mk_rsrc(a.pw + row, n * 4), ww ? lane * 4 : kOOB);
    sent |= xs.count_msgs ? (1u << s) : 0u;
    snapm |= xs.snapped ? (1u << s) : 0u;
  }
  bst_mask<MT>(sent, opt_rsrc(static_cast<const MT *>(a.sent), g0, n), lane);
  bst_mask<MT>(snapm, opt_rsrc(static_cast<const MT *>(a.snap), g0, n), lane);
}

#ifndef QE_SEND16_WAVES  // A/B knob: the 16-bit send kernel's wave budget (1 = none)
#define QE_SEND16_WAVES 1
#endif
template <int S, typename MT, bool N16 = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(N16 ? QE_SEND16_WAVES : 1))) void
k_progress_send(PArgs a) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  __shared__ uint32_t lds_w[kBlock / 64][kSendTPW][64];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t ntiles = (a.G + 63) / 64;
  const uint32_t chunk = a.chunk;  // <= kSendTPW (host-checked)
  const uint64_t t0 = (static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + wv) * chunk;
  const uint32_t nt =
      t0 < ntiles ? static_cast<uint32_t>(ntiles - t0 < chunk ? ntiles - t0 : chunk) : 0u;
  if (nt == 0) return;  // no block-level barrier below
  // the chunk's want masks (a tile past the chunk: n = 0, mask 0)
#pragma unroll
  for (int k = 0; k < kSendTPW; k++) {
    const uint64_t t = t0 + k;
    const uint32_t n = static_cast<uint32_t>(k) < nt ? tile_n(a.G, t) : 0u;
    lds_w[wv][k][lane] =
        ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.want) + t * 64, n * sizeof(MT)), lane) &
        kFull;
  }
  // tile k of the chunk, or past the end (no loads, no stores, want 0)
  auto tix = [&](uint32_t k) -> uint64_t { return k < nt ? t0 + k : ntiles; };
  auto want_of = [&](uint32_t k) -> uint32_t { return k < nt ? lds_w[wv][k][lane] : 0u; };
  SendSet<S, N16> xa, xb;
  ps_issue<S, N16>(a, tix(0), lane, want_of(0), xa);
  for (uint32_t k = 0; k < nt; k += 2) {
    ps_issue<S, N16>(a, tix(k + 1), lane, want_of(k + 1), xb);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the sends
    ps_finish<S, MT, N16>(a, tix(k), lane, want_of(k), xa);
    ps_issue<S, N16>(a, tix(k + 2), lane, want_of(k + 2), xa);
    __builtin_amdgcn_sched_barrier(0);
    ps_finish<S, MT, N16>(a, tix(k + 1), lane, want_of(k + 1), xb);
  }
}

// qe_propose (ABI 6): MsgProp on every group's leader (stepLeader,
// raft/raft.go:1019-1076), appendEntry (:621-642) and the bcastAppend that
// follows (:515-522).  One lane per group, a wave per 64-group tile: the
// proposal, the gates (no Progress of its own, a transfer in progress, the
// conf-change refusals against pendingConfIndex / the joint state, the
// uncommitted-size limit), then for the groups that append every slot's
// Match (Committed) and the tracked slots' Next and word in one batch of
// loads, the leader's own MaybeUpdate(lastIndex) and maybeCommit in
// registers, and one sendAppend per other tracked peer (memory-form ring
// append, as qe_progress_send).  Proposals arrive as a batch and a group
// appends once per launch, so a launch is one MsgProp per group.
constexpr uint64_t kPropSalt = 0x9E6C63D0676A9A99ull;

// (the 16-bit form's ring registers would drop it from 4 waves/SIMD to 3:
// its budget is held at 4, 128 VGPRs)
#ifndef QE_PROPOSE16_WAVES  // A/B knob (1 = no budget: 149 VGPRs, 3 waves)
#define QE_PROPOSE16_WAVES 4
#endif
#ifndef QE_PROPOSE16_PF  // A/B knob: 0 = each ring loaded at its peer's turn
#define QE_PROPOSE16_PF 1
#endif
template <int S, typename MT, bool MASKED, bool JOINT, bool ACCT, bool N16 = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(N16 ? QE_PROPOSE16_WAVES : 1))) void
k_propose(PArgs a) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  constexpr uint32_t MB = sizeof(MT);
  uint64_t cnt[Q_N] = {0, 0, 0, 0};
  Acct<ACCT> ac;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
  const uint64_t ntiles = (a.G + 63) / 64;
  const uint64_t maxu = a.max_unc ? a.max_unc : ~0ull;  // 0 = noLimit
  const bool app_only = (a.prop_flags & QE_PROP_APPEND_ONLY) != 0;
  // Loads in three stages per tile, software-pipelined across the wave's
  // tiles so one round trip per tile is exposed: A (the proposal count,
  // lastIndex, committed) and B (the masks, self slot, transferee, payload,
  // conf-change count and uncommitted size of the proposing groups) of tile
  // t+1 are issued during tile t, before any of tile t's stores (vmcnt
  // counts loads and stores in one issue order); C (term start, firstIndex,
  // every slot's Match, Next and word of the groups that pass the MsgProp
  // gates) at the top of tile t.  Size-dropped proposals (decided after C
  // is issued) load C rows they do not use; nothing is counted for them.
  // (1.618 -> 1.602 ms, profiles/r05/propose_pipe_ab.txt: the round trips
  // are not what bounds it; its ring appends write whole sectors, as the
  // send kernel's do)
  struct PA {
    uint32_t ne;
    uint64_t li, c0;
  };
  struct PBk {
    uint32_t trk, self, ltr, mi, mo, ncc;
    uint64_t sz, us;
  };
  auto load_a = [&](uint64_t t, PA &x) {
    const uint32_t n = t < ntiles ? tile_n(a.G, t) : 0u;  // past the end: nothing
    const uint64_t g0 = t * 64;
    x.ne = bld32(mk_rsrc(a.prop_n + g0, n * 4), lane * 4);
    x.li = bld64(mk_rsrc(a.last_index_rw + g0, n * 8), lane * 8);
    x.c0 = bld64(mk_rsrc(a.committed + g0, n * 8), lane * 8);
  };
  auto load_b = [&](uint64_t t, const PA &x, PBk &y) {
    const uint32_t n = t < ntiles ? tile_n(a.G, t) : 0u;
    const uint64_t g0 = t * 64;
    const bool prop = x.ne != 0;
    const uint32_t o1 = prop ? lane : kOOB;
    y.trk = a.tracked ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.tracked) + g0, n * MB), lane) & kFull)
                      : kFull;
    y.self = a.self_slot ? bld8(mk_rsrc(a.self_slot + g0, n), o1) : 0xFFu;
    y.ltr = a.transferee ? bld8(mk_rsrc(a.transferee + g0, n), o1) : 0xFFu;
    y.mi = MASKED ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.inc) + g0, n * MB), lane) & kFull)
                  : kFull;
    y.mo = JOINT ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.out) + g0, n * MB), lane) & kFull)
                 : 0u;
    y.sz = a.prop_payload ? bld64(mk_rsrc(a.prop_payload + g0, n * 8), prop ? lane * 8 : kOOB) : 0;
    y.ncc = a.max_cc ? bld8(mk_rsrc(a.cc_count + g0, n), o1) : 0u;
    y.us = bld64(opt_rsrc(a.unc, g0, n), prop ? lane * 8 : kOOB);
  };
  PA ha;
  PBk hb;
  load_a(wave, ha);
  load_b(wave, ha, hb);
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    const uint64_t g0 = t * 64;
    const uint32_t n = tile_n(a.G, t);
    const bool live = lane < n;
    const uint32_t o8 = lane * 8, o4 = lane * 4;
    const uint32_t ne = ha.ne;
    const bool prop = ne != 0;
    // lastIndex and committed of every group (the checksum covers them)
    const rsrc_t r_li = mk_rsrc(a.last_index_rw + g0, n * 8), r_c = mk_rsrc(a.committed + g0, n * 8);
    uint64_t li = ha.li;
    const uint64_t c0 = ha.c0;
    uint64_t c = c0;
    ac.add(live, 4);
    uint32_t res = QE_PROP_NONE, refused = 0, sentm = 0, snapm = 0;
    const uint32_t trk = hb.trk, self = hb.self, ltr = hb.ltr, mi = hb.mi, mo = hb.mo;
    const bool member = self < static_cast<uint32_t>(S) && ((trk >> self) & 1u) != 0;
    // (appendEntry alone skips the MsgProp gates but needs the leader's
    // Progress: the reference's MaybeUpdate on a missing one panics)
    res = !prop ? QE_PROP_NONE
                : (!member ? QE_PROP_DROPPED_NOT_MEMBER
                           : ((!app_only && ltr < static_cast<uint32_t>(S)) ? QE_PROP_DROPPED_TRANSFER
                                                                            : QE_PROP_OK));
    const bool go = res == QE_PROP_OK;
    // stage C of this tile
    const uint32_t k8 = go ? o8 : kOOB;
    const uint64_t ts = bld64(mk_rsrc(a.term_start + g0, n * 8), k8);
    const uint64_t fi = bld64(mk_rsrc(a.first_index + g0, n * 8), k8);
    const uint64_t sn = a.snap_index ? bld64(mk_rsrc(a.snap_index + g0, n * 8), k8) : fi - 1;
    uint64_t mt[S], nx[S];
    uint32_t pw[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const bool ld = go && ((trk >> s) & 1u) && (!app_only || self == static_cast<uint32_t>(s));
      mt[s] = bld64(mk_rsrc(a.match + row, n * 8), k8);
      nx[s] = bld64(mk_rsrc(a.next + row, n * 8), ld ? o8 : kOOB);
      pw[s] = bld32(mk_rsrc(a.pw + row, n * 4), ld ? o4 : kOOB);
    }
    // this tile's stage-B values the gates below still use (named before the
    // next tile's loads take the struct)
    const uint64_t sz_ld = hb.sz, us = hb.us;
    const uint32_t ncc_ld = hb.ncc;
    // stages A and B of the wave's next tile, before this tile's stores
    load_a(t + nwaves, ha);
    load_b(t + nwaves, ha, hb);
    if (__builtin_amdgcn_ballot_w64(prop)) {
      ac.add(prop, (a.self_slot ? 1 : 0) + (a.tracked ? MB : 0) + (a.transferee ? 1 : 0));
      uint64_t sz = go ? sz_ld : 0;
      ac.add(go, (a.prop_payload ? 8 : 0) + (a.max_cc ? 1 : 0));
      // conf-change entries (:1034-1072): refused ones become empty
      // EntryNormal entries (no payload), an accepted one sets
      // pendingConfIndex to its index
      // a proposal listing more conf-change entries than max_cc is refused
      // whole (QE_PROP_BAD_CC: nothing appended, no state changes), never
      // clamped silently
      const bool bad_cc = go && ncc_ld > a.max_cc;
      res = bad_cc ? QE_PROP_BAD_CC : res;
      const uint32_t ncc = (go && !bad_cc) ? ncc_ld : 0u;
      bool out_counted = false;
      if (__builtin_amdgcn_ballot_w64(ncc > 0)) {
        const bool cl = ncc > 0;
        const rsrc_t r_pci = mk_rsrc(a.pci + g0, n * 8);
        uint64_t pci = bld64(r_pci, cl ? o8 : kOOB);
        const uint64_t pci0 = pci;
        const uint64_t applied = bld64(mk_rsrc(a.applied + g0, n * 8), cl ? o8 : kOOB);
        const bool joint = mo != 0u;  // len(Voters[1]) > 0
        ac.add(cl, (a.out ? MB : 0) + 16);
        out_counted = cl && a.out != nullptr;
        for (uint32_t k = 0; k < a.max_cc; k++) {
          const bool on = k < ncc;
          if (!__builtin_amdgcn_ballot_w64(on)) break;
          const uint64_t row = static_cast<uint64_t>(k) * a.cc_stride + g0;
          const uint32_t pos = bld32(mk_rsrc(a.cc_pos + row, n * 4), on ? o4 : kOOB);
          const bool leave = bld8(mk_rsrc(a.cc_leave + row, n), on ? lane : kOOB) != 0;
          const uint32_t csz = bld32(mk_rsrc(a.cc_size + row, n * 4), on ? o4 : kOOB);
          ac.add(on, 9);
          if (on) {
            const bool pending = pci > applied;  // alreadyPending
            if (pending || (joint && !leave) || (!joint && leave)) {
              refused |= 1u << k;
            } else {
              pci = li + pos + 1;
              sz += csz;
            }
          }
        }
        const bool wpci = cl && pci != pci0;
        bst64(pci, r_pci, wpci ? o8 : kOOB);
        ac.add(wpci, 8);
      }
      // appendEntry -> increaseUncommittedSize (:1761-1779)
      const rsrc_t r_unc = opt_rsrc(a.unc, g0, n);
      ac.add(go && !bad_cc && a.unc, 8);
      const bool drop = go && !bad_cc && us > 0 && sz > 0 && us + sz > maxu;
      res = drop ? QE_PROP_DROPPED_SIZE : res;
      const bool ok = go && !bad_cc && !drop;
      bst64(us + sz, r_unc, (ok && sz) ? o8 : kOOB);
      ac.add(ok && a.unc && sz, 8);
      const uint64_t li2 = li + ne;  // raftLog.append
      bst64(li2, r_li, ok ? o8 : kOOB);
      ac.add(ok, 16 + 8 + 8 + (app_only ? 0 : 8 + (a.snap_index ? 8 : 0)) + (MASKED ? MB : 0) +
                     ((JOINT && !out_counted) ? MB : 0));
      if (__builtin_amdgcn_ballot_w64(ok)) {
        ac.add(ok, 8 * S + 12);  // every Match; the leader's Next + word
        // Progress[r.id].MaybeUpdate(lastIndex) (progress.go:144-153)
        uint64_t sm = 0, sx = 0;
        uint32_t sw = 0;
#pragma unroll
        for (int s = 0; s < S; s++) {
          const bool is = self == static_cast<uint32_t>(s);
          sm = is ? mt[s] : sm;
          sx = is ? nx[s] : sx;
          sw = is ? pw[s] : sw;
        }
        PR ps;
        ps.match = sm;
        ps.next = sx;
        pr_unpack(ps, sw);
        const bool up = sm < li2;
        if (up) {
          ps.match = li2;
          ps.probe_sent = 0;
        }
        if (ps.next < li2 + 1) ps.next = li2 + 1;
        const uint32_t nws = pr_pack(ps);
        // maybeCommit (raft.go:585-588, log.go:325-331)
        uint64_t vals[S];
#pragma unroll
        for (int s = 0; s < S; s++) vals[s] = self == static_cast<uint32_t>(s) ? ps.match : mt[s];
        const uint64_t mci = mci_of<S, MASKED, JOINT>(vals, mi, mo);
        if (ok && mci > c && mci >= ts && mci <= li2) c = mci;
        // bcastAppend: one sendAppend per other tracked peer; the leader's
        // own slot takes its MaybeUpdate in the same row stores
        PSend x;
        x.F = a.F;
        x.me = a.max_ents;
        x.fi = fi;
        x.li = li2;
        x.snap = sn;
        x.lb = lane * a.FP * 4;
        x.eb = N16 ? 2u : 4u;
        x.row = N16;  // the 16-bit form: each target's ring rewritten whole (ABI 8)
        // the 16-bit rings, each loaded one peer ahead of its turn (4
        // registers; all S with stage C would cost a wave per SIMD)
        auto ring16_ld = [&](int s) -> u32x4 {
          const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
          const bool on = ok && ((trk >> s) & 1u) && (!app_only || self == static_cast<uint32_t>(s)) &&
                          ((pw[s] >> QE_PW_COUNT_SHIFT) & 0xFFu) != 0;
          return bld128(mk_rsrc(a.infl16 + row * QE_RING16_MAX_F, n * 16), on ? lane * 16 : kOOB);
        };
        u32x4 raw_nx = {0, 0, 0, 0};
        if constexpr (N16 && QE_PROPOSE16_PF) raw_nx = ring16_ld(0);
#pragma unroll
        for (int s = 0; s < S; s++) {
          const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
          const bool is_self = ok && self == static_cast<uint32_t>(s);
          const bool tgt = ok && !app_only && ((trk >> s) & 1u) && self != static_cast<uint32_t>(s);
          u32x4 raw_cur = raw_nx;
          if constexpr (N16 && QE_PROPOSE16_PF) {
            if (s + 1 < S) raw_nx = ring16_ld(s + 1);
          }
          PR p;
          p.match = mt[s];
          p.next = nx[s];
          pr_unpack(p, pw[s]);
          p.pending = 0;
          p.reset = 0;
          {
            const uint64_t rb = row * a.FP;
            x.rlo = mk_rsrc(a.ilo + rb, n * a.FP * 4);
            x.rhi = mk_rsrc(a.ihi + rb, n * a.FP * 4);
            if constexpr (N16) x.r16 = mk_rsrc(a.infl16 + row * QE_RING16_MAX_F, n * 16);
          }
          x.count_msgs = 0;
          x.first_index = 0;
          x.snapped = false;
          PRun run{0, 0, 0};
          const uint32_t rep_old = p.rep;
          if (__builtin_amdgcn_ballot_w64(tgt)) send_burst<ACCT>(p, true, tgt ? 1u : 0u, x, run, ac);
          // the 16-bit form: a target's ring re-based on its new Next; the
          // leader's own re-based if its MaybeUpdate moved its Next while it
          // held entries (never, from becomeLeader on: nothing is sent to it)
          uint32_t nws_s = nws;
          if constexpr (N16) {
            const bool rl = (tgt || is_self) && p.count > 0;
            const u32x4 raw = QE_PROPOSE16_PF ? raw_cur : bld128(x.r16, rl ? lane * 16 : kOOB);
            PR q = p;
            if (is_self) q = ps;
            ring_append_n16(q, x, run, tgt || is_self, nx[s], rep_old, raw, a.FP);
            if (is_self) nws_s = pr_pack(q);
            else p.rep = q.rep;
          }
          const uint32_t nw = pr_pack(p);
          const bool wn = tgt && p.next != nx[s], ww = tgt && nw != pw[s], wp = tgt && x.snapped;
          const bool sn_ = is_self && ps.next != sx, sw_ = is_self && nws_s != sw;
          if (__builtin_amdgcn_ballot_w64(is_self && up))
            bst64(ps.match, mk_rsrc(a.match + row, n * 8), (is_self && up) ? o8 : kOOB);
          if (__builtin_amdgcn_ballot_w64(wn || sn_))
            bst64(is_self ? ps.next : p.next, mk_rsrc(a.next + row, n * 8), (wn || sn_) ? o8 : kOOB);
          if (__builtin_amdgcn_ballot_w64(ww || sw_))
            bst32(is_self ? nws_s : nw, mk_rsrc(a.pw + row, n * 4), (ww || sw_) ? o4 : kOOB);
          if (__builtin_amdgcn_ballot_w64(wp))
            bst64(p.pending, mk_rsrc(a.pending + row, n * 8), wp ? o8 : kOOB);
          ac.add(tgt, 12);
          ac.add(wn, 8);
          ac.add(tgt && ((nw ^ pw[s]) & ~QE_PW_RING_MASK) != 0, 4);
          ac.add(wp, 8);
          ac.add(is_self && up, 8);
          ac.add(sn_, 8);
          ac.add(is_self && ((nws_s ^ sw) & ~QE_PW_RING_MASK) != 0, 4);
          sentm |= (tgt && x.count_msgs) ? (1u << s) : 0u;
          snapm |= (tgt && x.snapped) ? (1u << s) : 0u;
        }
        bst64(c, r_c, c != c0 ? o8 : kOOB);
        ac.add(c != c0, 8);
        li = ok ? li2 : li;
      }
    }
    bst8(res, mk_rsrc(a.prop_result + g0, n), lane);
    if (a.cc_refused) bst8(refused, mk_rsrc(a.cc_refused + g0, n), lane);
    if (a.sent) bst_mask<MT>(sentm, opt_rsrc(static_cast<const MT *>(a.sent), g0, n), lane);
    if (a.snap) bst_mask<MT>(snapm, opt_rsrc(static_cast<const MT *>(a.snap), g0, n), lane);
    ac.add(live, 1 + (a.cc_refused ? 1 : 0) + (a.sent ? MB : 0) + (a.snap ? MB : 0));
    if (live) {
      const uint64_t gh = (a.goff + g0 + lane) * kPhi;
      cnt[Q_GROUPS] += 1;
      cnt[Q_SUM] += c;
      cnt[Q_ADV] += c != c0;
      cnt[Q_CSUM] += mix64(gh ^ kPropSalt ^ (static_cast<uint64_t>(res) << 60) ^ li) +
                     mix64(gh ^ c ^ (static_cast<uint64_t>(sentm) << 40));
    }
  }
  if (a.stats) {
    const int idx[Q_N] = {QE_STAT_GROUPS, QE_STAT_COMMIT_SUM, QE_STAT_COMMIT_ADVANCED,
                          QE_STAT_CHECKSUM};
    block_stats_add<Q_N, kBlock>(cnt, idx, a.stats);
  }
  acct_flush<ACCT>(ac, a.acct);
}

// qe_switch_config (ABI 7): raft.switchToConfig (raft/raft.go:1651-1700) on
// every group whose configuration was just switched.  One lane per group, a
// wave per 64-group tile, two round trips per tile: A (the switched flag,
// the leader's slot, the tracked / Voters masks, the transferee) of the
// wave's next tile is issued during this tile, before its stores; B (the
// log model, every voter's Match, every tracked slot's Next and word -- the
// probe's targets, a superset of the bcast's) at the top of the tile for the
// groups that get past switchToConfig's early returns.  maybeCommit and its
// term gate in registers, then one maybeSendAppend per target (memory-form
// ring appends, as qe_progress_send).
constexpr uint64_t kSwitchSalt = 0x2545F4914F6CDD1Dull;

#ifndef QE_SWITCH16_WAVES  // A/B knob: the 16-bit switch kernel's wave budget (1 = none)
#define QE_SWITCH16_WAVES 1
#endif
#ifndef QE_SWITCH16_ISSUE  // A/B knob: 1 = the 16-bit rings prefetched with round trip B
#define QE_SWITCH16_ISSUE 0
#endif
template <int S, typename MT, bool MASKED, bool JOINT, bool ACCT, bool N16 = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(N16 ? QE_SWITCH16_WAVES : 1))) void
k_switch_config(PArgs a) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  constexpr uint32_t MB = sizeof(MT);
  uint64_t cnt[Q_N] = {0, 0, 0, 0};
  Acct<ACCT> ac;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
  const uint64_t ntiles = (a.G + 63) / 64;
  struct SA {
    uint32_t sw, self, trk, mi, mo, ltr;
    uint64_t c0;  // committed of every group (the statistics cover it)
  };
  auto load_a = [&](uint64_t t, SA &x) {
    const uint32_t n = t < ntiles ? tile_n(a.G, t) : 0u;  // past the end: nothing
    const uint64_t g0 = t * 64;
    x.sw = a.sw_switched ? bld8(mk_rsrc(a.sw_switched + g0, n), lane) : (lane < n ? 1u : 0u);
    const uint32_t o1 = x.sw ? lane : kOOB;
    x.self = a.self_slot ? bld8(mk_rsrc(a.self_slot + g0, n), o1) : 0xFFu;
    x.trk = a.tracked ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.tracked) + g0, n * MB),
                                       x.sw ? lane : kOOB) & kFull)
                      : kFull;
    x.mi = MASKED ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.inc) + g0, n * MB),
                                   x.sw ? lane : kOOB) & kFull)
                  : kFull;
    x.mo = JOINT ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.out) + g0, n * MB),
                                  x.sw ? lane : kOOB) & kFull)
                 : 0u;
    x.ltr = a.transferee ? bld8(mk_rsrc(a.transferee + g0, n), o1) : 0xFFu;
    x.c0 = bld64(mk_rsrc(a.committed + g0, n * 8), lane * 8);
  };
  SA ha;
  load_a(wave, ha);
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    const uint64_t g0 = t * 64;
    const uint32_t n = tile_n(a.G, t);
    const bool live = lane < n;
    const uint32_t o8 = lane * 8, o4 = lane * 4;
    const SA h = ha;
    const bool sw = live && h.sw != 0;
    ac.add(live, (a.sw_switched ? 1 : 0) + 8);
    ac.add(sw, (a.self_slot ? 1 : 0) + (a.tracked ? MB : 0) + (MASKED ? MB : 0) + (JOINT ? MB : 0) +
                   (a.transferee ? 1 : 0));
    // the early returns (:1663-1680): no Progress of its own, or a learner
    // (tracked, in neither half); no incoming voters
    const bool member = h.self < static_cast<uint32_t>(S) && ((h.trk >> h.self) & 1u) != 0;
    const bool learner = member && (((h.mi | h.mo) >> h.self) & 1u) == 0;
    uint32_t res = !sw ? QE_SW_NONE
                       : ((!member || learner) ? QE_SW_REMOVED : (h.mi == 0 ? QE_SW_NO_VOTERS : QE_SW_PROBE));
    const bool go = res == QE_SW_PROBE;
    // round trip B of this tile
    const uint32_t k8 = go ? o8 : kOOB;
    const rsrc_t r_c = mk_rsrc(a.committed + g0, n * 8);
    const uint64_t c0 = h.c0;
    const uint64_t ts = bld64(mk_rsrc(a.term_start + g0, n * 8), k8);
    const uint64_t li = bld64(mk_rsrc(a.last_index + g0, n * 8), k8);
    const uint64_t fi = bld64(mk_rsrc(a.first_index + g0, n * 8), k8);
    const uint64_t sn = a.snap_index ? bld64(mk_rsrc(a.snap_index + g0, n * 8), k8) : fi - 1;
    const uint32_t vm = h.mi | h.mo;
    uint64_t mt[S], nx[S];
    uint32_t pw[S];
    // ABI 8: the 16-bit rings of the targets, prefetched with round trip B
    // (QE_SWITCH16_ISSUE; the default loads each one target ahead)
    u32x4 rg[(N16 && QE_SWITCH16_ISSUE) ? S : 1];
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const uint32_t tgt = go ? h.trk : 0u;
      mt[s] = bld64(mk_rsrc(a.match + row, n * 8), bit_off(go ? vm : 0u, s, o8));
      nx[s] = bld64(mk_rsrc(a.next + row, n * 8), bit_off(tgt, s, o8));
      pw[s] = bld32(mk_rsrc(a.pw + row, n * 4), bit_off(tgt, s, o4));
      if constexpr (N16 && QE_SWITCH16_ISSUE)
        rg[s] = bld128(mk_rsrc(a.infl16 + row * QE_RING16_MAX_F, n * 16), bit_off(tgt, s, lane * 16));
    }
    // round trip A of the wave's next tile, before this tile's stores
    load_a(t + nwaves, ha);
    uint64_t c = c0;
    uint32_t sentm = 0, snapm = 0, ltr = h.ltr;
    if (__builtin_amdgcn_ballot_w64(go)) {
      ac.add(go, 24 + (a.snap_index ? 8 : 0) + 8 * popc(vm));  // term start, lastIndex,
                                                                // firstIndex, snapshot, Match
      // maybeCommit (raft.go:585-588, log.go:325-331): the new config's
      // CommittedIndex and the term gate
      uint64_t vals[S];
#pragma unroll
      for (int s = 0; s < S; s++) vals[s] = mt[s];
      const uint64_t mci = mci_of<S, MASKED, JOINT>(vals, h.mi, h.mo);
      const bool adv = go && mci > c0 && mci >= ts && mci <= li;
      c = adv ? mci : c0;
      res = adv ? QE_SW_BCAST : res;
      // bcastAppend (sendIfEmpty, not the leader) or the probe of every
      // tracked peer (maybeSendAppend(id, false), the leader included)
      const uint32_t selfb = member ? (1u << h.self) : 0u;
      const uint32_t tg = go ? (adv ? (h.trk & ~selfb) : h.trk) : 0u;
      PSend x;
      x.F = a.F;
      x.me = a.max_ents;
      x.fi = fi;
      x.li = li;
      x.snap = sn;
      x.lb = lane * a.FP * 4;
      x.eb = N16 ? 2u : 4u;
      x.row = N16;  // the 16-bit form: each target's ring rewritten whole (ABI 8)
      auto ring16_ld = [&](int s) -> u32x4 {
        const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
        const bool on = ((tg >> s) & 1u) != 0 && ((pw[s] >> QE_PW_COUNT_SHIFT) & 0xFFu) != 0;
        return bld128(mk_rsrc(a.infl16 + row * QE_RING16_MAX_F, n * 16), on ? lane * 16 : kOOB);
      };
      u32x4 raw_nx = {0, 0, 0, 0};
      if constexpr (N16 && !QE_SWITCH16_ISSUE) raw_nx = ring16_ld(0);
#pragma unroll
      for (int s = 0; s < S; s++) {
        const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
        const bool on = ((tg >> s) & 1u) != 0;
        u32x4 raw = raw_nx;
        if constexpr (N16 && !QE_SWITCH16_ISSUE) {
          if (s + 1 < S) raw_nx = ring16_ld(s + 1);
        }
        if constexpr (N16 && QE_SWITCH16_ISSUE) raw = rg[s];
        PR p;
        p.match = mt[s];
        p.next = nx[s];
        pr_unpack(p, pw[s]);
        p.pending = 0;
        p.reset = 0;
        {
          const uint64_t rb = row * a.FP;
          x.rlo = mk_rsrc(a.ilo + rb, n * a.FP * 4);
          x.rhi = mk_rsrc(a.ihi + rb, n * a.FP * 4);
          if constexpr (N16) x.r16 = mk_rsrc(a.infl16 + row * QE_RING16_MAX_F, n * 16);
        }
        x.count_msgs = 0;
        x.first_index = 0;
        x.snapped = false;
        PRun run{0, 0, 0};
        const uint32_t rep_old = p.rep;
        if (__builtin_amdgcn_ballot_w64(on)) send_burst<ACCT>(p, adv, on ? 1u : 0u, x, run, ac);
        if constexpr (N16) ring_append_n16(p, x, run, on, nx[s], rep_old, raw, a.FP);
        const uint32_t nw = pr_pack(p);
        const bool wn = on && p.next != nx[s], ww = on && nw != pw[s], wp = on && x.snapped;
        if (__builtin_amdgcn_ballot_w64(wn)) bst64(p.next, mk_rsrc(a.next + row, n * 8), wn ? o8 : kOOB);
        if (__builtin_amdgcn_ballot_w64(ww)) bst32(nw, mk_rsrc(a.pw + row, n * 4), ww ? o4 : kOOB);
        if (__builtin_amdgcn_ballot_w64(wp)) bst64(p.pending, mk_rsrc(a.pending + row, n * 8), wp ? o8 : kOOB);
        ac.add(on, 12);
        ac.add(wn, 8);
        ac.add(on && ((nw ^ pw[s]) & ~QE_PW_RING_MASK) != 0, 4);
        ac.add(wp, 8);
        sentm |= (on && x.count_msgs) ? (1u << s) : 0u;
        snapm |= (on && x.snapped) ? (1u << s) : 0u;
      }
      bst64(c, r_c, c != c0 ? o8 : kOOB);
      ac.add(c != c0, 8);
      // abortLeaderTransfer when the transferee is no voter of the new
      // config (:1694-1697)
      const bool abort = go && ltr < static_cast<uint32_t>(S) && ((vm >> ltr) & 1u) == 0;
      if (abort) {
        ltr = 0xFFu;
        res |= QE_SW_TRANSFER_ABORTED;
      }
      if (a.transferee && __builtin_amdgcn_ballot_w64(abort))
        bst8(0xFFu, mk_rsrc(a.transferee + g0, n), abort ? lane : kOOB);
      ac.add(abort, 1);
    }
    bst8(res, mk_rsrc(a.sw_result + g0, n), lane);
    if (a.sent) bst_mask<MT>(sentm, opt_rsrc(static_cast<const MT *>(a.sent), g0, n), lane);
    if (a.snap) bst_mask<MT>(snapm, opt_rsrc(static_cast<const MT *>(a.snap), g0, n), lane);
    ac.add(live, 1 + (a.sent ? MB : 0) + (a.snap ? MB : 0));
    if (live) {
      const uint64_t gh = (a.goff + g0 + lane) * kPhi;
      cnt[Q_GROUPS] += 1;
      cnt[Q_SUM] += c;
      cnt[Q_ADV] += c != c0;
      cnt[Q_CSUM] += mix64(gh ^ kSwitchSalt ^ (static_cast<uint64_t>(res) << 56) ^ c) +
                     mix64(gh ^ kSentSalt ^ (static_cast<uint64_t>(sentm) << 40) ^
                           (static_cast<uint64_t>(snapm) << 20));
    }
  }
  if (a.stats) {
    const int idx[Q_N] = {QE_STAT_GROUPS, QE_STAT_COMMIT_SUM, QE_STAT_COMMIT_ADVANCED,
                          QE_STAT_CHECKSUM};
    block_stats_add<Q_N, kBlock>(cnt, idx, a.stats);
  }
  acct_flush<ACCT>(ac, a.acct);
}

// qe_become_leader (ABI 7): raft.becomeLeader (raft/raft.go:724-759) with the
// reset it starts with (:590-613), the empty entry's appendEntry and, with
// QE_BL_BCAST, stepCandidate's bcastAppend.  One lane per group, a wave per
// tile; reset writes every tracked slot's Progress without reading it (the
// new values are constants of lastIndex), so a group costs its log model,
// one write per Progress field and the probes' sends.
constexpr uint64_t kLeaderSalt = 0x6A09E667BB67AE85ull;

template <int S, typename MT, bool MASKED, bool JOINT>
__global__ __launch_bounds__(kBlock) void k_become_leader(PArgs a) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  constexpr uint32_t MB = sizeof(MT);
  uint64_t cnt[Q_N] = {0, 0, 0, 0};
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
  const uint64_t ntiles = (a.G + 63) / 64;
  const bool bcast = (a.bl_flags & QE_BL_BCAST) != 0;
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    const uint64_t g0 = t * 64;
    const uint32_t n = tile_n(a.G, t);
    const bool live = lane < n;
    const uint32_t o8 = lane * 8, o4 = lane * 4;
    const bool el = a.bl_elected ? bld8(mk_rsrc(a.bl_elected + g0, n), lane) != 0 : live;
    const uint32_t o1 = el ? lane : kOOB;
    const uint32_t self = a.self_slot ? bld8(mk_rsrc(a.self_slot + g0, n), o1) : 0xFFu;
    const uint32_t trk =
        a.tracked ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.tracked) + g0, n * MB), lane) & kFull)
                  : kFull;
    const uint32_t mi = MASKED ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.inc) + g0, n * MB), lane) & kFull)
                               : kFull;
    const uint32_t mo = JOINT ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.out) + g0, n * MB), lane) & kFull)
                              : 0u;
    const rsrc_t r_li = mk_rsrc(a.last_index + g0, n * 8), r_c = mk_rsrc(a.committed + g0, n * 8);
    const uint64_t li = bld64(r_li, el ? o8 : kOOB);
    const uint64_t c0 = bld64(r_c, o8);
    const uint32_t rc = (a.R && a.run_count) ? bld8(mk_rsrc(a.run_count + g0, n), o1) : 0u;
    const bool member = self < static_cast<uint32_t>(S) && ((trk >> self) & 1u) != 0;
    // (a full run table refuses only when a new run is needed; checked
    // against the last run's term below, conservatively here)
    const uint32_t res = !el ? QE_BL_NONE
                             : (!member ? QE_BL_NOT_MEMBER
                                        : ((a.R && rc >= a.R) ? QE_BL_RUNS_FULL : QE_BL_LEADER));
    const bool go = res == QE_BL_LEADER;
    const uint32_t k8 = go ? o8 : kOOB;
    const uint64_t term = bld64(mk_rsrc(a.bl_term + g0, n * 8), k8);
    const uint64_t fi = bld64(mk_rsrc(a.first_index + g0, n * 8), k8);
    const uint64_t sn = a.snap_index ? bld64(mk_rsrc(a.snap_index + g0, n * 8), k8) : fi - 1;
    uint64_t c = c0;
    uint32_t sentm = 0, snapm = 0;
    if (__builtin_amdgcn_ballot_w64(go)) {
      const uint64_t li2 = li + 1;  // the empty entry (appendEntry)
      // the log model enters the term: a run of `term` from lastIndex + 1 --
      // unless the log's last run has that term already (a bootstrap
      // snapshot of the new leader's own term): the term then starts there
      uint64_t ts2 = li2;
      if (a.R) {
        bool same = false;
        for (uint32_t r = 0; r < a.R; r++) {  // the last run, a row per lane
          const bool on = go && rc == r + 1;
          if (!__builtin_amdgcn_ballot_w64(on)) continue;
          const uint64_t row = static_cast<uint64_t>(r) * a.stride + g0;
          const uint64_t f = bld64(mk_rsrc(a.run_first + row, n * 8), on ? o8 : kOOB);
          const uint64_t tt = bld64(mk_rsrc(a.run_term + row, n * 8), on ? o8 : kOOB);
          if (on && tt == term) {
            same = true;
            ts2 = f;
          }
        }
        for (uint32_t r = 0; r < a.R; r++) {
          const bool on = go && !same && rc == r;
          if (!__builtin_amdgcn_ballot_w64(on)) continue;
          const uint64_t row = static_cast<uint64_t>(r) * a.stride + g0;
          bst64(li2, mk_rsrc(a.run_first + row, n * 8), on ? o8 : kOOB);
          bst64(term, mk_rsrc(a.run_term + row, n * 8), on ? o8 : kOOB);
        }
        bst8(rc + 1, mk_rsrc(a.run_count + g0, n), (go && !same) ? lane : kOOB);
      }
      bst64(ts2, mk_rsrc(a.term_start + g0, n * 8), k8);
      bst64(li2, r_li, k8);
      if (a.transferee) bst8(0xFFu, mk_rsrc(a.transferee + g0, n), go ? lane : kOOB);
      if (a.read_acks) {  // newReadOnly: nothing pending, the old numbers never reused
        const uint32_t qn = bld8(mk_rsrc(a.read_count + g0, n), go ? lane : kOOB);
        const uint32_t qh = bld32(mk_rsrc(a.read_head + g0, n * 4), go ? o4 : kOOB);
        const uint32_t q = qn < a.read_cap ? qn : a.read_cap;
        bst32(qh + q, mk_rsrc(a.read_head + g0, n * 4), go ? o4 : kOOB);
        bst8(0u, mk_rsrc(a.read_count + g0, n), go ? lane : kOOB);
      }
      if (a.bl_pci) bst64(li, mk_rsrc(a.bl_pci + g0, n * 8), k8);
      if (a.bl_unc) bst64(0, mk_rsrc(a.bl_unc + g0, n * 8), k8);
      // maybeCommit with the leader's own Match at the empty entry (the
      // others are 0 after reset): a one-voter config commits it
      uint64_t vals[S];
#pragma unroll
      for (int s = 0; s < S; s++) vals[s] = self == static_cast<uint32_t>(s) ? li2 : 0;
      const uint64_t mci = mci_of<S, MASKED, JOINT>(vals, mi, mo);
      if (go && mci > c0 && mci >= ts2 && mci <= li2) c = mci;
      bst64(c, r_c, c != c0 ? o8 : kOOB);
      PSend x;
      x.F = a.F;
      x.me = a.max_ents;
      x.fi = fi;
      x.li = li2;
      x.snap = sn;
      x.lb = lane * a.FP * 4;
      x.row = false;
#pragma unroll
      for (int s = 0; s < S; s++) {
        const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
        const bool tr = go && ((trk >> s) & 1u) != 0;
        const bool is_self = self == static_cast<uint32_t>(s);
        PR p;  // reset: Match 0, Next lastIndex + 1, StateProbe, empty Inflights
        p.match = is_self ? li2 : 0;  // (the leader: lastIndex, then MaybeUpdate(li2))
        p.next = is_self ? li2 + 1 : li + 1;
        p.pending = 0;
        p.reset = 0;
        p.state = is_self ? QE_PR_REPLICATE : QE_PR_PROBE;
        p.probe_sent = p.recent_active = p.start = p.count = 0;
        p.rep = 0;
        const bool tgt = bcast && tr && !is_self;
        if (__builtin_amdgcn_ballot_w64(tgt)) {
          const uint64_t rb = row * a.FP;
          x.rlo = mk_rsrc(a.ilo + rb, n * a.FP * 4);
          x.rhi = mk_rsrc(a.ihi + rb, n * a.FP * 4);
          x.count_msgs = 0;
          x.first_index = 0;
          x.snapped = false;
          PRun run{0, 0, 0};
          Acct<false> ac;
          send_burst<false>(p, true, tgt ? 1u : 0u, x, run, ac);
          sentm |= (tgt && x.count_msgs) ? (1u << s) : 0u;
          snapm |= (tgt && x.snapped) ? (1u << s) : 0u;
        }
        const uint32_t off8 = tr ? o8 : kOOB;
        bst64(p.match, mk_rsrc(a.match + row, n * 8), off8);
        bst64(p.next, mk_rsrc(a.next + row, n * 8), off8);
        bst64(p.pending, mk_rsrc(a.pending + row, n * 8), off8);
        bst32(pr_pack(p), mk_rsrc(a.pw + row, n * 4), tr ? o4 : kOOB);
      }
    }
    bst8(res, mk_rsrc(a.bl_result + g0, n), lane);
    if (a.sent) bst_mask<MT>(sentm, opt_rsrc(static_cast<const MT *>(a.sent), g0, n), lane);
    if (a.snap) bst_mask<MT>(snapm, opt_rsrc(static_cast<const MT *>(a.snap), g0, n), lane);
    if (live) {
      const uint64_t gh = (a.goff + g0 + lane) * kPhi;
      cnt[Q_GROUPS] += 1;
      cnt[Q_SUM] += c;
      cnt[Q_ADV] += c != c0;
      cnt[Q_CSUM] += mix64(gh ^ kLeaderSalt ^ (static_cast<uint64_t>(res) << 56) ^ c) +
                     mix64(gh ^ kSentSalt ^ (static_cast<uint64_t>(sentm) << 40) ^
                           (static_cast<uint64_t>(snapm) << 20));
    }
  }
  if (a.stats) {
    const int idx[Q_N] = {QE_STAT_GROUPS, QE_STAT_COMMIT_SUM, QE_STAT_COMMIT_ADVANCED,
                          QE_STAT_CHECKSUM};
    block_stats_add<Q_N, kBlock>(cnt, idx, a.stats);
  }
}

// qe_heartbeat (ABI 6): MsgBeat -> bcastHeartbeat (raft/raft.go:524-541):
// per group the context of the newest pending ReadIndex request, per peer
// (every tracked slot but the leader's) Commit = min(Match, committed)
// (sendHeartbeat :494-510).  One lane per group, a wave per tile; the Match
// rows of the peers sent to are read, their commit rows written.  Two round
// trips per tile: the masks, committed and queue head, then every Match row
// before the tile's first store.  A wave's next tile's header is issued
// between them (at the default one tile per wave it lies past the end; more
// tiles per wave are slower, profiles/r06/heartbeat_tpw.txt).  Every row is
// touched once per launch: non-temporal loads and stores.
// (0.239 -> 0.225 ms, profiles/r06/heartbeat_ab2.txt)
template <int S, typename MT>
__global__ __launch_bounds__(kBlock) void k_heartbeat(PArgs a) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
  const uint64_t ntiles = (a.G + 63) / 64;
  // a tile's masks, committed and ReadIndex queue head (past the end: zeros)
  struct HB {
    uint32_t trk, self, qn, qh;
    uint64_t c;
  };
  auto load_h = [&](uint64_t t, HB &h) {
    const uint32_t n = t < ntiles ? tile_n(a.G, t) : 0u;
    const uint64_t g0 = t * 64;
    h.trk = a.tracked ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.tracked) + g0, n * sizeof(MT)), lane) &
                         kFull)
                      : kFull;
    h.self = a.self_slot ? bld8<kNT>(mk_rsrc(a.self_slot + g0, n), lane) : 0xFFu;
    h.c = bld64<kNT>(mk_rsrc(a.committed + g0, n * 8), lane * 8);
    h.qn = h.qh = 0;
    if (a.hb_ctx && a.read_acks) {
      h.qn = bld8<kNT>(mk_rsrc(a.read_count + g0, n), lane);
      h.qh = bld32<kNT>(mk_rsrc(a.read_head + g0, n * 4), lane * 4);
    }
  };
  HB h;
  load_h(wave, h);
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    const uint64_t g0 = t * 64;
    const uint32_t n = tile_n(a.G, t);
    const uint32_t o8 = lane * 8;
    const uint32_t selfb = h.self < static_cast<uint32_t>(S) ? (1u << h.self) : 0u;
    const uint32_t to = lane < n ? (h.trk & ~selfb) : 0u;
    const uint64_t c = h.c;
    const uint32_t qn = h.qn, qh = h.qh;
    // every peer's Match row in one round trip, before the tile's first
    // store (a buffer store orders the loads after it: one dependent round
    // trip per slot otherwise)
    uint64_t m[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      m[s] = bld64<kNT>(mk_rsrc(a.match + row, n * 8), bit_off(to, s, o8));
    }
    load_h(t + nwaves, h);  // the wave's next tile, before this tile's stores
    if (a.hb_ctx) {
      const uint32_t q = qn < a.read_cap ? qn : a.read_cap;
      const uint32_t cx = q ? qh + q - 1u : 0u;  // lastPendingRequestCtx
      bst32<kNT>(cx, mk_rsrc(a.hb_ctx + g0, n * 4), lane * 4);
    }
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      bst64<kNT>(m[s] < c ? m[s] : c, mk_rsrc(a.hb_commit + row, n * 8), bit_off(to, s, o8));
    }
    if (a.sent) bst_mask<MT>(to, opt_rsrc(static_cast<const MT *>(a.sent), g0, n), lane);
  }
}

// qe_check_quorum: MsgCheckQuorum (raft/raft.go:997-1018) over the resident
// Progress words.  One lane per group; each wave owns a chunk of up to
// kSendTPW tiles (as qe_progress_send): the chunk's masks (Voters[0] |
// Voters[1] << 16, tracked) are staged in LDS first, so a tile's word loads
// depend on an LDS read, and two register sets keep tile k+1's words in
// flight while tile k is decided and stored.  Only the tracked slots' words
// are loaded, only changed words are stored.
template <int S>
struct CQTile {
  uint32_t mio, trk, self;
  uint32_t w[S];
};

template <int S>
__device__ __forceinline__ void cq_issue(const PArgs &a, uint64_t t, uint32_t lane, uint32_t mio,
                                         uint32_t trk, CQTile<S> &x) {
  const uint64_t g0 = t * 64;
  const uint32_t n = tile_n(a.G, t);
  x.mio = mio;
  x.trk = trk;
  x.self = a.self_slot ? bld8(mk_rsrc(a.self_slot + g0, n), lane) : 0xFFu;
#pragma unroll
  for (int s = 0; s < S; s++)
    x.w[s] = bld32(mk_rsrc(a.pw + static_cast<uint64_t>(s) * a.stride + g0, n * 4),
                   bit_off(trk, s, lane * 4));
}

template <int S, bool JOINT>
__device__ __forceinline__ void cq_finish(const PArgs &a, uint64_t t, uint32_t lane,
                                          const CQTile<S> &x, uint64_t (&cnt)[3]) {
  const uint64_t g0 = t * 64;
  const uint32_t n = tile_n(a.G, t);
  const uint32_t trk = x.trk, mi = x.mio & 0xFFFFu, mo = JOINT ? (x.mio >> 16) : 0u;
  // the leader sees itself active (when it still has a Progress)
  const uint32_t selfb = x.self < static_cast<uint32_t>(S) ? ((1u << x.self) & trk) : 0u;
  uint32_t ra = 0;
#pragma unroll
  for (int s = 0; s < S; s++) ra |= ((x.w[s] >> 3) & 1u) << s;
  ra = (ra & trk) | selfb;
  // QuorumActive: every voter with a Progress votes its RecentActive
  const uint32_t present = (mi | mo) & trk;
  const bool qa = joint_vote(mi, mo, present, ra & present) == kVoteWon;
  // Visit: RecentActive = false for every tracked peer but the leader
#pragma unroll
  for (int s = 0; s < S; s++) {
    const uint32_t nw =
        (x.w[s] & ~QE_PF_RECENT_ACTIVE) | (((selfb >> s) & 1u) ? QE_PF_RECENT_ACTIVE : 0u);
    const bool wr = ((trk >> s) & 1u) && nw != x.w[s];
    // a row some lane changes is stored for every tracked lane (unchanged
    // words rewritten as loaded): whole 64-B sectors instead of the partial
    // ones of changed words only, 0.137 -> 0.120 ms (profiles/r03/cq_fullrow_ab.txt)
#ifdef QE_CQ_CHANGED_ONLY  // A/B knob: store only the changed words
    const bool wf = wr;
#else
    const bool wf = (trk >> s) & 1u;
#endif
    if (__builtin_amdgcn_ballot_w64(wr))
      bst32(nw, mk_rsrc(a.pw + static_cast<uint64_t>(s) * a.stride + g0, n * 4),
            wf ? lane * 4 : kOOB);
  }
  if (a.qactive) bst8(qa ? 1u : 0u, mk_rsrc(a.qactive + g0, n), lane);
  if (lane < n) {
    cnt[0] += 1;
    cnt[1] += qa ? 0u : 1u;
    cnt[2] += mix64(((a.goff + g0 + lane) * kPhi) ^ (static_cast<uint64_t>(ra) << 32) ^
                    (qa ? kQuorumSalt : 0ull));
  }
}

template <int S, typename MT, bool MASKED, bool JOINT>
__global__ __launch_bounds__(kBlock) void k_check_quorum(PArgs a) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  __shared__ uint32_t lds_m[kBlock / 64][kSendTPW][64];
  __shared__ uint32_t lds_t[kBlock / 64][kSendTPW][64];
  uint64_t cnt[3] = {0, 0, 0};
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t ntiles = (a.G + 63) / 64;
  const uint64_t t0 = (static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + wv) * a.chunk;
  const uint32_t nt =
      t0 < ntiles ? static_cast<uint32_t>(ntiles - t0 < a.chunk ? ntiles - t0 : a.chunk) : 0u;
  if (nt > 0) {
    const bool staged = MASKED || a.tracked;
    if (staged) {
      uint32_t mv[kSendTPW], tv[kSendTPW];
#pragma unroll
      for (int k = 0; k < kSendTPW; k++) {
        const uint64_t g0 = (t0 + k) * 64;
        const uint32_t n = static_cast<uint32_t>(k) < nt ? tile_n(a.G, t0 + k) : 0u;
        const uint32_t mi =
            MASKED ? ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.inc) + g0, n * sizeof(MT)), lane)
                   : kFull;
        const uint32_t mo =
            JOINT ? ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.out) + g0, n * sizeof(MT)), lane)
                  : 0u;
        mv[k] = (mi & kFull) | ((mo & kFull) << 16);
        tv[k] = a.tracked ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.tracked) + g0,
                                                   n * sizeof(MT)), lane) & kFull)
                          : kFull;
      }
#pragma unroll
      for (int k = 0; k < kSendTPW; k++) {
        lds_m[wv][k][lane] = mv[k];
        lds_t[wv][k][lane] = tv[k];
      }
    }
    auto tix = [&](uint32_t k) -> uint64_t { return k < nt ? t0 + k : ntiles; };
    auto mio_of = [&](uint32_t k) -> uint32_t {
      return k < nt ? (staged ? lds_m[wv][k][lane] : kFull) : 0u;
    };
    auto trk_of = [&](uint32_t k) -> uint32_t {
      return k < nt ? (staged ? lds_t[wv][k][lane] : kFull) : 0u;
    };
    CQTile<S> xa, xb;
    cq_issue<S>(a, tix(0), lane, mio_of(0), trk_of(0), xa);
    for (uint32_t k = 0; k < nt; k += 2) {
      cq_issue<S>(a, tix(k + 1), lane, mio_of(k + 1), trk_of(k + 1), xb);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the decision
      cq_finish<S, JOINT>(a, tix(k), lane, xa, cnt);
      cq_issue<S>(a, tix(k + 2), lane, mio_of(k + 2), trk_of(k + 2), xa);
      __builtin_amdgcn_sched_barrier(0);
      cq_finish<S, JOINT>(a, tix(k + 1), lane, xb, cnt);
    }
  }
  if (a.stats) {
    const int idx[3] = {QE_STAT_GROUPS, QE_STAT_STEPDOWNS, QE_STAT_CHECKSUM};
    block_stats_add<3, kBlock>(cnt, idx, a.stats);
  }
}

// qe_read_index: MsgReadIndex on the leader (stepLeader, raft/raft.go:
// 1078-1096; sendMsgReadIndexResponse :1827-1843).  One lane per group, a
// wave per 64-group tile; the queue word of a group that queues is rewritten
// whole (entry `count` = the leader's own ack), or (ABI 7) the new entry's
// overflow slot is written when the word is full.  With keys, the pending
// requests' keys are compared first (addRequest's duplicate check, a loop
// over the group's pending entries: rare and short).
template <int S, typename MT, bool MASKED, bool JOINT>
__global__ __launch_bounds__(kBlock) void k_read_index(PArgs a) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  using QT = typename std::conditional<sizeof(MT) == 1, uint32_t, uint64_t>::type;
  constexpr uint32_t EW = 8 * sizeof(MT);
  constexpr uint32_t kRQ = QE_READ_QUEUE;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
  const uint64_t ntiles = (a.G + 63) / 64;
  const uint32_t cap = a.read_cap;
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    const uint64_t g0 = t * 64;
    const uint32_t n = tile_n(a.G, t);
    const uint32_t o8 = lane * 8, o4 = lane * 4;
    const bool req = bld8(mk_rsrc(a.ri_request + g0, n), lane) != 0;
    uint32_t res = QE_RI_NONE, ctx = 0;
    uint64_t c = 0;
    if (__builtin_amdgcn_ballot_w64(req)) {
      const uint32_t mi =
          MASKED ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.inc) + g0, n * sizeof(MT)), lane) &
                    kFull)
                 : kFull;
      const uint32_t mo =
          JOINT ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.out) + g0, n * sizeof(MT)), lane) &
                   kFull)
                : 0u;
      const uint32_t ro = req ? o8 : kOOB;
      c = bld64(mk_rsrc(a.committed + g0, n * 8), ro);
      const uint64_t ts = bld64(mk_rsrc(a.term_start + g0, n * 8), ro);
      const uint64_t li = bld64(mk_rsrc(a.last_index + g0, n * 8), ro);
      const bool single = popc(mi) == 1 && mo == 0;  // ProgressTracker.IsSingleton
      const bool in_term = c >= ts && c <= li;       // committedEntryInCurrentTerm
      res = single ? QE_RI_RESPOND
                   : (!in_term ? QE_RI_POSTPONED : (a.lease_based ? QE_RI_RESPOND : QE_RI_QUEUED));
      res = req ? res : QE_RI_NONE;
      const bool qd = res == QE_RI_QUEUED;  // ReadOnlySafe: addRequest + recvAck(r.id)
      if (__builtin_amdgcn_ballot_w64(qd)) {
        const uint32_t qo = qd ? o4 : kOOB;
        uint32_t qn = bld8(mk_rsrc(a.read_count + g0, n), qd ? lane : kOOB);
        uint32_t qh = bld32(mk_rsrc(a.read_head + g0, n * 4), qo);
        QT q;
        if constexpr (sizeof(QT) == 4)
          q = bld32(mk_rsrc(static_cast<const QT *>(a.read_acks) + g0, n * 4), qo);
        else
          q = bld64(mk_rsrc(static_cast<const QT *>(a.read_acks) + g0, n * 8), qd ? o8 : kOOB);
        const uint64_t key = a.ri_key ? bld64(mk_rsrc(a.ri_key + g0, n * 8), qd ? o8 : kOOB) : 0;
        qn = qn < cap ? qn : cap;  // (a count above the capacity is invalid input)
        // an empty queue starts over at context 1 when its head is 0 (a
        // fresh state, or numbers that wrapped exactly)
        if (qn == 0 && qh == 0) qh = 1;
        // addRequest's duplicate check (read_only.go:57-60)
        bool dup = false;
        const rsrc_t r_key = a.ri_key ? mk_rsrc(a.read_keys + g0 * cap, n * cap * 8) : mk_rsrc(nullptr, 0);
        for (uint32_t j = 0; __builtin_amdgcn_ballot_w64(a.ri_key && qd && !dup && j < qn); j++) {
          const bool on = a.ri_key && qd && !dup && j < qn;
          const uint64_t kj = bld64(r_key, on ? (lane * cap + (qh + j) % cap) * 8 : kOOB);
          if (on && kj == key) {
            dup = true;
            ctx = qh + j;
          }
        }
        res = (qd && dup) ? QE_RI_DUPLICATE : res;
        const bool full = qn >= cap || qh + qn == 0u;
        res = (qd && !dup && full) ? QE_RI_FULL : res;
        const bool add = qd && !dup && !full;
        const uint32_t self = a.self_slot ? bld8(mk_rsrc(a.self_slot + g0, n), add ? lane : kOOB) : 0xFFu;
        const uint32_t selfb = self < static_cast<uint32_t>(S) ? (1u << self) : 0u;
        if (add) ctx = qh + qn;
        const bool in_word = qn < kRQ;
        // entries past the count are dead: the word is rewritten canonical
        const QT live = qn >= kRQ ? q : static_cast<QT>(q & ((static_cast<QT>(1) << (EW * qn)) - 1u));
        const QT nq = static_cast<QT>(live | (static_cast<QT>(selfb) << (EW * (in_word ? qn : 0u))));
        if (__builtin_amdgcn_ballot_w64(add)) {
          const bool ww = add && in_word;
          if constexpr (sizeof(QT) == 4)
            bst32(nq, mk_rsrc(static_cast<QT *>(a.read_acks) + g0, n * 4), ww ? o4 : kOOB);
          else
            bst64(nq, mk_rsrc(static_cast<QT *>(a.read_acks) + g0, n * 8), ww ? o8 : kOOB);
          if (__builtin_amdgcn_ballot_w64(add && !in_word))  // ABI 7: the overflow ring
            ovf_st<MT>(selfb, ovf_rsrc<MT>(a, g0, n), (add && !in_word) ? ovf_off(a, lane, ctx, sizeof(MT)) : kOOB);
          if (a.ri_key) bst64(key, r_key, add ? (lane * cap + ctx % cap) * 8 : kOOB);
          bst32(qh, mk_rsrc(a.read_head + g0, n * 4), add ? o4 : kOOB);
          bst8(qn + 1, mk_rsrc(a.read_count + g0, n), add ? lane : kOOB);
        }
      }
    }
    bst8(res, mk_rsrc(a.ri_result + g0, n), lane);
    const bool wc = res == QE_RI_QUEUED || res == QE_RI_DUPLICATE;
    if (a.ri_ctx && __builtin_amdgcn_ballot_w64(wc))
      bst32(ctx, mk_rsrc(a.ri_ctx + g0, n * 4), wc ? o4 : kOOB);
    const bool wi = res == QE_RI_RESPOND || res == QE_RI_QUEUED;
    if (a.ri_index && __builtin_amdgcn_ballot_w64(wi))
      bst64(c, mk_rsrc(a.ri_index + g0, n * 8), wi ? o8 : kOOB);
  }
}

}  // namespace qe
