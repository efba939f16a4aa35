// qe_progress.hpp — qe_progress_step: the leader-side Progress state machine
// (stepLeader, raft/raft.go:1099-1338) with the sends it triggers executed
// where the reference executes them.  One group per lane, tiles of 64 groups.
//
// Every access goes through a per-tile buffer descriptor (wave-uniform base,
// 32-bit lane offset, num_records clipping the ragged last tile), as in the
// stream commit/vote kernel (qe_stream.hpp): a conditional access is an
// unconditional load or store whose offset is pushed out of range when its
// condition is false (no traffic, no branch, loads return 0).  Accesses that
// are rare for a whole wave (PendingSnapshot of Snapshot-state peers, the
// Inflights scan, the term-run table) sit behind real branches, so a wave
// with no such peer skips them and waits for nothing.
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
// The per-peer loads are software-pipelined: slot s+1's Progress loads are
// issued before slot s's Inflights loads.
#pragma once
#include "qe_stream.hpp"

namespace qe {

#ifndef QE_RING_CHUNK
#define QE_RING_CHUNK 8
#endif
constexpr int kRingChunk = QE_RING_CHUNK;

__device__ __forceinline__ uint64_t bld64(rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ uint32_t bld8(rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
}
__device__ __forceinline__ void bst64(uint64_t v, rsrc_t r, uint32_t off) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 0);
}
__device__ __forceinline__ void bst8(uint32_t v, rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(v), r, off, 0, 0);
}
template <typename MT>
__device__ __forceinline__ void bst_mask(uint32_t v, rsrc_t r, uint32_t lane) {
  if constexpr (sizeof(MT) == 1)
    __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(v), r, lane, 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(v), r, lane * 2, 0, 0);
}

// Byte accounting of the instrumented variant (ACCT): the bytes of every
// access the kernel requests (offset in range), i.e. the algorithmic bytes
// of the round at field granularity.
template <bool ACCT>
struct Acct {
  uint64_t b = 0;
  __device__ __forceinline__ void add(bool on, uint32_t bytes) {
    if constexpr (ACCT) b += on ? bytes : 0u;
  }
};

struct PB {  // per-peer loads of one slot
  uint64_t mt, ix, nx, hn, lt;  // mt, ix: re-read (L2-resident since round trips 1-2)
  uint32_t fl, st, ct;
  uint64_t rw[kRingChunk];  // the whole Inflights row when F <= kRingChunk
};

// Loads of slot row `row` (= s*stride + tile0): the Progress fields of a
// touched peer, RejectHint/LogTerm of a reject, and (F <= kRingChunk) the
// peer's whole Inflights row when FreeLE may run -- its position within the
// row (start) is not needed to issue the loads, so they go out together.
template <bool ACCT>
__device__ __forceinline__ void pb_load(const PArgs &a, uint64_t row, uint32_t n, uint32_t lane,
                                        bool touched, bool rej, bool has_ix, bool ring, PB &b,
                                        Acct<ACCT> &ac) {
  constexpr int CH = kRingChunk;
  const uint32_t o8 = touched ? lane * 8 : kOOB, o1 = touched ? lane : kOOB;
  b.mt = bld64(mk_rsrc(a.match + row, n * 8), o8);
  b.ix = bld64(mk_rsrc(a.mindex + row, n * 8), has_ix ? lane * 8 : kOOB);
  b.nx = bld64(mk_rsrc(a.next + row, n * 8), o8);
  b.fl = bld8(mk_rsrc(a.flags + row, n), o1);
  b.st = bld8(mk_rsrc(a.istart + row, n), o1);
  b.ct = bld8(mk_rsrc(a.icount + row, n), o1);
  b.hn = bld64(mk_rsrc(a.mhint + row, n * 8), rej ? lane * 8 : kOOB);
  b.lt = bld64(mk_rsrc(a.mlogterm + row, n * 8), rej ? lane * 8 : kOOB);
  ac.add(touched, 11);
  ac.add(rej, 16);
  const uint32_t F = a.F;
  if (F <= CH) {
    const rsrc_t r = mk_rsrc(a.ibuf + row * F, n * F * 8);
#pragma unroll
    for (int k = 0; k < CH; k++)
      b.rw[k] = bld64(r, ring && static_cast<uint32_t>(k) < F ? (lane * F + k) * 8 : kOOB);
  } else {
#pragma unroll
    for (int k = 0; k < CH; k++) b.rw[k] = 0;
  }
}

#ifndef QE_PSTEP_WAVES
#define QE_PSTEP_WAVES 3  // min waves per SIMD requested (VGPR budget)
#endif

// One peer's send side: raft.maybeSendAppend (raft/raft.go:432-492).
struct PSend {
  rsrc_t ring;
  uint32_t ring0, F, me;
  uint64_t fi, li, snap;
  uint32_t count_msgs;  // messages sent to this peer this round (saturating)
  uint64_t first_index; // m.Index of the first of them
  bool snapped;
  // Inflights entries this round appended: nadd of them, the first a0, each
  // next one min(lastIndex, previous + me) (OptimisticUpdate moves Next to
  // last+1 and the next MsgApp ends me-1 entries later)
  uint64_t a0;
  uint32_t nadd;
};

// `k` consecutive raft.maybeSendAppend(to, send_if_empty) calls on one peer
// (raft/raft.go:432-492), k = kLoop: `for maybeSendAppend(to, false) {}`.
// Consecutive calls have a closed form: a paused peer gets nothing; with no
// entries (Next > lastIndex) every call sends an empty MsgApp if
// sendIfEmpty, else none; Next < firstIndex: nothing unless sendIfEmpty,
// then one MsgSnap to a recently active peer (BecomeSnapshot pauses it);
// Probe: one MsgApp, ProbeSent pauses it; Replicate: one MsgApp per chunk
// of max_ents entries (OptimisticUpdate + Inflights.Add) until the ring is
// full or Next passes lastIndex, then empty MsgApps for the remaining calls
// if sendIfEmpty.  Straight-line code per lane; the only loop is the
// Inflights append loop (wave-uniform trip count).
constexpr uint32_t kLoop = 0xFFFFFFFFu;

template <bool ACCT>
__device__ __forceinline__ void send_burst(PR &p, bool sei, uint32_t k, PSend &x, Acct<ACCT> &ac) {
  const bool go = k > 0 && !pr_paused(p, x.F);
  const bool empty = p.next > x.li;
  const bool comp = !empty && p.next < x.fi;  // entries() fails with ErrCompacted
  uint64_t idx0 = p.next - 1;
  uint32_t nmsg = (go && empty && sei) ? k : 0u;  // kLoop only comes with sei == false
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
  const uint32_t lim = repl ? (room < k ? room : k) : 0u;
  uint32_t added = 0;
  while (__builtin_amdgcn_ballot_w64(added < lim && p.next <= x.li)) {
    const bool on = added < lim && p.next <= x.li;
    uint64_t last = x.li;
    if (x.me) {
      const uint64_t l = p.next + (x.me - 1);
      if (l >= p.next && l < last) last = l;
    }
    uint32_t pos = p.start + p.count;
    if (pos >= x.F) pos -= x.F;
    if (pos >= x.F) pos = 0;  // invalid Inflights.start: stay inside the row
    bst64(last, x.ring, on ? (x.ring0 + pos) * 8 : kOOB);
    ac.add(on, 8);
    x.a0 = (on && x.nadd == 0) ? last : x.a0;
    x.nadd += on ? 1u : 0u;
    p.next = on ? last + 1 : p.next;
    p.count += on ? 1u : 0u;
    added += on ? 1u : 0u;
  }
  if (repl) {
    nmsg = added;
    if (sei && added < k && p.count < x.F && p.next > x.li) nmsg += k - added;  // empties
  }
  if (nmsg) {
    if (x.count_msgs == 0) x.first_index = idx0;
    const uint32_t c = x.count_msgs + (nmsg < 255u ? nmsg : 255u);
    x.count_msgs = c < 255u ? c : 255u;
  }
}

// Inflights.FreeLE(to) (raft/tracker/inflights.go:87-113) given fr_old, the
// number of this round's c_old initial entries (from start) that are <= to,
// stopping at the first that is not; the entries this round appended follow
// them (closed form, PSend).  Exactly min(count, freed + 1) entries are
// examined, as the reference's loop does.
template <bool ACCT>
__device__ __forceinline__ void free_le(PR &p, uint64_t to, uint32_t c_old, uint32_t fr_old,
                                        const PSend &x, Acct<ACCT> &ac) {
  uint32_t fr = fr_old;
  if (fr == c_old) {
    uint64_t v = x.a0;
    for (uint32_t j = 0; j < x.nadd && v <= to; j++) {
      fr++;
      const uint64_t w = v + x.me;
      v = (x.me == 0 || w < v || w > x.li) ? x.li : w;
      if (x.me == 0) break;  // noLimit: one MsgApp carries every entry
    }
  }
  ac.add(p.count > 0, 8 * (fr + 1 < p.count ? fr + 1 : p.count));
  if (fr > 0) {
    p.count -= fr;
    uint32_t st2 = p.start + fr;
    while (st2 >= x.F) st2 -= x.F;
    p.start = p.count == 0 ? 0 : st2;
  }
}

// Initial ring entries <= to, from start: row-resident form (F <= kRingChunk).
__device__ __forceinline__ uint32_t row_prefix_le(const uint64_t (&rw)[kRingChunk], uint32_t F,
                                                  uint32_t start, uint32_t c_old, uint64_t to) {
  uint32_t pm = 0;
#pragma unroll
  for (int k = 0; k < kRingChunk; k++)
    pm |= (static_cast<uint32_t>(k) < F && rw[k] <= to) ? (1u << k) : 0u;
  const uint32_t full = (1u << F) - 1u;
  const uint32_t st = start < F ? start : 0u;
  const uint32_t rk = ((pm >> st) | (pm << (F - st))) & full;  // bit k: entry of rank k
  const uint32_t run = __builtin_ctz(~rk);                     // <= F
  return run < c_old ? run : c_old;
}
// rw[pos] as masked ORs: a select chain here is turned into an indexed load
// by the compiler, which would move the whole row to scratch memory
__device__ __forceinline__ uint64_t row_at(const uint64_t (&rw)[kRingChunk], uint32_t pos) {
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < kRingChunk; k++)
    v |= rw[k] & (0ull - static_cast<uint64_t>(pos == static_cast<uint32_t>(k)));
  return v;
}
// The same from memory (F > kRingChunk): e[] holds the first min(CH, c_old)
// entries from start, loaded after the peer's Progress arrived.
template <bool ACCT>
__device__ __forceinline__ uint32_t mem_prefix_le(const uint64_t (&e)[kRingChunk], uint32_t npre,
                                                  uint32_t start, uint32_t c_old, uint64_t to,
                                                  const PSend &x) {
  uint32_t fr = 0;
  bool go = true;
#pragma unroll
  for (int k = 0; k < kRingChunk; k++) {
    go = go && static_cast<uint32_t>(k) < npre && e[k] <= to;
    fr += go ? 1u : 0u;
  }
  if (fr == npre && fr < c_old) {
    uint32_t pos = start + fr;
    while (pos >= x.F) pos -= x.F;
    while (fr < c_old && bld64(x.ring, (x.ring0 + pos) * 8) <= to) {
      fr++;
      if (++pos >= x.F) pos -= x.F;
    }
  }
  return fr;
}

template <int S, typename MT, bool MASKED, bool JOINT, int RM, bool ACCT>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kBlock),
                          amdgpu_waves_per_eu(S <= 6 ? QE_PSTEP_WAVES : 1))) void
k_progress_step(PArgs a) {
  constexpr int CH = kRingChunk;
  constexpr uint32_t kFull = (1u << S) - 1u;
  uint64_t cnt[P_N] = {0, 0, 0, 0, 0};
  Acct<ACCT> ac;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave =
      static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) +
      __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
  const uint64_t ntiles = (a.G + 63) / 64;
  const uint32_t F = a.F;
  const bool row_ring = F <= CH;  // wave-uniform
  const uint32_t o8 = lane * 8;
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    const uint64_t g0 = t * 64;
    const uint32_t n = tile_n(a.G, t);
    const bool live = lane < n;
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
    const uint32_t ltr = a.transferee ? bld8(mk_rsrc(a.transferee + g0, n), lane) : 0xFFu;
    const uint64_t li = bld64(mk_rsrc(a.last_index + g0, n * 8), o8);
    const uint64_t fi = bld64(mk_rsrc(a.first_index + g0, n * 8), o8);
    const uint64_t ts = bld64(mk_rsrc(a.term_start + g0, n * 8), o8);
    const rsrc_t r_commit = mk_rsrc(a.committed + g0, n * 8);
    const uint64_t c0 = bld64(r_commit, o8);
    const uint64_t snap_ld = a.snap_index ? bld64(mk_rsrc(a.snap_index + g0, n * 8), o8) : 0;
    const uint32_t rc = bld8(mk_rsrc(a.run_count + g0, n), lane);
    ac.add(live, (MASKED ? sizeof(MT) : 0) + (JOINT ? sizeof(MT) : 0) +
                     (a.tracked ? sizeof(MT) : 0) + (a.self_slot ? 1 : 0) +
                     (a.transferee ? 1 : 0) + 32 + (a.snap_index ? 8 : 0) + 1);
    uint64_t m0[S];
    uint32_t ty[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const bool tr = (trk >> s) & 1u;
      m0[s] = bld64(mk_rsrc(a.match + row, n * 8), o8);
      ty[s] = bld8(mk_rsrc(a.mtype + row, n), tr ? lane : kOOB);
      ac.add(live, 8);
      ac.add(live && tr, 1);
    }
    const uint32_t nr = rc < a.R ? rc : a.R;
    // message kinds, 4 bits per slot, for the rolled phase-2 loop (kinds
    // above QE_MSG_UNREACHABLE are "no message")
    uint64_t tys = 0;
#pragma unroll
    for (int s = 0; s < S; s++)
      tys |= static_cast<uint64_t>(ty[s] <= QE_MSG_UNREACHABLE ? ty[s] : 15u) << (4 * s);
    // ---- round trip 2: m.Index of every MsgAppResp, the term-run table of
    // a group with a reject, and slot 0's peer loads ----
    uint64_t ix[S];
    uint32_t rej_any = 0;
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const bool has_ix = ty[s] == QE_MSG_APP_RESP || ty[s] == QE_MSG_APP_RESP_REJECT;
      ix[s] = bld64(mk_rsrc(a.mindex + row, n * 8), has_ix ? o8 : kOOB);
      ac.add(has_ix, 8);
      rej_any |= ty[s] == QE_MSG_APP_RESP_REJECT ? 1u : 0u;
    }
    uint64_t rf[RM], rt[RM];
#pragma unroll
    for (int r = 0; r < RM; r++) {
      const uint32_t off = (rej_any && static_cast<uint32_t>(r) < nr) ? o8 : kOOB;
      const uint64_t rrow = static_cast<uint64_t>(r) * a.stride + g0;
      rf[r] = bld64(mk_rsrc(a.run_first + rrow, n * 8), off);
      rt[r] = bld64(mk_rsrc(a.run_term + rrow, n * 8), off);
    }
    bool runs_counted = false;  // ACCT: the table counts once, when first used
    auto ty_of = [&](uint32_t s) -> uint32_t { return static_cast<uint32_t>(tys >> (4 * s)) & 15u; };
    auto has_ix_of = [&](uint32_t s) -> bool {
      const uint32_t t = ty_of(s);
      return t == QE_MSG_APP_RESP || t == QE_MSG_APP_RESP_REJECT;
    };
    PB cur;
    {  // slot 0, before phase 1: every possible event
      const uint32_t t0 = ty_of(0);
      const bool msg = t0 >= QE_MSG_APP_RESP && t0 <= QE_MSG_UNREACHABLE;
      const bool ld = (trk & 1u) && (msg || self != 0u);
      pb_load<ACCT>(a, g0, n, lane, ld, t0 == QE_MSG_APP_RESP_REJECT, has_ix_of(0),
                    ld && (t0 == QE_MSG_APP_RESP || t0 == QE_MSG_HEARTBEAT_RESP), cur, ac);
    }
    // ---- phase 1: MaybeUpdate + maybeCommit in message order -> bcasts ----
    uint64_t c = c0;
    uint32_t bset = 0, upd = 0, nbc = 0;
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
            c = mci;
            bset |= 1u << s;
            nbc++;
          }
        }
      }
    }
    // ---- phase 2: every peer's event sequence ----
    PSend x;
    x.F = F;
    x.me = a.max_ents;
    x.fi = fi;
    x.li = li;
    x.snap = a.snap_index ? snap_ld : fi - 1;
    uint32_t sent = 0, snapm = 0, tnow = 0;
    auto touched_of = [&](uint32_t s) -> bool {
      const bool tr = (trk >> s) & 1u;
      const uint32_t t = ty_of(s);
      const bool msg = t >= QE_MSG_APP_RESP && t <= QE_MSG_UNREACHABLE;
      return tr && (msg || (bset != 0 && s != self));
    };
    auto ring_of = [&](uint32_t s) -> bool {  // FreeLE may run for this peer
      const uint32_t t = ty_of(s);
      return touched_of(s) && ((t == QE_MSG_APP_RESP && ((upd >> s) & 1u)) ||
                               t == QE_MSG_HEARTBEAT_RESP);
    };
    // rolled over the slots (one copy of the per-peer code; the next slot's
    // loads are issued before this slot's work)
#pragma unroll 1
    for (uint32_t s = 0; s < static_cast<uint32_t>(S); s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const uint32_t tt = ty_of(s);
      const bool touched = touched_of(s);
      PB nxt;
      if (s + 1 < static_cast<uint32_t>(S))
        pb_load<ACCT>(a, row + a.stride, n, lane, touched_of(s + 1),
                      ty_of(s + 1) == QE_MSG_APP_RESP_REJECT, has_ix_of(s + 1), ring_of(s + 1), nxt,
                      ac);
      PR p;
      p.match = cur.mt;
      p.next = cur.nx;
      p.state = cur.fl & QE_PF_STATE;
      p.probe_sent = (cur.fl & QE_PF_PROBE_SENT) != 0;
      p.recent_active = (cur.fl & QE_PF_RECENT_ACTIVE) != 0;
      p.start = cur.st;
      p.count = cur.ct;
      p.pending = 0;
      p.reset = 0;
      // PendingSnapshot is read only in StateSnapshot (every other state only
      // ever overwrites it)
      const bool need_pd = touched && p.state == QE_PR_SNAPSHOT;
      uint64_t pd0 = 0;
      if (__builtin_amdgcn_ballot_w64(need_pd)) {
        pd0 = bld64(mk_rsrc(a.pending + row, n * 8), need_pd ? o8 : kOOB);
        ac.add(need_pd, 8);
      }
      p.pending = pd0;
      x.ring = mk_rsrc(a.ibuf + row * F, n * F * 8);
      x.ring0 = lane * F;
      const bool up = (upd >> s) & 1u;
      const uint32_t c_old = p.count;
      // F > kRingChunk: cur.rw (unused by that path) takes the first
      // entries from start, loaded after the Progress arrived
      uint64_t e[CH];
#pragma unroll
      for (int k = 0; k < CH; k++) e[k] = 0;
      uint32_t npre = 0;
      if (!row_ring) {
        const bool scan = ring_of(s) && p.state == QE_PR_REPLICATE;
        npre = scan ? (c_old < CH ? c_old : CH) : 0u;
        if (__builtin_amdgcn_ballot_w64(npre > 0)) {
#pragma unroll
          for (int k = 0; k < CH; k++) {
            uint32_t pos = p.start + k;
            if (pos >= F) pos -= F;
            if (pos >= F) pos = 0;  // invalid Inflights.start: stay inside the row
            e[k] = bld64(x.ring, static_cast<uint32_t>(k) < npre ? (x.ring0 + pos) * 8 : kOOB);
          }
        }
      }
      x.count_msgs = 0;
      x.first_index = 0;
      x.snapped = false;
      x.nadd = 0;
      x.a0 = 0;
      // The peer's events in order: k1 bcast sends (from accepts of earlier
      // slots), its own message, that message's sendAppend (k2), the
      // `for maybeSendAppend(from, false) {}` loop (lp), k3 bcast sends (from
      // later slots).
      const bool bcast_target = touched && s != self;
      const uint32_t below = (1u << s) - 1u;
      const uint32_t k1 = bcast_target ? popc(bset & below) : 0u;
      const uint32_t k3 = bcast_target ? popc(bset & ~below & ~(1u << s)) : 0u;
      uint32_t k2 = 0;
      bool lp = false, updated = false;
      send_burst<ACCT>(p, true, k1, x, ac);
      if (touched) {
        if (tt == QE_MSG_APP_RESP_REJECT) {  // raft.go:1109-1236
          p.recent_active = 1;
          uint64_t probe = cur.hn;
          if (cur.lt > 0) {
            probe = find_conflict_by_term<RM>(rf, rt, nr, li, probe, cur.lt);
            ac.add(!runs_counted, 16 * nr);
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
          cnt[P_VIOL] += (idx > li);
          const bool old_paused = pr_paused(p, F);
          if (up) {  // MaybeUpdate (progress.go:144-153)
            p.match = idx;
            updated = true;
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
              const uint32_t fo = row_ring ? row_prefix_le(cur.rw, F, p.start, c_old, idx)
                                           : mem_prefix_le<ACCT>(e, npre, p.start, c_old, idx, x);
              free_le<ACCT>(p, idx, c_old, fo, x, ac);
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
            if (c_old == 0) first = x.a0;
            else if (row_ring) first = row_at(cur.rw, p.start < F ? p.start : 0u);
            else first = e[0];
            const uint32_t fo = row_ring ? row_prefix_le(cur.rw, F, p.start, c_old, first)
                                         : mem_prefix_le<ACCT>(e, npre, p.start, c_old, first, x);
            free_le<ACCT>(p, first, c_old, fo, x, ac);
          }
          k2 = p.match < li ? 1u : 0u;
        } else if (tt == QE_MSG_SNAP_STATUS || tt == QE_MSG_SNAP_STATUS_REJECT) {  // :1310-1331
          if (p.state == QE_PR_SNAPSHOT) {
            if (tt == QE_MSG_SNAP_STATUS_REJECT) p.pending = 0;
            pr_become_probe(p);
            p.probe_sent = 1;
          }
        } else if (tt == QE_MSG_UNREACHABLE) {  // :1332-1338
          if (p.state == QE_PR_REPLICATE) pr_become_probe(p);
        }
      }
      send_burst<ACCT>(p, true, k2, x, ac);
      send_burst<ACCT>(p, false, lp ? kLoop : 0u, x, ac);
      send_burst<ACCT>(p, true, k3, x, ac);
      // ---- stores: the peer's new Progress (unchanged words and bytes skipped) ----
      const uint32_t w8 = touched ? o8 : kOOB, w1 = touched ? lane : kOOB;
      const uint32_t fl = p.state | (p.probe_sent ? QE_PF_PROBE_SENT : 0u) |
                          (p.recent_active ? QE_PF_RECENT_ACTIVE : 0u);
      const bool wm = updated, wn = touched && p.next != cur.nx;
      const bool wp = touched && (p.pending != pd0 || p.reset);
      const bool wf = touched && fl != cur.fl, ws = touched && p.start != cur.st;
      const bool wc = touched && p.count != cur.ct;
      bst64(p.match, mk_rsrc(a.match + row, n * 8), wm ? o8 : kOOB);
      bst64(p.next, mk_rsrc(a.next + row, n * 8), wn ? w8 : kOOB);
      bst64(p.pending, mk_rsrc(a.pending + row, n * 8), wp ? w8 : kOOB);
      bst8(fl, mk_rsrc(a.flags + row, n), wf ? w1 : kOOB);
      bst8(p.start, mk_rsrc(a.istart + row, n), ws ? w1 : kOOB);
      bst8(p.count, mk_rsrc(a.icount + row, n), wc ? w1 : kOOB);
      bst8(x.count_msgs, opt_rsrc(a.msg_count, row, n), lane);
      bst64(x.first_index, opt_rsrc(a.msg_index, row, n), x.count_msgs ? o8 : kOOB);
      ac.add(wm, 8);
      ac.add(wn, 8);
      ac.add(wp, 8);
      ac.add(wf, 1);
      ac.add(ws, 1);
      ac.add(wc, 1);
      ac.add(live && a.msg_count, 1);
      ac.add(x.count_msgs && a.msg_index, 8);
      sent |= x.count_msgs ? (1u << s) : 0u;
      snapm |= x.snapped ? (1u << s) : 0u;
      if (s + 1 < static_cast<uint32_t>(S)) cur = nxt;
    }
    bst64(c, r_commit, c != c0 ? o8 : kOOB);
    const uint32_t bc = nbc;
    bst_mask<MT>(sent, opt_rsrc(static_cast<const MT *>(a.sent), g0, n), lane);
    bst_mask<MT>(snapm, opt_rsrc(static_cast<const MT *>(a.snap), g0, n), lane);
    bst_mask<MT>(tnow, opt_rsrc(static_cast<const MT *>(a.tnow), g0, n), lane);
    bst8(bc, opt_rsrc(static_cast<const uint8_t *>(a.bcast), g0, n), lane);
    ac.add(live && c != c0, 8);
    ac.add(live && a.sent, sizeof(MT));
    ac.add(live && a.snap, sizeof(MT));
    ac.add(live && a.tnow, sizeof(MT));
    ac.add(live && a.bcast, 1);
    if (live) {
      cnt[P_GROUPS] += 1;
      cnt[P_SUM] += c;
      cnt[P_ADV] += (c != c0);
      const uint64_t tag =
          (static_cast<uint64_t>(sent) << 40) | (static_cast<uint64_t>(bc) << 62);
      cnt[P_CSUM] += mix64(((a.goff + g0 + lane) * kPhi) ^ c ^ tag);
    }
  }
  if (a.stats) {
    const int idx[P_N] = {QE_STAT_GROUPS, QE_STAT_COMMIT_SUM, QE_STAT_COMMIT_ADVANCED,
                          QE_STAT_INVARIANT_VIOLATIONS, QE_STAT_CHECKSUM};
    block_stats_add<P_N, kBlock>(cnt, idx, a.stats);
  }
  if constexpr (ACCT) {
    uint64_t b = ac.b;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) b += __shfl_xor(b, d, 64);
    if (lane == 0 && a.acct) atomicAdd(reinterpret_cast<unsigned long long *>(a.acct),
                                       static_cast<unsigned long long>(b));
  }
}

// qe_progress_send: raft.sendAppend / maybeSendAppend(to, send_if_empty)
// once for every slot of want[g] (bcastAppend after a proposal,
// raft/raft.go:515-522).  PendingSnapshot is never read (BecomeSnapshot
// only writes it).
template <int S, typename MT>
__global__ __launch_bounds__(kBlock) void k_progress_send(PArgs a) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  Acct<false> ac;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave =
      static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) +
      __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
  const uint64_t ntiles = (a.G + 63) / 64;
  const uint32_t o8 = lane * 8;
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    const uint64_t g0 = t * 64;
    const uint32_t n = tile_n(a.G, t);
    const uint32_t w =
        ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.want) + g0, n * sizeof(MT)), lane) & kFull;
    PSend x;
    x.F = a.F;
    x.me = a.max_ents;
    x.fi = bld64(mk_rsrc(a.first_index + g0, n * 8), w ? o8 : kOOB);
    x.li = bld64(mk_rsrc(a.last_index + g0, n * 8), w ? o8 : kOOB);
    x.snap = a.snap_index ? bld64(mk_rsrc(a.snap_index + g0, n * 8), w ? o8 : kOOB) : x.fi - 1;
    uint32_t sent = 0, snapm = 0;
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const bool on = (w >> s) & 1u;
      const uint32_t r8 = on ? o8 : kOOB, r1 = on ? lane : kOOB;
      PR p;
      p.match = 0;
      p.next = bld64(mk_rsrc(a.next + row, n * 8), r8);
      const uint32_t fl = bld8(mk_rsrc(a.flags + row, n), r1);
      p.state = fl & QE_PF_STATE;
      p.probe_sent = (fl & QE_PF_PROBE_SENT) != 0;
      p.recent_active = (fl & QE_PF_RECENT_ACTIVE) != 0;
      p.start = bld8(mk_rsrc(a.istart + row, n), r1);
      p.count = bld8(mk_rsrc(a.icount + row, n), r1);
      p.pending = 0;
      p.reset = 0;
      const uint64_t nx0 = p.next;
      const uint32_t st0 = p.start, ct0 = p.count;
      x.ring = mk_rsrc(a.ibuf + row * a.F, n * a.F * 8);
      x.ring0 = lane * a.F;
      x.count_msgs = 0;
      x.snapped = false;
      x.nadd = 0;
      x.a0 = 0;
      send_burst<false>(p, a.send_if_empty != 0, on ? 1u : 0u, x, ac);
      const uint32_t f2 = p.state | (p.probe_sent ? QE_PF_PROBE_SENT : 0u) |
                          (p.recent_active ? QE_PF_RECENT_ACTIVE : 0u);
      bst64(p.next, mk_rsrc(a.next + row, n * 8), on && p.next != nx0 ? o8 : kOOB);
      bst64(p.pending, mk_rsrc(a.pending + row, n * 8), on && x.snapped ? o8 : kOOB);
      bst8(f2, mk_rsrc(a.flags + row, n), on && f2 != fl ? lane : kOOB);
      bst8(p.start, mk_rsrc(a.istart + row, n), on && p.start != st0 ? lane : kOOB);
      bst8(p.count, mk_rsrc(a.icount + row, n), on && p.count != ct0 ? lane : kOOB);
      sent |= x.count_msgs ? (1u << s) : 0u;
      snapm |= x.snapped ? (1u << s) : 0u;
    }
    bst_mask<MT>(sent, opt_rsrc(static_cast<const MT *>(a.sent), g0, n), lane);
    bst_mask<MT>(snapm, opt_rsrc(static_cast<const MT *>(a.snap), g0, n), lane);
  }
}

}  // namespace qe
