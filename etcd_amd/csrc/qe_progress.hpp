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

constexpr int kRingChunk = 8;

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

struct PB {  // per-peer Progress loads of one slot
  uint64_t nx, hn, lt;
  uint32_t fl, st, ct;
};

// Progress loads of slot row `row` (= s*stride + tile0).
template <bool ACCT>
__device__ __forceinline__ void pb_load(const PArgs &a, uint64_t row, uint32_t n, uint32_t lane,
                                        bool touched, bool rej, PB &b, Acct<ACCT> &ac) {
  const uint32_t o8 = touched ? lane * 8 : kOOB, o1 = touched ? lane : kOOB;
  b.nx = bld64(mk_rsrc(a.next + row, n * 8), o8);
  b.fl = bld8(mk_rsrc(a.flags + row, n), o1);
  b.st = bld8(mk_rsrc(a.istart + row, n), o1);
  b.ct = bld8(mk_rsrc(a.icount + row, n), o1);
  b.hn = bld64(mk_rsrc(a.mhint + row, n * 8), rej ? lane * 8 : kOOB);
  b.lt = bld64(mk_rsrc(a.mlogterm + row, n * 8), rej ? lane * 8 : kOOB);
  ac.add(touched, 11);
  ac.add(rej, 16);
}

#ifndef QE_PSTEP_WAVES
#define QE_PSTEP_WAVES 3  // min waves per SIMD requested (VGPR budget: 151 at S=5, no scratch)
#endif

// One peer's send side: raft.maybeSendAppend (raft/raft.go:432-492).
struct PSend {
  rsrc_t ring;
  uint32_t ring0, F, me;
  uint64_t fi, li, snap;
  uint32_t count_msgs;  // messages sent to this peer this round (saturating)
  uint64_t first_index; // m.Index of the first of them
  bool snapped;
};

template <bool ACCT>
__device__ __forceinline__ bool send_append(PR &p, bool send_if_empty, PSend &x, Acct<ACCT> &ac) {
  if (pr_paused(p, x.F)) return false;
  uint64_t mindex;
  if (p.next > x.li) {  // entries(Next) = (nil, nil): empty MsgApp only if sendIfEmpty
    if (!send_if_empty) return false;
    mindex = p.next - 1;
  } else if (p.next < x.fi) {  // ErrCompacted: the sendIfEmpty check comes first (:442-444)
    if (!send_if_empty || !p.recent_active) return false;
    pr_reset(p, QE_PR_SNAPSHOT);  // BecomeSnapshot(snapshot index) (:468)
    p.pending = x.snap;
    x.snapped = true;
    mindex = x.snap;
  } else {
    uint64_t last = x.li;
    if (x.me) {
      const uint64_t l = p.next + (x.me - 1);
      if (l >= p.next && l < last) last = l;
    }
    mindex = p.next - 1;
    if (p.state == QE_PR_REPLICATE) {  // OptimisticUpdate + Inflights.Add (:478-482)
      p.next = last + 1;
      uint32_t pos = p.start + p.count;
      if (pos >= x.F) pos -= x.F;
      if (pos >= x.F) pos = 0;  // invalid Inflights.start: stay inside the row
      bst64(last, x.ring, (x.ring0 + pos) * 8);
      ac.add(true, 8);
      p.count++;
    } else if (p.state == QE_PR_PROBE) {
      p.probe_sent = 1;
    }
  }
  if (x.count_msgs == 0) x.first_index = mindex;
  if (x.count_msgs < 255) x.count_msgs++;
  return true;
}

// Inflights.FreeLE(to) (raft/tracker/inflights.go:87-113).  e[] holds the
// first min(kRingChunk, npre) live entries from `start` (loaded before this
// round's sends appended any); the rest, if the scan gets there, come from
// memory (the ring row is written in program order by this lane).
template <bool ACCT>
__device__ __forceinline__ void free_le(PR &p, uint64_t to, const uint64_t (&e)[kRingChunk],
                                        uint32_t npre, const PSend &x, Acct<ACCT> &ac) {
  constexpr int CH = kRingChunk;
  uint32_t fr = 0;
  bool go = true;
#pragma unroll
  for (int k = 0; k < CH; k++) {
    go = go && static_cast<uint32_t>(k) < npre && e[k] <= to;
    fr += go ? 1u : 0u;
  }
  if (fr == npre && fr < p.count) {  // beyond the prefetched entries
    uint32_t pos = p.start + fr;
    while (pos >= x.F) pos -= x.F;
    while (fr < p.count) {
      const uint64_t v = bld64(x.ring, (x.ring0 + pos) * 8);
      ac.add(true, 8);
      if (v > to) break;
      fr++;
      if (++pos >= x.F) pos -= x.F;
    }
  }
  if (fr > 0) {
    p.count -= fr;
    uint32_t st2 = p.start + fr;
    while (st2 >= x.F) st2 -= x.F;
    p.start = p.count == 0 ? 0 : st2;
  }
}

template <int S, typename MT, bool MASKED, bool JOINT, int RM, bool ACCT>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kBlock),
                          amdgpu_waves_per_eu(QE_PSTEP_WAVES))) void k_progress_step(PArgs a) {
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
  const uint32_t o8 = lane * 8;
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    const uint64_t g0 = t * 64;
    const uint32_t n = tile_n(a.G, t);
    const bool live = lane < n;
    // ---- A: per group ----
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
    const uint32_t nr = rc < a.R ? rc : a.R;
    ac.add(live, (MASKED ? sizeof(MT) : 0) + (JOINT ? sizeof(MT) : 0) +
                     (a.tracked ? sizeof(MT) : 0) + (a.self_slot ? 1 : 0) +
                     (a.transferee ? 1 : 0) + 32 + (a.snap_index ? 8 : 0) + 1);
    uint64_t vals[S];
    uint32_t ty[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const bool tr = (trk >> s) & 1u;
      vals[s] = bld64(mk_rsrc(a.match + row, n * 8), o8);
      ty[s] = bld8(mk_rsrc(a.mtype + row, n), tr ? lane : kOOB);
      ac.add(live, 8);
      ac.add(live && tr, 1);
    }
    // m.Index of every MsgAppResp (accept or reject)
    uint64_t ix[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const bool has_ix = ty[s] == QE_MSG_APP_RESP || ty[s] == QE_MSG_APP_RESP_REJECT;
      ix[s] = bld64(mk_rsrc(a.mindex + row, n * 8), has_ix ? o8 : kOOB);
      ac.add(has_ix, 8);
    }
    // ---- phase 1: MaybeUpdate + maybeCommit in message order -> bcasts ----
    uint64_t m0[S];
#pragma unroll
    for (int s = 0; s < S; s++) m0[s] = vals[s];
    uint64_t c = c0;
    uint32_t bset = 0, upd = 0, nbc = 0;
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
    // ---- phase 2: every peer's event sequence ----
    PSend x;
    x.F = F;
    x.me = a.max_ents;
    x.fi = fi;
    x.li = li;
    x.snap = a.snap_index ? snap_ld : fi - 1;
    uint64_t rf[RM], rt[RM];
#pragma unroll
    for (int r = 0; r < RM; r++) rf[r] = rt[r] = 0;
    bool have_runs = false;
    uint32_t sent = 0, snapm = 0, tnow = 0;
    auto touched_of = [&](int s) -> bool {
      const bool tr = (trk >> s) & 1u;
      const bool msg = ty[s] >= QE_MSG_APP_RESP && ty[s] <= QE_MSG_UNREACHABLE;
      return tr && (msg || (bset != 0 && static_cast<uint32_t>(s) != self));
    };
    PB cur;
    pb_load<ACCT>(a, g0, n, lane, touched_of(0), ty[0] == QE_MSG_APP_RESP_REJECT, cur, ac);
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const uint32_t tt = ty[s];
      const bool touched = touched_of(s);
      PB nxt;
      if (s + 1 < S)
        pb_load<ACCT>(a, row + a.stride, n, lane, touched_of(s + 1),
                      ty[s + 1] == QE_MSG_APP_RESP_REJECT, nxt, ac);
      PR p;
      p.match = m0[s];
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
      // term runs, once per group, when a reject needs findConflictByTerm
      const bool need_runs = touched && tt == QE_MSG_APP_RESP_REJECT && cur.lt > 0 && !have_runs;
      if (__builtin_amdgcn_ballot_w64(need_runs)) {
#pragma unroll
        for (int r = 0; r < RM; r++) {
          const uint32_t off = (need_runs && static_cast<uint32_t>(r) < nr) ? o8 : kOOB;
          const uint64_t rrow = static_cast<uint64_t>(r) * a.stride + g0;
          const uint64_t f = bld64(mk_rsrc(a.run_first + rrow, n * 8), off);
          const uint64_t m = bld64(mk_rsrc(a.run_term + rrow, n * 8), off);
          ac.add(need_runs && static_cast<uint32_t>(r) < nr, 16);
          rf[r] = need_runs ? f : rf[r];
          rt[r] = need_runs ? m : rt[r];
        }
      }
      have_runs = have_runs || need_runs;
      // Inflights entries a FreeLE of this round may scan: an accept that
      // raises Match of a Replicate peer, or a heartbeat response of a
      // Replicate peer whose ring is (or will be, after this round's
      // earlier sends) full
      x.ring = mk_rsrc(a.ibuf + row * F, n * F * 8);
      x.ring0 = lane * F;
      const bool repl = p.state == QE_PR_REPLICATE;
      const bool up = (upd >> s) & 1u;
      const bool scan = touched && repl && ((tt == QE_MSG_APP_RESP && up) ||
                                            tt == QE_MSG_HEARTBEAT_RESP);
      const uint32_t npre = scan ? (p.count < CH ? p.count : CH) : 0u;
      uint64_t e[CH];
#pragma unroll
      for (int k = 0; k < CH; k++) e[k] = 0;
      if (__builtin_amdgcn_ballot_w64(npre > 0)) {
#pragma unroll
        for (int k = 0; k < CH; k++) {
          uint32_t pos = p.start + k;
          if (pos >= F) pos -= F;
          if (pos >= F) pos = 0;  // invalid Inflights.start: stay inside the row
          e[k] = bld64(x.ring, static_cast<uint32_t>(k) < npre ? (x.ring0 + pos) * 8 : kOOB);
          ac.add(static_cast<uint32_t>(k) < npre, 8);
        }
      }
      x.count_msgs = 0;
      x.first_index = 0;
      x.snapped = false;
      // The peer's events in order: k1 bcast sends (from accepts of earlier
      // slots), its own message (handler), the handler's sendAppend (k2),
      // the `for maybeSendAppend(from, false) {}` loop (lp), k3 bcast sends
      // (from later slots).  One send_append call site per slot.
      const bool bcast_target = touched && static_cast<uint32_t>(s) != self;
      const uint32_t below = (1u << s) - 1u;
      uint32_t k1 = bcast_target ? popc(bset & below) : 0u;
      uint32_t k3 = bcast_target ? popc(bset & ~below & ~(1u << s)) : 0u;
      uint32_t k2 = 0;
      bool lp = false, handled = !touched, updated = false;
      for (;;) {
        bool sei;
        if (k1) {
          k1--;
          sei = true;
        } else if (!handled) {
          handled = true;
          if (tt == QE_MSG_APP_RESP_REJECT) {  // raft.go:1109-1236
            p.recent_active = 1;
            uint64_t probe = cur.hn;
            if (cur.lt > 0) probe = find_conflict_by_term<RM>(rf, rt, nr, li, probe, cur.lt);
            bool decr;  // MaybeDecrTo(m.Index, probe), progress.go:170-193
            if (p.state == QE_PR_REPLICATE) {
              decr = ix[s] > p.match;
              if (decr) p.next = p.match + 1;
            } else {
              decr = (p.next - 1 == ix[s]);
              if (decr) {
                const uint64_t m = ix[s] < probe + 1 ? ix[s] : probe + 1;
                p.next = m > 1 ? m : 1;
                p.probe_sent = 0;
              }
            }
            if (decr && p.state == QE_PR_REPLICATE) pr_become_probe(p);
            k2 = decr ? 1u : 0u;
          } else if (tt == QE_MSG_APP_RESP) {  // raft.go:1237-1282
            p.recent_active = 1;
            const uint64_t idx = ix[s];
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
                free_le<ACCT>(p, idx, e, npre, x, ac);
              }
              // bcastAppend of this accept (skips the leader) / sendAppend
              // if it was paused; then the send loop
              k2 = ((bset >> s) & 1u) ? (static_cast<uint32_t>(s) != self ? 1u : 0u)
                                      : (old_paused ? 1u : 0u);
              lp = true;
              if (static_cast<uint32_t>(s) == ltr && p.match == li) tnow |= 1u << s;
            }
          } else if (tt == QE_MSG_HEARTBEAT_RESP) {  // raft.go:1284-1294
            p.recent_active = 1;
            p.probe_sent = 0;
            if (p.state == QE_PR_REPLICATE && p.count == F) {
              uint64_t first;  // FreeFirstOne = FreeLE(buffer[start])
              if (npre > 0) {
                first = e[0];
              } else {
                uint32_t pos = p.start;
                while (pos >= F) pos -= F;
                first = bld64(x.ring, (x.ring0 + pos) * 8);
                ac.add(true, 8);
              }
              free_le<ACCT>(p, first, e, npre, x, ac);
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
          continue;
        } else if (k2) {
          k2--;
          sei = true;
        } else if (lp) {
          sei = false;
        } else if (k3) {
          k3--;
          sei = true;
        } else {
          break;
        }
        const bool r = send_append<ACCT>(p, sei, x, ac);
        if (!sei && !r) lp = false;
      }
      // ---- stores: the peer's new Progress (unchanged words and bytes skipped) ----
      const uint32_t w8 = touched ? o8 : kOOB, w1 = touched ? lane : kOOB;
      const uint32_t fl = p.state | (p.probe_sent ? QE_PF_PROBE_SENT : 0u) |
                          (p.recent_active ? QE_PF_RECENT_ACTIVE : 0u);
      const bool wm = updated, wn = touched && p.next != cur.nx, wp = touched && (p.pending != pd0 || p.reset);
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
      if (s + 1 < S) cur = nxt;
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
      if (on) send_append<false>(p, a.send_if_empty != 0, x, ac);
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
