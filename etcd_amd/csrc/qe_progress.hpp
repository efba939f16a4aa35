// qe_progress.hpp — qe_progress_step kernel (leader-side Progress state
// machine, raft/raft.go:1106-1296), one group per lane, tiles of 64 groups.
//
// Every access goes through a per-tile buffer descriptor (wave-uniform base,
// 32-bit lane offset, num_records clipping the ragged last tile), as in the
// stream commit/vote kernel (qe_stream.hpp): no 64-bit address arithmetic
// per lane, and a conditional access is an unconditional load or store whose
// offset is pushed out of range when its condition is false (the hardware
// drops it: no traffic, no branch, loads return 0).
//
// The reference's per-message work is a chain of dependent memory accesses
// (message -> Progress -> Inflights scan -> log terms).  Here the loads are
// grouped into stages whose addresses are known together:
//   A  per group: masks, committed, termStart, lastIndex, run count; per slot:
//      message type and Match (all slots: maybeCommit reads every Match)
//   B  per slot with a message: Next, PendingSnapshot, flags, Inflights
//      start/count, m.Index (+ RejectHint/LogTerm of a reject)
//   C  the first 8 Inflights entries FreeLE will scan, and (once per group)
//      the run table when a reject needs findConflictByTerm
// and software-pipelined over the slots: slot s+1's B loads are issued
// before slot s's C loads, so every slot after the first costs one memory
// round trip.  The state machine runs in registers, slots in ascending
// (message) order.
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

struct PB {  // stage-B registers of one slot
  uint64_t nx, pd, ix, hn, lt;
  uint32_t fl, st, ct;
};

// Stage B of slot row `row` (= s*stride + tile0) for message type t.
__device__ __forceinline__ void pb_load(const PArgs &a, uint64_t row, uint32_t n, uint32_t lane,
                                        uint32_t t, PB &b) {
  const bool msg = t >= QE_MSG_APP_RESP && t <= QE_MSG_HEARTBEAT_RESP;
  const bool has_ix = t == QE_MSG_APP_RESP || t == QE_MSG_APP_RESP_REJECT;
  const bool rej = t == QE_MSG_APP_RESP_REJECT;
  const uint32_t o8 = msg ? lane * 8 : kOOB, o1 = msg ? lane : kOOB;
  b.nx = bld64(mk_rsrc(a.next + row, n * 8), o8);
  b.pd = bld64(mk_rsrc(a.pending + row, n * 8), o8);
  b.fl = bld8(mk_rsrc(a.flags + row, n), o1);
  b.st = bld8(mk_rsrc(a.istart + row, n), o1);
  b.ct = bld8(mk_rsrc(a.icount + row, n), o1);
  b.ix = bld64(mk_rsrc(a.mindex + row, n * 8), has_ix ? lane * 8 : kOOB);
  b.hn = bld64(mk_rsrc(a.mhint + row, n * 8), rej ? lane * 8 : kOOB);
  b.lt = bld64(mk_rsrc(a.mlogterm + row, n * 8), rej ? lane * 8 : kOOB);
}

#ifndef QE_PSTEP_WAVES
#define QE_PSTEP_WAVES 1  // min waves per SIMD requested (VGPR budget)
#endif

template <int S, typename MT, bool MASKED, bool JOINT, int RM>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kBlock),
                          amdgpu_waves_per_eu(QE_PSTEP_WAVES))) void k_progress_step(PArgs a) {
  constexpr int CH = kRingChunk;
  constexpr uint32_t kFull = (1u << S) - 1u;
  uint64_t cnt[P_N] = {0, 0, 0, 0, 0};
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
    // ---- A ----
    const uint32_t mi =
        MASKED ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.inc) + g0, n * sizeof(MT)), lane) &
                  kFull)
               : kFull;
    const uint32_t mo =
        JOINT ? (ld_mask_r<MT>(mk_rsrc(static_cast<const MT *>(a.out) + g0, n * sizeof(MT)), lane) &
                 kFull)
              : 0u;
    const uint64_t li = bld64(mk_rsrc(a.last_index + g0, n * 8), o8);
    const uint64_t ts = bld64(mk_rsrc(a.term_start + g0, n * 8), o8);
    const rsrc_t r_commit = mk_rsrc(a.committed + g0, n * 8);
    const uint64_t c0 = bld64(r_commit, o8);
    const uint32_t rc = bld8(mk_rsrc(a.run_count + g0, n), lane);
    const uint32_t nr = rc < a.R ? rc : a.R;
    uint64_t vals[S];
    uint32_t ty[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      vals[s] = bld64(mk_rsrc(a.match + row, n * 8), o8);
      ty[s] = bld8(mk_rsrc(a.mtype + row, n), lane);
    }
    uint64_t rf[RM], rt[RM];
#pragma unroll
    for (int r = 0; r < RM; r++) rf[r] = rt[r] = 0;
    bool have_runs = false;
    uint64_t c = c0;
    uint32_t send = 0, bc = 0;
    PB cur;
    pb_load(a, g0, n, lane, ty[0], cur);
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint64_t row = static_cast<uint64_t>(s) * a.stride + g0;
      const uint32_t tt = ty[s];
      // ---- B of the next slot, in flight with this slot's C ----
      PB nxt;
      if (s + 1 < S) pb_load(a, row + a.stride, n, lane, ty[s + 1], nxt);
      // ---- C: term runs, once per group, when a reject needs them ----
      const bool need_runs = tt == QE_MSG_APP_RESP_REJECT && cur.lt > 0 && !have_runs;
#pragma unroll
      for (int r = 0; r < RM; r++) {
        const uint32_t off = (need_runs && static_cast<uint32_t>(r) < nr) ? o8 : kOOB;
        const uint64_t rrow = static_cast<uint64_t>(r) * a.stride + g0;
        const uint64_t f = bld64(mk_rsrc(a.run_first + rrow, n * 8), off);
        const uint64_t m = bld64(mk_rsrc(a.run_term + rrow, n * 8), off);
        rf[r] = need_runs ? f : rf[r];
        rt[r] = need_runs ? m : rt[r];
      }
      have_runs = have_runs || need_runs;
      // ---- C: FreeLE scan (inflights.go:87-113): an accept that raises
      // Match of a Replicate peer frees entries <= m.Index; a heartbeat
      // response on a full ring frees entries <= the first (FreeFirstOne) ----
      const bool repl = (cur.fl & QE_PF_STATE) == QE_PR_REPLICATE;
      const bool acc = tt == QE_MSG_APP_RESP && repl && cur.ix <= li && vals[s] < cur.ix;
      const bool hb = tt == QE_MSG_HEARTBEAT_RESP && repl && cur.ct == F;
      const uint32_t nscan = (acc || hb) ? (cur.ct < CH ? cur.ct : CH) : 0u;
      // this tile's rings of slot s: one row of F entries per lane
      const rsrc_t r_ring = mk_rsrc(a.ibuf + row * F, n * F * 8);
      const uint32_t ring0 = lane * F;
      uint64_t e[CH];
#pragma unroll
      for (int k = 0; k < CH; k++) {
        uint32_t pos = cur.st + k;
        if (pos >= F) pos -= F;
        if (pos >= F) pos = 0;  // corrupt Inflights.start: stay inside the row
        e[k] = bld64(r_ring, static_cast<uint32_t>(k) < nscan ? (ring0 + pos) * 8 : kOOB);
      }
      uint32_t fr = 0;
      {
        const uint64_t to = hb ? e[0] : cur.ix;
        bool go = true;
#pragma unroll
        for (int k = 0; k < CH; k++) {
          go = go && static_cast<uint32_t>(k) < nscan && e[k] <= to;
          fr += go ? 1u : 0u;
        }
        if (fr == CH && cur.ct > CH) {  // MaxInflightMsgs > 8: scan on
          uint32_t pos = cur.st + CH;
          if (pos >= F) pos -= F;
          if (pos >= F) pos = 0;
          while (fr < cur.ct && bld64(r_ring, (ring0 + pos) * 8) <= to) {
            fr++;
            if (++pos >= F) pos -= F;
          }
        }
      }
      // ---- the state machine for this slot's message ----
      const bool msg = tt >= QE_MSG_APP_RESP && tt <= QE_MSG_HEARTBEAT_RESP;
      PR p;
      p.match = vals[s];
      p.next = cur.nx;
      p.pending = cur.pd;
      p.state = cur.fl & QE_PF_STATE;
      p.probe_sent = (cur.fl & QE_PF_PROBE_SENT) != 0;
      p.recent_active = 1;
      p.start = cur.st;
      p.count = cur.ct;
      bool updated = false;
      if (tt == QE_MSG_APP_RESP_REJECT) {
        uint64_t probe = cur.hn;
        if (cur.lt > 0) probe = find_conflict_by_term<RM>(rf, rt, nr, li, probe, cur.lt);
        bool decr;  // MaybeDecrTo(m.Index, probe)
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
        if (decr) {
          if (p.state == QE_PR_REPLICATE) pr_become_probe(p);
          send |= 1u << s;
        }
      } else if (tt == QE_MSG_APP_RESP) {
        const uint64_t idx = cur.ix;
        if (idx > li) {
          cnt[P_VIOL] += 1;
        } else {
          const bool old_paused = pr_paused(p, F);
          if (p.match < idx) {  // MaybeUpdate
            p.match = idx;
            updated = true;
            p.probe_sent = 0;
          }
          if (p.next < idx + 1) p.next = idx + 1;
          if (updated) {
            if (p.state == QE_PR_PROBE) {
              pr_become_replicate(p);
            } else if (p.state == QE_PR_SNAPSHOT && p.match >= p.pending) {
              pr_become_probe(p);
              pr_become_replicate(p);
            } else if (p.state == QE_PR_REPLICATE && fr > 0) {
              p.count -= fr;
              uint32_t st2 = p.start + fr;
              if (st2 >= F) st2 -= F;
              p.start = p.count == 0 ? 0 : st2;
            }
            vals[s] = p.match;
            const uint64_t mci = mci_of<S, MASKED, JOINT>(vals, mi, mo);
            if (mci > c && mci >= ts && mci <= li) {
              c = mci;
              bc = 1;
            } else if (old_paused) {
              send |= 1u << s;
            }
          }
        }
      } else if (tt == QE_MSG_HEARTBEAT_RESP) {
        p.probe_sent = 0;
        if (p.state == QE_PR_REPLICATE && p.count == F && fr > 0) {
          p.count -= fr;
          uint32_t st2 = p.start + fr;
          if (st2 >= F) st2 -= F;
          p.start = p.count == 0 ? 0 : st2;
        }
        if (p.match < li) send |= 1u << s;
      }
      // ---- stores: the peer's new Progress (unchanged words and bytes skipped) ----
      const uint32_t w8 = msg ? o8 : kOOB, w1 = msg ? lane : kOOB;
      const uint32_t fl = p.state | (p.probe_sent ? QE_PF_PROBE_SENT : 0u) | QE_PF_RECENT_ACTIVE;
      bst64(p.match, mk_rsrc(a.match + row, n * 8), updated ? o8 : kOOB);
      bst64(p.next, mk_rsrc(a.next + row, n * 8), p.next != cur.nx ? w8 : kOOB);
      bst64(p.pending, mk_rsrc(a.pending + row, n * 8), p.pending != cur.pd ? w8 : kOOB);
      bst8(fl, mk_rsrc(a.flags + row, n), fl != cur.fl ? w1 : kOOB);
      bst8(p.start, mk_rsrc(a.istart + row, n), p.start != cur.st ? w1 : kOOB);
      bst8(p.count, mk_rsrc(a.icount + row, n), p.count != cur.ct ? w1 : kOOB);
      if (s + 1 < S) cur = nxt;
    }
    bst64(c, r_commit, o8);
    bst_mask<MT>(send, opt_rsrc(static_cast<const MT *>(a.send_mask), g0, n), lane);
    bst8(bc, opt_rsrc(static_cast<const uint8_t *>(a.bcast), g0, n), lane);
    if (lane < n) {
      cnt[P_GROUPS] += 1;
      cnt[P_SUM] += c;
      cnt[P_ADV] += (c != c0);
      const uint64_t tag =
          (static_cast<uint64_t>(send) << 40) | (static_cast<uint64_t>(bc) << 62);
      cnt[P_CSUM] += mix64(((a.goff + g0 + lane) * kPhi) ^ c ^ tag);
    }
  }
  if (a.stats) {
    const int idx[P_N] = {QE_STAT_GROUPS, QE_STAT_COMMIT_SUM, QE_STAT_COMMIT_ADVANCED,
                          QE_STAT_INVARIANT_VIOLATIONS, QE_STAT_CHECKSUM};
    block_stats_add<P_N, kBlock>(cnt, idx, a.stats);
  }
}

}  // namespace qe
