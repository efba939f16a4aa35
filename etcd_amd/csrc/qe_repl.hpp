// qe_repl.hpp — software-pipelined lockstep replication round
// (qe_replication_round, "stream" kernel; config 4 of BASELINE.json).
//
// Same per-group semantics as k_replication (qe_kernels.hpp):
// Progress.MaybeUpdate on every responding slot (raft/tracker/progress.go:
// 144-153), CommittedIndex over Match, the term-gated commit advance
// (raft/log.go:325-331, :233-241) and the ReadIndex quorum
// (raft/read_only.go:68-76).  Layout of the work, as in k_cv_stream
// (qe_stream.hpp):
//   * one group per lane, 64-group tiles addressed through buffer
//     descriptors (num_records clips the ragged last tile);
//   * a wave owns a chunk of up to QE_STREAM_TPW tiles whose four masks
//     (voters inc/out, responders, read acks) are staged in LDS first, so a
//     tile's row loads depend on an LDS read only;
//   * a slot that does not respond needs neither its resp index nor its
//     Next, and a slot outside the voters that does not respond needs no
//     Match: those loads get an out-of-range offset (dropped, no traffic);
//   * MaybeUpdate writes Match / Next only when they change, and committed
//     only when it advances (the reference assigns only on change too):
//     an unchanged word is a store with an out-of-range offset;
//   * two register sets, tile k+1's loads in flight while tile k computes.
#pragma once
#include "qe_stream.hpp"

namespace qe {

template <int S>
struct RTile {
  uint64_t m[S], n[S], r[S];
  uint64_t ts, li, cm;
};

// Chunk-local masks in LDS: [0] = inc | out << 16, [1] = resp | acks << 16.
template <int S, bool MASKED, bool JOINT, bool NTL>
__device__ __forceinline__ void rs_issue(const RArgs &a, uint64_t t, uint32_t lane, uint32_t vm,
                                         uint32_t ra, RTile<S> &x) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  const uint64_t tile0 = t * 64;
  const uint32_t n = tile_n(a.G, t);
  const uint32_t off = lane * 8;
  const int aux = NTL ? 2 : 0;
  const uint32_t rm = ra & kFull;
  const uint32_t voters = MASKED ? ((vm | (vm >> 16)) & kFull) : kFull;
  const uint32_t need_m = voters | rm;
#pragma unroll
  for (int s = 0; s < S; s++) {
    const uint64_t row = static_cast<uint64_t>(s) * a.stride + tile0;
    const uint32_t om = bit_off(need_m, s, off);
    const uint32_t orr = bit_off(rm, s, off);
    x.m[s] = __builtin_bit_cast(
        uint64_t, __builtin_amdgcn_raw_buffer_load_b64(mk_rsrc(a.match + row, n * 8), om, 0, aux));
    x.n[s] = __builtin_bit_cast(
        uint64_t, __builtin_amdgcn_raw_buffer_load_b64(mk_rsrc(a.next + row, n * 8), orr, 0, aux));
    x.r[s] = __builtin_bit_cast(
        uint64_t, __builtin_amdgcn_raw_buffer_load_b64(mk_rsrc(a.resp + row, n * 8), orr, 0, aux));
  }
  x.ts = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(
                                          mk_rsrc(a.term_start + tile0, n * 8), off, 0, aux));
  x.li = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(
                                          mk_rsrc(a.last_index + tile0, n * 8), off, 0, aux));
  x.cm = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(
                                          mk_rsrc(a.committed + tile0, n * 8), off, 0, aux));
}

template <int S, bool MASKED, bool JOINT, bool NTS>
__device__ __forceinline__ void rs_finish(const RArgs &a, uint64_t t, uint32_t lane,
                                          bool want_stats, uint32_t vm, uint32_t ra,
                                          RTile<S> &x, uint64_t (&cnt)[R_N]) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  const uint64_t tile0 = t * 64;
  const uint32_t n = tile_n(a.G, t);
  const uint32_t off = lane * 8;
  const int aux = NTS ? 2 : 0;
  const uint32_t inc = MASKED ? (vm & kFull) : kFull;
  const uint32_t out = JOINT ? ((vm >> 16) & kFull) : 0u;
  const uint32_t rm = ra & kFull, acks = (ra >> 16) & kFull;
  uint64_t sel[S];
#pragma unroll
  for (int s = 0; s < S; s++) {
    const bool resp = (rm >> s) & 1u;
    const uint64_t row = static_cast<uint64_t>(s) * a.stride + tile0;
    const bool um = resp && x.m[s] < x.r[s];          // MaybeUpdate: Match < n
    const bool un = resp && x.n[s] < x.r[s] + 1;      // Next = max(Next, n+1)
    const uint64_t m = um ? x.r[s] : x.m[s];
    const uint64_t nx = un ? x.r[s] + 1 : x.n[s];
    sel[s] = m;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, m),
                                          mk_rsrc(a.match + row, n * 8), um ? off : kOOB, 0, aux);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, nx),
                                          mk_rsrc(a.next + row, n * 8), un ? off : kOOB, 0, aux);
  }
  const uint64_t mci = (!JOINT && !MASKED) ? select_fixed<S>(sel) : joint_committed<S>(sel, inc, out);
  // raftLog.maybeCommit with term(i)==Term <=> term_start<=i<=last_index
  const uint32_t adv = (mci > x.cm && mci >= x.ts && mci <= x.li) ? 1u : 0u;
  const uint64_t cm = adv ? mci : x.cm;
  const uint32_t ro = a.read_acks ? (joint_vote(inc, out, acks, acks) == kVoteWon) : 0u;
  if (want_stats && lane < n) {
    cnt[R_GROUPS] += 1;
    cnt[R_SUM] += cm;
    cnt[R_ADV] += adv;
    cnt[R_READ] += ro;
    cnt[R_VIOL] += (mci > x.li);
    const uint64_t tag = (static_cast<uint64_t>(ro) << 62) | (static_cast<uint64_t>(adv) << 61);
    cnt[R_CSUM] += mix64(((a.goff + tile0 + lane) * kPhi) ^ cm ^ tag);
  }
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, cm),
                                        mk_rsrc(a.committed + tile0, n * 8), adv ? off : kOOB, 0,
                                        aux);
  __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(ro), opt_rsrc(a.read_ok, tile0, n),
                                       lane, 0, aux);
  __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(adv), opt_rsrc(a.adv, tile0, n), lane,
                                       0, aux);
}

template <int S, bool MASKED, bool JOINT, typename MT, bool NTL, bool NTS>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kBlock),
                          amdgpu_waves_per_eu(QE_STREAM_WAVES))) void k_repl_stream(RArgs a) {
  constexpr int TPW = QE_STREAM_TPW;
  __shared__ uint32_t lds_v[kBlock / 64][TPW][64];
  __shared__ uint32_t lds_r[kBlock / 64][TPW][64];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t ntiles = (a.G + 63) / 64;
  const uint32_t chunk = a.chunk;  // <= TPW (host-checked)
  const uint64_t t0 = (static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + w) * chunk;
  const uint32_t nt =
      t0 < ntiles ? static_cast<uint32_t>(ntiles - t0 < chunk ? ntiles - t0 : chunk) : 0u;
  const bool want_stats = a.stats != nullptr;
  uint64_t cnt[R_N];
#pragma unroll
  for (int i = 0; i < R_N; i++) cnt[i] = 0;
  if (nt > 0) {
    {
      uint32_t mv[TPW], mr[TPW];
#pragma unroll
      for (int k = 0; k < TPW; k++) {
        const uint64_t tile0 = (t0 + k) * 64;
        const uint32_t n = tile_n(a.G, t0 + k);  // 0 past the chunk's end
        uint32_t v = 0, r = 0;
        if constexpr (MASKED) v = bld_mask<MT>(a.inc, tile0, n, lane);
        if constexpr (JOINT) v |= bld_mask<MT>(a.out, tile0, n, lane) << 16;
        r = ld_mask_r<MT>(opt_rsrc(static_cast<const MT *>(a.resp_mask), tile0, n), lane);
        r |= ld_mask_r<MT>(opt_rsrc(static_cast<const MT *>(a.read_acks), tile0, n), lane) << 16;
        mv[k] = v;
        mr[k] = r;
      }
#pragma unroll
      for (int k = 0; k < TPW; k++) {
        lds_v[w][k][lane] = mv[k];
        lds_r[w][k][lane] = mr[k];
      }
    }
    const uint64_t tend = t0 + nt;
    auto tix = [&](uint32_t k) -> uint64_t { return t0 + k < tend ? t0 + k : ntiles; };
    auto vm_of = [&](uint32_t k) -> uint32_t { return lds_v[w][k % TPW][lane]; };
    auto ra_of = [&](uint32_t k) -> uint32_t { return lds_r[w][k % TPW][lane]; };
    RTile<S> xa, xb;
    rs_issue<S, MASKED, JOINT, NTL>(a, tix(0), lane, vm_of(0), ra_of(0), xa);
    for (uint32_t k = 0; k < nt; k += 2) {
      rs_issue<S, MASKED, JOINT, NTL>(a, tix(k + 1), lane, vm_of(k + 1), ra_of(k + 1), xb);
      __builtin_amdgcn_sched_barrier(0);
      rs_finish<S, MASKED, JOINT, NTS>(a, tix(k), lane, want_stats, vm_of(k), ra_of(k), xa, cnt);
      rs_issue<S, MASKED, JOINT, NTL>(a, tix(k + 2), lane, vm_of(k + 2), ra_of(k + 2), xa);
      __builtin_amdgcn_sched_barrier(0);
      rs_finish<S, MASKED, JOINT, NTS>(a, tix(k + 1), lane, want_stats, vm_of(k + 1),
                                       ra_of(k + 1), xb, cnt);
    }
  }
  if (want_stats) {
    const int idx[R_N] = {QE_STAT_GROUPS, QE_STAT_COMMIT_SUM, QE_STAT_COMMIT_ADVANCED,
                          QE_STAT_READ_RELEASED, QE_STAT_INVARIANT_VIOLATIONS, QE_STAT_CHECKSUM};
    block_stats_add<R_N, kBlock>(cnt, idx, a.stats);
  }
}

}  // namespace qe
