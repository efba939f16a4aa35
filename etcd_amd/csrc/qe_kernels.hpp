// qe_kernels.hpp — MI355X (gfx950) kernels of the batched quorum engine.
//
// One lane owns one group: a slot row of the SoA arrays ([S][stride]) is one
// coalesced access per wave (512 B of u64 for a 64-group tile), addressed
// through a per-tile buffer descriptor whose num_records clips the ragged
// last tile.  The stream kernels (qe_stream.hpp) give each wave a chunk of
// tiles and keep tile k+1's loads in flight while tile k is decided; the
// Progress kernels (qe_progress.hpp) walk one tile per wave.  See DESIGN.md
// §2-§3.
#pragma once
// A/B knobs are for variant libraries built by
// scripts/build_variant*.sh, which define QE_VARIANT_BUILD; they only change
// code paths or launch shapes (the experiments that dropped work, the
// stamps and the LDS-DMA ring of round 4 left the product kernel in round 5:
// git show bdcd377:etcd_amd/csrc/qe_progress.hpp).  A product build with any
// of them set is refused, so a stray -D can never ship a library that
// computes something else.
#if !defined(QE_VARIANT_BUILD) &&                                                  \
    (defined(QE_CQ_CHANGED_ONLY) || defined(QE_STREAM_ALL_ROWS) || defined(QE_NO_RM8) || \
     defined(QE_RM16_WPB) || defined(QE_PSTEP_WAVES) || defined(QE_STREAM_TPW) ||        \
     defined(QE_STREAM_WAVES) || defined(QE_JOINT_MIN_WAVES) || defined(QE_LD_AUX) ||     \
     defined(QE_ST_AUX) || defined(QE_SEND_AUX) || defined(QE_NO_READ_OVF) ||              \
     defined(QE_SEND16_WAVES) || defined(QE_SWITCH16_WAVES) || defined(QE_PROPOSE16_WAVES) || defined(QE_PROPOSE16_PF) || \
     defined(QE_SEND16_ISSUE) || defined(QE_SWITCH16_ISSUE))
#error "A/B knob set in a product build: use scripts/build_variant*.sh (QE_VARIANT_BUILD)"
#endif
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>

#include "../../include/etcd_quorum.h"
#include "qe_device.hpp"

namespace qe {

constexpr int kBlock = 256;
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------
// Tuning knobs (qe_tune): occupancy of the persistent grid.
// ---------------------------------------------------------------------------
extern int g_blocks_per_cu;
extern int g_nontemporal;  // bit 0: loads, bit 1: stores
extern int g_cv_kernel;    // qe_commit_vote: 0 pair kernel, 1 stream kernel, -1 default
extern int g_repl_kernel;  // qe_replication_round: 0 pair kernel, 1 stream kernel, -1 default

inline int num_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0)
      v = 256;
    cached[dev] = v;
  }
  return cached[dev];
}

// Grid: with g_tiles_per_wave == 0 a persistent grid of min(work, CUs x
// resident blocks per CU) (`occ` = hipOccupancyMaxActiveBlocksPerMultiprocessor,
// capped by g_blocks_per_cu); with g_tiles_per_wave = T > 0 each wave walks
// T tiles and the hardware dispatcher keeps refilling CUs as blocks retire.
// g_tiles_per_wave < 0 (default) picks the per-kernel `auto_tpw` measured best
// (DESIGN.md §6).
extern int g_tiles_per_wave;
inline unsigned grid_for(uint64_t work_waves, int occ, int auto_tpw = 0) {
  const uint64_t need = (work_waves + (kBlock / 64) - 1) / (kBlock / 64);
  const int tpw = g_tiles_per_wave >= 0 ? g_tiles_per_wave : auto_tpw;
  uint64_t g;
  if (tpw > 0) {
    g = (need + tpw - 1) / tpw;
  } else {
    int per_cu = occ > 0 ? occ : 4;
    if (g_blocks_per_cu > 0 && g_blocks_per_cu < per_cu) per_cu = g_blocks_per_cu;
    const uint64_t cap = static_cast<uint64_t>(num_cus()) * per_cu;
    g = need < cap ? need : cap;
  }
  if (g > 0x7FFFFFFFull) g = 0x7FFFFFFFull;
  return static_cast<unsigned>(g ? g : 1);
}

template <typename K>
inline int occupancy(K kernel) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, kBlock, 0) != hipSuccess) n = 0;
  return n;
}

// ---------------------------------------------------------------------------
// Loads/stores of a pair of adjacent groups.
// ---------------------------------------------------------------------------
// GUARD = false: the caller knows the whole tile is in range (wave-uniform
// fast path, no per-element branches between the loads).
template <bool VEC, bool NT, bool GUARD = true>
__device__ __forceinline__ void ld_u64_pair(const uint64_t *p, uint64_t g0, uint64_t G,
                                            uint64_t &lo, uint64_t &hi) {
  if (VEC && (!GUARD || g0 + 1 < G)) {
    const u64x2 *q = reinterpret_cast<const u64x2 *>(p + g0);
    u64x2 x = NT ? __builtin_nontemporal_load(q) : *q;
    lo = x.x;
    hi = x.y;
  } else {
    lo = g0 < G ? p[g0] : 0;
    hi = g0 + 1 < G ? p[g0 + 1] : 0;
  }
}

template <bool VEC, bool NT = false, bool GUARD = true>
__device__ __forceinline__ void st_u64_pair(uint64_t *p, uint64_t g0, uint64_t G, uint64_t lo,
                                            uint64_t hi) {
  if (VEC && (!GUARD || g0 + 1 < G)) {
    u64x2 x;
    x.x = lo;
    x.y = hi;
    if (NT) __builtin_nontemporal_store(x, reinterpret_cast<u64x2 *>(p + g0));
    else *reinterpret_cast<u64x2 *>(p + g0) = x;
  } else {
    if (g0 < G) p[g0] = lo;
    if (g0 + 1 < G) p[g0 + 1] = hi;
  }
}

// Mask pairs: uint8 masks load as one uint16, uint16 masks as one uint32.
template <typename MT, bool VEC, bool GUARD = true>
__device__ __forceinline__ void ld_mask_pair(const void *p, uint64_t g0, uint64_t G,
                                             uint32_t &lo, uint32_t &hi) {
  const MT *m = static_cast<const MT *>(p);
  if (VEC && (!GUARD || g0 + 1 < G)) {
    if constexpr (sizeof(MT) == 1) {
      const uint32_t x = *reinterpret_cast<const uint16_t *>(m + g0);
      lo = x & 0xFFu;
      hi = x >> 8;
    } else {
      const uint32_t x = *reinterpret_cast<const uint32_t *>(m + g0);
      lo = x & 0xFFFFu;
      hi = x >> 16;
    }
  } else {
    lo = g0 < G ? m[g0] : 0u;
    hi = g0 + 1 < G ? m[g0 + 1] : 0u;
  }
}

template <typename MT, bool VEC, bool GUARD = true>
__device__ __forceinline__ void st_mask_pair(void *p, uint64_t g0, uint64_t G, uint32_t lo,
                                             uint32_t hi) {
  MT *m = static_cast<MT *>(p);
  if (VEC && (!GUARD || g0 + 1 < G)) {
    if constexpr (sizeof(MT) == 1) {
      *reinterpret_cast<uint16_t *>(m + g0) = static_cast<uint16_t>(lo | (hi << 8));
    } else {
      *reinterpret_cast<uint32_t *>(m + g0) = lo | (hi << 16);
    }
  } else {
    if (g0 < G) m[g0] = static_cast<MT>(lo);
    if (g0 + 1 < G) m[g0 + 1] = static_cast<MT>(hi);
  }
}

// uint8 outputs: a pair is one uint16 store.
template <bool VEC, bool NT = false, bool GUARD = true>
__device__ __forceinline__ void st_u8_pair(uint8_t *p, uint64_t g0, uint64_t G, uint32_t lo,
                                           uint32_t hi) {
  if (VEC && (!GUARD || g0 + 1 < G)) {
    const uint16_t x = static_cast<uint16_t>(lo | (hi << 8));
    if (NT) __builtin_nontemporal_store(x, reinterpret_cast<uint16_t *>(p + g0));
    else *reinterpret_cast<uint16_t *>(p + g0) = x;
  } else {
    if (g0 < G) p[g0] = static_cast<uint8_t>(lo);
    if (g0 + 1 < G) p[g0 + 1] = static_cast<uint8_t>(hi);
  }
}

// ---------------------------------------------------------------------------
// Fused CommittedIndex + VoteResult + TallyVotes (qe_commit_vote).
// MODE 0: fixed MajorityConfig of all S slots (compile-time rank)
// MODE 1: masked MajorityConfig (inc_mask)
// MODE 2: JointConfig (inc_mask, out_mask)
// ---------------------------------------------------------------------------
struct CVArgs {
  uint64_t G, goff, stride;
  const uint64_t *match;
  const void *inc, *out, *learner, *voted, *granted;
  uint64_t *commit;
  uint8_t *vote, *gcount, *rcount;
  uint64_t *stats;
  uint32_t chunk;  // k_cv_stream: tiles per wave, 1..QE_STREAM_TPW (set by the launcher)
};

enum { C_GROUPS, C_INF, C_SUM, C_ZERO, C_WON, C_LOST, C_PEND, C_GR, C_RJ, C_VIOL, C_CSUM, C_N };

template <int S, int MODE>
__device__ __forceinline__ void eval_group(uint64_t (&v)[S], uint32_t inc, uint32_t out,
                                           uint32_t learner, uint32_t voted, uint32_t granted,
                                           uint64_t &commit, uint32_t &vote, uint32_t &gc,
                                           uint32_t &rc, uint32_t top = S) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  if constexpr (MODE == 0) {
    commit = select_fixed<S>(v);
    inc = kFull;
    out = 0;
  } else {
    if constexpr (MODE == 1) out = 0;
    commit = joint_committed_top<S>(v, inc, out, top);
  }
  vote = joint_vote(inc, out, voted, granted);
  const uint32_t voters = (inc | out) & ~learner;
  gc = popc(voted & granted & voters);
  rc = popc(voted & ~granted & voters);
}

// Per-thread statistics of qe_commit_vote: counts in 32 bits (a thread sees
// far fewer than 2^32 groups), sums in 64 bits -- fewer live VGPRs.
struct CVStats {
  uint32_t groups = 0, inf = 0, zero = 0, won = 0, lost = 0, pend = 0, gr = 0, rj = 0, viol = 0;
  uint64_t sum = 0, csum = 0;
};

// Voter masks (JointConfig halves) of one tile.
template <typename MT, int MODE, int PAIRS, bool VEC, bool GUARD>
__device__ __forceinline__ void cv_masks(const CVArgs &a, uint64_t t, int lane,
                                         uint32_t (&mi)[PAIRS][2], uint32_t (&mo)[PAIRS][2]) {
  constexpr uint64_t kTile = 64ull * PAIRS;
#pragma unroll
  for (int j = 0; j < PAIRS; j++) {
    const uint64_t g0 = 2 * (t * kTile + j * 64 + lane);
    ld_mask_pair<MT, VEC, GUARD>(a.inc, g0, a.G, mi[j][0], mi[j][1]);
    if constexpr (MODE == 2) ld_mask_pair<MT, VEC, GUARD>(a.out, g0, a.G, mo[j][0], mo[j][1]);
    else mo[j][0] = mo[j][1] = 0;
  }
}

// One tile (64 lanes x PAIRS pairs) of qe_commit_vote.  GUARD = false on
// every tile that lies wholly inside [0, G): then no load or store carries a
// bounds branch and all the tile's loads issue back to back.  Masked modes
// receive this tile's voter masks (mi/mo, loaded one tile ahead) and prefetch
// the next tile's into mi_n/mo_n after issuing this tile's loads, so the
// dependent mask -> row-skip decision costs no extra memory round trip.
template <int S, int MODE, typename MT, int PAIRS, bool VEC, bool NTL, bool NTS, bool GUARD>
__device__ __forceinline__ void cv_tile(const CVArgs &a, uint64_t t, int lane, bool want_stats,
                                        CVStats &st, const uint32_t (&mi_in)[PAIRS][2],
                                        const uint32_t (&mo_in)[PAIRS][2], uint64_t tn,
                                        uint64_t ntiles, uint64_t nfull,
                                        uint32_t (&mi_n)[PAIRS][2], uint32_t (&mo_n)[PAIRS][2]) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  constexpr uint64_t kTile = 64ull * PAIRS;
  const uint64_t G = a.G;
  uint64_t v[PAIRS][2][S];
  uint32_t mi[PAIRS][2], mo[PAIRS][2], ml[PAIRS][2], vd[PAIRS][2], gr[PAIRS][2];
  // ---- slot rows no group of this wave uses (learner / empty slots) are
  // not fetched at all ----
  uint32_t used = kFull;
  if constexpr (MODE >= 1) {
    uint32_t u = 0;
#pragma unroll
    for (int j = 0; j < PAIRS; j++)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        mi[j][h] = mi_in[j][h];
        mo[j][h] = mo_in[j][h];
        u |= mi[j][h] | mo[j][h];
      }
    used = wave_or(u) & kFull;
  } else {
#pragma unroll
    for (int j = 0; j < PAIRS; j++) {
      mi[j][0] = mi[j][1] = kFull;
      mo[j][0] = mo[j][1] = 0;
    }
  }
  // ---- issue every remaining load of the tile (bytes in flight) ----
#pragma unroll
  for (int j = 0; j < PAIRS; j++) {
    const uint64_t g0 = 2 * (t * kTile + j * 64 + lane);
#pragma unroll
    for (int s = 0; s < S; s++) {
      if (MODE == 0 || ((used >> s) & 1u))
        ld_u64_pair<VEC, NTL, GUARD>(a.match + s * a.stride, g0, G, v[j][0][s], v[j][1][s]);
      else
        v[j][0][s] = v[j][1][s] = 0;  // no group of the wave has a voter here
    }
    if (a.learner) ld_mask_pair<MT, VEC, GUARD>(a.learner, g0, G, ml[j][0], ml[j][1]);
    else ml[j][0] = ml[j][1] = 0;
    if (a.voted) {
      ld_mask_pair<MT, VEC, GUARD>(a.voted, g0, G, vd[j][0], vd[j][1]);
      if (a.granted) ld_mask_pair<MT, VEC, GUARD>(a.granted, g0, G, gr[j][0], gr[j][1]);
      else gr[j][0] = gr[j][1] = 0;
    } else {
      vd[j][0] = vd[j][1] = gr[j][0] = gr[j][1] = 0;
    }
  }
  // ---- prefetch the next tile's voter masks ----
  if constexpr (MODE >= 1) {
    if (tn < ntiles) {
      if (VEC && tn < nfull) cv_masks<MT, MODE, PAIRS, VEC, false>(a, tn, lane, mi_n, mo_n);
      else cv_masks<MT, MODE, PAIRS, VEC, true>(a, tn, lane, mi_n, mo_n);
    }
  }
  // ---- compute + store ----
#pragma unroll
  for (int j = 0; j < PAIRS; j++) {
    const uint64_t g0 = 2 * (t * kTile + j * 64 + lane);
    uint64_t c[2];
    uint32_t vt[2], gc[2], rc[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t inc = mi[j][h] & kFull, out = mo[j][h] & kFull, lrn = ml[j][h] & kFull;
      const uint32_t vv = vd[j][h] & kFull, gg = gr[j][h] & kFull;
      eval_group<S, MODE>(v[j][h], inc, out, lrn, vv, gg, c[h], vt[h], gc[h], rc[h]);
      if (want_stats && (!GUARD || g0 + h < G)) {
        st.groups += 1;
        st.inf += (c[h] == kInf);
        st.sum += (c[h] == kInf) ? 0 : c[h];
        st.zero += (c[h] == 0);
        st.won += (vt[h] == kVoteWon);
        st.lost += (vt[h] == kVoteLost);
        st.pend += (vt[h] == kVotePending);
        st.gr += gc[h];
        st.rj += rc[h];
        st.viol += ((lrn & (inc | out)) != 0);
        const uint64_t tag = static_cast<uint64_t>(vt[h] | (gc[h] << 2) | (rc[h] << 7)) << 52;
        st.csum += mix64(((a.goff + g0 + h) * kPhi) ^ c[h] ^ tag);
      }
    }
    if (a.commit) st_u64_pair<VEC, NTS, GUARD>(a.commit, g0, G, c[0], c[1]);
    if (a.vote) st_u8_pair<VEC, NTS, GUARD>(a.vote, g0, G, vt[0], vt[1]);
    if (a.gcount) st_u8_pair<VEC, NTS, GUARD>(a.gcount, g0, G, gc[0], gc[1]);
    if (a.rcount) st_u8_pair<VEC, NTS, GUARD>(a.rcount, g0, G, rc[0], rc[1]);
  }
}

#ifndef QE_JOINT_MIN_WAVES
#define QE_JOINT_MIN_WAVES 1  // min waves per SIMD requested for the joint kernel
#endif
template <int S, int MODE, typename MT, int PAIRS, bool VEC, bool NTL, bool NTS>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kBlock),
                          amdgpu_waves_per_eu(MODE == 2 ? QE_JOINT_MIN_WAVES : 1)))
void k_commit_vote(CVArgs a) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const uint64_t nwaves = (static_cast<uint64_t>(gridDim.x) * kBlock) >> 6;
  const uint64_t npairs = (a.G + 1) >> 1;
  constexpr uint64_t kTile = 64ull * PAIRS;
  const uint64_t ntiles = (npairs + kTile - 1) / kTile;
  const uint64_t nfull = a.G / (2 * kTile);  // tiles wholly inside [0, G)
  const bool want_stats = a.stats != nullptr;

  CVStats st;
  uint32_t mi[PAIRS][2] = {}, mo[PAIRS][2] = {};
  if constexpr (MODE >= 1) {
    if (wave < ntiles) {
      if (VEC && wave < nfull) cv_masks<MT, MODE, PAIRS, VEC, false>(a, wave, lane, mi, mo);
      else cv_masks<MT, MODE, PAIRS, VEC, true>(a, wave, lane, mi, mo);
    }
  }
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    uint32_t mi_n[PAIRS][2], mo_n[PAIRS][2];
    if (VEC && t < nfull)
      cv_tile<S, MODE, MT, PAIRS, VEC, NTL, NTS, false>(a, t, lane, want_stats, st, mi, mo,
                                                        t + nwaves, ntiles, nfull, mi_n, mo_n);
    else
      cv_tile<S, MODE, MT, PAIRS, VEC, NTL, NTS, true>(a, t, lane, want_stats, st, mi, mo,
                                                       t + nwaves, ntiles, nfull, mi_n, mo_n);
    if constexpr (MODE >= 1) {
#pragma unroll
      for (int j = 0; j < PAIRS; j++)
#pragma unroll
        for (int h = 0; h < 2; h++) {
          mi[j][h] = mi_n[j][h];
          mo[j][h] = mo_n[j][h];
        }
    }
  }
  if (want_stats) {
    uint64_t cnt[C_N] = {st.groups, st.inf, st.sum, st.zero, st.won, st.lost,
                         st.pend,   st.gr,  st.rj,  st.viol, st.csum};
    const int idx[C_N] = {QE_STAT_GROUPS,     QE_STAT_COMMIT_INF,   QE_STAT_COMMIT_SUM,
                          QE_STAT_COMMIT_ZERO, QE_STAT_VOTE_WON,    QE_STAT_VOTE_LOST,
                          QE_STAT_VOTE_PENDING, QE_STAT_GRANTED,    QE_STAT_REJECTED,
                          QE_STAT_INVARIANT_VIOLATIONS, QE_STAT_CHECKSUM};
    block_stats_add<C_N, kBlock>(cnt, idx, a.stats);
  }
}

// ---------------------------------------------------------------------------
// Lockstep replication round (qe_replication_round).
// ---------------------------------------------------------------------------
struct RArgs {
  uint64_t G, goff, stride;
  uint64_t *match, *next, *committed;
  const uint64_t *term_start, *last_index, *resp;
  const void *inc, *out, *resp_mask, *read_acks;
  uint8_t *read_ok, *adv;
  uint64_t *stats;
  uint32_t chunk;  // k_repl_stream: tiles per wave chunk
};

enum { R_GROUPS, R_SUM, R_ADV, R_READ, R_VIOL, R_CSUM, R_N };

template <int S, bool JOINT, bool MASKED, typename MT, bool VEC, bool NT, bool GUARD>
__device__ __forceinline__ void repl_tile(const RArgs &a, uint64_t t, int lane, bool want_stats,
                                          uint64_t (&cnt)[R_N]) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  const uint64_t G = a.G;
  const uint64_t g0 = 2 * (t * 64 + lane);
  uint32_t mi[2], mo[2], rm[2], ack[2];
  if (MASKED) ld_mask_pair<MT, VEC, GUARD>(a.inc, g0, G, mi[0], mi[1]);
  else mi[0] = mi[1] = kFull;
  if (JOINT) ld_mask_pair<MT, VEC, GUARD>(a.out, g0, G, mo[0], mo[1]);
  else mo[0] = mo[1] = 0;
  if (a.resp_mask) ld_mask_pair<MT, VEC, GUARD>(a.resp_mask, g0, G, rm[0], rm[1]);
  else rm[0] = rm[1] = 0;
  if (a.read_acks) ld_mask_pair<MT, VEC, GUARD>(a.read_acks, g0, G, ack[0], ack[1]);
  else ack[0] = ack[1] = 0;
  uint64_t ts[2], li[2], cm[2];
  ld_u64_pair<VEC, NT, GUARD>(a.term_start, g0, G, ts[0], ts[1]);
  ld_u64_pair<VEC, NT, GUARD>(a.last_index, g0, G, li[0], li[1]);
  ld_u64_pair<VEC, NT, GUARD>(a.committed, g0, G, cm[0], cm[1]);

  // Progress.MaybeUpdate on every responding slot (progress.go:144-153),
  // streamed slot by slot: read match/next/resp, update, write back.
  uint64_t sel[2][S];
#pragma unroll
  for (int s = 0; s < S; s++) {
    uint64_t m[2], n[2], r[2];
    ld_u64_pair<VEC, NT, GUARD>(a.match + s * a.stride, g0, G, m[0], m[1]);
    ld_u64_pair<VEC, NT, GUARD>(a.next + s * a.stride, g0, G, n[0], n[1]);
    ld_u64_pair<VEC, NT, GUARD>(a.resp + s * a.stride, g0, G, r[0], r[1]);
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const bool resp = (rm[h] >> s) & 1u;
      m[h] = (resp && m[h] < r[h]) ? r[h] : m[h];
      n[h] = (resp && n[h] < r[h] + 1) ? r[h] + 1 : n[h];
      sel[h][s] = m[h];
    }
    st_u64_pair<VEC, NT, GUARD>(a.match + s * a.stride, g0, G, m[0], m[1]);
    st_u64_pair<VEC, NT, GUARD>(a.next + s * a.stride, g0, G, n[0], n[1]);
  }

  uint32_t ro[2], adv[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t inc = mi[h] & kFull, out = mo[h] & kFull;
    const uint64_t mci = (!JOINT && !MASKED) ? select_fixed<S>(sel[h])
                                             : joint_committed<S>(sel[h], inc, out);
    // raftLog.maybeCommit with term(i)==Term <=> term_start<=i<=last_index
    adv[h] = (mci > cm[h] && mci >= ts[h] && mci <= li[h]) ? 1u : 0u;
    cm[h] = adv[h] ? mci : cm[h];
    const uint32_t acks = ack[h] & kFull;
    ro[h] = a.read_acks ? (joint_vote(inc, out, acks, acks) == kVoteWon) : 0u;
    if (want_stats && (!GUARD || g0 + h < G)) {
      cnt[R_GROUPS] += 1;
      cnt[R_SUM] += cm[h];
      cnt[R_ADV] += adv[h];
      cnt[R_READ] += ro[h];
      cnt[R_VIOL] += (mci > li[h]);
      const uint64_t tag = (static_cast<uint64_t>(ro[h]) << 62) | (static_cast<uint64_t>(adv[h]) << 61);
      cnt[R_CSUM] += mix64(((a.goff + g0 + h) * kPhi) ^ cm[h] ^ tag);
    }
  }
  st_u64_pair<VEC, NT, GUARD>(a.committed, g0, G, cm[0], cm[1]);
  if (a.read_ok) st_u8_pair<VEC, NT, GUARD>(a.read_ok, g0, G, ro[0], ro[1]);
  if (a.adv) st_u8_pair<VEC, NT, GUARD>(a.adv, g0, G, adv[0], adv[1]);
}

template <int S, bool JOINT, bool MASKED, typename MT, bool VEC, bool NT>
__global__ __launch_bounds__(kBlock) void k_replication(RArgs a) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const uint64_t nwaves = (static_cast<uint64_t>(gridDim.x) * kBlock) >> 6;
  const uint64_t npairs = (a.G + 1) >> 1;
  const uint64_t ntiles = (npairs + 63) / 64;
  const uint64_t nfull = a.G / 128;
  const bool want_stats = a.stats != nullptr;
  uint64_t cnt[R_N];
#pragma unroll
  for (int i = 0; i < R_N; i++) cnt[i] = 0;
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    if (VEC && t < nfull)
      repl_tile<S, JOINT, MASKED, MT, VEC, NT, false>(a, t, lane, want_stats, cnt);
    else
      repl_tile<S, JOINT, MASKED, MT, VEC, NT, true>(a, t, lane, want_stats, cnt);
  }
  if (want_stats) {
    const int idx[R_N] = {QE_STAT_GROUPS, QE_STAT_COMMIT_SUM, QE_STAT_COMMIT_ADVANCED,
                          QE_STAT_READ_RELEASED, QE_STAT_INVARIANT_VIOLATIONS, QE_STAT_CHECKSUM};
    block_stats_add<R_N, kBlock>(cnt, idx, a.stats);
  }
}

// ---------------------------------------------------------------------------
// Randomized election simulation (qe_election_steps).  Group state stays in
// registers across `steps` fused steps; ALU/RNG-bound.
// ---------------------------------------------------------------------------
struct EArgs {
  uint64_t G, goff;
  uint64_t *term;
  uint8_t *state;
  void *voted, *granted;
  const uint8_t *self_slot;
  const void *inc, *out, *learner;
  uint64_t seed, step0;
  uint32_t steps, p_drop, p_grant, flags, p_active;
  const void *sresp, *sgrant;
  const uint8_t *shup;
  uint64_t sstride;
  uint64_t *stats;
};

enum { E_GROUPS, E_ELEC, E_LEAD, E_DOWN, E_WON, E_LOST, E_PEND, E_GR, E_RJ, E_VIOL, E_CSUM, E_N };

// One TallyVotes with the invariant checks; counts into the
// per-lane 32-bit step counters.  JOINT = false: Voters[1] is empty for every
// group (no out mask), so JointConfig.VoteResult is the incoming half's
// MajorityConfig.VoteResult and the half-swap symmetry holds by construction.
template <bool JOINT>
__device__ __forceinline__ uint32_t elec_tally(uint32_t mi, uint32_t mo, uint32_t ml, uint32_t vd,
                                               uint32_t gr, uint32_t gbefore,
                                               uint32_t (&cnt)[E_N]) {
  if constexpr (!JOINT) mo = 0;
  const uint32_t voters = (mi | mo) & ~ml;
  const uint32_t gcn = popc(vd & gr & voters), rcn = popc(vd & ~gr & voters);
  const uint32_t res = JOINT ? joint_vote(mi, mo, vd, gr) : majority_vote(mi, vd, gr);
  const uint32_t sym = JOINT ? joint_vote(mo, mi, vd, gr) : res;
  const uint32_t n0 = popc(mi), n1 = JOINT ? popc(mo) : 0u;
  const bool won_ok = (n0 == 0 || popc(gr & vd & mi) >= n0 / 2 + 1) &&
                      (n1 == 0 || popc(gr & vd & mo) >= n1 / 2 + 1);
  cnt[E_VIOL] += (sym != res) + (res == kVoteWon && !won_ok) + (gcn < gbefore);
  cnt[E_GR] += gcn;
  cnt[E_RJ] += rcn;
  cnt[E_WON] += (res == kVoteWon);
  cnt[E_LOST] += (res == kVoteLost);
  cnt[E_PEND] += (res == kVotePending);
  return res;
}

// raft.campaign (raft/raft.go:785-803): PreVote -> becomePreCandidate (term
// kept), else becomeCandidate (term+1); votes reset; self-vote; a won
// (single-voter) tally moves on to the election / leadership.
template <bool JOINT>
__device__ __forceinline__ void elec_campaign(bool pre, uint32_t mi, uint32_t mo, uint32_t ml,
                                              uint32_t self, uint64_t &t, uint32_t &sta,
                                              uint32_t &vd, uint32_t &gr, uint32_t (&cnt)[E_N]) {
  bool go = true;
  if (pre) {
    sta = QE_STATE_PRE_CANDIDATE;
    vd = self;
    gr = self;
    go = elec_tally<JOINT>(mi, mo, ml, vd, gr, 0u, cnt) == kVoteWon;
  }
  if (go) {
    t += 1;
    sta = QE_STATE_CANDIDATE;
    vd = self;
    gr = self;
    cnt[E_ELEC] += 1;
    if (elec_tally<JOINT>(mi, mo, ml, vd, gr, 0u, cnt) == kVoteWon) {
      sta = QE_STATE_LEADER;
      cnt[E_LEAD] += 1;
    }
  }
}

// OPT: bit 0 PreVote, bit 1 CheckQuorum, bit 2 scripted responses, bit 3
// joint (an out mask is given) -- compile-time, so the plain simulation
// carries none of their branches.
template <int S, typename MT, int OPT>
__global__ __launch_bounds__(kBlock) void k_election(EArgs a) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  constexpr bool pre = (OPT & 1) != 0, cq = (OPT & 2) != 0, scripted = (OPT & 4) != 0;
  constexpr bool joint = (OPT & 8) != 0;
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const uint64_t nthreads = static_cast<uint64_t>(gridDim.x) * kBlock;
  uint64_t cnt[E_N];
#pragma unroll
  for (int i = 0; i < E_N; i++) cnt[i] = 0;
  const MT *incp = static_cast<const MT *>(a.inc), *outp = static_cast<const MT *>(a.out);
  const MT *lrnp = static_cast<const MT *>(a.learner);
  MT *vdp = static_cast<MT *>(a.voted), *grp = static_cast<MT *>(a.granted);
  const MT *srp = static_cast<const MT *>(a.sresp), *sgp = static_cast<const MT *>(a.sgrant);

  for (uint64_t g = tid; g < a.G; g += nthreads) {
    const uint64_t gid = a.goff + g;
    const uint32_t mi = incp ? (incp[g] & kFull) : kFull;
    const uint32_t mo = (joint && outp) ? (outp[g] & kFull) : 0u;
    const uint32_t ml = lrnp ? (lrnp[g] & kFull) : 0u;
    const uint32_t sidx = a.self_slot[g] % S;
    const uint32_t self = 1u << sidx;
    const uint32_t voters = mi | mo;
    const bool promotable = (self & voters) != 0 && (self & ml) == 0;
    uint64_t t = a.term[g];
    uint32_t sta = a.state[g];
    uint32_t vd = vdp[g] & kFull, gr = grp[g] & kFull;
    // campaign sends (pre)vote requests to Voters.IDs() (raft.go:813-834)
    const uint32_t peers = voters & ~self;
    // counter-based RNG key (oracle/quorum_oracle.c elec_gkey), once per group
    const uint64_t gk64 = mix64(a.seed + gid * kPhi) ^ 0x6A09E667F3BCC909ull;
    const uint32_t gkey = static_cast<uint32_t>(gk64) ^ static_cast<uint32_t>(gk64 >> 32);
    // 32-bit step counters per chunk of <= 2^24 steps (no overflow: at most
    // 2 tallies x 16 grants per step), flushed into the 64-bit totals
    for (uint32_t k0 = 0; promotable && k0 < a.steps; k0 += (1u << 24)) {
      const uint32_t kend = a.steps - k0 < (1u << 24) ? a.steps : k0 + (1u << 24);
      uint32_t c32[E_N];
#pragma unroll
      for (int i = 0; i < E_N; i++) c32[i] = 0;
      for (uint32_t k = k0; k < kend; k++) {
        const uint64_t step = a.step0 + k;
        const uint32_t hb = gkey + static_cast<uint32_t>(step) * 0x9E3779B1u;
        uint32_t resp = 0, val = 0;
        bool hup = false;
        if constexpr (scripted) {
          const uint64_t so = static_cast<uint64_t>(k) * a.sstride + g;
          resp = srp[so] & peers;
          val = sgp[so] & resp;
          hup = a.shup && a.shup[so] != 0;
        }
        // One set of slot draws per step, d = fmix32(gkey + step*C1 + s*C2
        // (+ C3 for a leader's CheckQuorum round)) (oracle elec_draw), for
        // the S - 1 slots other than self (its draw is never used): a wave
        // mixing leaders and candidates hashes once, not once per branch.
        const bool ldr = cq && sta == QE_STATE_LEADER;
        const bool camp = !ldr && (sta == QE_STATE_FOLLOWER || sta == QE_STATE_LEADER || hup);
        if constexpr (!scripted) {
          if (!camp) {
            const uint32_t off = ldr ? 0x27D4EB2Fu : 0u;
#pragma unroll
            for (int j = 0; j + 1 < S; j++) {
              const uint32_t s = static_cast<uint32_t>(j) + (static_cast<uint32_t>(j) >= sidx ? 1u : 0u);
              const uint32_t d = fmix32(hb + s * 0x85EBCA77u + off);
              const bool peer = ((peers >> s) & 1u) != 0;
              const uint32_t lo = d & 0xFFFFu;
              // a leader: heard from within the election timeout (p_active);
              // a candidate: the response delivered (p_drop) and granted
              const bool deliver = peer && (ldr ? lo < a.p_active : lo >= a.p_drop);
              resp |= deliver ? (1u << s) : 0u;
              val |= (deliver && (d >> 16) < a.p_grant) ? (1u << s) : 0u;
            }
          }
        }
        if (ldr) {
          // CheckQuorum round (raft.go:997-1018)
          const uint32_t recent = resp | self;
          const uint32_t present = voters & ~ml;
          const bool qa = (joint ? joint_vote(mi, mo, present, recent & present)
                                 : majority_vote(mi, present, recent & present)) == kVoteWon;
          const bool qb = joint ? joint_vote(mo, mi, present, recent & present) == kVoteWon : qa;
          c32[E_VIOL] += (qa != qb);
          if (!qa) {
            sta = QE_STATE_FOLLOWER;
            c32[E_DOWN] += 1;
          }
        } else if (camp) {
          elec_campaign<joint>(pre, mi, mo, ml, self, t, sta, vd, gr, c32);
        } else {
          const uint32_t gbefore = popc(gr & vd & ~ml & voters);
          const uint32_t fresh = resp & ~vd;  // RecordVote: first vote sticks
          vd |= fresh;
          gr |= fresh & val;
          const uint32_t res = elec_tally<joint>(mi, mo, ml, vd, gr, gbefore, c32);
          if (res == kVoteWon) {
            if (sta == QE_STATE_PRE_CANDIDATE) {
              elec_campaign<joint>(false, mi, mo, ml, self, t, sta, vd, gr, c32);
            } else {
              sta = QE_STATE_LEADER;
              c32[E_LEAD] += 1;
            }
          } else if (res == kVoteLost) {
            sta = QE_STATE_FOLLOWER;
            c32[E_DOWN] += 1;
          }
        }
      }
      c32[E_GROUPS] = kend - k0;
#pragma unroll
      for (int i = 0; i < E_N; i++) cnt[i] += c32[i];
    }
    a.term[g] = t;
    a.state[g] = static_cast<uint8_t>(sta);
    vdp[g] = static_cast<MT>(vd);
    grp[g] = static_cast<MT>(gr);
    const uint64_t tag = (static_cast<uint64_t>(sta) << 62) | (static_cast<uint64_t>(vd) << 40) |
                         (static_cast<uint64_t>(gr) << 24);
    cnt[E_CSUM] += mix64((gid * kPhi) ^ t ^ tag);
  }
  if (a.stats) {
    const int idx[E_N] = {QE_STAT_GROUPS,    QE_STAT_ELECTIONS,  QE_STAT_LEADERS,
                          QE_STAT_STEPDOWNS, QE_STAT_VOTE_WON,   QE_STAT_VOTE_LOST,
                          QE_STAT_VOTE_PENDING, QE_STAT_GRANTED, QE_STAT_REJECTED,
                          QE_STAT_INVARIANT_VIOLATIONS, QE_STAT_CHECKSUM};
    block_stats_add<E_N, kBlock>(cnt, idx, a.stats);
  }
}

// ---------------------------------------------------------------------------
// Progress state machine (qe_progress_step / qe_progress_send).  Per-peer
// state lives in slot-SoA rows, the Inflights ring in [S][F][stride] rows
// (F = MaxInflightMsgs, entry-major).
// ---------------------------------------------------------------------------
struct PArgs {
  uint64_t G, goff, stride;
  uint32_t F, R;
  uint64_t *match, *next, *pending;
  uint32_t *pw;  // [S][stride] packed per-peer words (QE_PW_*)
  uint32_t *ilo, *ihi;  // Inflights rings, lane-major [S][stride][FP] (ABI 4)
  uint16_t *infl16;     // ABI 8: the 16-bit form [S][stride][8], or null
  uint32_t FP;          // QE_RING_PITCH(F)
  uint64_t *committed;
  const uint64_t *term_start, *first_index, *last_index, *snap_index;
  const uint64_t *run_first, *run_term;
  const uint8_t *run_count;
  const void *inc, *out, *tracked;
  const uint8_t *self_slot;
  uint8_t *transferee;  // rw (ABI 5: MsgTransferLeader)
  uint32_t max_ents;
  // ReadIndex queue (ABI 5): acks [G][QE_READ_QUEUE] mask-typed, head, count;
  // ABI 7: capacity (host-normalised: >= QE_READ_QUEUE), the overflow ring
  // [G][read_cap] mask-typed, the request keys [G][read_cap]
  void *read_acks;
  uint32_t *read_head;
  uint8_t *read_count;
  uint32_t read_cap;
  void *read_ovf;
  uint64_t *read_keys;
  // step messages and outputs
  const uint8_t *mtype;
  const uint64_t *mindex, *mhint, *mlogterm;
  void *sent, *snap, *tnow;
  uint8_t *bcast, *msg_count;
  uint64_t *msg_index, *acct;
  const uint32_t *read_ctx;
  uint8_t *read_released, *term_commit;
  uint64_t *term_commit_index;
  uint64_t *stats;
  // read index (qe_read_index)
  const uint8_t *ri_request;
  const uint64_t *ri_key;  // ABI 7: request keys (NULL: no duplicate check)
  uint8_t *ri_result;
  uint32_t *ri_ctx;
  uint64_t *ri_index;
  uint32_t lease_based;
  // send
  const void *want;
  uint32_t send_if_empty;
  uint32_t chunk;  // k_progress_send: tiles per wave chunk
  // check quorum
  uint8_t *qactive;
  // propose (qe_propose, ABI 6)
  const uint32_t *prop_n;
  const uint64_t *prop_payload;
  uint32_t max_cc, prop_flags;
  uint64_t cc_stride;
  const uint8_t *cc_count, *cc_leave;
  const uint32_t *cc_pos, *cc_size;
  const uint64_t *applied;
  uint64_t *pci, *unc;
  uint64_t max_unc;
  uint8_t *prop_result, *cc_refused;
  uint64_t *last_index_rw;
  // heartbeat (qe_heartbeat, ABI 6)
  uint64_t *hb_commit;
  uint32_t *hb_ctx;
  // switchToConfig (qe_switch_config, ABI 7)
  const uint8_t *sw_switched;
  uint8_t *sw_result;
  // becomeLeader (qe_become_leader, ABI 7)
  const uint8_t *bl_elected;
  const uint64_t *bl_term;
  uint32_t bl_flags;
  uint64_t *bl_pci, *bl_unc;
  uint8_t *bl_result;
};

struct PR {
  uint64_t match, next, pending;
  uint32_t state, probe_sent, recent_active, start, count;
  uint32_t reset;  // ResetState ran: PendingSnapshot must be written back
  uint32_t rep;    // the word's ring representation bits (QE_PW_RING_MASK)
};

// The packed per-peer word (include/etcd_quorum.h QE_PW_*).
__device__ __forceinline__ void pr_unpack(PR &p, uint32_t w) {
  p.state = w & QE_PF_STATE;
  p.probe_sent = (w >> 2) & 1u;
  p.recent_active = (w >> 3) & 1u;
  p.start = (w >> QE_PW_START_SHIFT) & 0xFFu;
  p.count = (w >> QE_PW_COUNT_SHIFT) & 0xFFu;
  p.rep = w & QE_PW_RING_MASK;
}
__device__ __forceinline__ uint32_t pr_pack(const PR &p) {
  return p.state | (p.probe_sent ? QE_PF_PROBE_SENT : 0u) |
         (p.recent_active ? QE_PF_RECENT_ACTIVE : 0u) | (p.start << QE_PW_START_SHIFT) |
         (p.count << QE_PW_COUNT_SHIFT) | p.rep;
}

__device__ __forceinline__ void pr_reset(PR &p, uint32_t st) {  // progress.go:84-90
  p.reset = 1;
  p.probe_sent = 0;
  p.pending = 0;
  p.state = st;
  p.count = 0;
  p.start = 0;
  p.rep = 0;  // an empty ring: epoch 0, not wide (canonical)
}
__device__ __forceinline__ void pr_become_probe(PR &p) {  // progress.go:112-125
  if (p.state == QE_PR_SNAPSHOT) {
    const uint64_t ps = p.pending;
    pr_reset(p, QE_PR_PROBE);
    const uint64_t x = p.match + 1, y = ps + 1;
    p.next = x > y ? x : y;
  } else {
    pr_reset(p, QE_PR_PROBE);
    p.next = p.match + 1;
  }
}
__device__ __forceinline__ void pr_become_replicate(PR &p) {  // progress.go:127-131
  pr_reset(p, QE_PR_REPLICATE);
  p.next = p.match + 1;
}
__device__ __forceinline__ bool pr_paused(const PR &p, uint32_t F) {  // progress.go:201-212
  // Probe: ProbeSent; Replicate: Inflights.Full(); Snapshot: always (as
  // selects, not a branch chain)
  const bool probe = p.state == QE_PR_PROBE, repl = p.state == QE_PR_REPLICATE;
  return probe ? p.probe_sent != 0 : (repl ? p.count == F : true);
}

// raftLog.findConflictByTerm (raft/log.go:147-168) on the term-run model,
// over the group's run table held in registers: walking down index by index
// while term(index) > t is the same as jumping to the end of the run below,
// run by run (term(i) = term of the highest run r with run_first[r] <= i,
// 0 below run 0 or above lastIndex, as oracle/quorum_oracle.c orc_log_term).
template <int RM>
__device__ __forceinline__ uint64_t find_conflict_by_term(const uint64_t (&rf)[RM],
                                                          const uint64_t (&rt)[RM], uint32_t nr,
                                                          uint64_t li, uint64_t index,
                                                          uint64_t t) {
  if (index > li || nr == 0) return index;
  uint64_t cur = index;
  bool done = false;
#pragma unroll
  for (int r = RM - 1; r >= 0; r--) {
    if (!done && static_cast<uint32_t>(r) < nr && rf[r] <= cur) {
      if (rt[r] <= t) done = true;
      else cur = rf[r] - 1;
    }
  }
  return cur;
}

template <int S, bool MASKED, bool JOINT>
__device__ __forceinline__ uint64_t mci_of(const uint64_t (&vals)[S], uint32_t inc, uint32_t out) {
  uint64_t v[S];
#pragma unroll
  for (int s = 0; s < S; s++) v[s] = vals[s];
  if constexpr (!MASKED && !JOINT) return select_fixed<S>(v);
  else return joint_committed<S>(v, inc, out);
}

enum { P_GROUPS, P_SUM, P_ADV, P_VIOL, P_READ, P_CSUM, P_N };
enum { Q_GROUPS, Q_SUM, Q_ADV, Q_CSUM, Q_N };  // k_propose, k_switch_config

// k_progress_step: qe_progress.hpp

// k_progress_send: qe_progress.hpp

// ---------------------------------------------------------------------------
// Small bitmap kernels: QuorumActive, RecordVote.
// ---------------------------------------------------------------------------
template <typename MT>
__global__ __launch_bounds__(kBlock) void k_quorum_active(uint64_t G, uint32_t full,
                                                          const void *inc, const void *out,
                                                          const void *learner,
                                                          const void *recent, uint8_t *active) {
  const MT *pi = static_cast<const MT *>(inc), *po = static_cast<const MT *>(out);
  const MT *pl = static_cast<const MT *>(learner), *pr = static_cast<const MT *>(recent);
  for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; g < G;
       g += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint32_t mi = pi ? (pi[g] & full) : full, mo = po ? (po[g] & full) : 0u;
    const uint32_t ml = pl ? (pl[g] & full) : 0u;
    const uint32_t present = (mi | mo | ml) & ~ml;  // votes[id] for non-learners
    const uint32_t ra = pr[g] & present;
    active[g] = joint_vote(mi, mo, present, ra) == kVoteWon;
  }
}

template <typename MT>
__global__ __launch_bounds__(kBlock) void k_vote_result(uint64_t G, uint32_t full,
                                                        const void *inc, const void *out,
                                                        const void *voted, const void *granted,
                                                        uint8_t *vote) {
  const MT *pi = static_cast<const MT *>(inc), *po = static_cast<const MT *>(out);
  const MT *pv = static_cast<const MT *>(voted), *pg = static_cast<const MT *>(granted);
  for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; g < G;
       g += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint32_t mi = pi ? (pi[g] & full) : full, mo = po ? (po[g] & full) : 0u;
    const uint32_t vd = pv ? (pv[g] & full) : 0u;
    const uint32_t gr = (pv && pg) ? (pg[g] & full) : 0u;
    vote[g] = static_cast<uint8_t>(joint_vote(mi, mo, vd, gr));
  }
}

template <typename MT>
__global__ __launch_bounds__(kBlock) void k_record_votes(uint64_t G, uint32_t full, void *voted,
                                                         void *granted, const void *resp,
                                                         const void *value) {
  MT *pv = static_cast<MT *>(voted), *pg = static_cast<MT *>(granted);
  const MT *pr = static_cast<const MT *>(resp), *px = static_cast<const MT *>(value);
  for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; g < G;
       g += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint32_t vd = pv[g], fresh = pr[g] & full & ~vd;
    pv[g] = static_cast<MT>(vd | fresh);
    pg[g] = static_cast<MT>(pg[g] | (fresh & px[g]));
  }
}

// ---------------------------------------------------------------------------
// Synthetic generator (bit-identical with oracle/quorum_oracle.c).
// ---------------------------------------------------------------------------
struct GArgs {
  uint64_t G, goff, stride;
  uint32_t S;
  uint64_t *match;
  void *inc, *out, *learner, *voted, *granted;
  qe_gen_params p;
};

__device__ __forceinline__ uint32_t rotl_s(uint32_t m, uint32_t r, uint32_t S) {
  const uint32_t full = (1u << S) - 1u;
  m &= full;
  if (r == 0) return m;
  return ((m << r) | (m >> (S - r))) & full;
}

template <typename MT>
__global__ __launch_bounds__(kBlock) void k_gen(GArgs a) {
  const uint32_t S = a.S;
  const uint32_t full = (1u << S) - 1u;
  for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; g < a.G;
       g += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint64_t gid = a.goff + g;
    const uint64_t hb = hash4(a.p.seed, gid, 0xFFFFu, 0);
    uint32_t mi, mo, ml;
    if (a.p.mask_mode == 0 || a.p.mask_mode == 2) {
      uint32_t ni = a.p.n_inc ? a.p.n_inc : S;
      if (ni > S) ni = S;
      uint32_t no = a.p.n_out > S ? S : a.p.n_out;
      if (no == 0) {
        mi = (1u << ni) - 1u;
        mo = 0;
        ml = full & ~mi;
      } else {
        const uint32_t omin = (ni + no > S) ? ni + no - S : 0;
        const uint32_t omax = ni < no ? ni : no;
        const uint64_t okey = a.p.mask_mode == 2 ? (gid >> 20) : (hb >> 8);
        const uint32_t o = omin + static_cast<uint32_t>(okey % (omax - omin + 1));
        const uint32_t uni = ni + no - o;
        mi = (1u << ni) - 1u;
        mo = ((1u << no) - 1u) << (ni - o);
        ml = full & ~((1u << uni) - 1u);
      }
      const uint32_t r = a.p.mask_mode == 2 ? 0u : static_cast<uint32_t>((hb >> 16) % S);
      mi = rotl_s(mi, r, S);
      mo = rotl_s(mo, r, S);
      ml = rotl_s(ml, r, S);
    } else {
      const uint64_t hm = hash4(a.p.seed, gid, 0xFFFEu, 0);
      mi = static_cast<uint32_t>(hm) & full;
      mo = ((hm >> 48) & 3u) == 0 ? 0u : (static_cast<uint32_t>(hm >> 16) & full);
      ml = static_cast<uint32_t>(hm >> 32) & full;
      if (((hm >> 50) & 7u) != 0) ml &= ~(mi | mo);
    }
    if (a.inc) static_cast<MT *>(a.inc)[g] = static_cast<MT>(mi);
    if (a.out) static_cast<MT *>(a.out)[g] = static_cast<MT>(mo);
    if (a.learner) static_cast<MT *>(a.learner)[g] = static_cast<MT>(ml);
    if (a.match) {
      for (uint32_t s = 0; s < S; s++) {
        const uint64_t h = hash4(a.p.seed, gid, s, 1);
        uint64_t v;
        if (static_cast<uint32_t>(h & 0xFFFFu) < a.p.p_absent_q16) v = 0;
        else if (a.p.dist == 0) v = (hb >> 2) + ((h >> 40) & 0xFFFFu);
        else if (a.p.dist == 1) v = h >> 1;
        else v = (h >> 40) & 3u;
        a.match[s * a.stride + g] = v;
      }
    }
    if (a.voted || a.granted) {
      uint32_t vd = 0, gr = 0;
      for (uint32_t s = 0; s < S; s++) {
        const uint64_t h = hash4(a.p.seed, gid, s, 2);
        if (static_cast<uint32_t>(h & 0xFFFFu) < a.p.p_voted_q16) {
          vd |= 1u << s;
          if (static_cast<uint32_t>((h >> 16) & 0xFFFFu) < a.p.p_granted_q16) gr |= 1u << s;
        }
      }
      if (a.voted) static_cast<MT *>(a.voted)[g] = static_cast<MT>(vd);
      if (a.granted) static_cast<MT *>(a.granted)[g] = static_cast<MT>(gr);
    }
  }
}

}  // namespace qe
