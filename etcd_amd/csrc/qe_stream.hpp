// qe_stream.hpp — software-pipelined qe_commit_vote ("stream" kernel).
//
// One group per lane, tiles of 64 groups.  Each wave owns a contiguous chunk
// of up to TPW tiles.  Every global access goes through a per-tile buffer
// descriptor whose num_records clips the ragged last tile, so the last tile
// needs no guarded code path, and a slot the lane's group does not use is
// given an out-of-range offset, so its load is dropped by the bounds check:
// no memory traffic and no branch around the load.
//
// The chunk's voter masks (inc | out << 16) are staged into LDS once at the
// start of the chunk.  The next tile's row loads then depend only on an LDS
// read (lgkmcnt), not on a vector load queued behind the current tile's rows
// (vmcnt retires in order).  Two register sets, with the tile loop unrolled
// by two, keep tile t+1's rows in flight while tile t runs the selection
// network.  See DESIGN.md §3.
#pragma once
#include "qe_kernels.hpp"

namespace qe {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;  // > any num_records used here: load returns 0

// off when bit s of mask is set, else off | kOOB (dropped by the bounds
// check): a shift and one v_and_or_b32 instead of a compare and a select.
// off < 2^31.
__device__ __forceinline__ uint32_t bit_off(uint32_t mask, int s, uint32_t off) {
  return ((~mask << (31 - s)) & kOOB) | off;
}

__device__ __forceinline__ rsrc_t mk_rsrc(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, static_cast<int>(bytes),
                                           0x00020000);
}

template <typename MT>
__device__ __forceinline__ uint32_t bld_mask(const void *base, uint64_t tile0, uint32_t n,
                                             uint32_t lane) {
  const rsrc_t r = mk_rsrc(static_cast<const MT *>(base) + tile0, n * sizeof(MT));
  if constexpr (sizeof(MT) == 1)
    return __builtin_amdgcn_raw_buffer_load_b8(r, lane, 0, 0);
  else
    return __builtin_amdgcn_raw_buffer_load_b16(r, lane * 2, 0, 0);
}

// Per-tile inputs other than the voter masks.
struct STile {
  uint32_t lrn, vd, gr;
};

// Groups of tile t inside [0, G) (0 past the end: every access is dropped).
__device__ __forceinline__ uint32_t tile_n(uint64_t G, uint64_t t) {
  const uint64_t tile0 = t * 64;
  const uint64_t rem = G > tile0 ? G - tile0 : 0;
  return rem < 64 ? static_cast<uint32_t>(rem) : 64u;
}

// Optional array: a null pointer gets num_records 0, so its loads return 0
// and its stores are dropped, without a branch.
template <typename T>
__device__ __forceinline__ rsrc_t opt_rsrc(const T *p, uint64_t tile0, uint32_t n) {
  return p ? mk_rsrc(p + tile0, n * sizeof(T)) : mk_rsrc(p, 0);
}

template <typename MT>
__device__ __forceinline__ uint32_t ld_mask_r(rsrc_t r, uint32_t lane) {
  if constexpr (sizeof(MT) == 1)
    return __builtin_amdgcn_raw_buffer_load_b8(r, lane, 0, 0);
  else
    return __builtin_amdgcn_raw_buffer_load_b16(r, lane * 2, 0, 0);
}

template <int S, int MODE, typename MT, bool NTL>
__device__ __forceinline__ void st_issue(const CVArgs &a, uint64_t t, uint32_t lane, uint32_t use,
                                         uint32_t top, uint64_t (&v)[S], STile &x) {
  const uint64_t tile0 = t * 64;
  const uint32_t n = tile_n(a.G, t);
  const uint32_t off = lane * 8;
#pragma unroll
  for (int s = 0; s < S; s++) {
    const rsrc_t r = mk_rsrc(a.match + s * a.stride + tile0, n * 8);
    const uint32_t o = MODE == 0 ? off : bit_off(use, s, off);
#ifndef QE_STREAM_ALL_ROWS  // A/B knob: issue every slot row's load
    // slots >= top (scalar) hold no voter of the chunk: no instruction at all
    // (a fully dropped load still costs an issue slot of the memory path)
    if (MODE != 0 && static_cast<uint32_t>(s) >= top) {
      v[s] = 0;
      continue;
    }
#endif
    v[s] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, NTL ? 2 : 0));
  }
  const MT *lp = static_cast<const MT *>(a.learner), *vp = static_cast<const MT *>(a.voted);
  const MT *gp = a.voted ? static_cast<const MT *>(a.granted) : nullptr;
  x.lrn = ld_mask_r<MT>(opt_rsrc(lp, tile0, n), lane);
  x.vd = ld_mask_r<MT>(opt_rsrc(vp, tile0, n), lane);
  x.gr = ld_mask_r<MT>(opt_rsrc(gp, tile0, n), lane);
}

template <int S, int MODE, bool NTS>
__device__ __forceinline__ void st_finish(const CVArgs &a, uint64_t t, uint32_t lane,
                                          bool want_stats, uint32_t mio, uint32_t top,
                                          uint64_t (&v)[S], const STile &x, CVStats &st) {
  constexpr uint32_t kFull = (1u << S) - 1u;
  const uint64_t tile0 = t * 64;
  const uint32_t n = tile_n(a.G, t);
  const uint32_t inc = MODE == 0 ? kFull : (mio & kFull);
  const uint32_t out = MODE == 2 ? ((mio >> 16) & kFull) : 0u;
  const uint32_t lrn = x.lrn & kFull, vv = x.vd & kFull, gg = x.gr & kFull;
  uint64_t c;
  uint32_t vt, gc, rc;
  eval_group<S, MODE>(v, inc, out, lrn, vv, gg, c, vt, gc, rc, top);
  if (want_stats && lane < n) {
    st.groups += 1;
    st.inf += (c == kInf);
    st.sum += (c == kInf) ? 0 : c;
    st.zero += (c == 0);
    st.won += (vt == kVoteWon);
    st.lost += (vt == kVoteLost);
    st.pend += (vt == kVotePending);
    st.gr += gc;
    st.rj += rc;
    st.viol += ((lrn & (inc | out)) != 0);
    const uint64_t tag = static_cast<uint64_t>(vt | (gc << 2) | (rc << 7)) << 52;
    st.csum += mix64(((a.goff + tile0 + lane) * kPhi) ^ c ^ tag);
  }
  const int aux = NTS ? 2 : 0;
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, c), opt_rsrc(a.commit, tile0, n),
                                        lane * 8, 0, aux);
  __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(vt), opt_rsrc(a.vote, tile0, n), lane,
                                       0, aux);
  __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(gc), opt_rsrc(a.gcount, tile0, n),
                                       lane, 0, aux);
  __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(rc), opt_rsrc(a.rcount, tile0, n),
                                       lane, 0, aux);
}

#ifndef QE_STREAM_TPW
#define QE_STREAM_TPW 8  // tiles per wave chunk (LDS: 256 B per tile per wave)
#endif

#ifndef QE_STREAM_WAVES
#define QE_STREAM_WAVES 1  // min waves per SIMD requested (VGPR budget)
#endif

template <int S, int MODE, typename MT, bool NTL, bool NTS>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kBlock),
                          amdgpu_waves_per_eu(QE_STREAM_WAVES))) void k_cv_stream(CVArgs a) {
  constexpr int TPW = QE_STREAM_TPW;
  __shared__ uint32_t lds_m[kBlock / 64][TPW][64];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t ntiles = (a.G + 63) / 64;
  const uint32_t chunk = a.chunk;  // <= TPW (host-checked)
  const uint64_t t0 = (static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + w) * chunk;
  const uint32_t nt =
      t0 < ntiles ? static_cast<uint32_t>(ntiles - t0 < chunk ? ntiles - t0 : chunk) : 0u;
  const bool want_stats = a.stats != nullptr;
  CVStats st;
  uint32_t top = S;
  if (nt > 0) {
    // ---- stage the chunk's voter masks in LDS (one exposed latency per chunk) ----
    if constexpr (MODE >= 1) {
      uint32_t mv[TPW];
#pragma unroll
      for (int k = 0; k < TPW; k++) {
        const uint64_t tile0 = (t0 + k) * 64;
        const uint32_t n = tile_n(a.G, t0 + k);  // 0 past the chunk's end
        uint32_t m = bld_mask<MT>(a.inc, tile0, n, lane);
        if constexpr (MODE == 2) m |= bld_mask<MT>(a.out, tile0, n, lane) << 16;
        mv[k] = m;
      }
      uint32_t any = 0;
#pragma unroll
      for (int k = 0; k < TPW; k++) {
        lds_m[w][k][lane] = mv[k];
        any |= mv[k];
      }
      // slots >= top hold no voter of any group in the chunk (wave-uniform)
      top = __builtin_amdgcn_readfirstlane(
          32u - __builtin_clz(wave_or((any | (any >> 16)) & 0xFFFFu) | 1u));
    }
    auto use_of = [&](uint32_t k) -> uint32_t {
      if constexpr (MODE == 0) return 0u;
      const uint32_t m = lds_m[w][k][lane];
      return MODE == 2 ? ((m | (m >> 16)) & 0xFFFFu) : m;
    };
    auto mio_of = [&](uint32_t k) -> uint32_t {
      if constexpr (MODE == 0) return 0u;
      return lds_m[w][k][lane];
    };
    // Branch-free body: a tile index past the chunk (odd nt, or the
    // prefetch after the last tile) has n = 0, so its loads return 0, its
    // stores are dropped and it adds nothing to the statistics.
    const uint64_t tend = t0 + nt;
    auto tix = [&](uint32_t k) -> uint64_t { return t0 + k < tend ? t0 + k : ntiles; };
    uint64_t va[S], vb[S];
    STile xa, xb;
    st_issue<S, MODE, MT, NTL>(a, tix(0), lane, use_of(0), top, va, xa);
    for (uint32_t k = 0; k < nt; k += 2) {
      // tile k from set A while tile k+1 streams into set B, then swap
      st_issue<S, MODE, MT, NTL>(a, tix(k + 1), lane, use_of((k + 1) % TPW), top, vb, xb);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the compute
      st_finish<S, MODE, NTS>(a, tix(k), lane, want_stats, mio_of(k), top, va, xa, st);
      st_issue<S, MODE, MT, NTL>(a, tix(k + 2), lane, use_of((k + 2) % TPW), top, va, xa);
      __builtin_amdgcn_sched_barrier(0);
      st_finish<S, MODE, NTS>(a, tix(k + 1), lane, want_stats, mio_of((k + 1) % TPW), top, vb,
                              xb, st);
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

}  // namespace qe
