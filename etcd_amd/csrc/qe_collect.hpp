// qe_collect.hpp — qe_collect: the groups a batch step changed, as a dense
// list in ascending group order.
//
// The consumer is the host's Ready loop: raft only reports a HardState when
// it differs from the previous one (raft/node.go:571-573, newReady; the
// RawNode keeps prevHardSt, raft/rawnode.go:152-176), so after a batched
// round the host needs the groups whose commit advanced (the `adv` flags of
// qe_replication_round) and their new index -- not all G words over PCIe.
//
// Three passes over 4096-group chunks (256 threads x 16 flags):
//   count    per-chunk number of selected groups;
//   scan     one block: exclusive prefix of the chunk counts, and the total;
//   scatter  per chunk, in 16 rounds of 256 consecutive groups: the selected
//            groups of a round at consecutive positions (coalesced stores).
// The count pass reads flags as 16-B vectors when the array is 16-B aligned;
// values (optional) are gathered for the selected groups only.
// Measured (64M groups, half flagged, values gathered): 0.224 ms; with the
// scatter's gathers/stores under per-round exec-mask branches (each round's
// load waited on before its store) 0.285; writing each thread's 16-group
// run itself (strided stores) 1.14 ms; reading the scatter's flags a byte
// per round instead of staging them through LDS 0.31.
// Round 5 (profiles/r05/collect_ab.txt, rocprofv3 per kernel): the count
// pass as one wave per chunk with four loads per lane in flight 18.1 ->
// 16.0 us; the scan with each thread's counts held in registers (17.4 us)
// or staged through 128 KB of LDS (13.0 us) was slower than this one
// (10.3 us): a single block's scan is latency, not access width.
#pragma once
#include "qe_stream.hpp"

namespace qe {

constexpr uint32_t kCollectPer = 16;                    // flags per thread
constexpr uint32_t kCollectChunk = kBlock * kCollectPer;  // groups per block

__device__ __forceinline__ uint32_t collect_bits(const uint8_t *flags, uint64_t G, uint64_t g,
                                                 bool vec) {
  // bit i: flag g + i is set
  uint32_t m = 0;
  if (vec && g + kCollectPer <= G) {
    const uint4 v = *reinterpret_cast<const uint4 *>(flags + g);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int b = 0; b < 4; b++) m |= ((w[k] >> (8 * b)) & 0xFFu) ? (1u << (4 * k + b)) : 0u;
  } else {
#pragma unroll
    for (uint32_t i = 0; i < kCollectPer; i++)
      m |= (g + i < G && flags[g + i] != 0) ? (1u << i) : 0u;
  }
  return m;
}

// Count: one wave per chunk (four chunks per block, no block barrier); lane
// l holds groups [16 l, 16 l + 16) of each of the chunk's four 1024-group
// quarters, so a lane's four 16-B loads are independent and in flight
// together.  Nonzero bytes are counted four to a word: ((w & 0x7F..) +
// 0x7F..) | w has the high bit of every nonzero byte set.
constexpr uint32_t kCountWaves = kBlock / 64;  // chunks per count block

__device__ __forceinline__ uint32_t nz_bytes(uint32_t w) {
  return __builtin_popcount((((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u);
}

__global__ __launch_bounds__(kBlock) void k_collect_count(const uint8_t *flags, uint64_t G, bool vec,
                                                          uint64_t nb, uint32_t *counts) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kCountWaves + (threadIdx.x >> 6);
  if (b >= nb) return;  // (wave-uniform; no barrier below)
  const uint64_t base = b * kCollectChunk;
  uint32_t c = 0;
  if (vec && base + kCollectChunk <= G) {  // a full chunk, 16-B aligned
    uint4 v[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; q++)
      v[q] = *reinterpret_cast<const uint4 *>(flags + base + (q * 64 + lane) * kCollectPer);
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) c += nz_bytes(v[q].x) + nz_bytes(v[q].y) + nz_bytes(v[q].z) + nz_bytes(v[q].w);
  } else {
#pragma unroll
    for (uint32_t q = 0; q < 4; q++)
      c += __builtin_popcount(collect_bits(flags, G, base + (q * 64 + lane) * kCollectPer, vec));
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if (lane == 0) counts[b] = c;
}

// One block: offsets[b] = sum of counts[0..b), *out_count = the total.
// Thread t owns the contiguous range [t*per, (t+1)*per) of the chunk
// counts; a wave scan (shuffles, no barriers) and one block step over the 16
// wave totals replace the barrier-per-step Hillis-Steele scan (28 us -> a
// few us for 16K chunks: it was the second-longest part of qe_collect).
__global__ __launch_bounds__(1024) void k_collect_scan(const uint32_t *counts, uint64_t nb,
                                                       uint64_t *offsets, uint64_t *out_count) {
  __shared__ uint64_t wtot[16];
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  // per: a multiple of 4, so a thread's range is 16-byte aligned and read
  // as uint4 loads (the counts array starts 16-byte aligned: the scratch is
  // 8-byte aligned and the counts follow nb u64 offsets -- see qe_collect)
  const uint64_t per = ((nb + 1023) / 1024 + 3) & ~3ull;
  const uint64_t b0 = t * per < nb ? t * per : nb, b1 = b0 + per < nb ? b0 + per : nb;
  const bool vec = (reinterpret_cast<uintptr_t>(counts) & 15u) == 0;
  uint64_t s = 0;
  if (vec) {
    uint64_t b = b0;
    for (; b + 4 <= b1; b += 4) {
      const uint4 v = *reinterpret_cast<const uint4 *>(counts + b);
      s += static_cast<uint64_t>(v.x) + v.y + v.z + v.w;
    }
    for (; b < b1; b++) s += counts[b];
  } else {
    for (uint64_t b = b0; b < b1; b++) s += counts[b];
  }
  uint64_t inc = s;  // inclusive scan of the thread sums within the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(inc, d, 64);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  uint64_t before = 0, all = 0;
#pragma unroll
  for (uint32_t k = 0; k < 16; k++) {
    before += k < w ? wtot[k] : 0ull;
    all += wtot[k];
  }
  uint64_t run = before + inc - s;
  uint64_t b = b0;
  if (vec && (reinterpret_cast<uintptr_t>(offsets) & 15u) == 0) {
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    for (; b + 4 <= b1; b += 4) {
      const uint4 v = *reinterpret_cast<const uint4 *>(counts + b);
      const uint64_t o1 = run + v.x, o2 = o1 + v.y, o3 = o2 + v.z;
      *reinterpret_cast<u64x2 *>(offsets + b) = u64x2{run, o1};
      *reinterpret_cast<u64x2 *>(offsets + b + 2) = u64x2{o2, o3};
      run = o3 + v.w;
    }
  }
  for (; b < b1; b++) {
    offsets[b] = run;
    run += counts[b];
  }
  if (t == 1023) *out_count = all;
}

// Scatter: the chunk is walked in kCollectPer rounds of kBlock consecutive
// groups (thread t takes group base + r*kBlock + t), so the selected groups
// of a round land at consecutive positions in lane order: a wave's stores
// are one contiguous run (ballot + mbcnt for the rank inside the wave, the
// waves' counts through LDS for the block), not 16-entry runs per thread.
__global__ __launch_bounds__(kBlock) void k_collect_scatter(const uint8_t *flags, uint64_t G,
                                                            bool vec, uint64_t goff,
                                                            const uint64_t *perm,
                                                            const uint64_t *values,
                                                            const uint64_t *offsets,
                                                            uint64_t *out_groups,
                                                            uint64_t *out_values) {
  __shared__ uint32_t wcnt[kCollectPer][kBlock / 64];
  __shared__ uint32_t lflag[kCollectChunk / 4];  // the chunk's flags, a byte each
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kCollectChunk;
  // the chunk's flags: one 16-B load per thread (full, aligned chunks), then
  // read back round-major from LDS
  const bool full = vec && base + kCollectChunk <= G;  // block-uniform
  if (full) {
    const uint4 v = *reinterpret_cast<const uint4 *>(flags + base + tid * kCollectPer);
    *reinterpret_cast<uint4 *>(&lflag[tid * 4]) = v;
    __syncthreads();
  }
  const uint8_t *l8 = reinterpret_cast<const uint8_t *>(lflag);
  bool f[kCollectPer];
  uint32_t rank[kCollectPer];
#pragma unroll
  for (uint32_t r = 0; r < kCollectPer; r++) {
    const uint64_t g = base + r * kBlock + tid;
    f[r] = full ? l8[r * kBlock + tid] != 0 : (g < G && flags[g] != 0);
    const uint64_t bal = __builtin_amdgcn_ballot_w64(f[r]);
    rank[r] = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bal >> 32),
                                        __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bal), 0u));
    if (lane == 0) wcnt[r][w] = static_cast<uint32_t>(__builtin_popcountll(bal));
  }
  __syncthreads();
  // Stores and gathers through buffer descriptors based at the chunk: an
  // unselected lane's offset is kOOB (dropped), so every round's loads are
  // issued back to back without exec-mask branches and the stores follow.
  const uint32_t nc = static_cast<uint32_t>(G - base < kCollectChunk ? G - base : kCollectChunk);
  const uint64_t pos0 = offsets[blockIdx.x];
  const rsrc_t rog = mk_rsrc(out_groups ? out_groups + pos0 : nullptr, out_groups ? kCollectChunk * 8 : 0);
  const rsrc_t rov = mk_rsrc(out_values ? out_values + pos0 : nullptr, out_values ? kCollectChunk * 8 : 0);
  const rsrc_t rv = mk_rsrc(values ? values + base : nullptr, values ? nc * 8 : 0);
  const rsrc_t rp = mk_rsrc(perm ? perm + base : nullptr, perm ? nc * 8 : 0);
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  uint32_t po[kCollectPer];
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t r = 0; r < kCollectPer; r++) {
    uint32_t before = 0, all = 0;
#pragma unroll
    for (uint32_t k = 0; k < kBlock / 64; k++) {
      before += k < w ? wcnt[r][k] : 0u;
      all += wcnt[r][k];
    }
    po[r] = f[r] ? (pos + before + rank[r]) * 8 : kOOB;
    pos += all;
  }
  if (out_values) {
    u32x2 v[kCollectPer];
#pragma unroll
    for (uint32_t r = 0; r < kCollectPer; r++)
      v[r] = __builtin_amdgcn_raw_buffer_load_b64(rv, f[r] ? (r * kBlock + tid) * 8 : kOOB, 0, 0);
#pragma unroll
    for (uint32_t r = 0; r < kCollectPer; r++) __builtin_amdgcn_raw_buffer_store_b64(v[r], rov, po[r], 0, 0);
  }
  if (out_groups) {
    if (perm) {
      u32x2 v[kCollectPer];
#pragma unroll
      for (uint32_t r = 0; r < kCollectPer; r++)
        v[r] = __builtin_amdgcn_raw_buffer_load_b64(rp, f[r] ? (r * kBlock + tid) * 8 : kOOB, 0, 0);
#pragma unroll
      for (uint32_t r = 0; r < kCollectPer; r++)
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(u32x2, goff + __builtin_bit_cast(uint64_t, v[r])), rog, po[r], 0, 0);
    } else {
#pragma unroll
      for (uint32_t r = 0; r < kCollectPer; r++)
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(u32x2, goff + base + r * kBlock + tid), rog, po[r], 0, 0);
    }
  }
}

}  // namespace qe
