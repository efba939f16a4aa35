// qe_device.hpp — device-side building blocks of the batched quorum engine
// (gfx950).  Pure integer work: 64-bit compare/select networks, popcount vote
// logic, a counter-based hash.  No MFMA: the path is HBM-bound.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qe {

constexpr uint64_t kInf = ~0ull;
constexpr uint64_t kPhi = 0x9E3779B97F4A7C15ull;
constexpr uint32_t kVotePending = 1, kVoteLost = 2, kVoteWon = 3;

// splitmix64 finalizer; identical to oracle/quorum_oracle.c:orc_mix64.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// MurmurHash3 32-bit finalizer (oracle/quorum_oracle.c orc_fmix32).
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint64_t hash4(uint64_t seed, uint64_t gid, uint32_t lane,
                                          uint32_t stream) {
  uint64_t k = (static_cast<uint64_t>(stream) << 32) | lane;
  return mix64(mix64(seed + gid * kPhi) ^ (k * 0xD6E8FEB86659FD93ull));
}

__device__ __forceinline__ uint32_t popc(uint32_t x) { return __builtin_popcount(x); }

// ---------------------------------------------------------------------------
// Sorting networks (Batcher odd-even merge sort for arbitrary n, built at
// compile time).  Only the comparators that feed the selected rank survive
// dead-code elimination, so `select_fixed<N>` costs a partial network.
// ---------------------------------------------------------------------------
struct CE {
  int a, b;
};

template <int N>
struct Batcher {
  static constexpr int count() {
    int c = 0;
    for (int p = 1; p < N; p <<= 1)
      for (int k = p; k >= 1; k >>= 1)
        for (int j = k % p; j + k < N; j += 2 * k)
          for (int i = 0; i < k && i < N - j - k; i++)
            if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) c++;
    return c;
  }
  static constexpr int kSize = count();
  struct Net {
    CE e[kSize > 0 ? kSize : 1];
  };
  static constexpr Net make() {
    Net n{};
    int c = 0;
    for (int p = 1; p < N; p <<= 1)
      for (int k = p; k >= 1; k >>= 1)
        for (int j = k % p; j + k < N; j += 2 * k)
          for (int i = 0; i < k && i < N - j - k; i++)
            if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) n.e[c++] = CE{i + j, i + j + k};
    return n;
  }
  static constexpr Net kNet = make();
};

__device__ __forceinline__ void cmpx(uint64_t &a, uint64_t &b) {
  const bool sw = b < a;
  const uint64_t lo = sw ? b : a;
  const uint64_t hi = sw ? a : b;
  a = lo;
  b = hi;
}

__device__ __forceinline__ void cmpx_p(uint64_t &a, uint32_t &pa, uint64_t &b, uint32_t &pb) {
  const bool sw = b < a;
  const uint64_t lo = sw ? b : a, hi = sw ? a : b;
  const uint32_t plo = sw ? pb : pa, phi = sw ? pa : pb;
  a = lo;
  b = hi;
  pa = plo;
  pb = phi;
}

// (N/2+1)-th largest of N values = ascending position N-(N/2+1)
// (raft/quorum/majority.go:165-171).  v is clobbered.
template <int N>
__device__ __forceinline__ uint64_t select_fixed(uint64_t (&v)[N]) {
  constexpr auto net = Batcher<N>::kNet;
#pragma unroll
  for (int c = 0; c < Batcher<N>::kSize; c++) cmpx(v[net.e[c].a], v[net.e[c].b]);
  return v[N - (N / 2 + 1)];
}

// Masked joint selection.  Slot values are sorted once with a 2-bit payload
// (bit0: member of JointConfig[0], bit1: member of JointConfig[1]); walking
// from the top, the k-th member of a half is that half's (n/2+1)-th largest
// acked index.  An empty half yields inf (majority.go:128-132), and the joint
// result is the min of the halves (joint.go:49-56).  This is the general
// (64-bit) path.
template <int S>
__device__ __forceinline__ uint64_t joint_committed_wide(uint64_t (&v)[S], const uint32_t (&pay)[S],
                                                         uint32_t n0, uint32_t n1) {
  uint32_t p[S];
#pragma unroll
  for (int s = 0; s < S; s++) p[s] = pay[s];
  constexpr auto net = Batcher<S>::kNet;
#pragma unroll
  for (int c = 0; c < Batcher<S>::kSize; c++)
    cmpx_p(v[net.e[c].a], p[net.e[c].a], v[net.e[c].b], p[net.e[c].b]);
  const uint32_t k0 = n0 / 2 + 1, k1 = n1 / 2 + 1;
  uint32_t c0 = 0, c1 = 0;
  uint64_t r0 = n0 ? 0 : kInf, r1 = n1 ? 0 : kInf;
#pragma unroll
  for (int q = S - 1; q >= 0; q--) {
    const uint32_t m0 = p[q] & 1u, m1 = p[q] >> 1;
    c0 += m0;
    c1 += m1;
    r0 = (m0 && c0 == k0) ? v[q] : r0;
    r1 = (m1 && c1 == k1) ? v[q] : r1;
  }
  return r0 < r1 ? r0 : r1;
}

// Fast path (exact): when every nonzero value of the group shares bits 29..63
// (followers of one leader ack indexes close to each other; checked as "same
// high word and same bits 29..60" with two 32-bit maxima), a nonzero value
// v maps order-preservingly onto the 30-bit offset (v & (2^29 - 1)) | 2^29
// and zero onto offset 0.  Key = offset << 2 | payload is a 32-bit word, and
// a comparator is one v_min_u32 plus one v_max_u32 instead of a 64-bit
// compare and six selects.  Slots outside both halves keep payload 0: they
// sort with the rest and are never selected.  Groups whose nonzero values
// differ above bit 28 take the 64-bit payload sort.
//
// Selection without a walk: after the sort, the payload bits of all S
// positions are gathered into one word P (one v_alignbit per position).  The
// k-th largest member of a half with n members is its (n-k+1)-th member from
// the bottom, i.e. the lowest set bit of the half's membership bits after
// clearing the n-k = (n-1)/2 lowest ones.  Keys ascend with position, so
// min(CI(half 0), CI(half 1)) (joint.go:49-56) is the key at the lower of the
// two positions: the lowest set bit of the OR of both cleared masks.  An
// empty half contributes no bit (its CommittedIndex is inf,
// majority.go:128-132); both empty gives inf.

// k[q] for a per-lane index q < S: a binary select tree over q's bits.
template <int S>
__device__ __forceinline__ uint32_t pick_lane(const uint32_t (&k)[S], uint32_t q) {
  uint32_t c[S];
#pragma unroll
  for (int i = 0; i < S; i++) c[i] = k[i];
  int n = S;
#pragma unroll
  for (int bit = 0; (1 << bit) < S; bit++) {
    // all-ones where q has this bit: one v_bfi_b32 per pair (a select on a
    // compare would be folded back into an index compare chain)
    const uint32_t m = 0u - ((q >> bit) & 1u);
#pragma unroll
    for (int i = 0; i < (n + 1) / 2; i++)
      c[i] = 2 * i + 1 < n ? ((c[2 * i + 1] & m) | (c[2 * i] & ~m)) : c[2 * i];
    n = (n + 1) / 2;
  }
  return c[0];
}

// Clears the d lowest set bits of x, for d <= DMAX.
template <int DMAX>
__device__ __forceinline__ uint32_t clear_low_bits(uint32_t x, uint32_t d) {
#pragma unroll
  for (int i = 0; i < DMAX; i++) x = static_cast<uint32_t>(i) < d ? (x & (x - 1u)) : x;
  return x;
}

template <int S>
__device__ __forceinline__ uint64_t joint_committed(uint64_t (&v)[S], uint32_t inc,
                                                    uint32_t out) {
  static_assert(S >= 1 && S <= 16, "slot count");
  constexpr uint32_t kM = (1u << 29) - 1u;
  // every nonzero value must share its high word and bits 29..60 with the
  // maxima of those fields over the group (zeros never raise a maximum)
  uint32_t y[S];
  uint32_t hmax = 0, ymax = 0;
#pragma unroll
  for (int s = 0; s < S; s++) {
    const uint32_t lo = static_cast<uint32_t>(v[s]), hi = static_cast<uint32_t>(v[s] >> 32);
    y[s] = __builtin_amdgcn_alignbit(hi, lo, 29);  // bits 29..60 of v
    ymax = y[s] > ymax ? y[s] : ymax;
    hmax = hi > hmax ? hi : hmax;
  }
  bool fast = true;
#pragma unroll
  for (int s = 0; s < S; s++)
    fast &= ((y[s] == ymax) & (static_cast<uint32_t>(v[s] >> 32) == hmax)) | (v[s] == 0);
  const uint32_t n0 = popc(inc), n1 = popc(out);
  if (!fast) {
    uint32_t pay[S];
#pragma unroll
    for (int s = 0; s < S; s++) pay[s] = ((inc >> s) & 1u) | (((out >> s) & 1u) << 1);
    return joint_committed_wide<S>(v, pay, n0, n1);
  }
  uint32_t k[S];
#pragma unroll
  for (int s = 0; s < S; s++) {
    const uint32_t pay = ((inc >> s) & 1u) | (((out >> s) & 1u) << 1);
    const uint32_t off = v[s] != 0 ? ((static_cast<uint32_t>(v[s]) & kM) | (1u << 29)) : 0u;
    k[s] = (off << 2) | pay;
  }
  constexpr auto net = Batcher<S>::kNet;
#pragma unroll
  for (int c = 0; c < Batcher<S>::kSize; c++) {
    const uint32_t x = k[net.e[c].a], yv = k[net.e[c].b];
    k[net.e[c].a] = x < yv ? x : yv;
    k[net.e[c].b] = x < yv ? yv : x;
  }
  // position q's payload lands at bits B + 2q, B + 2q + 1
  constexpr int B = 32 - 2 * S;
  uint32_t P = 0;
#pragma unroll
  for (int q = 0; q < S; q++) P = __builtin_amdgcn_alignbit(k[q], P, 2);
  const uint32_t h0 = P & 0x55555555u, h1 = (P >> 1) & 0x55555555u;
  constexpr int DMAX = (S - 1) / 2;
  const uint32_t x0 = clear_low_bits<DMAX>(h0, (n0 - 1u) >> 1);
  const uint32_t x1 = clear_low_bits<DMAX>(h1, (n1 - 1u) >> 1);
  const uint32_t x = x0 | x1;
  if (x == 0) return kInf;  // both halves empty
  const uint32_t q = (static_cast<uint32_t>(__builtin_ctz(x)) - B) >> 1;
  const uint32_t off = pick_lane<S>(k, q) >> 2;
  if (off == 0) return 0;
  const uint32_t lo = (ymax << 29) | (off & kM);
  return (static_cast<uint64_t>(hmax) << 32) | lo;
}

// joint_committed over the first `top` slots only, where `top` is
// wave-uniform and no lane of the wave has a voter in slots >= top (the
// shape-bucketed layout puts every voter in the low slots).
// The smaller network is picked with a scalar branch; slots >= top hold
// only absent, non-member values, which never change a result.
template <int S, int N>
__device__ __forceinline__ uint64_t joint_committed_first(const uint64_t (&v)[S], uint32_t inc,
                                                          uint32_t out) {
  uint64_t w[N];
#pragma unroll
  for (int i = 0; i < N; i++) w[i] = v[i];
  return joint_committed<N>(w, inc, out);
}

template <int S>
__device__ __forceinline__ uint64_t joint_committed_top(uint64_t (&v)[S], uint32_t inc,
                                                        uint32_t out, uint32_t top) {
  if constexpr (S >= 6) {
    if (top <= S - 5) return joint_committed_first<S, S - 5>(v, inc, out);
    if (top <= S - 4) return joint_committed_first<S, S - 4>(v, inc, out);
    if (top <= S - 3) return joint_committed_first<S, S - 3>(v, inc, out);
    if (top <= S - 2) return joint_committed_first<S, S - 2>(v, inc, out);
    if (top <= S - 1) return joint_committed_first<S, S - 1>(v, inc, out);
  }
  return joint_committed<S>(v, inc, out);
}

// MajorityConfig.VoteResult over slot bitmaps (raft/quorum/majority.go:178-210).
__device__ __forceinline__ uint32_t majority_vote(uint32_t member, uint32_t voted,
                                                  uint32_t granted) {
  const uint32_t n = popc(member);
  const uint32_t yes = popc(member & voted & granted);
  const uint32_t no = popc(member & voted & ~granted);
  const uint32_t missing = n - yes - no;
  const uint32_t q = n / 2 + 1;
  const uint32_t r = yes >= q ? kVoteWon : (yes + missing >= q ? kVotePending : kVoteLost);
  return n == 0 ? kVoteWon : r;
}

// JointConfig.VoteResult (raft/quorum/joint.go:61-75).
__device__ __forceinline__ uint32_t joint_vote(uint32_t inc, uint32_t out, uint32_t voted,
                                               uint32_t granted) {
  const uint32_t r1 = majority_vote(inc, voted, granted);
  const uint32_t r2 = majority_vote(out, voted, granted);
  if (r1 == r2) return r1;
  return (r1 == kVoteLost || r2 == kVoteLost) ? kVoteLost : kVotePending;
}

// ---------------------------------------------------------------------------
// Wave / block reductions.
// ---------------------------------------------------------------------------
// OR of a 32-bit value over the 64 lanes, returned wave-uniform (SGPR).
__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x |= __shfl_xor(x, off, 64);
  return __builtin_amdgcn_readfirstlane(x);
}

// ---------------------------------------------------------------------------
// Statistics counters.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    uint32_t lo = static_cast<uint32_t>(x), hi = static_cast<uint32_t>(x >> 32);
    lo = __shfl_xor(lo, off, 64);
    hi = __shfl_xor(hi, off, 64);
    x += (static_cast<uint64_t>(hi) << 32) | lo;
  }
  return x;
}

// Adds NC per-thread counters into the sharded stats buffer: wave sums, then
// LDS across the block's waves, then NC lanes of wave 0 issue one atomic each.
template <int NC, int BLOCK>
__device__ __forceinline__ void block_stats_add(uint64_t (&c)[NC], const int (&idx)[NC],
                                                uint64_t *stats) {
  __shared__ uint64_t red[BLOCK / 64][NC];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NC; i++) {
    const uint64_t s = wave_sum_u64(c[i]);
    if (lane == 0) red[w][i] = s;
  }
  __syncthreads();
  if (threadIdx.x < NC) {
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < BLOCK / 64; k++) s += red[k][threadIdx.x];
    int which = 0;
#pragma unroll
    for (int i = 0; i < NC; i++)
      if (i == static_cast<int>(threadIdx.x)) which = idx[i];
    const int shard = blockIdx.x & 63;  // QE_STATS_SHARDS
    atomicAdd(reinterpret_cast<unsigned long long *>(stats + shard * 16 + which),
              static_cast<unsigned long long>(s));
  }
}

}  // namespace qe
