// qe_inst.hip — per-slot-count instantiations of the hot kernels.  Compiled
// once per S (1..16) with -DQE_S=<S> so the 16 variants build in parallel.
#include "qe_dispatch.hpp"

#ifndef QE_S
#error "compile with -DQE_S=<slots>"
#endif
#ifndef QE_PAIRS
#define QE_PAIRS ((QE_S) <= 8 ? 2 : 1)  // adjacent-group pairs per lane per tile
#endif

namespace qe {

namespace {
constexpr int S = QE_S;
using MT = std::conditional<(S <= 8), uint8_t, uint16_t>::type;

template <int MODE, bool VEC, bool NTL, bool NTS>
int launch_cv_k(const CVArgs &a, hipStream_t st) {
  constexpr int kPairs = QE_PAIRS;
  auto kern = k_commit_vote<S, MODE, MT, kPairs, VEC, NTL, NTS>;
  static int occ = occupancy(kern);
  const uint64_t npairs = (a.G + 1) / 2;
  const uint64_t tiles = (npairs + 64 * kPairs - 1) / (64 * kPairs);
  hipLaunchKernelGGL(kern, dim3(grid_for(tiles, occ, MODE == 2 ? 8 : 1)), dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

// Chunk (tiles per wave): QE_STREAM_TPW on large batches; a batch too small
// to give every CU 32 waves at that chunk gets shorter chunks (>= 2, so the
// two-set pipeline still overlaps), trading per-wave pipelining for waves in
// flight.  g_tiles_per_wave > 0 overrides (clamped to QE_STREAM_TPW).
template <int MODE, bool NTL, bool NTS>
int launch_cv_stream(CVArgs a, hipStream_t st) {
  auto kern = k_cv_stream<S, MODE, MT, NTL, NTS>;
  const uint64_t tiles = (a.G + 63) / 64;
  uint64_t chunk;
  if (g_tiles_per_wave > 0) {
    chunk = static_cast<uint64_t>(g_tiles_per_wave);
  } else {
    const uint64_t waves = static_cast<uint64_t>(num_cus()) * 32;
    chunk = (tiles + waves - 1) / waves;
    if (chunk < 2) chunk = 2;
  }
  if (chunk > QE_STREAM_TPW) chunk = QE_STREAM_TPW;
  a.chunk = static_cast<uint32_t>(chunk);
  const uint64_t per_block = (kBlock / 64) * chunk;
  const uint64_t blocks = (tiles + per_block - 1) / per_block;
  if (blocks > 0x7FFFFFFFull) return QE_ERANGE;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

template <int MODE>
int launch_cv(const CVArgs &a, bool vec, hipStream_t st) {
  // default: the stream kernel (measured faster in every mode);
  // it addresses each 64-group tile through buffer descriptors and needs
  // no row alignment
  const int which = g_cv_kernel >= 0 ? g_cv_kernel : 1;
  if (which == 1) {
    switch (g_nontemporal & 3) {
      case 1: return launch_cv_stream<MODE, true, false>(a, st);
      case 2: return launch_cv_stream<MODE, false, true>(a, st);
      case 3: return launch_cv_stream<MODE, true, true>(a, st);
      default: return launch_cv_stream<MODE, false, false>(a, st);
    }
  }
  if (!vec) return launch_cv_k<MODE, false, false, false>(a, st);
  switch (g_nontemporal & 3) {
    case 1: return launch_cv_k<MODE, true, true, false>(a, st);
    case 2: return launch_cv_k<MODE, true, false, true>(a, st);
    case 3: return launch_cv_k<MODE, true, true, true>(a, st);
    default: return launch_cv_k<MODE, true, false, false>(a, st);
  }
}
}  // namespace

#define QE_CAT2(a, b) a##b
#define QE_CAT(a, b) QE_CAT2(a, b)

int QE_CAT(dispatch_cv_, QE_S)(const CVArgs &a, int mode, bool vec, hipStream_t st) {
  switch (mode) {
    case 0: return launch_cv<0>(a, vec, st);
    case 1: return launch_cv<1>(a, vec, st);
    default: return launch_cv<2>(a, vec, st);
  }
}

template <bool J, bool M, bool V, bool NT>
static int launch_repl_k(const RArgs &a, hipStream_t st) {
  auto kern = k_replication<S, J, M, MT, V, NT>;
  static int occ = occupancy(kern);
  const uint64_t tiles = ((a.G + 1) / 2 + 63) / 64;
  hipLaunchKernelGGL(kern, dim3(grid_for(tiles, occ, 1)), dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

// non-temporal state traffic whenever qe_tune("nontemporal") has both bits
template <bool J, bool M, bool V>
static int launch_repl(const RArgs &a, hipStream_t st) {
  if (V && (g_nontemporal & 3) == 3) return launch_repl_k<J, M, V, true>(a, st);
  return launch_repl_k<J, M, V, false>(a, st);
}

// Stream replication kernel (qe_repl.hpp); chunking as launch_cv_stream.
template <bool M, bool J, bool NTL, bool NTS>
static int launch_repl_stream(RArgs a, hipStream_t st) {
  auto kern = k_repl_stream<S, M, J, MT, NTL, NTS>;
  const uint64_t tiles = (a.G + 63) / 64;
  uint64_t chunk;
  if (g_tiles_per_wave > 0) {
    chunk = static_cast<uint64_t>(g_tiles_per_wave);
  } else {
    const uint64_t waves = static_cast<uint64_t>(num_cus()) * 32;
    chunk = (tiles + waves - 1) / waves;
    if (chunk < 2) chunk = 2;
  }
  if (chunk > QE_STREAM_TPW) chunk = QE_STREAM_TPW;
  a.chunk = static_cast<uint32_t>(chunk);
  const uint64_t per_block = (kBlock / 64) * chunk;
  const uint64_t blocks = (tiles + per_block - 1) / per_block;
  if (blocks > 0x7FFFFFFFull) return QE_ERANGE;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

template <bool M, bool J>
static int launch_repl_s(const RArgs &a, hipStream_t st) {
  switch (g_nontemporal & 3) {
    case 1: return launch_repl_stream<M, J, true, false>(a, st);
    case 2: return launch_repl_stream<M, J, false, true>(a, st);
    case 3: return launch_repl_stream<M, J, true, true>(a, st);
    default: return launch_repl_stream<M, J, false, false>(a, st);
  }
}

int QE_CAT(dispatch_repl_, QE_S)(const RArgs &a, bool masked, bool joint, bool vec,
                                 hipStream_t st) {
  if (g_repl_kernel != 0) {  // default: stream kernel (no alignment requirement)
    if (joint) return launch_repl_s<true, true>(a, st);
    if (masked) return launch_repl_s<true, false>(a, st);
    return launch_repl_s<false, false>(a, st);
  }
  if (vec) {
    if (joint) return launch_repl<true, true, true>(a, st);
    if (masked) return launch_repl<false, true, true>(a, st);
    return launch_repl<false, false, true>(a, st);
  }
  if (joint) return launch_repl<true, true, false>(a, st);
  if (masked) return launch_repl<false, true, false>(a, st);
  return launch_repl<false, false, false>(a, st);
}

template <int OPT>
static int launch_elec(const EArgs &a, hipStream_t st) {
  auto kern = k_election<S, MT, OPT>;
  static int occ = occupancy(kern);
  const uint64_t waves = (a.G + 63) / 64;
  hipLaunchKernelGGL(kern, dim3(grid_for(waves, occ, 1)), dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

int QE_CAT(dispatch_elec_, QE_S)(const EArgs &a, hipStream_t st) {
  const int opt = (a.flags & 3u) | (a.sresp ? 4 : 0) | (a.out ? 8 : 0);
  switch (opt) {
#define QE_E(o) \
  case o: return launch_elec<o>(a, st);
    QE_E(0) QE_E(1) QE_E(2) QE_E(3) QE_E(4) QE_E(5) QE_E(6) QE_E(7)
    QE_E(8) QE_E(9) QE_E(10) QE_E(11) QE_E(12) QE_E(13) QE_E(14)
#undef QE_E
    default: return launch_elec<15>(a, st);
  }
}

}  // namespace qe
