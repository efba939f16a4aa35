// qe_inst.hip — per-slot-count instantiations of the hot kernels.  Compiled
// once per S (1..16) with -DQE_S=<S> so the 16 variants build in parallel.
#include "qe_dispatch.hpp"

#ifndef QE_S
#error "compile with -DQE_S=<slots>"
#endif

namespace qe {

namespace {
constexpr int S = QE_S;
using MT = std::conditional<(S <= 8), uint8_t, uint16_t>::type;

template <int MODE>
int launch_cv(const CVArgs &a, bool vec, hipStream_t st) {
  constexpr int kPairs = 2;
  const uint64_t npairs = (a.G + 1) / 2;
  const uint64_t tiles = (npairs + 64 * kPairs - 1) / (64 * kPairs);
  const unsigned grid = grid_for(tiles);
  if (vec) {
    if (g_nontemporal)
      hipLaunchKernelGGL((k_commit_vote<S, MODE, MT, kPairs, true, true>), dim3(grid),
                         dim3(kBlock), 0, st, a);
    else
      hipLaunchKernelGGL((k_commit_vote<S, MODE, MT, kPairs, true, false>), dim3(grid),
                         dim3(kBlock), 0, st, a);
  } else {
    hipLaunchKernelGGL((k_commit_vote<S, MODE, MT, kPairs, false, false>), dim3(grid),
                       dim3(kBlock), 0, st, a);
  }
  return hip_status(hipGetLastError());
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

int QE_CAT(dispatch_repl_, QE_S)(const RArgs &a, bool masked, bool joint, bool vec,
                                 hipStream_t st) {
  const uint64_t tiles = ((a.G + 1) / 2 + 63) / 64;
  const unsigned grid = grid_for(tiles);
#define QE_RL(J, M, V) \
  hipLaunchKernelGGL((k_replication<S, J, M, MT, V>), dim3(grid), dim3(kBlock), 0, st, a)
  if (vec) {
    if (joint) QE_RL(true, true, true);
    else if (masked) QE_RL(false, true, true);
    else QE_RL(false, false, true);
  } else {
    if (joint) QE_RL(true, true, false);
    else if (masked) QE_RL(false, true, false);
    else QE_RL(false, false, false);
  }
#undef QE_RL
  return hip_status(hipGetLastError());
}

int QE_CAT(dispatch_elec_, QE_S)(const EArgs &a, hipStream_t st) {
  const uint64_t cap = static_cast<uint64_t>(num_cus()) * g_blocks_per_cu;
  const uint64_t need = (a.G + kBlock - 1) / kBlock;
  const unsigned grid = static_cast<unsigned>(need < cap ? (need ? need : 1) : cap);
  hipLaunchKernelGGL((k_election<S, MT>), dim3(grid), dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

}  // namespace qe
