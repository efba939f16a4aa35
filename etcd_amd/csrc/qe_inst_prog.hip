// qe_inst_prog.hip — per-slot-count instantiations of the Progress state
// machine kernels (qe_progress.hpp).  Compiled once per S (1..16) with
// -DQE_S=<S>, separately from qe_inst.hip so the two kernel families rebuild
// independently.
#include "qe_dispatch.hpp"

#ifndef QE_S
#error "compile with -DQE_S=<slots>"
#endif

namespace qe {

namespace {
constexpr int S = QE_S;
using MT = std::conditional<(S <= 8), uint8_t, uint16_t>::type;
}  // namespace

#define QE_CAT2(a, b) a##b
#define QE_CAT(a, b) QE_CAT2(a, b)

template <int RM, bool ACCT, int WPB = kBlock / 64>
static int launch_progress_step(const PArgs &a, bool masked, bool joint, hipStream_t st) {
  // the same waves as the 4-wave grid, in blocks of WPB waves
  const uint64_t nb = static_cast<uint64_t>(grid_for((a.G + 63) / 64, 0, 1)) * ((kBlock / 64) / WPB);
  const dim3 grid(static_cast<unsigned>(nb < 0x7FFFFFFFull ? nb : 0x7FFFFFFFull));
  const dim3 blk(64 * WPB);
  if (joint)
    hipLaunchKernelGGL((k_progress_step<S, MT, true, true, RM, ACCT, WPB>), grid, blk, 0, st, a);
  else if (masked)
    hipLaunchKernelGGL((k_progress_step<S, MT, true, false, RM, ACCT, WPB>), grid, blk, 0, st, a);
  else
    hipLaunchKernelGGL((k_progress_step<S, MT, false, false, RM, ACCT, WPB>), grid, blk, 0, st, a);
  return hip_status(hipGetLastError());
}

// kind 0: qe_progress_step, 1: qe_progress_send, 2: qe_progress_step with
// byte accounting (instrumented variant, measurement only)
int QE_CAT(dispatch_progress_, QE_S)(const PArgs &a, int kind, bool masked, bool joint,
                                     hipStream_t st) {
  if (kind == 1) {
    hipLaunchKernelGGL((k_progress_send<S, MT>), dim3(grid_for((a.G + 63) / 64, 0, 1)),
                       dim3(kBlock), 0, st, a);
    return hip_status(hipGetLastError());
  }
  // run table (staged in LDS, l_run): 4 runs cover the common leader log (one
  // or two older terms before the current one); 8 keep the block's LDS at
  // 52 KB (3 blocks per CU at S = 5, where 16 runs' 84 KB allow one);
  // up to QE_MAX_LOG_RUNS otherwise
  if (kind == 2) return launch_progress_step<QE_MAX_LOG_RUNS, true>(a, masked, joint, st);
  if (a.R <= 4) return launch_progress_step<4, false>(a, masked, joint, st);
#ifndef QE_NO_RM8  // A/B knob: without the 8-run kernel
  if (a.R <= 8) return launch_progress_step<8, false>(a, masked, joint, st);
#endif
#ifdef QE_RM16_WPB  // A/B knob: waves per block of the 16-run kernel
  return launch_progress_step<QE_MAX_LOG_RUNS, false, QE_RM16_WPB>(a, masked, joint, st);
#else
  return launch_progress_step<QE_MAX_LOG_RUNS, false, 1>(a, masked, joint, st);
#endif
}

}  // namespace qe
