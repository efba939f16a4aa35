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

template <int RM, bool ACCT, bool RD, int WPB = kBlock / 64, bool P = false, bool N16 = false>
static int launch_progress_step_p(const PArgs &a, bool masked, bool joint, hipStream_t st) {
  // the same waves as the 4-wave grid, in blocks of WPB waves
  const uint64_t nb = static_cast<uint64_t>(grid_for((a.G + 63) / 64, 0, 1)) * ((kBlock / 64) / WPB);
  const dim3 grid(static_cast<unsigned>(nb < 0x7FFFFFFFull ? nb : 0x7FFFFFFFull));
  const dim3 blk(64 * WPB);
  if (joint)
    hipLaunchKernelGGL((k_progress_step<S, MT, true, true, RM, ACCT, RD, WPB, P, N16>), grid, blk, 0, st, a);
  else if (masked)
    hipLaunchKernelGGL((k_progress_step<S, MT, true, false, RM, ACCT, RD, WPB, P, N16>), grid, blk, 0, st, a);
  else
    hipLaunchKernelGGL((k_progress_step<S, MT, false, false, RM, ACCT, RD, WPB, P, N16>), grid, blk, 0, st, a);
  return hip_status(hipGetLastError());
}

// ABI 8, the 16-bit Inflights form (host-checked: F <= 8, S <= 9, at most 4
// log runs): the pipelined kernels, and the rolled one for the byte count
static int launch_progress_step_n16(const PArgs &a, bool acct, bool masked, bool joint,
                                    hipStream_t st) {
  if constexpr (S <= QE_RING16_MAX_SLOTS) {
    if (acct) return launch_progress_step_p<4, true, true, kBlock / 64, false, true>(a, masked, joint, st);
    if (a.read_acks) return launch_progress_step_p<4, false, true, kBlock / 64, true, true>(a, masked, joint, st);
    return launch_progress_step_p<4, false, false, kBlock / 64, true, true>(a, masked, joint, st);
  }
  return QE_EINVAL;
}

// the pipelined slot loop (qe_progress.hpp) for rings in row form, up to 9
// slots and the 4-run table (3 waves/SIMD; with the 8-run table it needs
// 176-195 VGPRs from S = 6, 2 waves); the rolled loop otherwise
template <int RM, bool ACCT, bool RD, int WPB = kBlock / 64>
static int launch_progress_step(const PArgs &a, bool masked, bool joint, hipStream_t st) {
  if constexpr (S <= 9 && RM <= 4 && !ACCT) {
    if (a.F <= kRingChunk) return launch_progress_step_p<RM, ACCT, RD, WPB, true>(a, masked, joint, st);
  }
  return launch_progress_step_p<RM, ACCT, RD, WPB, false>(a, masked, joint, st);
}

// qe_progress_send: chunks of up to kSendTPW tiles per wave (as the stream
// commit kernel: a batch too small to give every CU 32 waves at that chunk
// gets shorter chunks, >= 2 so the two register sets still overlap)
static int launch_progress_send(PArgs a, hipStream_t st) {
  const uint64_t tiles = (a.G + 63) / 64;
  const uint64_t waves = static_cast<uint64_t>(num_cus()) * 32;
  uint64_t chunk = g_tiles_per_wave > 0 ? static_cast<uint64_t>(g_tiles_per_wave)
                                        : (tiles + waves - 1) / waves;
  if (chunk < 2) chunk = 2;
  if (chunk > static_cast<uint64_t>(kSendTPW)) chunk = kSendTPW;
  a.chunk = static_cast<uint32_t>(chunk);
  const uint64_t per_block = (kBlock / 64) * chunk;
  const uint64_t blocks = (tiles + per_block - 1) / per_block;
  if (blocks > 0x7FFFFFFFull) return QE_ERANGE;
  if constexpr (S <= QE_RING16_MAX_SLOTS) {
    if (a.infl16) {
      hipLaunchKernelGGL((k_progress_send<S, MT, true>), dim3(static_cast<unsigned>(blocks)),
                         dim3(kBlock), 0, st, a);
      return hip_status(hipGetLastError());
    }
  }
  hipLaunchKernelGGL((k_progress_send<S, MT>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
                     0, st, a);
  return hip_status(hipGetLastError());
}

static int launch_check_quorum(PArgs a, bool masked, bool joint, hipStream_t st) {
  // the chunking of qe_progress_send (kSendTPW tiles per wave at most)
  const uint64_t tiles = (a.G + 63) / 64;
  const uint64_t waves = static_cast<uint64_t>(num_cus()) * 32;
  uint64_t chunk = g_tiles_per_wave > 0 ? static_cast<uint64_t>(g_tiles_per_wave)
                                        : (tiles + waves - 1) / waves;
  if (chunk < 2) chunk = 2;
  if (chunk > static_cast<uint64_t>(kSendTPW)) chunk = kSendTPW;
  a.chunk = static_cast<uint32_t>(chunk);
  const uint64_t per_block = (kBlock / 64) * chunk;
  const uint64_t blocks = (tiles + per_block - 1) / per_block;
  if (blocks > 0x7FFFFFFFull) return QE_ERANGE;
  const dim3 grid(static_cast<unsigned>(blocks));
  if (joint) hipLaunchKernelGGL((k_check_quorum<S, MT, true, true>), grid, dim3(kBlock), 0, st, a);
  else if (masked) hipLaunchKernelGGL((k_check_quorum<S, MT, true, false>), grid, dim3(kBlock), 0, st, a);
  else hipLaunchKernelGGL((k_check_quorum<S, MT, false, false>), grid, dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

template <bool RD>
static int step_runs(const PArgs &a, bool masked, bool joint, hipStream_t st) {
  if (a.R <= 4) return launch_progress_step<4, false, RD>(a, masked, joint, st);
#ifndef QE_NO_RM8  // A/B knob: without the 8-run kernel
  if (a.R <= 8) return launch_progress_step<8, false, RD>(a, masked, joint, st);
#endif
#ifdef QE_RM16_WPB  // A/B knob: waves per block of the 16-run kernel
  return launch_progress_step<QE_MAX_LOG_RUNS, false, RD, QE_RM16_WPB>(a, masked, joint, st);
#else
  return launch_progress_step<QE_MAX_LOG_RUNS, false, RD, 1>(a, masked, joint, st);
#endif
}

static int launch_read_index(const PArgs &a, bool masked, bool joint, hipStream_t st) {
  const dim3 grid(grid_for((a.G + 63) / 64, 0, 1));
  if (joint) hipLaunchKernelGGL((k_read_index<S, MT, true, true>), grid, dim3(kBlock), 0, st, a);
  else if (masked) hipLaunchKernelGGL((k_read_index<S, MT, true, false>), grid, dim3(kBlock), 0, st, a);
  else hipLaunchKernelGGL((k_read_index<S, MT, false, false>), grid, dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

template <bool ACCT, bool N16 = false>
static int launch_propose(const PArgs &a, bool masked, bool joint, hipStream_t st) {
  if constexpr (!N16 && S <= QE_RING16_MAX_SLOTS) {
    if (a.infl16) return launch_propose<ACCT, true>(a, masked, joint, st);
  }
  const dim3 grid(grid_for((a.G + 63) / 64, 0, 1));
  if (joint) hipLaunchKernelGGL((k_propose<S, MT, true, true, ACCT, N16>), grid, dim3(kBlock), 0, st, a);
  else if (masked) hipLaunchKernelGGL((k_propose<S, MT, true, false, ACCT, N16>), grid, dim3(kBlock), 0, st, a);
  else hipLaunchKernelGGL((k_propose<S, MT, false, false, ACCT, N16>), grid, dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

template <bool ACCT, bool N16 = false>
static int launch_switch_config(const PArgs &a, bool masked, bool joint, hipStream_t st) {
  if constexpr (!N16 && S <= QE_RING16_MAX_SLOTS) {
    if (a.infl16) return launch_switch_config<ACCT, true>(a, masked, joint, st);
  }
  const dim3 grid(grid_for((a.G + 63) / 64, 0, 1));
  if (joint) hipLaunchKernelGGL((k_switch_config<S, MT, true, true, ACCT, N16>), grid, dim3(kBlock), 0, st, a);
  else if (masked) hipLaunchKernelGGL((k_switch_config<S, MT, true, false, ACCT, N16>), grid, dim3(kBlock), 0, st, a);
  else hipLaunchKernelGGL((k_switch_config<S, MT, false, false, ACCT, N16>), grid, dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

static int launch_become_leader(const PArgs &a, bool masked, bool joint, hipStream_t st) {
  const dim3 grid(grid_for((a.G + 63) / 64, 0, 1));
  if (joint) hipLaunchKernelGGL((k_become_leader<S, MT, true, true>), grid, dim3(kBlock), 0, st, a);
  else if (masked) hipLaunchKernelGGL((k_become_leader<S, MT, true, false>), grid, dim3(kBlock), 0, st, a);
  else hipLaunchKernelGGL((k_become_leader<S, MT, false, false>), grid, dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

static int launch_heartbeat(const PArgs &a, hipStream_t st) {
  const dim3 grid(grid_for((a.G + 63) / 64, 0, 1));
  hipLaunchKernelGGL((k_heartbeat<S, MT>), grid, dim3(kBlock), 0, st, a);
  return hip_status(hipGetLastError());
}

// kind 0: qe_progress_step, 1: qe_progress_send, 2: qe_progress_step with
// byte accounting (instrumented variant, measurement only), 3:
// qe_check_quorum, 4: qe_read_index, 5: qe_propose, 6: qe_propose with byte
// accounting, 7: qe_heartbeat, 8: qe_switch_config, 9: qe_switch_config with
// byte accounting, 10: qe_become_leader
int QE_CAT(dispatch_progress_, QE_S)(const PArgs &a, int kind, bool masked, bool joint,
                                     hipStream_t st) {
  if (kind == 1) return launch_progress_send(a, st);
  if (kind == 3) return launch_check_quorum(a, masked, joint, st);
  if (kind == 4) return launch_read_index(a, masked, joint, st);
  if (kind == 5) return launch_propose<false>(a, masked, joint, st);
  if (kind == 6) return launch_propose<true>(a, masked, joint, st);
  if (kind == 7) return launch_heartbeat(a, st);
  if (kind == 8) return launch_switch_config<false>(a, masked, joint, st);
  if (kind == 9) return launch_switch_config<true>(a, masked, joint, st);
  if (kind == 10) return launch_become_leader(a, masked, joint, st);
  // run table (staged in LDS, l_run): 4 runs cover the common leader log (one
  // or two older terms before the current one); 8 keep the block's LDS at
  // 52 KB (3 blocks per CU at S = 5, where 16 runs' 84 KB allow one);
  // up to QE_MAX_LOG_RUNS otherwise
  // ReadIndex tracking (a.read_acks) takes a variant of its own: its queue
  // state costs registers the rounds without reads should not pay
  if (a.infl16 && (kind == 0 || kind == 2)) return launch_progress_step_n16(a, kind == 2, masked, joint, st);
  if (kind == 2) return launch_progress_step<QE_MAX_LOG_RUNS, true, true>(a, masked, joint, st);
  if (a.read_acks) return step_runs<true>(a, masked, joint, st);
  return step_runs<false>(a, masked, joint, st);
}

}  // namespace qe
