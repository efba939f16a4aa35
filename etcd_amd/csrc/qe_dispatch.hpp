// qe_dispatch.hpp — declarations shared by the per-S instantiation objects
// (qe_inst.hip) and the C ABI (qe_api.hip).
#pragma once
#include "qe_kernels.hpp"
#include "qe_stream.hpp"
#include "qe_progress.hpp"
#include "qe_repl.hpp"

namespace qe {

int hip_status(hipError_t e);

#define QE_DECL_S(n)                                                                   \
  int dispatch_cv_##n(const CVArgs &a, int mode, bool vec, hipStream_t st);           \
  int dispatch_repl_##n(const RArgs &a, bool masked, bool joint, bool vec,            \
                        hipStream_t st);                                               \
  int dispatch_elec_##n(const EArgs &a, hipStream_t st);                            \
  int dispatch_progress_##n(const PArgs &a, int kind, bool masked, bool joint,        \
                            hipStream_t st);
QE_DECL_S(1) QE_DECL_S(2) QE_DECL_S(3) QE_DECL_S(4) QE_DECL_S(5) QE_DECL_S(6) QE_DECL_S(7)
QE_DECL_S(8) QE_DECL_S(9) QE_DECL_S(10) QE_DECL_S(11) QE_DECL_S(12) QE_DECL_S(13)
QE_DECL_S(14) QE_DECL_S(15) QE_DECL_S(16)
#undef QE_DECL_S

}  // namespace qe
