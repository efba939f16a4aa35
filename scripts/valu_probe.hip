// valu_probe.hip — issue cost of the VALU instruction classes the election
// kernel (k_election) executes, on gfx950, at full occupancy: every CU runs
// 8 waves per SIMD, each wave a loop of 32 independent instructions of ONE
// kind per iteration (8 chains of 4, so no dependent stall at 8 waves), so
// the kernel is VALU-issue bound.  Printed per kind: ms per launch, SIMD
// cycles per wave64 instruction at 2.4 GHz, and the instruction count (the
// shader clock itself comes from GRBM_GUI_ACTIVE of the --pmc pass), from which
// scripts/valu_cost.py weights the election's VALU mix (VERDICT r04 item 8:
// v_mul_lo_u32 is not full rate, so an instruction count understates the
// SIMD time).  The same binary under rocprofv3 --pmc gives what
// SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU / SQ_THREAD_CYCLES_VALU report for a
// known instruction stream.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

typedef unsigned int u32;
typedef unsigned long long u64;

constexpr int kIters = 4096;
constexpr int kPerIter = 32;

// one instruction of each chain: "op a_i, a_i, k" for i = 0..7
#define R8(T) T(0) T(1) T(2) T(3) T(4) T(5) T(6) T(7)
// 3-source kinds read a second chain's register as the third operand (three
// distinct VGPRs, as compiled code has them; a repeated register measured
// half rate)
#define R8P(T) T(0, 1) T(1, 2) T(2, 3) T(3, 4) T(4, 5) T(5, 6) T(6, 7) T(7, 0)
#define I_ADD(i) "v_add_u32 %" #i ", %" #i ", %8\n"
#define I_XOR(i) "v_xor_b32 %" #i ", %" #i ", %8\n"
#define I_MUL(i) "v_mul_lo_u32 %" #i ", %" #i ", %8\n"
#define I_MUL24(i) "v_mul_u32_u24 %" #i ", %" #i ", %8\n"
#define I_BCNT(i) "v_bcnt_u32_b32 %" #i ", %" #i ", %8\n"
#define I_BITOP3(i, j) "v_bitop3_b32 %" #i ", %" #i ", %8, %" #j " bitop3:0x96\n"
#define I_CND(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, vcc\n"
#define I_MUL16(i) "v_mul_lo_u16 %" #i ", %" #i ", %8\n"
#define I_ADD3(i, j) "v_add3_u32 %" #i ", %" #i ", %8, %" #j "\n"
// 64-bit kinds: a_i are VGPR pairs
#define I_MAD64(i) "v_mad_u64_u32 %" #i ", vcc, %8, %8, %" #i "\n"
#define I_LSHLADD64(i) "v_lshl_add_u64 %" #i ", %" #i ", 1, %" #i "\n"
#define I_SHR64(i) "v_lshrrev_b64 %" #i ", 1, %" #i "\n"
#define I_MOV(i) "v_mov_b32 %" #i ", %8\n"
#define I_CMP(i) "v_cmp_gt_u32_e64 vcc, %" #i ", %8\n"
#define I_AND(i) "v_and_b32 %" #i ", %" #i ", %8\n"
#define I_OR3(i, j) "v_or3_b32 %" #i ", %" #i ", %8, %" #j "\n"
#define I_SHR(i) "v_lshrrev_b32 %" #i ", 1, %" #i "\n"
#define I_SUB(i) "v_sub_u32 %" #i ", %" #i ", %8\n"
#define I_CND32(i) "v_cndmask_b32_e32 %" #i ", %" #i ", %8, vcc\n"
#define I_MIN(i) "v_min_u32 %" #i ", %" #i ", %8\n"
#define I_MAX(i) "v_max_u32 %" #i ", %" #i ", %8\n"
#define I_SHL(i) "v_lshlrev_b32 %" #i ", 1, %" #i "\n"
#define I_ALIGN(i, j) "v_alignbit_b32 %" #i ", %" #i ", %" #j ", 3\n"
#define I_ANDOR(i, j) "v_and_or_b32 %" #i ", %" #i ", %8, %" #j "\n"
#define I_RDL(i) "v_readlane_b32 s" #i "6, %" #i ", 5\n"    // SGPR spill reload shape
#define I_WRL(i) "v_writelane_b32 %" #i ", s" #i "6, 7\n"   // SGPR spill store shape
#define OPS(T) R8(T) R8(T) R8(T) R8(T)  // 32 instructions, 8 independent chains of 4
#define OPS3(T) R8P(T) R8P(T) R8P(T) R8P(T)

#define KINDS(X)                                                         \
  X(0, u32, I_ADD, "v_add_u32") X(1, u32, I_XOR, "v_xor_b32")           \
  X(2, u32, I_MUL, "v_mul_lo_u32") X(3, u32, I_MUL24, "v_mul_u32_u24")  \
  X(4, u32, I_BCNT, "v_bcnt_u32_b32") X3(5, u32, I_BITOP3, "v_bitop3_b32") \
  X(6, u32, I_CND, "v_cndmask_b32") X(7, u32, I_MUL16, "v_mul_lo_u16")  \
  X3(8, u32, I_ADD3, "v_add3_u32") X(9, u64, I_MAD64, "v_mad_u64_u32")   \
  X(10, u64, I_LSHLADD64, "v_lshl_add_u64") X(11, u64, I_SHR64, "v_lshrrev_b64") \
  X(12, u32, I_MOV, "v_mov_b32") X(13, u32, I_CMP, "v_cmp_gt_u32")                 \
  X(14, u32, I_AND, "v_and_b32") X3(15, u32, I_OR3, "v_or3_b32")                    \
  X(16, u32, I_SHR, "v_lshrrev_b32") X(17, u32, I_SUB, "v_sub_u32")                \
  X(18, u32, I_CND32, "v_cndmask_b32_e32")                                        \
  XS(19, u32, I_RDL, "v_readlane_b32") XS(20, u32, I_WRL, "v_writelane_b32")        \
  X(21, u32, I_MIN, "v_min_u32") X(22, u32, I_MAX, "v_max_u32")                    \
  X(23, u32, I_SHL, "v_lshlrev_b32") X3(24, u32, I_ALIGN, "v_alignbit_b32")        \
  X3(25, u32, I_ANDOR, "v_and_or_b32")
constexpr int kKinds = 26;

template <int KIND, typename T>
__device__ __forceinline__ void body(T &a0, T &a1, T &a2, T &a3, T &a4, T &a5, T &a6, T &a7,
                                     u32 k) {
#define X(K, TY, I, NAME)                                                                      \
  if constexpr (KIND == K)                                                                     \
    asm volatile(OPS(I) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                 "+v"(a7)                                                                      \
                 : "v"(k)                                                                      \
                 : "vcc");
#define X3(K, TY, I, NAME)                                                                     \
  if constexpr (KIND == K)                                                                     \
    asm volatile(OPS3(I) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),         \
                 "+v"(a6), "+v"(a7)                                                            \
                 : "v"(k)                                                                      \
                 : "vcc");
#define XS(K, TY, I, NAME)                                                                     \
  if constexpr (KIND == K)                                                                     \
    asm volatile(OPS(I) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                 "+v"(a7)                                                                      \
                 : "v"(k)                                                                      \
                 : "s6", "s16", "s26", "s36", "s46", "s56", "s66", "s76");
  KINDS(X)
#undef X
#undef X3
#undef XS
}

template <int KIND, typename T>
__global__ __launch_bounds__(256) void k_valu(u32 *sink, u32 seed) {
  T a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
    a6 = a0 + 6, a7 = a0 + 7;
  const u32 k = seed | 1u;
  for (int i = 0; i < kIters; i++) body<KIND, T>(a0, a1, a2, a3, a4, a5, a6, a7, k);
  const T r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (r == static_cast<T>(0x12345678u)) sink[0] = static_cast<u32>(r);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
  u32 *sink;
  hipMalloc(&sink, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double waves = static_cast<double>(blocks) * 4;
  const double insts = waves * kIters * kPerIter;  // wave64 instructions per launch
  const double per_simd = insts / (cus * 4.0);
  for (int kind = 0; kind < kKinds; kind++) {
    const char *name = "";
    for (int rep = 0; rep < 4; rep++) {
      hipEventRecord(e0);
      switch (kind) {
#define X(K, TY, I, NAME)                                                             \
  case K:                                                                             \
    name = NAME;                                                                      \
    hipLaunchKernelGGL((k_valu<K, TY>), dim3(blocks), dim3(256), 0, 0, sink, 3u);     \
    break;
#define X3 X
#define XS X
        KINDS(X)
#undef X
#undef X3
#undef XS
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 3)
        printf("%-16s %9.4f ms  %7.3f SIMD-cycles/inst at 2.4 GHz  insts %.6e\n", name, ms,
               ms * 1e6 * 2.4 / per_simd, insts);
    }
  }
  return 0;
}
