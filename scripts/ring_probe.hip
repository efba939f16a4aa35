// ring_probe.hip — Inflights ring layouts for the Progress step (not part of
// the product).  G peers, each with an 8-entry u64 ring:
//   em   entry-major [8][G]: entry k of 64 peers is one 512-B row; a ring is
//        8 dwordx2 instructions
//   lm   lane-major [G][8]: a peer's ring is 64 contiguous bytes; 4 dwordx4
//        instructions, each lane touching its own 64-B line
// Loads (sum of the ring) and stores (the whole ring), with every lane or a
// random 60 % of the lanes active.  Prints ms, moved GB/s and cycles per
// instruction per CU (256 CUs at 2.4 GHz).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ bool active(size_t g, int k, int pct) {
  unsigned h = (unsigned)g * 0x9E3779B1u + k * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return pct >= 100 || (h % 100u) < (unsigned)pct;
}

template <int PCT>
__global__ __launch_bounds__(256) void em_load(const u64 *R, u64 *out, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  u64 acc = 0;
  const bool on = active(g, 0, PCT);
#pragma unroll
  for (int k = 0; k < 8; k++)
    if (on) acc += R[k * G + g];
  out[g] = acc;
}
template <int PCT>
__global__ __launch_bounds__(256) void lm_load(const u64 *R, u64 *out, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  u64 acc = 0;
  const bool on = active(g, 0, PCT);
  const u64x2 *r = reinterpret_cast<const u64x2 *>(R + g * 8);
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (on) {
      const u64x2 v = r[k];
      acc += v.x + v.y;
    }
  out[g] = acc;
}
template <int PCT>
__global__ __launch_bounds__(256) void em_store(u64 *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  const bool on = active(g, 0, PCT);
#pragma unroll
  for (int k = 0; k < 8; k++)
    if (on) R[k * G + g] = g + k;
}
template <int PCT>
__global__ __launch_bounds__(256) void lm_store(u64 *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  const bool on = active(g, 0, PCT);
  u64x2 *r = reinterpret_cast<u64x2 *>(R + g * 8);
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (on) r[k] = u64x2{g + 2 * k, g + 2 * k + 1};
}

template <typename F>
static float bench(F f) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 3; i++) f();
  std::vector<float> ms;
  for (int i = 0; i < 10; i++) {
    (void)hipEventRecord(a);
    f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float t = 0;
    (void)hipEventElapsedTime(&t, a, b);
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  return ms[ms.size() / 2];
}

static void rep(const char *n, float ms, double bytes, double instr) {
  printf("%-16s %.3f ms  %5.0f GB/s  %5.1f cyc/instr/CU\n", n, ms, bytes / (ms * 1e-3) / 1e9,
         ms * 1e-3 * 2.4e9 * 256 / instr);
}

int main() {
  const size_t G = 32ull << 20;
  u64 *R, *o;
  if (hipMalloc(&R, G * 64) || hipMalloc(&o, G * 8)) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(R, 1, G * 64);
  const dim3 grid(G / 256), blk(256);
  const double tiles = G / 64.0;
  float t;
  t = bench([&] { hipLaunchKernelGGL(em_load<100>, grid, blk, 0, 0, R, o, G); });
  rep("em load 100%", t, 72.0 * G, tiles * 9);
  t = bench([&] { hipLaunchKernelGGL(lm_load<100>, grid, blk, 0, 0, R, o, G); });
  rep("lm load 100%", t, 72.0 * G, tiles * 5);
  t = bench([&] { hipLaunchKernelGGL(em_load<60>, grid, blk, 0, 0, R, o, G); });
  rep("em load 60%", t, (0.6 * 64 + 8) * G, tiles * 9);
  t = bench([&] { hipLaunchKernelGGL(lm_load<60>, grid, blk, 0, 0, R, o, G); });
  rep("lm load 60%", t, (0.6 * 64 + 8) * G, tiles * 5);
  t = bench([&] { hipLaunchKernelGGL(em_store<100>, grid, blk, 0, 0, R, G); });
  rep("em store 100%", t, 64.0 * G, tiles * 8);
  t = bench([&] { hipLaunchKernelGGL(lm_store<100>, grid, blk, 0, 0, R, G); });
  rep("lm store 100%", t, 64.0 * G, tiles * 4);
  t = bench([&] { hipLaunchKernelGGL(em_store<60>, grid, blk, 0, 0, R, G); });
  rep("em store 60%", t, 0.6 * 64 * G, tiles * 8);
  t = bench([&] { hipLaunchKernelGGL(lm_store<60>, grid, blk, 0, 0, R, G); });
  rep("lm store 60%", t, 0.6 * 64 * G, tiles * 4);
  (void)hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
