// append_probe_gm.hip — a bcastAppend's Inflights appends by ring-block
// layout across slots (not part of the product; round-4 verdict item 6).
// G groups x S = 5 peers, 8-entry 32-bit rings (32 B per peer); one bcast
// appends one entry to each of the 4 followers (slots 1..4), each at its
// own data-dependent ring position (0..7), as qe_progress_send does.
//   sm   slot-major  [S][G][8]  (ABI 4: a slot's ring block of a tile is 2 KB)
//   gm   group-major [G][S][8]  (a group's 5 rings contiguous: 160 B)
//   gm8  group-major, slots padded to 8 ([G][8][8], 256 B per group)
//   gmq  group-major, the 4 appends of a group issued by 4 adjacent lanes
//        (a lane quad per group, 16 groups per wave, one store per lane)
// Prints ms, appended GB/s (4-byte entries) and cycles per wave-append per CU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32;

__device__ __forceinline__ u32 pos_of(size_t g, u32 s) {
  u32 h = (u32)g * 0x9E3779B1u + s * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h & 7u;
}

__global__ __launch_bounds__(256) void sm(u32 *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
#pragma unroll
  for (u32 s = 1; s < 5; s++) R[(s * G + g) * 8 + pos_of(g, s)] = (u32)g + s;
}
__global__ __launch_bounds__(256) void gm(u32 *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
#pragma unroll
  for (u32 s = 1; s < 5; s++) R[(g * 5 + s) * 8 + pos_of(g, s)] = (u32)g + s;
}
__global__ __launch_bounds__(256) void gm8(u32 *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
#pragma unroll
  for (u32 s = 1; s < 5; s++) R[(g * 8 + s) * 8 + pos_of(g, s)] = (u32)g + s;
}
__global__ __launch_bounds__(256) void gmq(u32 *R, size_t G) {
  const size_t t = blockIdx.x * 256ull + threadIdx.x;  // 4 lanes per group
  const size_t g = t >> 2;
  const u32 s = 1 + (u32)(t & 3);
  R[(g * 5 + s) * 8 + pos_of(g, s)] = (u32)g + s;
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

static void rep(const char *n, float ms, double G) {
  const double appends = 4.0 * G;
  printf("%-6s %.3f ms  %6.0f GB/s appended  %6.1f cyc/wave-append/CU\n", n, ms,
         appends * 4 / (ms * 1e-3) / 1e9, ms * 1e-3 * 2.4e9 * 256 / (appends / 64.0));
}

int main() {
  const size_t G = 16ull << 20;
  void *R;
  if (hipMalloc(&R, G * 256)) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(R, 1, G * 256);
  u32 *R32 = static_cast<u32 *>(R);
  const dim3 blk(256);
  float t;
  for (int rep_i = 0; rep_i < 2; rep_i++) {
    t = bench([&] { hipLaunchKernelGGL(sm, dim3(G / 256), blk, 0, 0, R32, G); });
    rep("sm", t, G);
    t = bench([&] { hipLaunchKernelGGL(gm, dim3(G / 256), blk, 0, 0, R32, G); });
    rep("gm", t, G);
    t = bench([&] { hipLaunchKernelGGL(gm8, dim3(G / 256), blk, 0, 0, R32, G); });
    rep("gm8", t, G);
    t = bench([&] { hipLaunchKernelGGL(gmq, dim3(4 * G / 256), blk, 0, 0, R32, G); });
    rep("gmq", t, G);
  }
  (void)hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
