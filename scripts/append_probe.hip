// append_probe.hip — cost of Inflights appends (Inflights.Add at a
// data-dependent ring position, raft/tracker/inflights.go:55-71) by ring
// layout and entry width (not part of the product).  G peers, 8-entry rings,
// each peer appends one entry at its own random position p (0..7):
//   em64 / em32   entry-major [8][G]: entry k of 64 peers is one row
//   tb64 / tb32   tile-blocked [G/64][8][64]: a tile's ring block is contiguous
//   lm64 / lm32   lane-major [G][8]: a peer's ring is contiguous
// "scatter": one store instruction, each lane at its own position;
// "rows": 8 row stores, lane active in row p only (the step's ring_flush);
// "rmw":  the whole ring loaded and stored back (full sectors).
// Prints ms, appended GB/s (entry bytes) and cycles per wave per CU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;
typedef unsigned int u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32 pos_of(size_t g) {
  u32 h = (u32)g * 0x9E3779B1u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h & 7u;
}

template <typename T>
__global__ __launch_bounds__(256) void em_scatter(T *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  R[pos_of(g) * G + g] = (T)(g + 1);
}
template <typename T>
__global__ __launch_bounds__(256) void tb_scatter(T *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  R[(g >> 6) * 512 + pos_of(g) * 64 + (g & 63)] = (T)(g + 1);
}
template <typename T>
__global__ __launch_bounds__(256) void lm_scatter(T *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  R[g * 8 + pos_of(g)] = (T)(g + 1);
}
template <typename T>
__global__ __launch_bounds__(256) void em_rows(T *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  const u32 p = pos_of(g);
#pragma unroll
  for (u32 k = 0; k < 8; k++)
    if (p == k) R[k * G + g] = (T)(g + 1);
}
template <typename T>
__global__ __launch_bounds__(256) void tb_rows(T *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  const u32 p = pos_of(g);
#pragma unroll
  for (u32 k = 0; k < 8; k++)
    if (p == k) R[(g >> 6) * 512 + k * 64 + (g & 63)] = (T)(g + 1);
}
// lane-major u32 ring = 32 B per peer: two dwordx4 loads + two stores
__global__ __launch_bounds__(256) void lm32_rmw(u32 *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  u32x4 *r = reinterpret_cast<u32x4 *>(R + g * 8);
  u32x4 a = r[0], b = r[1];
  const u32 p = pos_of(g), v = (u32)(g + 1);
  a.x = p == 0 ? v : a.x; a.y = p == 1 ? v : a.y; a.z = p == 2 ? v : a.z; a.w = p == 3 ? v : a.w;
  b.x = p == 4 ? v : b.x; b.y = p == 5 ? v : b.y; b.z = p == 6 ? v : b.z; b.w = p == 7 ? v : b.w;
  r[0] = a;
  r[1] = b;
}
// lane-major u16 ring = 16 B per peer (round 6: the 16-bit offsets the
// Inflights rings would need): one dwordx4 load + one store;
// two peers share a 32-B sector
typedef unsigned short u16;
__global__ __launch_bounds__(256) void lm16_rmw(u16 *R, size_t G) {
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  u32x4 *r = reinterpret_cast<u32x4 *>(R + g * 8);
  u32x4 a = r[0];
  const u32 p = pos_of(g), v = (u32)(g + 1) & 0xFFFFu;
  const u32 sh = (p & 1u) * 16u, keep = ~(0xFFFFu << sh), nv = v << sh;
  a.x = (p >> 1) == 0 ? (a.x & keep) | nv : a.x;
  a.y = (p >> 1) == 1 ? (a.y & keep) | nv : a.y;
  a.z = (p >> 1) == 2 ? (a.z & keep) | nv : a.z;
  a.w = (p >> 1) == 3 ? (a.w & keep) | nv : a.w;
  r[0] = a;
}
// tile-blocked u32 block (2 KB per 64 peers) loaded and stored whole, 16 B
// per lane per instruction, the append applied through LDS
__global__ __launch_bounds__(256) void tb32_rmw(u32 *R, size_t G) {
  __shared__ u32 l[4][512];
  const size_t g = blockIdx.x * 256ull + threadIdx.x;
  const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  u32x4 *blk = reinterpret_cast<u32x4 *>(R + (g >> 6) * 512);
  const u32x4 a = blk[lane], b = blk[64 + lane];
  *reinterpret_cast<u32x4 *>(&l[w][lane * 4]) = a;
  *reinterpret_cast<u32x4 *>(&l[w][256 + lane * 4]) = b;
  __builtin_amdgcn_wave_barrier();
  l[w][pos_of(g) * 64 + lane] = (u32)(g + 1);
  __builtin_amdgcn_wave_barrier();
  blk[lane] = *reinterpret_cast<u32x4 *>(&l[w][lane * 4]);
  blk[64 + lane] = *reinterpret_cast<u32x4 *>(&l[w][256 + lane * 4]);
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

static void rep(const char *n, float ms, double G, int bytes) {
  printf("%-14s %.3f ms  %6.0f GB/s appended  %6.1f cyc/wave/CU\n", n, ms,
         G * bytes / (ms * 1e-3) / 1e9, ms * 1e-3 * 2.4e9 * 256 / (G / 64.0));
}

int main() {
  const size_t G = 32ull << 20;
  void *R;
  if (hipMalloc(&R, G * 64)) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(R, 1, G * 64);
  const dim3 grid(G / 256), blk(256);
  u64 *R64 = static_cast<u64 *>(R);
  u32 *R32 = static_cast<u32 *>(R);
  float t;
  t = bench([&] { hipLaunchKernelGGL(em_scatter<u64>, grid, blk, 0, 0, R64, G); });
  rep("em64 scatter", t, G, 8);
  t = bench([&] { hipLaunchKernelGGL(em_scatter<u32>, grid, blk, 0, 0, R32, G); });
  rep("em32 scatter", t, G, 4);
  t = bench([&] { hipLaunchKernelGGL(tb_scatter<u64>, grid, blk, 0, 0, R64, G); });
  rep("tb64 scatter", t, G, 8);
  t = bench([&] { hipLaunchKernelGGL(tb_scatter<u32>, grid, blk, 0, 0, R32, G); });
  rep("tb32 scatter", t, G, 4);
  t = bench([&] { hipLaunchKernelGGL(lm_scatter<u64>, grid, blk, 0, 0, R64, G); });
  rep("lm64 scatter", t, G, 8);
  t = bench([&] { hipLaunchKernelGGL(lm_scatter<u32>, grid, blk, 0, 0, R32, G); });
  rep("lm32 scatter", t, G, 4);
  t = bench([&] { hipLaunchKernelGGL(em_rows<u64>, grid, blk, 0, 0, R64, G); });
  rep("em64 rows", t, G, 8);
  t = bench([&] { hipLaunchKernelGGL(em_rows<u32>, grid, blk, 0, 0, R32, G); });
  rep("em32 rows", t, G, 4);
  t = bench([&] { hipLaunchKernelGGL(tb_rows<u64>, grid, blk, 0, 0, R64, G); });
  rep("tb64 rows", t, G, 8);
  t = bench([&] { hipLaunchKernelGGL(tb_rows<u32>, grid, blk, 0, 0, R32, G); });
  rep("tb32 rows", t, G, 4);
  t = bench([&] { hipLaunchKernelGGL(lm32_rmw, grid, blk, 0, 0, R32, G); });
  rep("lm32 rmw", t, G, 4);
  t = bench([&] { hipLaunchKernelGGL(tb32_rmw, grid, blk, 0, 0, R32, G); });
  rep("tb32 rmw", t, G, 4);
  u16 *R16 = static_cast<u16 *>(R);
  t = bench([&] { hipLaunchKernelGGL(lm_scatter<u16>, grid, blk, 0, 0, R16, G); });
  rep("lm16 scatter", t, G, 2);
  t = bench([&] { hipLaunchKernelGGL(lm16_rmw, grid, blk, 0, 0, R16, G); });
  rep("lm16 rmw", t, G, 2);
  (void)hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
