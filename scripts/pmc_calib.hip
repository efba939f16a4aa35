// pmc_calib.hip — calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE (KiB) by
// access width on gfx950 (MI355X_MICROARCH.md §HBM: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
// Each kernel moves a KNOWN byte count over a 1 GiB region (4x the Infinity
// Cache), one wave per 64-lane row, in the widths the engine's kernels use:
//   r1 r2 r4 r8 r16    full-row loads of 1/2/4/8/16 B per lane (64..1024 B)
//   r8h                u64 row, every other lane (256 B read per 512-B row)
//   r16ring            16 B per lane at lane*32 (half of each lane's 32-B
//                      Inflights ring, the Progress step's ring load)
//   w1 w4 w8 w16       full-row stores
//   w4ring             one 4-B word per lane's 32-B ring (an Inflights.Add)
//   w16ring            16 B per lane at lane*32 (half a ring rewritten)
// The known bytes per launch are printed; scripts/pmc_calib.py divides them
// by the counters of the same kernels (separate --pmc passes).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned int u32;
typedef unsigned long long u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

constexpr size_t kRegion = 1ull << 30;

template <typename T>
__global__ __launch_bounds__(256) void rd(const T *__restrict__ p, size_t n, u32 *sink) {
  T acc{};
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) acc ^= p[i];
  if (acc == T(0x12345)) sink[0] = 1;
}
__global__ __launch_bounds__(256) void r16(const u32x4 *__restrict__ p, size_t n, u32 *sink) {
  u32 acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const u32x4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345u) sink[0] = 1;
}
__global__ __launch_bounds__(256) void r8h(const u64 *__restrict__ p, size_t n, u32 *sink) {
  u64 acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    if ((i & 1) == 0) acc ^= p[i];
  if (acc == 0x12345ull) sink[0] = 1;
}
// lane l of a row reads 16 B at l*32: n = number of 32-B rings
__global__ __launch_bounds__(256) void r16ring(const u32x4 *__restrict__ p, size_t n, u32 *sink) {
  u32 acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const u32x4 v = p[2 * i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345u) sink[0] = 1;
}
template <typename T>
__global__ __launch_bounds__(256) void wr(T *__restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) p[i] = T(i);
}
__global__ __launch_bounds__(256) void w16(u32x4 *__restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    p[i] = u32x4{(u32)i, 1u, 2u, 3u};
}
__global__ __launch_bounds__(256) void w4ring(u32 *__restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    u32 h = (u32)i * 0x9E3779B1u;
    h ^= h >> 15;
    p[8 * i + (h & 7u)] = (u32)i;
  }
}
__global__ __launch_bounds__(256) void w16ring(u32x4 *__restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    p[2 * i] = u32x4{(u32)i, 1u, 2u, 3u};
}

int main() {
  void *buf;
  u32 *sink;
  if (hipMalloc(&buf, kRegion) || hipMalloc(&sink, 64)) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(buf, 3, kRegion);
  const dim3 grid(256 * 32), blk(256);
  auto launch = [&](const char *name, double bytes, auto f) {
    for (int i = 0; i < 3; i++) f();
    (void)hipDeviceSynchronize();
    printf("%-8s known_bytes %.0f\n", name, bytes);
  };
  const size_t R = kRegion;
  launch("r1", R, [&] { hipLaunchKernelGGL(rd<unsigned char>, grid, blk, 0, 0, (const unsigned char *)buf, R, sink); });
  launch("r2", R, [&] { hipLaunchKernelGGL(rd<unsigned short>, grid, blk, 0, 0, (const unsigned short *)buf, R / 2, sink); });
  launch("r4", R, [&] { hipLaunchKernelGGL(rd<u32>, grid, blk, 0, 0, (const u32 *)buf, R / 4, sink); });
  launch("r8", R, [&] { hipLaunchKernelGGL(rd<u64>, grid, blk, 0, 0, (const u64 *)buf, R / 8, sink); });
  launch("r16", R, [&] { hipLaunchKernelGGL(r16, grid, blk, 0, 0, (const u32x4 *)buf, R / 16, sink); });
  launch("r8h", R / 2, [&] { hipLaunchKernelGGL(r8h, grid, blk, 0, 0, (const u64 *)buf, R / 8, sink); });
  launch("r16ring", R / 2, [&] { hipLaunchKernelGGL(r16ring, grid, blk, 0, 0, (const u32x4 *)buf, R / 32, sink); });
  launch("w1", R, [&] { hipLaunchKernelGGL(wr<unsigned char>, grid, blk, 0, 0, (unsigned char *)buf, R); });
  launch("w4", R, [&] { hipLaunchKernelGGL(wr<u32>, grid, blk, 0, 0, (u32 *)buf, R / 4); });
  launch("w8", R, [&] { hipLaunchKernelGGL(wr<u64>, grid, blk, 0, 0, (u64 *)buf, R / 8); });
  launch("w16", R, [&] { hipLaunchKernelGGL(w16, grid, blk, 0, 0, (u32x4 *)buf, R / 16); });
  launch("w4ring", R / 8, [&] { hipLaunchKernelGGL(w4ring, grid, blk, 0, 0, (u32 *)buf, R / 32); });
  launch("w16ring", R / 2, [&] { hipLaunchKernelGGL(w16ring, grid, blk, 0, 0, (u32x4 *)buf, R / 32); });
  printf("done\n");
  return 0;
}
