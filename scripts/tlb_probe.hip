// tlb_probe.hip — does the number of distinct arrays a wave touches per
// 64-group tile bound a many-field kernel (the Progress step touches ~100
// SoA rows per tile)?  Not part of the product.  Each wave reads K rows
// (u8: 64 B per row, or u64: 512 B) and writes one:
//   sep   K separate SoA arrays (row k of tile t at arr_k + 64 t)
//   blk   one tile-blocked array [tile][K][64]: a tile's K rows contiguous
// Same bytes, same instruction count; only the address pattern differs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int KMAX = 64;
template <typename T>
struct Arrs {
  const T *a[KMAX];
};

__device__ __forceinline__ rsrc_t mk(const void *p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}
template <typename T>
__device__ __forceinline__ unsigned long long ld(const T *p, unsigned lane) {
  if constexpr (sizeof(T) == 1) return __builtin_amdgcn_raw_buffer_load_b8(mk(p, 64), lane, 0, 0);
  else return __builtin_bit_cast(unsigned long long, __builtin_amdgcn_raw_buffer_load_b64(mk(p, 512), lane * 8, 0, 0));
}

template <int K, typename T>
__global__ __launch_bounds__(256) void k_sep(Arrs<T> A, T *out) {
  const size_t g0 = (blockIdx.x * 256ull) + (threadIdx.x & ~63u);
  const unsigned lane = threadIdx.x & 63;
  unsigned long long acc = 0;
#pragma unroll
  for (int k = 0; k < K; k++) acc ^= ld(A.a[k] + g0, lane) << (k & 7);
  out[g0 + lane] = (T)acc;
}

template <int K, typename T>
__global__ __launch_bounds__(256) void k_blk(const T *B, T *out) {
  const size_t t = blockIdx.x * 4ull + (threadIdx.x >> 6);
  const size_t g0 = t * 64;
  const unsigned lane = threadIdx.x & 63;
  const T *base = B + t * K * 64;
  unsigned long long acc = 0;
#pragma unroll
  for (int k = 0; k < K; k++) acc ^= ld(base + k * 64, lane) << (k & 7);
  out[g0 + lane] = (T)acc;
}

// u64 rows with a fraction P/8 of the lanes active (the others get an
// out-of-range offset: no traffic): does a masked row cost less?
template <int K, int P>
__global__ __launch_bounds__(256) void k_msk(Arrs<unsigned long long> A, unsigned long long *out) {
  const size_t g0 = (blockIdx.x * 256ull) + (threadIdx.x & ~63u);
  const unsigned lane = threadIdx.x & 63;
  unsigned long long acc = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    unsigned h = (unsigned)(g0 >> 6) * 0x9E3779B1u + k * 0x85EBCA77u + lane * 0xC2B2AE3Du;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    const bool on = P >= 8 || (P < 0 ? lane < (unsigned)(-8 * P) : (h & 7u) < (unsigned)P);
    acc ^= __builtin_bit_cast(unsigned long long, __builtin_amdgcn_raw_buffer_load_b64(
                                                       mk(A.a[k] + g0, 512), on ? lane * 8 : 0x80000000u, 0, 0))
           << (k & 7);
  }
  out[g0 + lane] = acc;
}

template <typename F>
static float bench(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; i++) f();
  std::vector<float> ms;
  for (int i = 0; i < 10; i++) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float t = 0;
    (void)hipEventElapsedTime(&t, a, b);
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  return ms[ms.size() / 2];
}

template <int K, typename T>
static void run(T *buf, T *out, size_t G) {
  Arrs<T> A;
  for (int k = 0; k < K; k++) A.a[k] = buf + k * G;
  const dim3 grid(G / 256);
  const float ts = bench([&] { hipLaunchKernelGGL((k_sep<K, T>), grid, dim3(256), 0, 0, A, out); });
  const float tb = bench([&] { hipLaunchKernelGGL((k_blk<K, T>), grid, dim3(256), 0, 0, buf, out); });
  const double bytes = (K + 1.0) * G * sizeof(T), instr = (G / 64.0) * (K + 1);
  auto cyc = [&](float ms) { return ms * 1e-3 * 2.4e9 * 256 / instr; };
  printf("u%-2d K=%2d  sep %.3f ms %5.0f GB/s %5.1f cyc/instr/CU   blk %.3f ms %5.0f GB/s %5.1f cyc/instr/CU\n",
         (int)(8 * sizeof(T)), K, ts, bytes / (ts * 1e-3) / 1e9, cyc(ts), tb, bytes / (tb * 1e-3) / 1e9, cyc(tb));
}

int main() {
  const size_t G = 8ull << 20;
  unsigned char *b1, *o1;
  unsigned long long *b8, *o8;
  if (hipMalloc(&b1, KMAX * G) || hipMalloc(&b8, KMAX * G * 8) || hipMalloc(&o1, G) || hipMalloc(&o8, G * 8)) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(b1, 3, KMAX * G);
  (void)hipMemset(b8, 5, KMAX * G * 8);
  run<8>(b1, o1, G);
  run<16>(b1, o1, G);
  run<32>(b1, o1, G);
  run<64>(b1, o1, G);
  run<8>(b8, o8, G);
  run<16>(b8, o8, G);
  run<32>(b8, o8, G);
  run<64>(b8, o8, G);
  {
    Arrs<unsigned long long> A;
    for (int k = 0; k < 16; k++) A.a[k] = b8 + k * G;
    const dim3 grid(G / 256);
    const double instr = (G / 64.0) * 17;
#define MSK(P)                                                                                    \
    {                                                                                             \
      const float t = bench([&] { hipLaunchKernelGGL((k_msk<16, P>), grid, dim3(256), 0, 0, A, o8); }); \
      printf("u64 K=16 lanes %d/8: %.3f ms  %5.0f GB/s moved  %5.1f cyc/instr/CU\n", P, t,            \
             (16.0 * (P < 0 ? -P : P) / 8 + 1) * G * 8 / (t * 1e-3) / 1e9, t * 1e-3 * 2.4e9 * 256 / instr);           \
    }
    MSK(8) MSK(6) MSK(4) MSK(2) MSK(1) MSK(-6) MSK(-4) MSK(-2) MSK(-1)
  }
  (void)hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
