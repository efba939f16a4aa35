// vmem_probe.hip — what bounds the byte-field kernels (Progress step,
// confchange)?  Not part of the product.  G groups, K byte arrays (SoA, one
// byte per group each), one byte written per group:
//   row    one buffer_load_ubyte per array per 64-group tile (K+1 vector
//          memory instructions per tile, 64 B each)
//   block  a 256-group block loads each array's 256 B with one dword
//          instruction of one wave, transposed through LDS (K/4+1 per tile)
//   row8   the same with u64 arrays (512 B per instruction)
// Prints ms, GB/s and cycles per vector memory instruction per CU
// (256 CUs at 2.4 GHz).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int KMAX = 16;
struct Arrs {
  const unsigned char *a[KMAX];
  const unsigned long long *w[KMAX];
};

__device__ __forceinline__ rsrc_t mk(const void *p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}

template <int K>
__global__ __launch_bounds__(256) void k_row(Arrs A, unsigned char *out, size_t G) {
  const size_t g0 = (blockIdx.x * 256ull) + (threadIdx.x & ~63u);
  const unsigned lane = threadIdx.x & 63;
  unsigned acc = 0;
#pragma unroll
  for (int k = 0; k < K; k++) acc ^= __builtin_amdgcn_raw_buffer_load_b8(mk(A.a[k] + g0, 64), lane, 0, 0) << (k & 7);
  __builtin_amdgcn_raw_buffer_store_b8((unsigned char)acc, mk(out + g0, 64), lane, 0, 0);
}

template <int K>
__global__ __launch_bounds__(256) void k_block(Arrs A, unsigned char *out, size_t G) {
  __shared__ unsigned lds[KMAX][64];
  const size_t b0 = blockIdx.x * 256ull;
  const unsigned w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < (K + 3) / 4; j++) {
    const unsigned k = 4 * j + w;
    if (k < K) lds[k][lane] = __builtin_amdgcn_raw_buffer_load_b32(mk(A.a[k] + b0, 256), lane * 4, 0, 0);
  }
  __syncthreads();
  const unsigned char *l8 = reinterpret_cast<const unsigned char *>(lds);
  unsigned acc = 0;
#pragma unroll
  for (int k = 0; k < K; k++) acc ^= (unsigned)l8[k * 256 + threadIdx.x] << (k & 7);
  __builtin_amdgcn_raw_buffer_store_b8((unsigned char)acc, mk(out + b0, 256), threadIdx.x, 0, 0);
}

template <int K>
__global__ __launch_bounds__(256) void k_row8(Arrs A, unsigned long long *out, size_t G) {
  const size_t g0 = (blockIdx.x * 256ull) + (threadIdx.x & ~63u);
  const unsigned lane = threadIdx.x & 63;
  unsigned long long acc = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    auto v = __builtin_amdgcn_raw_buffer_load_b64(mk(A.w[k] + g0, 512), lane * 8, 0, 0);
    acc ^= __builtin_bit_cast(unsigned long long, v) << (k & 7);
  }
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, acc), mk(out + g0, 512), lane * 8, 0, 0);
}

// u64 arrays, two rows per dwordx4 instruction: lanes 0-31 read 32 x 16 B
// of array 2j, lanes 32-63 of array 2j+1 (global addresses per lane)
template <int K>
__global__ __launch_bounds__(256) void k_row16(Arrs A, unsigned long long *out, size_t G) {
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  const size_t g0 = (blockIdx.x * 256ull) + (threadIdx.x & ~63u);
  const unsigned lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31;
  unsigned long long acc = 0;
#pragma unroll
  for (int j = 0; j < K / 2; j++) {
    const u64x2 v = *reinterpret_cast<const u64x2 *>(A.w[2 * j + h] + g0 + 2 * l);
    acc ^= (v.x + v.y) << (j & 7);
  }
  out[g0 + lane] = acc;
}

// partial writes: each wave stores K rows (u64 or u8); lane writes when a
// hash of (tile, row, lane) falls below P/8 (P = 8: every lane)
__device__ __forceinline__ unsigned hsh(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
template <int K, int P, typename T>
__global__ __launch_bounds__(256) void k_wr(T *const *W, size_t G) {
  const size_t g0 = (blockIdx.x * 256ull) + (threadIdx.x & ~63u);
  const unsigned lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < K; k++) {
    const bool on = P >= 8 || (hsh((unsigned)(g0 >> 6) * 131u + k * 977u + lane) & 7u) < (unsigned)P;
    if (on) W[k][g0 + lane] = (T)(g0 + lane + k);
  }
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
    float t;
    hipEventElapsedTime(&t, a, b);
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  return ms[ms.size() / 2];
}

static void report(const char *name, int K, float ms, double bytes, double instr_per_tile, size_t G) {
  const double tiles = G / 64.0;
  const double cyc = ms * 1e-3 * 2.4e9 * 256 / (tiles * instr_per_tile);
  printf("%-6s K=%2d  %.3f ms  %6.0f GB/s  %5.1f cycles/instr/CU\n", name, K, ms, bytes / (ms * 1e-3) / 1e9,
         cyc);
}

template <int K>
static void run(Arrs A, unsigned char *o, unsigned long long *o8, size_t G) {
  const dim3 grid(G / 256);
  float t = bench([&] { hipLaunchKernelGGL(k_row<K>, grid, dim3(256), 0, 0, A, o, G); });
  report("row", K, t, (K + 1.0) * G, K + 1, G);
  t = bench([&] { hipLaunchKernelGGL(k_block<K>, grid, dim3(256), 0, 0, A, o, G); });
  report("block", K, t, (K + 1.0) * G, (K + 3) / 4 + 1, G);
  t = bench([&] { hipLaunchKernelGGL(k_row8<K>, grid, dim3(256), 0, 0, A, o8, G); });
  report("row8", K, t, 8.0 * (K + 1.0) * G, K + 1, G);
  t = bench([&] { hipLaunchKernelGGL(k_row16<K>, grid, dim3(256), 0, 0, A, o8, G); });
  report("row16", K, t, 8.0 * (K + 1.0) * G, K / 2 + 1, G);
}

int main() {
  const size_t G = 16ull << 20;
  Arrs A;
  unsigned char *buf;
  unsigned long long *wbuf, *o8;
  unsigned char *o;
  if (hipMalloc(&buf, KMAX * G) || hipMalloc(&wbuf, KMAX * G * 8) || hipMalloc(&o, G) ||
      hipMalloc(&o8, G * 8)) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(buf, 3, KMAX * G);
  hipMemset(wbuf, 5, KMAX * G * 8);
  for (int k = 0; k < KMAX; k++) {
    A.a[k] = buf + k * G;
    A.w[k] = wbuf + k * G;
  }
  run<4>(A, o, o8, G);
  run<8>(A, o, o8, G);
  run<12>(A, o, o8, G);
  run<16>(A, o, o8, G);
  unsigned long long **W8;
  unsigned char **W1;
  hipMalloc(&W8, KMAX * sizeof(void *));
  hipMalloc(&W1, KMAX * sizeof(void *));
  hipMemcpy(W8, A.w, KMAX * sizeof(void *), hipMemcpyHostToDevice);
  hipMemcpy(W1, A.a, KMAX * sizeof(void *), hipMemcpyHostToDevice);
  const dim3 grid(G / 256);
  float t;
#define WR(P)                                                                                  \
  t = bench([&] { hipLaunchKernelGGL((k_wr<8, P, unsigned long long>), grid, dim3(256), 0, 0, W8, G); }); \
  report("wr8 P" #P, 8, t, 8.0 * 8 * G * P / 8, 8, G);                                          \
  t = bench([&] { hipLaunchKernelGGL((k_wr<8, P, unsigned char>), grid, dim3(256), 0, 0, W1, G); }); \
  report("wr1 P" #P, 8, t, 1.0 * 8 * G * P / 8, 8, G);
  WR(8) WR(6) WR(4) WR(1)
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
