// membw.hip — HBM ceiling probe for the quorum kernels' access mix (not part
// of the product).  Streams a 3.4 GB working set with 16-byte loads:
//   read   : pure read (a reduction; one word written per thread)
//   copy   : 1:1 read/write
//   mix41  : 40 B read + 1 u64 write per 16 B of pairs (≈ the 53 B/group
//            commit_vote mix: 42 B read, 11 B written)
// Each with plain and non-temporal accesses.  Prints GB/s (median of 20).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

template <bool NT>
__global__ void k_read(const u64x2 *__restrict__ p, size_t n, u64 *out) {
  u64 acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    u64x2 v = NT ? __builtin_nontemporal_load(p + i) : p[i];
    acc += v.x ^ v.y;
  }
  if (acc == 0x1234567) out[0] = acc;
}

template <bool NT>
__global__ void k_copy(const u64x2 *__restrict__ p, u64x2 *__restrict__ q, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    u64x2 v = NT ? __builtin_nontemporal_load(p + i) : p[i];
    if (NT) __builtin_nontemporal_store(v, q + i);
    else q[i] = v;
  }
}

// five SoA rows of pairs read, one row of pairs written (ratio 5:1)
template <bool NT>
__global__ void k_mix(const u64x2 *__restrict__ p, size_t rows_stride, u64x2 *__restrict__ q,
                      size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    u64x2 acc = {0, 0};
#pragma unroll
    for (int s = 0; s < 5; s++) {
      u64x2 v = NT ? __builtin_nontemporal_load(p + s * rows_stride + i) : p[s * rows_stride + i];
      acc.x += v.x;
      acc.y ^= v.y;
    }
    if (NT) __builtin_nontemporal_store(acc, q + i);
    else q[i] = acc;
  }
}

template <typename F>
static double bench(F f, double bytes) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 5; i++) f();
  std::vector<float> ms;
  for (int i = 0; i < 20; i++) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float t;
    hipEventElapsedTime(&t, a, b);
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  return bytes / (ms[ms.size() / 2] * 1e-3) / 1e9;
}

int main() {
  const size_t bytes = 3400ull << 20;  // 3.4 GB
  const size_t n = bytes / 16;
  u64x2 *p, *q;
  u64 *o;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&q, bytes) != hipSuccess ||
      hipMalloc(&o, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(p, 1, bytes);
  hipMemset(q, 0, bytes);
  for (int grid : {2048, 8192, 65536}) {
    const int blk = 256;
    printf("grid %d read     %.0f GB/s  nt %.0f GB/s\n", grid,
           bench([&] { hipLaunchKernelGGL(k_read<false>, dim3(grid), dim3(blk), 0, 0, p, n, o); },
                 (double)bytes),
           bench([&] { hipLaunchKernelGGL(k_read<true>, dim3(grid), dim3(blk), 0, 0, p, n, o); },
                 (double)bytes));
    printf("grid %d copy     %.0f GB/s  nt %.0f GB/s\n", grid,
           bench([&] { hipLaunchKernelGGL(k_copy<false>, dim3(grid), dim3(blk), 0, 0, p, q, n / 2); },
                 (double)bytes),
           bench([&] { hipLaunchKernelGGL(k_copy<true>, dim3(grid), dim3(blk), 0, 0, p, q, n / 2); },
                 (double)bytes));
    const size_t rn = n / 6;  // 5 read rows + 1 written row
    printf("grid %d mix5:1   %.0f GB/s  nt %.0f GB/s\n", grid,
           bench([&] { hipLaunchKernelGGL(k_mix<false>, dim3(grid), dim3(blk), 0, 0, p, rn, q, rn); },
                 6.0 * rn * 16),
           bench([&] { hipLaunchKernelGGL(k_mix<true>, dim3(grid), dim3(blk), 0, 0, p, rn, q, rn); },
                 6.0 * rn * 16));
  }
  return 0;
}
