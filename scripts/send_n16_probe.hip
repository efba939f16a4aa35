// send_n16_probe.hip -- the memory pattern of qe_progress_send (bcastAppend
// to 4 followers of 16M groups, F = 8) with 32-bit Inflights words (ABI 4:
// one 4-B store per append into the peer's own 32-B ring sector) against a
// 16-bit form (8 x u16 per peer, two peers per 32-B sector: the peer's 16-B
// ring read and written whole).  Not part of the product: a go / no-go probe
// for a 16-bit ring representation (round 6).  Both modes load firstIndex /
// lastIndex per group and Next + the packed word per follower, store Next +
// the word, and append one entry at ring position (start + count) % 8.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;

__device__ __forceinline__ rsrc_t mk(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint64_t ld64(rsrc_t r, uint32_t o) {
  return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, 2));
}
__device__ __forceinline__ uint32_t ld32(rsrc_t r, uint32_t o) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 2);
}
__device__ __forceinline__ void st64(uint64_t v, rsrc_t r, uint32_t o) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, o, 0, 2);
}
__device__ __forceinline__ void st32(uint32_t v, rsrc_t r, uint32_t o) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, o, 0, 2);
}

template <int MODE>  // 0: 32-bit words, scatter; 1: 16-bit ring, read + write whole
__global__ __launch_bounds__(256) void k_send(uint64_t G, uint64_t stride, const uint64_t *fi,
                                              const uint64_t *li, uint64_t *next, uint32_t *pw,
                                              uint32_t *r32, uint16_t *r16) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = blockIdx.x * 4ull + (threadIdx.x >> 6);
  const uint64_t nw = gridDim.x * 4ull;
  const uint64_t nt = (G + 63) / 64;
  for (uint64_t t = wave; t < nt; t += nw) {
    const uint64_t g0 = t * 64;
    const uint32_t n = (uint32_t)(G - g0 < 64 ? G - g0 : 64);
    const uint64_t f = ld64(mk(fi + g0, n * 8), lane * 8);
    const uint64_t l = ld64(mk(li + g0, n * 8), lane * 8);
    uint64_t nx[5];
    uint32_t w[5];
    u32x4 rg[5];
#pragma unroll
    for (int s = 1; s < 5; s++) {
      const uint64_t row = s * stride + g0;
      nx[s] = ld64(mk(next + row, n * 8), lane * 8);
      w[s] = ld32(mk(pw + row, n * 4), lane * 4);
      if (MODE == 1)
        rg[s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              mk(r16 + row * 8, n * 16), lane * 16, 0, 2));
    }
#pragma unroll
    for (int s = 1; s < 5; s++) {
      const uint64_t row = s * stride + g0;
      const uint32_t start = (w[s] >> 8) & 7, cnt = (w[s] >> 16) & 0xFF;
      const bool go = nx[s] <= l && nx[s] >= f && cnt < 8;
      const uint32_t pos = (start + cnt) & 7;
      const uint64_t v = nx[s] + 15 < l ? nx[s] + 15 : l;
      st64(v + 1, mk(next + row, n * 8), go ? lane * 8 : kOOB);
      st32(w[s] + (1u << 16), mk(pw + row, n * 4), go ? lane * 4 : kOOB);
      if (MODE == 0) {
        st32((uint32_t)v, mk(r32 + row * 8, n * 32), go ? lane * 32 + pos * 4 : kOOB);
      } else {
        // every live entry re-based on the new Next: offsets shift by the
        // append's advance, the new entry at offset 0
        const uint32_t d = (uint32_t)(v + 1 - nx[s]);
        u32x4 r = rg[s];
        const uint32_t dd = d | (d << 16);
        r.x += dd, r.y += dd, r.z += dd, r.w += dd;
        const uint32_t sh = 16 * (pos & 1), m = ~(0xFFFFu << sh);
        if ((pos >> 1) == 0) r.x &= m;
        if ((pos >> 1) == 1) r.y &= m;
        if ((pos >> 1) == 2) r.z &= m;
        if ((pos >> 1) == 3) r.w &= m;
        __builtin_amdgcn_raw_buffer_store_b128(r, mk(r16 + row * 8, n * 16), go ? lane * 16 : kOOB,
                                               0, 2);
      }
    }
  }
}

int main() {
  const uint64_t G = 1ull << 24, stride = G, S = 5;
  std::vector<uint64_t> hfi(G), hli(G), hnx(S * stride);
  std::vector<uint32_t> hpw(S * stride);
  uint64_t x = 88172645463325252ull;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  for (uint64_t g = 0; g < G; g++) {
    const uint64_t base = (1ull << 20) + rnd() % (1ull << 39);
    hfi[g] = base - 64;
    hli[g] = base + 128;
    for (uint64_t s = 0; s < S; s++) {
      hnx[s * stride + g] = base + 1 + rnd() % 4;
      hpw[s * stride + g] = 1u | 8u | ((uint32_t)(rnd() % 8) << 8) | ((uint32_t)(rnd() % 8) << 16);
    }
  }
  uint64_t *fi, *li, *nx, *nx0;
  uint32_t *pw, *pw0, *r32;
  uint16_t *r16;
  hipMalloc(&fi, G * 8);
  hipMalloc(&li, G * 8);
  hipMalloc(&nx, S * stride * 8);
  hipMalloc(&nx0, S * stride * 8);
  hipMalloc(&pw, S * stride * 4);
  hipMalloc(&pw0, S * stride * 4);
  hipMalloc(&r32, S * stride * 32);
  hipMalloc(&r16, S * stride * 16);
  hipMemcpy(fi, hfi.data(), G * 8, hipMemcpyHostToDevice);
  hipMemcpy(li, hli.data(), G * 8, hipMemcpyHostToDevice);
  hipMemcpy(nx0, hnx.data(), S * stride * 8, hipMemcpyHostToDevice);
  hipMemcpy(pw0, hpw.data(), S * stride * 4, hipMemcpyHostToDevice);
  hipMemset(r32, 0, S * stride * 32);
  hipMemset(r16, 0, S * stride * 16);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks = 256 * 8;
  for (int mode = 0; mode < 2; mode++) {
    float best = 1e9f, sum = 0.f;
    int reps = 0;
    for (int it = 0; it < 25; it++) {
      hipMemcpy(nx, nx0, S * stride * 8, hipMemcpyDeviceToDevice);
      hipMemcpy(pw, pw0, S * stride * 4, hipMemcpyDeviceToDevice);
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(k_send<0>, dim3(blocks), dim3(256), 0, 0, G, stride, fi, li, nx, pw, r32, r16);
      else hipLaunchKernelGGL(k_send<1>, dim3(blocks), dim3(256), 0, 0, G, stride, fi, li, nx, pw, r32, r16);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (it >= 5) {
        best = ms < best ? ms : best;
        sum += ms;
        reps++;
      }
    }
    printf("%s  mean %.4f ms  min %.4f ms\n", mode == 0 ? "ring32 scatter" : "ring16 rmw    ", sum / reps, best);
  }
  printf("done\n");
  return 0;
}
