// soffset_probe.hip — is a raw buffer access's SGPR offset (soffset) part of
// the range check against num_records on gfx950?  A 64-byte descriptor at
// the start of an 8 KiB buffer is read and written at voffset = lane*4 with
// soffset = 4096: if soffset is outside the check, lanes 0-15 reach bytes
// 4096..4159 (in range by voffset) and lanes 16-63 are dropped (voffset >=
// 64); every access stays inside the allocation either way.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned int u32;

__global__ void k_probe(u32 *buf, u32 *out) {
  const u32 lane = threadIdx.x;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 64, 0x00020000);
  const u32 v = __builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, 4096, 0);
  out[lane] = v;
  __builtin_amdgcn_raw_buffer_store_b32(0xABCD0000u + lane, r, lane * 4, 6144, 0);
}

int main() {
  u32 *buf, *out;
  if (hipMalloc(&buf, 8192) != hipSuccess || hipMalloc(&out, 256) != hipSuccess) return 1;
  u32 h[2048];
  for (int i = 0; i < 2048; i++) h[i] = i;
  if (hipMemcpy(buf, h, 8192, hipMemcpyHostToDevice) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, buf, out);
  u32 o[64];
  if (hipMemcpy(o, out, 256, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (hipMemcpy(h, buf, 8192, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int in_load = 0, in_store = 0, dropped_load = 0;
  for (int l = 0; l < 64; l++) {
    if (l < 16 && o[l] == static_cast<u32>(1024 + l)) in_load++;
    if (l >= 16 && o[l] == 0) dropped_load++;
  }
  for (int l = 0; l < 64; l++)
    if (h[1536 + l] == 0xABCD0000u + static_cast<u32>(l)) in_store++;
  printf("loads reaching soffset+voffset for voffset<64: %d/16, dropped voffset>=64: %d/48, stores landed: %d/64\n",
         in_load, dropped_load, in_store);
  printf("soffset %s the range check\n", (in_load == 16 && dropped_load == 48 && in_store == 16) ? "is OUTSIDE" : "is INSIDE or other");
  return 0;
}
