// Probe: buffer_load_dwordx4 ... lds (LDS-DMA) on gfx950 at byte-misaligned
// source offsets, and out-of-range lanes: does lane i's 16 bytes land at
// LDS base + 16 i with the bytes at that source offset (0 when out of range)?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const uint8_t *src, uint32_t *out) {
  __shared__ u32x4 s[64];
  const int t = threadIdx.x;
  s[t] = u32x4{0xdeadbeef, 0xdeadbeef, 0xdeadbeef, 0xdeadbeef};
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), 0, 4096, 0x00020000);
  const uint32_t off = t < 60 ? (uint32_t)(t * 37 + (t & 15)) : 0xFFFFF000u;  // lanes 60..63 out of range
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)s, 16, off, 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  const u32x4 v = s[t];
  out[4 * t] = v.x; out[4 * t + 1] = v.y; out[4 * t + 2] = v.z; out[4 * t + 3] = v.w;
}
int main() {
  uint8_t h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 13 + 5);
  uint8_t *d; uint32_t *o;
  if (hipMalloc(&d, 4096) || hipMalloc(&o, 64 * 16)) return 1;
  if (hipMemcpy(d, h, 4096, hipMemcpyHostToDevice)) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  uint32_t r[256];
  if (hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost)) return 1;
  int bad = 0, oob_zero = 0;
  for (int t = 0; t < 64; ++t) {
    uint32_t w[4] = {0, 0, 0, 0};
    if (t < 60) __builtin_memcpy(w, h + t * 37 + (t & 15), 16);
    int ok = 1;
    for (int j = 0; j < 4; ++j) ok &= r[4 * t + j] == w[j];
    if (t < 60) bad += !ok; else oob_zero += ok;
  }
  printf("lds-dma unaligned mismatches (of 60): %d; out-of-range lanes reading 0: %d of 4 (lane 60 word0 %08x)\n",
         bad, oob_zero, r[240]);
  return 0;
}
