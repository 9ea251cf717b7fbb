// Probe: do buffer_load_dwordx4 / global_load_dwordx4 at byte-misaligned
// addresses return the bytes at that address on gfx950 (unaligned mode)?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const uint8_t *src, uint32_t *out) {
  const int t = threadIdx.x;  // offset t (0..63)
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), 0, 4096, 0x00020000);
  u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)t, 0, 0);
  u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)t, 0, 2);
  const u32x4 *g = (const u32x4 *)(src + t);
  u32x4 c = *g;
  uint32_t *o = out + t * 12;
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  o[8] = c.x; o[9] = c.y; o[10] = c.z; o[11] = c.w;
}
int main() {
  uint8_t h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 7 + 3);
  uint8_t *d; uint32_t *o;
  hipMalloc(&d, 4096); hipMalloc(&o, 64 * 48);
  hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  uint32_t r[64 * 12];
  hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
  int bad[3] = {0, 0, 0};
  for (int t = 0; t < 64; ++t)
    for (int m = 0; m < 3; ++m) {
      uint32_t w[4];
      __builtin_memcpy(w, h + t, 16);
      for (int j = 0; j < 4; ++j) if (r[t * 12 + m * 4 + j] != w[j]) { bad[m]++; break; }
    }
  printf("unaligned mismatches (of 64 offsets): buffer default %d, buffer nt %d, global %d\n", bad[0], bad[1], bad[2]);
  return 0;
}
