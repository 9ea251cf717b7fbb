// tools/xcd_probe.hip -- what per-XCD work dealing can cost on MI355X
// (VERDICT r4 "do this" 5: deal a launch's units dynamically, one counter per
// XCD, so the launch has no second generation of waves).  Three questions:
//   1. placement: which XCD runs workgroup b (is it b % 8?);
//   2. throughput: how fast a resident grid (5120 waves) can take units from
//      counters -- one counter, eight counters by blockIdx % 8, eight by the
//      real XCC_ID -- at workgroup scope (the atomic stays in the XCD's own
//      L2) and at agent scope;
//   3. exactness: with per-XCC counters at workgroup scope, every unit is
//      taken exactly once (the counter is only ever touched from its own L2).
// Standalone: hipcc --offload-arch=gfx950 -O3 tools/xcd_probe.hip -o tools/xcd_probe
// Prints one JSON line per measurement.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 15u;
}

__global__ void k_place(uint32_t *out) {
  if ((threadIdx.x & 63u) == 0) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)(4u * gridDim.x * 4u), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(xcc_id(), r, 4u * (blockIdx.x * 4u + (threadIdx.x >> 6)), 0, 0);
  }
}

// Each wave takes units from its counter until the counter passes `quota`
// (mode 0: one counter; 1: eight by blockIdx % 8; 2: eight by XCC_ID), `chunk`
// units per take; every unit taken is marked in `seen` (a count per unit).
// SCOPE: 0 workgroup, 1 agent.
template <int SCOPE>
__global__ __launch_bounds__(256) void k_deal(uint32_t *ctr, uint32_t *seen, uint32_t units, uint32_t mode,
                                              uint32_t chunk, uint32_t spin) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t c = mode == 0 ? 0u : mode == 1 ? blockIdx.x % 8u : xcc_id() % 8u;
  const uint32_t per = mode == 0 ? units : units / 8u;
  const uint32_t base = mode == 0 ? 0u : c * per;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(seen, 0, (int)(4u * units), 0x00020000);
  uint32_t acc = 0;
  for (;;) {
    uint32_t u = 0;
    if (lane == 0)
      u = SCOPE == 0 ? __hip_atomic_fetch_add(ctr + 16u * c, chunk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                     : __hip_atomic_fetch_add(ctr + 16u * c, chunk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    u = __builtin_amdgcn_readfirstlane(u);
    if (u >= per) break;
    const uint32_t k = base + u + lane;
    if (lane < chunk && u + lane < per) {
      (void)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rs, (int)(4u * k), 0, 0);
    }
    for (uint32_t s = 0; s < spin; ++s) acc = acc * 1664525u + 1013904223u;  // stand-in for a unit's work
  }
  if (acc == 0x12345678u) (void)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rs, 0, 0, 0);
}

int main(int argc, char **argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 1280;
  uint32_t *d_place, *d_ctr, *d_seen;
  CHECK(hipMalloc(&d_place, 4u * blocks * 4u));
  CHECK(hipMalloc(&d_ctr, 4u * 16u * 8u));
  const uint32_t max_units = 1u << 18;
  CHECK(hipMalloc(&d_seen, 4u * max_units));
  // 1. placement
  hipLaunchKernelGGL(k_place, dim3(blocks), dim3(256), 0, 0, d_place);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> pl(blocks * 4u);
  CHECK(hipMemcpy(pl.data(), d_place, 4u * blocks * 4u, hipMemcpyDeviceToHost));
  int mod8 = 0, hist[16] = {};
  for (int b = 0; b < blocks; ++b) {
    mod8 += pl[4u * b] == (uint32_t)(b % 8);
    hist[pl[4u * b] & 15u]++;
  }
  printf("{\"probe\": \"placement\", \"blocks\": %d, \"xcc_eq_block_mod8\": %d, \"per_xcc\": [", blocks, mod8);
  for (int x = 0; x < 8; ++x) printf("%d%s", hist[x], x < 7 ? ", " : "]}\n");
  // 2./3. dealing
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (uint32_t units : {16384u, 65536u}) {
    for (uint32_t mode = 0; mode < 3; ++mode) {
      for (int scope = 0; scope < 2; ++scope) {
        for (uint32_t chunk : {1u, 4u}) {
          for (uint32_t spin : {0u, 400u}) {
            float best = 1e30f;
            uint32_t dup = 0, miss = 0;
            for (int rep = 0; rep < 5; ++rep) {
              CHECK(hipMemset(d_ctr, 0, 4u * 16u * 8u));
              CHECK(hipMemset(d_seen, 0, 4u * units));
              CHECK(hipDeviceSynchronize());
              CHECK(hipEventRecord(e0, 0));
              if (scope == 0)
                hipLaunchKernelGGL(k_deal<0>, dim3(blocks), dim3(256), 0, 0, d_ctr, d_seen, units, mode, chunk, spin);
              else
                hipLaunchKernelGGL(k_deal<1>, dim3(blocks), dim3(256), 0, 0, d_ctr, d_seen, units, mode, chunk, spin);
              CHECK(hipEventRecord(e1, 0));
              CHECK(hipEventSynchronize(e1));
              float ms = 0;
              CHECK(hipEventElapsedTime(&ms, e0, e1));
              best = ms < best ? ms : best;
              std::vector<uint32_t> seen(units);
              CHECK(hipMemcpy(seen.data(), d_seen, 4u * units, hipMemcpyDeviceToHost));
              for (uint32_t k = 0; k < units; ++k) {
                dup += seen[k] > 1;
                miss += seen[k] == 0;
              }
            }
            printf("{\"probe\": \"deal\", \"units\": %u, \"counters\": \"%s\", \"scope\": \"%s\", \"chunk\": %u, "
                   "\"spin\": %u, \"best_us\": %.2f, \"dup\": %u, \"miss\": %u}\n",
                   units, mode == 0 ? "one" : mode == 1 ? "block%8" : "xcc", scope ? "agent" : "workgroup", chunk,
                   spin, best * 1000.f, dup, miss);
            fflush(stdout);
          }
        }
      }
    }
  }
  return 0;
}
