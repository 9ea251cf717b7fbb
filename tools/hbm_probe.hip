// tools/hbm_probe.hip -- what HBM read bandwidth does this MI355X deliver to a
// plain streaming kernel?  The ceiling the checksum kernels are judged against
// in practice (the spec peak, 8 TB/s, is what roofline.peak uses).
//
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o tools/hbm_probe && tools/hbm_probe
//
// Reads a 2 GiB buffer (8x the 256 MiB Infinity Cache) with 16-byte loads:
// grid-stride loops with UNROLL independent loads per lane, global_load vs
// buffer_load, default vs nontemporal policy, several grid sizes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
      return 1;                                                             \
    }                                                                       \
  } while (0)

template <int UNROLL, int AUX>
__global__ __launch_bounds__(256) void rd_buffer(const uint8_t *p, uint32_t bytes, uint32_t *out) {
  auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), 0, (int)bytes, 0x00020000);
  const uint32_t nthr = gridDim.x * 256u;
  const uint32_t tid = blockIdx.x * 256u + threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t base = tid * 16u; base < bytes; base += nthr * 16u * UNROLL) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, base + (uint32_t)u * nthr * 16u, 0, AUX);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 0x9E3779B9u) out[tid] = acc;
}

template <int UNROLL>
__global__ __launch_bounds__(256) void rd_global(const u32x4 *p, uint64_t n, uint32_t *out) {
  const uint64_t nthr = (uint64_t)gridDim.x * 256u;
  const uint64_t tid = blockIdx.x * 256u + threadIdx.x;
  uint32_t acc = 0;
  for (uint64_t i = tid; i < n; i += nthr * UNROLL) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint64_t j = i + (uint64_t)u * nthr;
      v[u] = j < n ? p[j] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 0x9E3779B9u) out[tid] = acc;
}

// The checksum's access pattern without the checksum: the 16-byte envelope of
// every slot's datagram (nch chunks at slot * stride + env_off), flat chunk
// index space, grid-stride, UNROLL loads in flight per lane.
template <int UNROLL>
__global__ __launch_bounds__(256) void rd_slots(const uint8_t *p, uint32_t bytes, uint32_t nslots,
                                                uint32_t stride, uint32_t env_off, uint32_t nch,
                                                uint32_t *out) {
  auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), 0, (int)bytes, 0x00020000);
  const uint32_t nthr = gridDim.x * 256u;
  const uint32_t total = nslots * nch;
  uint32_t acc = 0;
  for (uint32_t c = blockIdx.x * 256u + threadIdx.x; c < total; c += nthr * UNROLL) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint32_t cc = c + (uint32_t)u * nthr;
      const uint32_t slot = cc / nch, k = cc - slot * nch;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(
          r, cc < total ? slot * stride + env_off + 16u * k : 0xFFFFF000u, 0, 2);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x * 256u + threadIdx.x] = acc;
}

__global__ void fill(uint32_t *p, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
    p[i] = (uint32_t)(i * 2654435761u);
}

template <typename F>
static double time_it(F launch, int reps, hipEvent_t a, hipEvent_t b, double *best) {
  std::vector<float> ms;
  for (int i = 0; i < reps + 2; ++i) {
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float t;
    hipEventElapsedTime(&t, a, b);
    if (i >= 2) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  *best = ms.front();
  return ms[ms.size() / 2];
}

int main() {
  const uint32_t bytes = 2u << 30;
  uint8_t *buf;
  uint32_t *out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64u << 20));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, (uint32_t *)buf, (uint64_t)bytes / 4);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  printf("{\"probe\": \"hbm_read\", \"bytes\": %u, \"results\": [\n", bytes);
  bool first = true;
  auto report = [&](const char *kind, int unroll, int aux, int grid, double med, double best) {
    printf("%s  {\"kind\": \"%s\", \"unroll\": %d, \"aux\": %d, \"grid\": %d, \"median_GBps\": %.1f, "
           "\"best_GBps\": %.1f}",
           first ? "" : ",\n", kind, unroll, aux, grid, bytes / med / 1e6, bytes / best / 1e6);
    first = false;
  };
  for (int grid : {1024, 2048, 4096, 8192, 16384}) {
    double best, med;
#define RB(U, AUX)                                                                                \
  med = time_it([&] { hipLaunchKernelGGL((rd_buffer<U, AUX>), dim3(grid), dim3(256), 0, 0, buf, bytes, out); }, \
                10, a, b, &best);                                                                 \
  report("buffer", U, AUX, grid, med, best);
    RB(4, 0) RB(8, 0) RB(16, 0) RB(4, 2) RB(8, 2) RB(16, 2)
    // other cache-policy bits (gfx950: bit 0 sc0, bit 1 nt, bit 4 sc1)
    RB(4, 1) RB(4, 3) RB(4, 16) RB(4, 17) RB(4, 18) RB(4, 19) RB(8, 18) RB(8, 19)
#define RG(U)                                                                                     \
  med = time_it([&] {                                                                             \
    hipLaunchKernelGGL((rd_global<U>), dim3(grid), dim3(256), 0, 0, (const u32x4 *)buf,            \
                       (uint64_t)bytes / 16, out);                                                \
  }, 10, a, b, &best);                                                                            \
  report("global", U, 0, grid, med, best);
    RG(4) RG(8) RG(16)
  }
  // slot layouts of the BASELINE configs: 1500 B in 2176 B slots, 9000 B in
  // 9216 B slots, 46 B in 64 B slots (IP at +142 / +142 / +14)
  struct L { uint32_t stride, ip_off, len; } lays[] = {{2176, 142, 1500}, {9216, 142, 9000}, {64, 14, 46}};
  for (auto ly : lays) {
    const uint32_t env = ly.ip_off & ~15u;
    const uint32_t nch = (ly.ip_off + ly.len + 15u) / 16u - env / 16u;
    const uint32_t nslots = (bytes - 4096) / ly.stride;
    const double useful = (double)nslots * ly.len;
    for (int grid : {2048, 4096, 8192, 16384}) {
      double best, med;
#define RS(U)                                                                                    \
  med = time_it([&] {                                                                            \
    hipLaunchKernelGGL((rd_slots<U>), dim3(grid), dim3(256), 0, 0, buf, bytes, nslots, ly.stride, \
                       env, nch, out);                                                           \
  }, 10, a, b, &best);                                                                           \
  printf(",\n  {\"kind\": \"slots\", \"stride\": %u, \"len\": %u, \"unroll\": %d, \"grid\": %d, "    \
         "\"useful_median_GBps\": %.1f, \"envelope_median_GBps\": %.1f, \"useful_best_GBps\": %.1f}", \
         ly.stride, ly.len, U, grid, useful / med / 1e6, (double)nslots * nch * 16 / med / 1e6,   \
         useful / best / 1e6);
      RS(4) RS(8) RS(16)
    }
    // one BASELINE-sized batch per launch, rotating over the 2 GiB buffer so no
    // launch finds its batch in the Infinity Cache
    const uint32_t per = ly.len == 46 ? (1u << 20) : 65536u;
    const uint32_t region = per * ly.stride + 4096;
    const int nreg = (int)(bytes / region);
    for (int grid : {1024, 2048, 4096, 8192}) {
      int it = 0;
      double best, med;
#define RB1(U)                                                                                    \
  med = time_it([&] {                                                                             \
    const uint32_t o = (uint32_t)(it++ % nreg) * region;                                          \
    hipLaunchKernelGGL((rd_slots<U>), dim3(grid), dim3(256), 0, 0, buf + o, region, per,          \
                       ly.stride, env, nch, out);                                                 \
  }, 16, a, b, &best);                                                                            \
  printf(",\n  {\"kind\": \"slots_batch\", \"packets\": %u, \"stride\": %u, \"len\": %u, \"unroll\": %d, " \
         "\"grid\": %d, \"median_us\": %.2f, \"useful_median_GBps\": %.1f, \"useful_best_GBps\": %.1f}",    \
         per, ly.stride, ly.len, U, grid, med * 1e3, (double)per * ly.len / med / 1e6,               \
         (double)per * ly.len / best / 1e6);
      RB1(2) RB1(4) RB1(8)
    }
  }
  printf("\n]}\n");
  return 0;
}
