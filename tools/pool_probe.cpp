// tools/pool_probe.cpp -- which of the GPU agents' memory pools the CPU may
// access (the drop-in service's device mailbox needs one it can write through
// the PCIe BAR).  Diagnostics only.
//   hipcc -O2 tools/pool_probe.cpp -o tools/pool_probe -lhsa-runtime64
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdio.h>
#include <string.h>

static hsa_agent_t g_cpu;
static hsa_status_t cpu_cb(hsa_agent_t a, void *) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU) {
    g_cpu = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t pool_cb(hsa_amd_memory_pool_t p, void *gpu) {
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  size_t size = 0;
  bool alloc = false;
  hsa_amd_memory_pool_access_t acc_cpu = HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SIZE, &size);
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  hsa_amd_agent_memory_pool_get_info(g_cpu, p, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &acc_cpu);
  printf("{\"segment\": %d, \"flags\": %u, \"size_mb\": %zu, \"alloc\": %d, \"cpu_access\": %d", (int)seg, flags,
         size >> 20, (int)alloc, (int)acc_cpu);
  if (seg == HSA_AMD_SEGMENT_GLOBAL && alloc && acc_cpu != HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED) {
    void *q = nullptr;
    hsa_status_t s1 = hsa_amd_memory_pool_allocate(p, 4096, 0, &q);
    hsa_status_t s2 = q ? hsa_amd_agents_allow_access(1, &g_cpu, nullptr, q) : HSA_STATUS_ERROR;
    int ok = 0;
    if (s1 == HSA_STATUS_SUCCESS && s2 == HSA_STATUS_SUCCESS) {
      volatile unsigned *w = (volatile unsigned *)q;
      w[0] = 0x12345678u;
      ok = w[0] == 0x12345678u;
    }
    printf(", \"alloc_status\": %d, \"allow_status\": %d, \"cpu_rw\": %d", (int)s1, (int)s2, ok);
    if (q) hsa_amd_memory_pool_free(q);
  }
  printf("}\n");
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t gpu_cb(hsa_agent_t a, void *) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) hsa_amd_agent_iterate_memory_pools(a, pool_cb, nullptr);
  return HSA_STATUS_SUCCESS;
}
int main() {
  if (hsa_init() != HSA_STATUS_SUCCESS) return 1;
  hsa_iterate_agents(cpu_cb, nullptr);
  hsa_iterate_agents(gpu_cb, nullptr);
  hsa_shut_down();
  return 0;
}
