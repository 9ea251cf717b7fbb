"""No kernel of the library can fault on an index (CPU test, no GPU needed).

Round 4's suite hit an intermittent hipErrorIllegalAddress.  Whatever index a
kernel computes -- from a descriptor, a stale mailbox, a wrong argument -- it
now reaches memory only through a buffer resource carrying the array's extent
(cksum_device.h, `Arr`), which the hardware range-checks: past the extent a
load reads zeros and a store or atomic is dropped.  This test reads the built
library's gfx950 code object and fails if any kernel has a memory
instruction that is not range-checked that way: a global_ / flat_ / scratch_
load, store or atomic, a scalar load through a pointer other than the
kernel-argument segment, or any scalar-cache write (tools/isa_audit.py).
"""
import os
import shutil

import pytest

from libunsod_amd._lib import LIB_PATH

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tools_ok():
    return (os.path.exists("/opt/rocm/llvm/bin/clang-offload-bundler") and
            os.path.exists("/opt/rocm/llvm/bin/llvm-objdump") and shutil.which("objcopy"))


@pytest.mark.skipif(not _tools_ok(), reason="LLVM / binutils tools not available")
def test_no_kernel_has_an_unchecked_memory_access():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from isa_audit import audit, demangle
    found = audit(LIB_PATH)
    assert len(found) > 150, len(found)
    assert any(k.startswith("mi_aql_rundma") for k in found) and "mi_aql_dropin_svc" in found
    bad = {k: dict(v) for k, v in found.items() if v}
    names = demangle(list(bad))
    assert not bad, {names.get(k, k): v for k, v in bad.items()}


BAD_KERNELS = r"""
#include <hip/hip_runtime.h>
#include <stdint.h>
__global__ void plain_store(uint32_t *out, const uint32_t *idx) { out[idx[threadIdx.x]] = 1u; }
__global__ void uniform_load(uint32_t *out, const uint32_t *tab, uint32_t k) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 64, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(tab[k], r, 0, 0, 0);
}
__global__ void bounded(uint32_t *out, uint32_t n) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)(4 * n), 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(7u, r, 4u * threadIdx.x, 0, 0);
}
"""


@pytest.mark.skipif(not (_tools_ok() and os.path.exists("/opt/rocm/bin/hipcc")), reason="hipcc not available")
def test_the_audit_catches_unchecked_accesses(tmp_path):
    """The checker itself: a plain global store through an index, and a
    uniform load through a user pointer (a scalar load), are reported; a
    buffer store is not."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from isa_audit import audit
    src = tmp_path / "bad.hip"
    src.write_text(BAD_KERNELS)
    so = tmp_path / "libbad.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", str(src), "-o", str(so)],
                   check=True, capture_output=True)
    found = {k: dict(v) for k, v in audit(str(so)).items()}
    plain = next(v for k, v in found.items() if "plain_store" in k)
    uni = next(v for k, v in found.items() if "uniform_load" in k)
    ok = next(v for k, v in found.items() if "bounded" in k)
    assert any(op.startswith("global_store") for op in plain), plain
    assert any(op.startswith("s_load from") for op in uni), uni
    assert not ok, ok
