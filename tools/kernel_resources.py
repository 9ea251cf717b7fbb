#!/usr/bin/env python3
"""Registers, scratch and LDS of the gfx950 kernels in a built object or .so
(from the code object's metadata notes).

    python tools/kernel_resources.py libunsod_amd/lib/obj/stream_kernels.o [NAME_SUBSTRING]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"


def kernels(path):
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "co.elf")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fat], check=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    out = {}
    for block in re.split(r"\n  - \.agpr_count:", notes)[1:]:
        g = lambda k: re.search(r"\.%s:\s+(\S+)" % k, block).group(1)  # noqa: E731
        out[g("name")] = dict(vgpr=int(g("vgpr_count")), sgpr=int(g("sgpr_count")),
                              scratch=int(g("private_segment_fixed_size")), lds=int(g("group_segment_fixed_size")),
                              vgpr_spill=int(g("vgpr_spill_count")), sgpr_spill=int(g("sgpr_spill_count")))
    return out


if __name__ == "__main__":
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, r in sorted(kernels(sys.argv[1]).items()):
        if pat in name:
            print(name, r)
