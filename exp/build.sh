#!/bin/bash
# Experiment builds of libmicksum.so (timing-only variants; results are wrong on purpose)
set -e
cd "$(dirname "$0")/.."
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -Ilibunsod_amd/csrc -DMI_EXP_$v $EXTRA \
    -c libunsod_amd/csrc/cksum_kernels.hip -o exp/k_$v.o
  gcc -O2 -fPIC -std=c11 -Iinclude -Ilibunsod_amd/csrc -c libunsod_amd/csrc/inet_dropin.c -o exp/d.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC exp/k_$v.o exp/d.o -o exp/lib_$v.so
done
