#!/bin/bash
# Build libmicksum variants for A/B runs on the GPU box: each NAME=FLAGS pair
# compiles cksum_kernels.hip with FLAGS (e.g. -DMI_RUN_PIPE=0) and links
# tools/ab/libmicksum_NAME.so; MI_CKSUM_LIB=tools/ab/libmicksum_NAME.so selects
# it in any tool or bench.py.  Builds run in parallel (one hipcc per variant).
set -e
cd "$(dirname "$0")/../../libunsod_amd/csrc"
make -s ../lib/obj/inet_dropin.o
for spec in "$@"; do
  (
    name=${spec%%=*}; flags=${spec#*=}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -I../../include -I. \
      ${flags//,/ } -c cksum_kernels.hip -o ../../tools/ab/k_$name.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC ../../tools/ab/k_$name.o ../lib/obj/inet_dropin.o \
      -o ../../tools/ab/libmicksum_$name.so -Wl,-soname,libmicksum.so -L/opt/rocm/lib -lhsa-runtime64
    echo "built tools/ab/libmicksum_$name.so ($flags)"
  ) &
done
wait
