#!/bin/bash
# Build libmicksum variants of the stream kernel for A/B runs on the GPU box
# (MI_CKSUM_LIB=tools/ab/libmicksum_<name>.so selects one).  Each NAME=FLAGS pair
# compiles stream_kernels.hip with FLAGS and links it with the main objects.
set -e
cd "$(dirname "$0")/../../libunsod_amd/csrc"
make -s ../lib/obj/cksum_kernels.o ../lib/obj/inet_dropin.o
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -I. $flags -c stream_kernels.hip \
    -o ../../tools/ab/stream_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC ../lib/obj/cksum_kernels.o ../../tools/ab/stream_$name.o \
    ../lib/obj/inet_dropin.o -o ../../tools/ab/libmicksum_$name.so -Wl,-soname,libmicksum.so -L/opt/rocm/lib -lhsa-runtime64
  echo "built tools/ab/libmicksum_$name.so ($flags)"
done
