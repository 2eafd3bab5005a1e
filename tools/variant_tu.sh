#!/bin/bash
# Variant copies of librmx.so with extra -D flags on ONE translation unit (timing A/B on the GPU box with
# RMX_LIB=vbuild/<name>/librmx.so):
#   bash tools/variant_tu.sh k_tail_s3 name "-DFOO=1" [name2 "-DBAR=2" ...]
set -e
cd "$(dirname "$0")/../recommendation-models_amd/csrc"
make -s librmx.so
TU=$1; shift
OBJS=$(ls *.o | grep -v "^$TU.o$" | tr '\n' ' ')
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -munsafe-fp-atomics -I../../include"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  out=../../vbuild/$name; mkdir -p $out
  /opt/rocm/bin/hipcc $FL $flags -c -o $out/$TU.o $TU.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/librmx.so $OBJS $out/$TU.o \
    -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
  echo "built vbuild/$name/librmx.so ($TU $flags)"
done
