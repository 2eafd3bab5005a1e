#!/bin/bash
# Variant / diagnostic copies of librmx.so: the listed translation units rebuilt with extra -D flags, linked
# with the in-tree objects of the others.  vbuild/ travels to the GPU box (build/ does not: .gpurunignore).
#   bash tools/vbuild.sh NAME "FLAGS" TU.hip [TU.hip ...]   ->  vbuild/NAME/librmx.so  (RMX_LIB=... to use)
set -e
name=$1; flags=$2; shift 2
cd "$(dirname "$0")/../recommendation-models_amd/csrc"
make -s librmx.so
out=../../vbuild/$name; mkdir -p $out
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -munsafe-fp-atomics -I../../include"
objs=""
for o in $(sed -n 's/^SRCS = //p' Makefile) parse.cpp; do
  b=${o%.*}.o
  if [[ " $* " == *" $o "* ]]; then objs="$objs $out/$b"; else objs="$objs $b"; fi
done
for tu in "$@"; do
  /opt/rocm/bin/hipcc $FL $flags -c -o $out/${tu%.hip}.o $tu &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/librmx.so $objs -L/opt/rocm/lib -lrccl -lpthread \
  -Wl,-rpath,/opt/rocm/lib
echo "vbuild/$name/librmx.so"
