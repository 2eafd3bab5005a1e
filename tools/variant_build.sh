#!/bin/bash
# Variant copies of librmx.so with extra -D flags on the GEMM translation units (timing A/B):
#   bash tools/variant_build.sh name "-DFOO=1 -DBAR=2" ...  ->  build/<name>/librmx.so (RMX_LIB=...)
set -e
cd "$(dirname "$0")/../recommendation-models_amd/csrc"
make -s librmx.so
OBJS="capi.o models.o k_gemm.o k_encoder.o k_interact.o shard.o train.o metric.o parse.o"
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -munsafe-fp-atomics -I../../include"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  out=../../build/$name; mkdir -p $out
  /opt/rocm/bin/hipcc $FL $flags -c -o $out/k_gemm_s3.o k_gemm_s3.hip &
  /opt/rocm/bin/hipcc $FL $flags -c -o $out/k_gemm_bf16.o k_gemm_bf16.hip &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/librmx.so $OBJS $out/k_gemm_s3.o $out/k_gemm_bf16.o \
    -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
done
