#!/bin/bash
# Diagnostic copies of librmx.so with RMX_GEMM_DIAG set in the split-GEMM TU (k_gemm.hpp):
# build/diag<d>/librmx.so, used as RMX_LIB=... for timing-only experiments (results are wrong).
set -e
cd "$(dirname "$0")/../recommendation-models_amd/csrc"
make -s librmx.so
OBJS="capi.o models.o k_gemm.o k_encoder.o k_interact.o shard.o train.o metric.o parse.o"
for d in "$@"; do
  out=../../build/diag$d; mkdir -p $out
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -munsafe-fp-atomics -I../../include \
    -DRMX_GEMM_DIAG=$d -c -o $out/k_gemm_s3.o k_gemm_s3.hip &
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -munsafe-fp-atomics -I../../include \
    -DRMX_GEMM_DIAG=$d -c -o $out/k_gemm_bf16.o k_gemm_bf16.hip &
done
wait
for d in "$@"; do
  out=../../build/diag$d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/librmx.so $OBJS $out/k_gemm_s3.o $out/k_gemm_bf16.o \
    -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
done
