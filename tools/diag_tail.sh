#!/bin/bash
# Timing-only copies of librmx.so with RMX_TAIL_DIAG set in k_tail.hip: tools/diag_lib/tail<d>/librmx.so,
# used as RMX_LIB=... (results are wrong).  Usage: tools/diag_tail.sh 1 2 4 8
set -e
cd "$(dirname "$0")/../recommendation-models_amd/csrc"
make -s librmx.so
OBJS="capi.o models.o k_gemm.o k_gemm_bf16.o k_gemm_s3.o k_encoder.o k_interact.o shard.o train.o metric.o parse.o"
for d in "$@"; do
  out=../../tools/diag_lib/tail$d; mkdir -p $out
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -munsafe-fp-atomics -I../../include \
    -DRMX_TAIL_DIAG=$d -c -o $out/k_tail.o k_tail.hip &
done
wait
for d in "$@"; do
  out=../../tools/diag_lib/tail$d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/librmx.so $OBJS $out/k_tail.o \
    -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
  rm -f $out/k_tail.o
done
