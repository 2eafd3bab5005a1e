#!/bin/bash
# A/B of variant librmx.so builds (build/<name>/librmx.so from tools/variant_build.sh) against the
# in-tree one, alternating:  bash tools/ab_lib.sh [--workload W] name [name ...]
set -u
W=deepfm
if [ "$1" = --workload ]; then W=$2; shift 2; fi
O=gpurun_out/ablib; mkdir -p $O
for round in 1 2; do
  for L in base "$@"; do
    if [ $L = base ]; then LIB=recommendation-models_amd/csrc/librmx.so; else LIB=build/$L/librmx.so; fi
    RMX_LIB=$LIB timeout -k 10 120 python bench.py --workload $W --steps 60 --warmup 10 --no-companion --no-cpu-baseline > $O/$L.json || exit 1
    python3 -c "
import json; d=json.load(open('$O/$L.json')); print('$L', round(d['value']/1e6,3), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})"
  done
done
