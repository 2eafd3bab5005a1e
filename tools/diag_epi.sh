#!/bin/bash
# Epilogue cost of the split-GEMM tower layers: base vs diag 32 (no activation stores) vs diag 512 (no
# stored-activation epilogue: no LDS transpose either), alternating twice.  Results are wrong in the
# diag builds: timing only.  Build first (CPU): bash tools/diag_build.sh 32 512
set -u
O=gpurun_out/diag_epi; mkdir -p $O
for round in 1 2; do
  for d in base 32 512; do
    if [ $d = base ]; then L=recommendation-models_amd/csrc/librmx.so; else L=build/diag$d/librmx.so; fi
    RMX_LIB=$L timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-companion --no-cpu-baseline > $O/$d.json 2> $O/$d.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/$d.json')); print('$d', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})" | tee -a $O/summary.txt
  done
done
