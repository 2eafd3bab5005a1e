#!/bin/bash
# Runs the DCN bf16 line under each diagnostic tail library (tools/diag_tail.sh) and the product one.
set -u
O=gpurun_out/diag_tail; mkdir -p $O
for d in ${DIAGS:-0 1 2 4 8 3 0}; do
  if [ $d = 0 ]; then L=recommendation-models_amd/csrc/librmx.so; else L=tools/diag_lib/tail$d/librmx.so; fi
  RMX_LIB=$L timeout -k 10 120 python bench.py --workload ${WL:-dcn_bf16} --steps 60 --warmup 5 --no-cpu-baseline > $O/d$d.json 2> $O/d$d.err || { tail $O/d$d.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/d$d.json') if l.startswith('{')][-1]); print('diag $d', round(d['value']/1e6,1), {k: v['avg_ms'] for k, v in d['stages'].items()})"
done
