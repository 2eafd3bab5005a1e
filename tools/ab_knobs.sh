#!/bin/bash
# A/B of kernel knobs on one box: bash tools/ab_knobs.sh <tag> <workload> "<k=v,...>" ["<k=v,...>" ...]
# ("-" = defaults); prints examples/s, ms/step and the per-stage times of each setting
set -u
TAG=$1; WL=$2; shift 2
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
i=0
for kv in "$@"; do
  args=""
  [ "$kv" != "-" ] && args="--set $kv"
  timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline --no-companion $args > $O/ab_$i.json 2> $O/ab_$i.err || { tail -5 $O/ab_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$O/ab_$i.json'))
print('%-28s %12.0f %8.4f ms' % ('$kv', d['value'], d['ms_per_step']), {k: v['avg_ms'] for k, v in d['stages'].items()})"
  i=$((i+1))
done
