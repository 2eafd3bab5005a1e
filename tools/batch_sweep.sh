#!/bin/bash
# Launch-batch sweep (the metric is examples/s; B is the launch batch, SURVEY.md §8d lists several)
set -u
O=gpurun_out/bsweep; mkdir -p $O
for B in 32768 65536 98304 131072 49152; do
  timeout -k 10 150 python bench.py --batch $B --steps 100 --warmup 10 --no-companion --no-cpu-baseline > $O/d$B.json 2> $O/d$B.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/d$B.json')); print('deepfm B=$B', round(d['value']/1e6,2), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})" | tee -a $O/summary.txt
done
for B in 8192 16384 32768; do
  timeout -k 10 200 python bench.py --workload xdeepfm --batch $B --steps 30 --warmup 5 --no-cpu-baseline > $O/x$B.json 2> $O/x$B.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/x$B.json')); print('xdeepfm B=$B', round(d['value']/1e6,3), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})" | tee -a $O/summary.txt
done
