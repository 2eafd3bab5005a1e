#!/bin/bash
# A/B of the bf16 tower variants: parity under the variant, then DCN / PNN bf16 lines per variant.
set -u
O=gpurun_out/bf16; mkdir -p $O
RMX_TEST_TUNING=tower_variant=6 timeout -k 10 600 python -u -m pytest tests/test_bf16.py tests/test_split_gemm.py -k "bf16 or dcn or pnn" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for w in dcn_bf16 pnn_bf16; do
  for v in ${VARS:-default 6 default 6}; do
    if [ $v = default ]; then SET=""; else SET="--set tower_variant=$v"; fi
    timeout -k 10 120 python bench.py --workload $w --steps 100 --warmup 10 --no-cpu-baseline $SET > $O/${w}_$v.json || exit 1
    python3 -c "
import json; d=json.load(open('$O/${w}_$v.json')); print('$w var=$v', round(d['value']/1e6,1), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})"
  done
done
