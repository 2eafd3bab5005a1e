#!/bin/bash
# A/B of split-GEMM tower tiles (knob s3_tower): parity under the variant, then DeepFM lines per variant.
set -u
O=gpurun_out/abtower; mkdir -p $O
V=${VAR:-3}
RMX_TEST_TUNING=s3_tower=$V timeout -k 10 600 python -u -m pytest tests/test_split_gemm.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 1 $V 1 $V; do
  timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-companion --no-cpu-baseline --set s3_tower=$v > $O/deepfm_$v.json || exit 1
  python3 -c "
import json; d=json.load(open('$O/deepfm_$v.json')); print('deepfm s3_tower=$v', round(d['value']/1e6,1), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})"
done
