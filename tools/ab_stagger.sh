#!/bin/bash
# A/B of the split-GEMM loop variants (knob s3_stagger 0 / 1 / 2): parity first, then DeepFM and xDeepFM lines.
set -u
O=gpurun_out/stag; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_split_gemm.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in ${STAG_VALUES:-0 1 2 0 1 2}; do
  timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-companion --no-cpu-baseline --set s3_stagger=$v > $O/deepfm_$v.json || exit 1
  python3 -c "
import json; d=json.load(open('$O/deepfm_$v.json')); print('deepfm stagger=$v', round(d['value']/1e6,1), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})"
done
for v in ${STAG_XVALUES:-1 2}; do
  timeout -k 10 200 python bench.py --workload xdeepfm --steps 20 --warmup 3 --no-cpu-baseline --set s3_stagger=$v > $O/xdeepfm_$v.json || exit 1
  python3 -c "
import json; d=json.load(open('$O/xdeepfm_$v.json')); print('xdeepfm stagger=$v', round(d['value']/1e6,3), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})"
done
