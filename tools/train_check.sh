#!/bin/bash
# GPU: backward parity tests + the two training benches (summary lines).
set -u
O=gpurun_out/tr; mkdir -p $O
timeout -k 10 400 python -m pytest tests/test_train.py -m gpu -q -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload deepfm_train --steps 50 > $O/d.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload xdeepfm_train --steps 10 --warmup 2 > $O/x.log 2>&1 || exit 1
for f in d x; do python -c "
import json; d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); print(d['config']['workload'], round(d['value']/1e6,3), 'M ex/s', d['ms_per_step']); print({k: v['avg_ms'] for k, v in d['stages'].items()})"; done
