set -u
O=gpurun_out/train; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for w in deepfm_train xdeepfm_train; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail $O/$w.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$w.json')); print('$w', round(d['value']/1e6,3), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})"
done
