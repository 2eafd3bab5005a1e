set -u
O=gpurun_out/shard; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_shard.py tests/test_threads.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for o in "" "--no-overlap"; do
  timeout -k 10 300 python bench.py --workload deepfm_sharded --steps 100 --warmup 10 --no-cpu-baseline $o > $O/sh$o.json 2> $O/sh$o.err || { tail $O/sh$o.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/sh$o.json')); print('sharded $o', round(d['value']/1e6,1), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})"
done
