set -u
O=gpurun_out/dd; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_shard.py -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
for a in "" "--no-dedupe" "--zipf 1.1" "--zipf 1.1 --no-dedupe"; do
  timeout -k 10 300 python bench.py --workload deepfm_sharded --no-cpu-baseline $a > $O/sh.log 2>&1 || exit 1
  echo "$a :: $(python -c "import json; d=json.loads(open('$O/sh.log').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), d['ms_per_step'], d['exchange'], d['stages'].get('shard_exchange'))")"
done
true

export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o sh -- python3 bench.py --workload deepfm_sharded --no-cpu-baseline --steps 20 --warmup 3 --zipf 1.1 > $O/prof.log 2>&1 || exit 1
python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/prof/*kernel_stats.csv')[0])): print('%-60s %5s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
