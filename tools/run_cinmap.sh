#!/bin/bash
# A/B of the split CIN's chunk map (knob cin_map): parity tests, then xDeepFM bench on / off
set -u
export TMPDIR=/tmp
O=gpurun_out/cinmap; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_split_gemm.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "cin or xdeepfm or variants" > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -3 $O/t1.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_train.py tests/test_golden.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "xdeepfm or XDEEPFM or cin" > $O/t2.log 2>&1 || { tail -40 $O/t2.log; exit 1; }
tail -3 $O/t2.log
timeout -k 10 300 python bench.py --workload xdeepfm --no-cpu-baseline > $O/b_on.json 2> $O/b_on.err || exit 1
timeout -k 10 300 python bench.py --workload xdeepfm --no-cpu-baseline --set cin_map=0 > $O/b_off.json 2> $O/b_off.err || exit 1
timeout -k 10 300 python bench.py --workload xdeepfm --no-cpu-baseline --set cin_map_lds=1 > $O/b_lds.json 2> $O/b_lds.err || exit 1
python3 - $O <<'PY'
import json, sys
for n in ("b_on", "b_off", "b_lds"):
    d = json.load(open(sys.argv[1] + "/" + n + ".json"))
    print(n, d["value"], d["ms_per_step"], {k: v["avg_ms"] for k, v in d["stages"].items()})
PY
