#!/bin/bash
# rocprofv3 kernel stats of one bench workload: bash tools/prof_quick.sh <tag> <workload> [bench args...]
set -u
TAG=$1; WL=$2; shift 2
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o $WL -- python3 bench.py --workload $WL --no-cpu-baseline "$@" > $O/log 2>&1 || exit 1
python3 - "$O" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/*kernel_stats.csv")[0])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:24]:
    print("%-90s %5s %9.1f us %5.1f%%" % (r["Name"][:90], r["Calls"], float(r["AverageNs"]) / 1e3,
                                         100 * float(r["TotalDurationNs"]) / tot))
PY
