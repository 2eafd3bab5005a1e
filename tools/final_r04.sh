#!/bin/bash
# Round-4 record on the GPU box (one phase per gpurun call, each step under its own time limit; the script
# stops at the first failing step).  Usage: bash tools/final_r04.sh OUTDIR tests|driver|lines|grid|pmc
set -u
export TMPDIR=/tmp
O=${1:-gpurun_out/final}; PHASE=${2:-tests}
mkdir -p "$O"
step() {  # step <name> <seconds> <command...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$O/steps.log"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$O/steps.log"
  tail -3 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
case $PHASE in
  tests)
    step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
    ;;
  driver)
    step bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5
    step prof_driver 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_driver" -o deepfm -- \
      python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-companion
    ;;
  lines)
    for wl in xdeepfm dcn_bf16 pnn_bf16; do
      step bench_$wl 600 python bench.py --workload $wl --no-companion
      step prof_$wl 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$wl" -o $wl -- \
        python3 bench.py --workload $wl --no-cpu-baseline --no-companion --steps 20 --warmup 5
    done
    step bench_deepfm_sharded 600 python bench.py --workload deepfm_sharded --no-companion
    ;;
  grid)
    step grid 1100 bash tools/grid_r04.sh "$O/grid"
    ;;
  pmc)
    step pmc 1100 bash tools/pmc_r04.sh "$O/pmc"
    ;;
esac
