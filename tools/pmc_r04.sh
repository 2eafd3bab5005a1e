#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, MI355X_MICROARCH.md §HBM) of the bench workloads, for
# profiles/traffic.json (tools/pmc_summary.py).  Usage: bash tools/pmc_r04.sh OUTDIR [workload ...]
set -u
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc}; shift || true
WLS=${*:-"deepfm xdeepfm dcn_bf16 pnn_bf16"}
mkdir -p "$O"
for wl in $WLS; do
  for pass in fetch write sq grbm; do
    case $pass in
      fetch) ctr="FETCH_SIZE" ;;
      write) ctr="WRITE_SIZE" ;;
      sq) ctr="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" ;;
      grbm) ctr="GRBM_GUI_ACTIVE GRBM_COUNT" ;;
    esac
    steps=5; [ "$wl" = xdeepfm ] && steps=3
    mkdir -p "$O/pmc_$wl"
    echo "== pmc_${wl}_$pass: $ctr" | tee -a "$O/steps.log"
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_$wl/$pass" -o "$pass" -- \
      python3 bench.py --workload "$wl" --steps $steps --warmup 2 --no-cpu-baseline --no-companion --settle-ms 0 \
      > "$O/pmc_$wl/$pass.log" 2>&1
    rc=$?
    echo "== pmc_${wl}_$pass rc=$rc" | tee -a "$O/steps.log"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
