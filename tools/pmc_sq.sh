#!/bin/bash
# SQ / LDS counters of one bench workload (one rocprofv3 --pmc pass per counter group, each under its own
# time limit).  Usage: bash tools/pmc_sq.sh OUTDIR TAG "bench args"
set -u
export TMPDIR=/tmp
O=$1; TAG=$2; ARGS=$3
mkdir -p "$O/$TAG"
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/$TAG/p$i" -o p$i -- \
    python3 bench.py $ARGS --steps 5 --warmup 2 --no-cpu-baseline --no-companion --settle-ms 0 > "$O/$TAG/p$i.log" 2>&1
  rc=$?
  echo "$TAG pass $i ($ctr) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
