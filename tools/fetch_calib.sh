#!/bin/bash
# FETCH_SIZE calibration for the forward path's read widths (tools/probe/fetch_calib.hip; build it
# first: hipcc --offload-arch=gfx950 -O3 -o tools/probe/fetch_calib tools/probe/fetch_calib.hip)
set -u
export TMPDIR=/tmp
O=gpurun_out/fetch_calib; mkdir -p $O
timeout -k 10 60 ./tools/probe/fetch_calib > $O/timing.txt 2>&1 || exit 1
cat $O/timing.txt
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- ./tools/probe/fetch_calib > $O/fetch.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 -L > $O/list.txt 2>&1 || exit 1
if grep -q "TCC_EA0_RDREQ_32B" $O/list.txt; then
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/rdreq -o rdreq -- ./tools/probe/fetch_calib > $O/rdreq.log 2>&1 || exit 1
fi
grep -o "TCC_EA0_RDREQ[A-Z0-9_]*" $O/list.txt | sort -u > $O/rdreq_names.txt || true
echo done
