#!/bin/bash
# A/B session on the gpurun box: split-GEMM parity, then knob sweeps with tools/tune.py.
# Usage: bash tools/ab.sh <tag> "<step>;<step>..."  where a step is  name|seconds|command
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
IFS=';' read -ra STEPS <<< "$2"
for s in "${STEPS[@]}"; do
  IFS='|' read -r name secs cmd <<< "$s"
  echo "== $name: $cmd" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -n 30 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
echo "== all done"
