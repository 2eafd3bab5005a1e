#!/bin/bash
# single-buffered dW (knob wgrad_sb): training GPU tests, then the training A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/sb
timeout -k 10 400 python -u -m pytest tests/test_train.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sb/t.log 2>&1; rc=$?
tail -3 gpurun_out/sb/t.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_knobs.sh sbx xdeepfm_train - wgrad_sb=0 && bash tools/ab_knobs.sh sbd deepfm_train - wgrad_sb=0 "wgrad_s3=1" "wgrad_s3=1,wgrad_sb=2"
