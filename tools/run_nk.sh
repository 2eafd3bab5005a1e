#!/bin/bash
# 208 x 128 dW tile (knob wgrad_nk): training GPU tests, then the training A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/nk
timeout -k 10 400 python -u -m pytest tests/test_train.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/nk/t.log 2>&1; rc=$?
tail -3 gpurun_out/nk/t.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_knobs.sh nkx xdeepfm_train - && bash tools/ab_knobs.sh nkd deepfm_train - wgrad_nk=2
