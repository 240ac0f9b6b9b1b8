#!/bin/bash
# round 5: per-entry fixed-point agreement (C3 int32, C4/C5 binned), full-size
# fixed point vs fp32, scale-16 training demo (binned vs fp32 atomics)
set -u
mkdir -p gpurun_out
TAG=${1:-a}
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread \
   tests/test_gpu_fx.py::test_fx_per_entry_agreement \
   tests/test_gpu_ml.py::test_full_size_fx_vs_fp32 > gpurun_out/r05_fx_$TAG.log 2>&1
rc=$?
# test failures (1) are measurements here; anything else (fault, abort, timeout) ends the call
[ $rc -le 1 ] || exit $rc
$T 500 python -u tools/train_demo.py 1000 4096 4 16 > gpurun_out/train_s16_$TAG.json 2> gpurun_out/train_s16_$TAG.err || exit $?
