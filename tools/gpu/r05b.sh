#!/bin/bash
# round 5: binned grid gradient, round-4 int22 records (_r04: HEAD before the
# change, built in-tree) against the e4m18 records: per-entry agreement
# (C3 int32, C4/C5 binned), full-size fixed point vs fp32, bin/fx GPU tests,
# scale-16 training demo (binned vs fp32 atomics)
set -u
mkdir -p gpurun_out
TAG=${1:-b}
export TMPDIR=/tmp
T="timeout -k 10"
PT="python -u -m pytest -v -s --timeout 200 --timeout-method thread"
ok() { [ $1 -le 1 ]; }   # pytest: 0 pass, 1 test failures (a measurement here); else stop
( cd _r04 && $T 300 $PT tests/test_gpu_fx.py::test_fx_per_entry_agreement ) > gpurun_out/r05_fx_old_$TAG.log 2>&1; ok $? || exit 9
$T 300 $PT tests/test_gpu_fx.py tests/test_gpu_bin.py tests/test_gpu_ml.py::test_full_size_fx_vs_fp32 > gpurun_out/r05_fx_new_$TAG.log 2>&1; ok $? || exit 8
$T 300 python -u tools/train_demo.py 1000 4096 4 16 > gpurun_out/train_s16_new_$TAG.json 2> gpurun_out/train_s16_new_$TAG.err || exit $?
( cd _r04 && $T 300 python -u tools/train_demo.py 1000 4096 4 16 ) > gpurun_out/train_s16_old_$TAG.json 2> gpurun_out/train_s16_old_$TAG.err || exit $?
