#!/bin/bash
# round 5: e4m18 records + bin-pass guards + split sum: bin / fx tests, the
# per-entry agreement with the reordered-fp32 floor, C3 / C4 / C5 bench lines
set -u
mkdir -p gpurun_out
TAG=${1:-d}
export TMPDIR=/tmp
T="timeout -k 10"
PT="python -u -m pytest -v -s -p no:cacheprovider --timeout 200 --timeout-method thread"
$T 400 $PT tests/test_gpu_bin.py tests/test_gpu_fx.py tests/test_gpu_ml.py::test_full_size_fx_vs_fp32 > gpurun_out/r05_tests_$TAG.log 2>&1
rc=$?; echo "tests rc $rc" >> gpurun_out/r05_tests_$TAG.log; [ $rc -le 1 ] || exit $rc
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
$T 300 python bench.py $X > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 8192 $X > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 300 python bench.py --models 4 --scale 16 --rays 4096 $X > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
echo done
