#!/bin/bash
# binned scatter: new tests, fx / ml tests, C5 / C4 / C3 bench
set -u
mkdir -p gpurun_out
TAG=${1:-b}
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_bin.py tests/test_gpu_fx.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_bin_$TAG.log 2>&1 || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 8192 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 300 python bench.py --models 4 --scale 16 --rays 4096 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
$T 400 python -u -m pytest tests/test_gpu_ml.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_ml_$TAG.log 2>&1 || exit $?
