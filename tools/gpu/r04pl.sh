#!/bin/bash
# merge plan with u16 ids: merged-order tests, DP tests, C5 bench (plan kernel time)
set -u
mkdir -p gpurun_out
TAG=${1:-pl}
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_ml.py tests/test_gpu_dist.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_pl_$TAG.log 2>&1 || exit $?
Q="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
$T 300 python bench.py --models 8 --scale 16 --rays 8192 $Q > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
echo done
