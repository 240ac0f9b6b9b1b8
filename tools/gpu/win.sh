#!/bin/bash
# 64-row walk windows: merged-backward tests, headline bench, phase ablation, C5
set -u
mkdir -p gpurun_out
TAG=${1:-w}
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_fx.py tests/test_gpu_ml.py tests/test_gpu_render.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_w_$TAG.log 2>&1 || exit $?
$T 200 python tools/ablate.py 0 4096 1 4097 > gpurun_out/ablate_$TAG.json 2> gpurun_out/ablate_$TAG.err || exit $?
Q="--cpu-rays 0 --dropin-step 0 --density-update 0 --test-time-rays 0"
$T 300 python bench.py $Q > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
$T 300 python bench.py $Q --models 8 --scale 16 --rays 8192 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 300 python bench.py $Q --models 4 --scale 16 --rays 4096 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
$T 300 python bench.py $Q --models 1 --rays 8192 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
