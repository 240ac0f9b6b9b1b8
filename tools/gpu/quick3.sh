#!/bin/bash
# quick check: fx + ml tests, fx headroom diag, headline bench, C4/C5 per GPU
set -u
mkdir -p gpurun_out
TAG=${1:-q}
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_fx.py tests/test_gpu_ml.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_q_$TAG.log 2>&1 || exit $?
$T 200 python tools/fx_diag.py 8192 12 adam > gpurun_out/fx_diag_$TAG.log 2>&1 || exit $?
$T 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
$T 300 python bench.py --models 4 --scale 16 --rays 4096 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 8192 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
