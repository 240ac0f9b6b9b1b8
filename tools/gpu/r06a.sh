#!/bin/bash
# round 6 first call: C3 training demo (int32 fixed point vs fp32 atomics,
# VERDICT r05 item 3) and the C3 / C5 bench lines at HEAD as this round's baseline
set -u
mkdir -p gpurun_out
TAG=${1:-r06a}
export TMPDIR=/tmp
T="timeout -k 10"
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
$T 300 python bench.py $Q > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || exit $?
$T 300 python bench.py $Q --models 8 --scale 16 --rays 8192 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 600 python -u tools/train_demo.py 1000 8192 2 0.5 > gpurun_out/train_demo_c3_$TAG.json 2> gpurun_out/train_demo_c3_$TAG.err || exit $?
echo done
