#!/bin/bash
# rocprofv3 kernel stats (C3, C5) at the final code, for profiles/r06/
set -u
mkdir -p gpurun_out
TAG=${1:-r06ab}
trap "find gpurun_out -name '*kernel_trace.csv' -delete" EXIT
export TMPDIR=/tmp
T="timeout -k 10"
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
$T 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 10 --warmup 3 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
$T 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profc5_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 10 --warmup 3 --models 8 --scale 16 --rays 8192 > gpurun_out/profc5_$TAG.log 2>&1 || exit $?
echo done
