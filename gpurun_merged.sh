#!/bin/bash
# merged-backward iteration: its tests, then bench merged vs split
set -u
mkdir -p gpurun_out
TAG=${1:-m}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ml.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --cpu-rays 0 --train-step 0 > gpurun_out/bench_${TAG}_merged.json 2> gpurun_out/bench_${TAG}_merged.err || exit $?
timeout -k 10 200 python bench.py --cpu-rays 0 --train-step 0 --split-bwd > gpurun_out/bench_${TAG}_split.json 2> gpurun_out/bench_${TAG}_split.err
