#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-i}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ml.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "int_grad or merged_backward_matches" > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ablate_ig.py > gpurun_out/ablate_$TAG.json 2> gpurun_out/ablate_$TAG.err
