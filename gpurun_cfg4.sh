#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-c}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ml.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
B="timeout -k 10 200 python bench.py --cpu-rays 0 --train-step 0 --steps 10 --warmup 3"
for h in 0 128 256 512; do
$B --head-chunk $h > gpurun_out/cfg_${TAG}_h$h.json 2>/dev/null || exit $?
done
