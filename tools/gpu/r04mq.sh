#!/bin/bash
# march with the next chunk's queries issued ahead: march parity tests, C3 / C5 march time
set -u
mkdir -p gpurun_out
TAG=${1:-mq}
export TMPDIR=/tmp
T="timeout -k 10"
$T 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ml.py tests/test_gpu_render.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_mq_$TAG.log 2>&1 || exit $?
$T 200 python tools/march_probe.py 2 0.5 8192 > gpurun_out/march_c3_$TAG.json 2> gpurun_out/march_c3_$TAG.err || exit $?
$T 200 python tools/march_probe.py 8 16 8192 > gpurun_out/march_c5_$TAG.json 2> gpurun_out/march_c5_$TAG.err || exit $?
echo done
