#!/bin/bash
# GPU-box job: merged-backward tests, tools/ablate.py timings, TCC_EA0_ATOMIC pass
set -u
mkdir -p gpurun_out
TAG=${1:-m}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ml.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ablate.py ${ABL:-0 1 4 32 s0 i0} > gpurun_out/ablate_$TAG.json 2> gpurun_out/ablate_$TAG.err || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d gpurun_out/pmca_$TAG -o run --output-format csv -- python3 bench.py --cpu-rays 0 --steps 3 --warmup 1 --train-step 0 > gpurun_out/pmca_$TAG.log 2>&1
