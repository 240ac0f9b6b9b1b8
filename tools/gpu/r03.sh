#!/bin/bash
# Round-3 check on the GPU box: GPU tests, smoke, headline bench (CPU
# baseline thread sweep), C2 through render(), and the self-launched
# 2-rank rehearsal (gloo, both ranks on GPU 0).
set -u
mkdir -p gpurun_out
TAG=${1:-r}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
timeout -k 10 300 python bench.py --models 1 --rays 8192 --cpu-rays 0 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
RADNERF_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --backend gloo --cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0 --steps 5 --warmup 2 > gpurun_out/bench_dp2_$TAG.json 2> gpurun_out/bench_dp2_$TAG.err || exit $?
