#!/bin/bash
# round 5: full GPU suite + smoke at HEAD, scale-16 training demo (e5m17
# binned vs fp32), 2-rank gloo rehearsal of the data-parallel step
set -u
mkdir -p gpurun_out
TAG=${1:-h}
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/gpu_suite_$TAG.log 2>&1 || exit $?
$T 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
$T 300 python -u tools/train_demo.py 1000 4096 4 16 > gpurun_out/train_s16_$TAG.json 2> gpurun_out/train_s16_$TAG.err || exit $?
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
RADNERF_DEVICE=0 $T 300 python bench.py --gpus 2 --backend gloo --models 8 --scale 16 --rays 4096 $X > gpurun_out/bench_dp2_c5_$TAG.json 2> gpurun_out/bench_dp2_c5_$TAG.err || exit $?
echo done
