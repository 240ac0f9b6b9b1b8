#!/bin/bash
# Round-3 check: changed GPU tests first (fx wrap / per-entry, density update,
# render), then the whole GPU suite, smoke, headline bench, C2 through
# render(), C5 pinned rank 0 simulated, self-launched 2-rank rehearsal.
set -u
mkdir -p gpurun_out
TAG=${1:-r}
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_fx.py tests/test_gpu_render.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_new_$TAG.log 2>&1 || exit $?
$T 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit $?
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
$T 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
$T 300 python bench.py --models 1 --rays 8192 --cpu-rays 0 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 65536 --pinned-sim 8 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 --train-step 0 --steps 10 --warmup 3 > gpurun_out/bench_c5pin_$TAG.json 2> gpurun_out/bench_c5pin_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 8192 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
RADNERF_DEVICE=0 $T 300 python bench.py --gpus 2 --backend gloo --cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0 --steps 5 --warmup 2 > gpurun_out/bench_dp2_$TAG.json 2> gpurun_out/bench_dp2_$TAG.err || exit $?
