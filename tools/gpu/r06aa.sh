#!/bin/bash
# validation of the 1/16 tail (tail chunks 1536 at K >= 8, scale 16): full GPU suite, smoke, C1 / C2 / C3 / C4 / C5 / pinned bench lines
set -u
mkdir -p gpurun_out
TAG=${1:-r06aa}
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 250 --timeout-method thread > gpurun_out/gpu_suite_$TAG.log 2>&1 || exit $?
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
$T 500 python bench.py > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || exit $?
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
$T 300 python bench.py --models 4 --scale 16 --rays 4096 $Q > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 8192 $Q > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 65536 --pinned-sim 8 --cpu-rays 0 $Q > gpurun_out/bench_c5pin_$TAG.json 2> gpurun_out/bench_c5pin_$TAG.err || exit $?
$T 300 python bench.py --models 1 --rays 1024 --cpu-rays 0 $Q > gpurun_out/bench_c1_$TAG.json 2> gpurun_out/bench_c1_$TAG.err || exit $?
$T 300 python bench.py --models 1 --rays 8192 --cpu-rays 0 $Q > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
echo done
