#!/bin/bash
# 128-B aligned binned issues: tests, C5 / C4 bench, C5 walk ablation, WRITE_SIZE pass
set -u
mkdir -p gpurun_out
TAG=${1:-al}
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_bin.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_bin_$TAG.log 2>&1 || exit $?
Q="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
$T 300 python bench.py --models 8 --scale 16 --rays 8192 $Q > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 300 python bench.py --models 4 --scale 16 --rays 4096 $Q > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
ABL_K=8 ABL_SCALE=16 ABL_RAYS=8192 $T 300 python3 tools/ablate.py 0 16 1 > gpurun_out/ablate_c5bin_$TAG.json 2> gpurun_out/ablate_c5bin_$TAG.err || exit $?
$T 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_c5bin_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 --models 8 --scale 16 --rays 8192 > gpurun_out/pmcw_c5bin_$TAG.log 2>&1 || exit $?
echo done
