#!/bin/bash
# round 5: chunk-size sweep of the merged passes after the walk / MLP changes
set -u
mkdir -p gpurun_out
TAG=${1:-j}
export TMPDIR=/tmp
T="timeout -k 10"
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
for mc in 512 768 1024 1280 1536; do
$T 300 python bench.py $X --max-chunk $mc > gpurun_out/sw_c3_mc${mc}_$TAG.json 2> gpurun_out/sw.err || exit $?
done
for mc in 1024 1536 2048; do
$T 300 python bench.py --models 8 --scale 16 --rays 8192 $X --max-chunk $mc > gpurun_out/sw_c5_mc${mc}_$TAG.json 2> gpurun_out/sw.err || exit $?
done
for mc in 768 1024 1536; do
$T 300 python bench.py --models 4 --scale 16 --rays 4096 $X --max-chunk $mc > gpurun_out/sw_c4_mc${mc}_$TAG.json 2> gpurun_out/sw.err || exit $?
done
for mc in 512 1024; do
$T 300 python bench.py --models 1 --rays 8192 $X --max-chunk $mc > gpurun_out/sw_c2_mc${mc}_$TAG.json 2> gpurun_out/sw.err || exit $?
done
echo done
