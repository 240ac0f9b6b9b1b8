#!/bin/bash
set -u
mkdir -p gpurun_out
T="timeout -k 10"
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0 --steps 20 --warmup 3"
for r in 1 2; do
for mc in 8192 12288 16384; do
$T 200 python bench.py --models 8 --scale 16 --rays 8192 $X --max-chunk $mc > gpurun_out/swn_c5_mc${mc}_$r.json 2> gpurun_out/swn.err || exit $?
$T 200 python bench.py --models 8 --scale 16 --rays 65536 --pinned-sim 8 $X --max-chunk $mc > gpurun_out/swn_c5pin_mc${mc}_$r.json 2> gpurun_out/swn.err || exit $?
done
done
echo done
