#!/bin/bash
# big-chunk sweep of the merged backward (dev tool): --max-chunk at C3 / C4 / C5
# (gpurun_out/swm_*.json), two rounds interleaved
set -u
mkdir -p gpurun_out
T="timeout -k 10"
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0 --steps 20 --warmup 3"
for r in 1 2; do
for mc in 6144 8192 12288; do
$T 200 python bench.py --models 8 --scale 16 --rays 8192 $X --max-chunk $mc > gpurun_out/swm_c5_mc${mc}_$r.json 2> gpurun_out/swm.err || exit $?
done
for mc in 3072 4096 6144; do
$T 200 python bench.py --models 4 --scale 16 --rays 4096 $X --max-chunk $mc > gpurun_out/swm_c4_mc${mc}_$r.json 2> gpurun_out/swm.err || exit $?
done
for mc in 1024 1536 2048; do
$T 200 python bench.py $X --max-chunk $mc > gpurun_out/swm_c3_mc${mc}_$r.json 2> gpurun_out/swm.err || exit $?
done
done
echo done
