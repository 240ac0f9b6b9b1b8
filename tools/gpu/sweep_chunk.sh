#!/bin/bash
# tail-chunk sweep of the merged passes (dev tool): --min-chunk at the
# renderer's big-chunk defaults, C3 / C4 / C5 (gpurun_out/sw5_*.json)
set -u
mkdir -p gpurun_out
T="timeout -k 10"
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
for mn in 256 512 1024 2048; do
$T 300 python bench.py --models 8 --scale 16 --rays 8192 $X --min-chunk $mn > gpurun_out/sw5_c5_mn${mn}.json 2> gpurun_out/sw5.err || exit $?
$T 300 python bench.py --models 4 --scale 16 --rays 4096 $X --min-chunk $mn > gpurun_out/sw5_c4_mn${mn}.json 2> gpurun_out/sw5.err || exit $?
$T 300 python bench.py $X --min-chunk $mn > gpurun_out/sw5_c3_mn${mn}.json 2> gpurun_out/sw5.err || exit $?
done
echo done
