#!/bin/bash
# head-chunk sweep of the merged backward (dev tool): --head-chunk at C3 / C5,
# two rounds interleaved (gpurun_out/swh_*.json)
set -u
mkdir -p gpurun_out
T="timeout -k 10"
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
for r in 1 2; do
for hc in 0 128 256 512; do
$T 200 python bench.py $X --steps 40 --warmup 5 --head-chunk $hc > gpurun_out/swh_c3_h${hc}_$r.json 2> gpurun_out/swh.err || exit $?
$T 200 python bench.py --models 8 --scale 16 --rays 8192 $X --steps 20 --warmup 3 --head-chunk $hc > gpurun_out/swh_c5_h${hc}_$r.json 2> gpurun_out/swh.err || exit $?
done
done
echo done
