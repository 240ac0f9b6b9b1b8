#!/bin/bash
# level-partitioned forward launch shapes (dev tool): --enc-blocks x
# --mlp-blocks at C3 and C5 (gpurun_out/swf_*.json)
set -u
mkdir -p gpurun_out
T="timeout -k 10"
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
for eb in 2048 4096 8192; do
for mb in 256 512 1024; do
$T 300 python bench.py $X --enc-blocks $eb --mlp-blocks $mb > gpurun_out/swf_c3_e${eb}_m${mb}.json 2> gpurun_out/swf.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 8192 $X --enc-blocks $eb --mlp-blocks $mb > gpurun_out/swf_c5_e${eb}_m${mb}.json 2> gpurun_out/swf.err || exit $?
done
done
echo done
