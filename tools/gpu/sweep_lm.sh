#!/bin/bash
# level-major encode schedule vs level groups (dev tool), C3 / C5, encode
# block counts; two rounds interleaved (gpurun_out/swl_*.json)
set -u
mkdir -p gpurun_out
T="timeout -k 10"
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
for r in 1 2; do
for v in "0 4096" "1 4096" "1 2048" "1 1024"; do
set -- $v
$T 200 python bench.py $X --steps 40 --warmup 5 --level-major $1 --enc-blocks $2 > gpurun_out/swl_c3_lm$1_e$2_$r.json 2> gpurun_out/swl.err || exit $?
$T 200 python bench.py --models 8 --scale 16 --rays 8192 $X --steps 20 --warmup 3 --level-major $1 --enc-blocks $2 > gpurun_out/swl_c5_lm$1_e$2_$r.json 2> gpurun_out/swl.err || exit $?
done
done
echo done
