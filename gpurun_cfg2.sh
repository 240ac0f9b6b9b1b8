#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-c}
B="timeout -k 10 200 python bench.py --cpu-rays 0 --train-step 0 --steps 10 --warmup 3"
for mc in 768 1024 1536 2048 3072; do
$B --max-chunk $mc > gpurun_out/cfg_${TAG}_mc$mc.json 2>/dev/null || exit $?
done
$B --scale 16 --models 8 --rays 8192 --max-chunk 2048 > gpurun_out/cfg_${TAG}_s16k8_mc2048.json 2>/dev/null || exit $?
$B --scale 16 --models 4 --rays 4096 --max-chunk 2048 > gpurun_out/cfg_${TAG}_s16k4_mc2048.json 2>/dev/null
