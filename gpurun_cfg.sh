#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-c}
B="timeout -k 10 200 python bench.py --cpu-rays 0 --train-step 0 --steps 10 --warmup 3"
$B --max-chunk 2048 > gpurun_out/cfg_${TAG}_mc2048.json 2>/dev/null || exit $?
$B --max-chunk 8192 > gpurun_out/cfg_${TAG}_mc8192.json 2>/dev/null || exit $?
$B --scale 16 --models 4 --rays 4096 > gpurun_out/cfg_${TAG}_s16k4.json 2>/dev/null || exit $?
$B --scale 16 --models 4 --rays 4096 --split-bwd > gpurun_out/cfg_${TAG}_s16k4_split.json 2>/dev/null || exit $?
$B --scale 16 --models 8 --rays 8192 > gpurun_out/cfg_${TAG}_s16k8.json 2>/dev/null || exit $?
$B --scale 16 --models 8 --rays 8192 --split-bwd > gpurun_out/cfg_${TAG}_s16k8_split.json 2>/dev/null || exit $?
$B --models 1 > gpurun_out/cfg_${TAG}_k1.json 2>/dev/null || exit $?
$B --models 1 --split-bwd > gpurun_out/cfg_${TAG}_k1_split.json 2>/dev/null
