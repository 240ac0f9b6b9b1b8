#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-c}
B="timeout -k 10 200 python bench.py --cpu-rays 0 --train-step 0 --steps 10 --warmup 3"
for mc in 512 768 1024 1536 2048; do
$B --max-chunk $mc > gpurun_out/cfg_${TAG}_mc$mc.json 2>/dev/null || exit $?
done
