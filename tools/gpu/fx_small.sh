#!/bin/bash
# fixed point on/off at small batches (C1, C2) and C3
set -u
mkdir -p gpurun_out
TAG=${1:-s}
export TMPDIR=/tmp
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
for fx in 1 0 1 0; do
  for cfg in "--models 1 --rays 1024" "--models 1 --rays 8192" "--models 2 --rays 8192"; do
    timeout -k 10 120 python bench.py $Q $cfg --grid-fx $fx >> gpurun_out/fx_small_$TAG.jsonl 2>/dev/null || exit $?
  done
done
