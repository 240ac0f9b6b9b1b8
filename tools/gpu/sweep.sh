#!/bin/bash
# GPU-box job: bench.py over a list of option sets, one JSON line each
# (usage: tools/gpu/sweep.sh TAG "opts1" "opts2" ...; each step time-limited,
# stops at the first failure).
set -u
mkdir -p gpurun_out
TAG=$1; shift
i=0
for opts in "$@"; do
  timeout -k 10 200 python bench.py --cpu-rays 0 --train-step 0 --steps 10 --warmup 3 $opts \
      > gpurun_out/sweep_${TAG}_$i.json 2> gpurun_out/sweep_${TAG}_$i.err || exit $?
  echo "$opts" > gpurun_out/sweep_${TAG}_$i.opts
  i=$((i + 1))
done
