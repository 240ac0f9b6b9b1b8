#!/bin/bash
# rocprofv3 kernel stats of the C5 per-GPU step (K=8, 8192 rays, scale 16)
set -u
TAG=${1:-r}
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5_$TAG -o run --output-format csv -- python3 $R/bench.py $Q --steps 10 --warmup 3 --models 8 --scale 16 --rays 8192 > $R/gpurun_out/prof_c5_$TAG.log 2>&1
rc=$?
find $R/gpurun_out/prof_c5_$TAG -name "*kernel_trace.csv" -delete
exit $rc
