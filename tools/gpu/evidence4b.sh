#!/bin/bash
# Round-4 evidence, part B (after part A's traffic.json was merged into
# profiles/): the headline line with the CPU baseline, C1/C2, C4/C5 per GPU
# (binned scatter), C5 pinned rank 0 simulated on one GPU, and the
# self-launched 2-rank rehearsal (gloo, both ranks on GPU 0) with its comm
# fields.
set -u
mkdir -p gpurun_out
TAG=${1:-r}
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
$T 300 python bench.py --models 1 --rays 8192 --cpu-rays 0 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
$T 300 python bench.py --models 1 --rays 1024 --cpu-rays 0 > gpurun_out/bench_c1_$TAG.json 2> gpurun_out/bench_c1_$TAG.err || exit $?
$T 300 python bench.py --models 4 --scale 16 --rays 4096 --cpu-rays 0 --dropin-step 0 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 8192 --cpu-rays 0 --dropin-step 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 65536 --pinned-sim 8 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 --train-step 0 --steps 10 --warmup 3 > gpurun_out/bench_c5pin_$TAG.json 2> gpurun_out/bench_c5pin_$TAG.err || exit $?
RADNERF_DEVICE=0 $T 300 python bench.py --gpus 2 --backend gloo --cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0 --steps 5 --warmup 2 > gpurun_out/bench_dp2_$TAG.json 2> gpurun_out/bench_dp2_$TAG.err || exit $?
echo done
