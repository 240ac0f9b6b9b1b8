#!/bin/bash
# round 6 evidence at HEAD, part 2: bench lines C1-C5 + pinned with part 1's
# PMC traffic (gpurun_out/traffic.json, merged back from part 1 and copied to
# profiles/r06/traffic_r06k.json), and the 2-rank gloo rehearsal
set -u
mkdir -p gpurun_out
TAG=${1:-r06k}
export TMPDIR=/tmp
T="timeout -k 10"
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
cp profiles/r06/traffic_r06k.json gpurun_out/traffic.json
TJ="--traffic-json gpurun_out/traffic.json"
$T 500 python bench.py $TJ > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || exit $?
$T 300 python bench.py --models 4 --scale 16 --rays 4096 --cpu-rays 0 $TJ > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 8192 --cpu-rays 0 $TJ > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 300 python bench.py --models 1 --rays 1024 --cpu-rays 0 $TJ > gpurun_out/bench_c1_$TAG.json 2> gpurun_out/bench_c1_$TAG.err || exit $?
$T 300 python bench.py --models 1 --rays 8192 --cpu-rays 0 $TJ > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 65536 --pinned-sim 8 --cpu-rays 0 $Q > gpurun_out/bench_c5pin_$TAG.json 2> gpurun_out/bench_c5pin_$TAG.err || exit $?
# the 2-rank data-parallel rehearsal on one GPU (gloo): the bounded-timeout
# process group, the six buckets and the exposed communication
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
RADNERF_DEVICE=0 $T 300 python bench.py --gpus 2 --backend gloo --models 8 --scale 16 --rays 4096 $X > gpurun_out/bench_dp2_c5_$TAG.json 2> gpurun_out/bench_dp2_c5_$TAG.err || exit $?
echo done
