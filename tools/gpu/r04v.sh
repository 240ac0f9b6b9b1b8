#!/bin/bash
# binned-scatter probe + tests + grid-bin A/B at C5, C4 and C3
set -u
mkdir -p gpurun_out
TAG=${1:-v}
export TMPDIR=/tmp
T="timeout -k 10"
$T 200 python3 tools/bin_probe.py c5 3 shuffled 0.125 > gpurun_out/binprobe_fp_$TAG.json 2> gpurun_out/binprobe_fp_$TAG.err || exit $?
$T 300 python3 tools/bin_probe.py c5 5 shuffled 1.0 > gpurun_out/binprobe_full_$TAG.json 2> gpurun_out/binprobe_full_$TAG.err || exit $?
$T 300 python -u -m pytest tests/test_gpu_bin.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_bin_$TAG.log 2>&1 || exit $?
Q="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
for gb in 1 0; do
  $T 300 python bench.py --models 8 --scale 16 --rays 8192 $Q --grid-bin $gb > gpurun_out/bench_c5_gb${gb}_$TAG.json 2> gpurun_out/bench_c5_gb${gb}_$TAG.err || exit $?
  $T 300 python bench.py --models 4 --scale 16 --rays 4096 $Q --grid-bin $gb > gpurun_out/bench_c4_gb${gb}_$TAG.json 2> gpurun_out/bench_c4_gb${gb}_$TAG.err || exit $?
  $T 300 python bench.py $Q --grid-bin $gb > gpurun_out/bench_c3_gb${gb}_$TAG.json 2> gpurun_out/bench_c3_gb${gb}_$TAG.err || exit $?
done
