#!/bin/bash
# round 5: merged-backward instruction diet (issue loop split by stream parity,
# packed ReLU masks, pipelined dW tiles): full GPU suite, C3 / C5 bench, C3
# chunk-size sweep, phase ablation
set -u
mkdir -p gpurun_out
TAG=${1:-i}
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/gpu_suite_$TAG.log 2>&1 || exit $?
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
for i in 1 2; do
$T 300 python bench.py $X > gpurun_out/bench_c3_${TAG}$i.json 2> gpurun_out/bench_c3_${TAG}$i.err || exit $?
done
for mc in 2048 3072 1024; do
$T 300 python bench.py $X --max-chunk $mc > gpurun_out/bench_c3_${TAG}_mc$mc.json 2> gpurun_out/bench_c3_${TAG}_mc$mc.err || exit $?
done
$T 300 python bench.py --models 8 --scale 16 --rays 8192 $X > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 300 python -u tools/ablate.py 0 4096 > gpurun_out/abl_c3_$TAG.json 2> gpurun_out/abl_c3_$TAG.err || exit $?
echo done
