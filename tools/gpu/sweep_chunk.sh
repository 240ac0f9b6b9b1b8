#!/bin/bash
# chunk-size checks of the merged passes (dev tool): GPU tests of the merged
# kernels, then bench lines at the renderer's defaults and the pinned layout /
# C1 with balanced vs plain big chunks (gpurun_out/sw4_*.json)
set -u
mkdir -p gpurun_out
T="timeout -k 10"
X="--cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0"
$T 400 python -u -m pytest tests/test_gpu_ml.py tests/test_gpu_fx.py tests/test_gpu_bin.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/sw4_tests.log 2>&1 || exit $?
$T 300 python bench.py $X > gpurun_out/sw4_c3_def.json 2> gpurun_out/sw4.err || exit $?
$T 300 python bench.py --models 4 --scale 16 --rays 4096 $X > gpurun_out/sw4_c4_def.json 2> gpurun_out/sw4.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 8192 $X > gpurun_out/sw4_c5_def.json 2> gpurun_out/sw4.err || exit $?
for b in 1 0; do
for mc in 1024 2048 4096 8192; do
$T 300 python bench.py --models 8 --scale 16 --rays 65536 --pinned-sim 8 $X --max-chunk $mc --balance-chunks $b > gpurun_out/sw4_pin_b${b}_mc${mc}.json 2> gpurun_out/sw4.err || exit $?
done
$T 300 python bench.py --models 1 --rays 1024 $X --balance-chunks $b > gpurun_out/sw4_c1_b${b}.json 2> gpurun_out/sw4.err || exit $?
done
echo done
