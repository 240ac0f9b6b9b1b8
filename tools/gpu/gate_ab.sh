#!/bin/bash
set -u
mkdir -p gpurun_out
X="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py tests/test_gpu_render.py tests/test_gpu_dist.py tests/test_gpu_ml.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_gbw2.log 2>&1 || exit $?
for r in 1 2; do for g in 0 1; do
timeout -k 10 200 python bench.py $X --steps 40 --warmup 5 --gate-partials $g > gpurun_out/gab_c3_g${g}_$r.json 2> gpurun_out/gab.err || exit $?
timeout -k 10 200 python bench.py $X --steps 20 --warmup 3 --models 8 --scale 16 --rays 8192 --gate-partials $g > gpurun_out/gab_c5_g${g}_$r.json 2> gpurun_out/gab.err || exit $?
done; done
echo done
