#!/bin/bash
# round 6: fp32 coarse levels in the binned scatter (bin_f32_levels): the GPU
# tests touched, then the count swept at C5 / C4 per GPU and the pinned C5
# rank (interleaved rounds)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 700 python -u -m pytest -x -v -p no:cacheprovider --timeout 250 --timeout-method thread tests/test_gpu_bin.py tests/test_gpu_fx.py tests/test_gpu_ml.py -k "bin or fx or full_size" --deselect tests/test_gpu_bin.py::test_bin_pass_refuses_corrupt_inputs > gpurun_out/tests_f32c_r06i.log 2>&1 || exit $?
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
C5="--models 8 --scale 16 --rays 8192 --steps 20 --warmup 3"
C4="--models 4 --scale 16 --rays 4096 --steps 30 --warmup 3"
P5="--models 8 --scale 16 --rays 65536 --pinned-sim 8 --steps 10 --warmup 2"
for r in 1 2; do
  for n in 0 8 9 10; do
    $T 200 python bench.py $Q $C5 --bin-f32-levels $n > gpurun_out/abi_c5_n${n}_$r.json 2> gpurun_out/abi_c5_n${n}_$r.err || exit $?
  done
  for n in 0 7 8 9; do
    $T 200 python bench.py $Q $C4 --bin-f32-levels $n > gpurun_out/abi_c4_n${n}_$r.json 2> gpurun_out/abi_c4_n${n}_$r.err || exit $?
  done
done
for n in 0 6 8 9 10; do
  $T 300 python bench.py $Q $P5 --bin-f32-levels $n > gpurun_out/abi_p5_n${n}.json 2> gpurun_out/abi_p5_n${n}.err || exit $?
done
echo done
