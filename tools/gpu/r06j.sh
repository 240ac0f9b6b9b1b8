#!/bin/bash
# A/B on one box: fx_mode 5 (the binned walk with levels 0-7 fp32 at compile
# time, this tree) vs fx_mode 4 (build/oldtree = the previous commit), C5 and
# C4 per GPU and the pinned rank, interleaved; the binned GPU tests first
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 250 --timeout-method thread tests/test_gpu_bin.py tests/test_gpu_fx.py tests/test_gpu_dist.py > gpurun_out/tests_m5_r06j.log 2>&1 || exit $?
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
C5="--models 8 --scale 16 --rays 8192 --steps 20 --warmup 3"
C4="--models 4 --scale 16 --rays 4096 --steps 30 --warmup 3"
P5="--models 8 --scale 16 --rays 65536 --pinned-sim 8"
for r in 1 2; do
  for v in old new; do
    B=bench.py; [ $v = old ] && B=build/oldtree/bench.py
    $T 200 python $B $Q $C5 > gpurun_out/abj_c5_${v}_$r.json 2> gpurun_out/abj_c5_${v}_$r.err || exit $?
    $T 200 python $B $Q $C4 > gpurun_out/abj_c4_${v}_$r.json 2> gpurun_out/abj_c4_${v}_$r.err || exit $?
  done
done
for v in old new; do
  B=bench.py; [ $v = old ] && B=build/oldtree/bench.py
  $T 300 python $B $Q $P5 > gpurun_out/abj_p5_${v}.json 2> gpurun_out/abj_p5_${v}.err || exit $?
done
echo done
