#!/bin/bash
# A/B on one box: the tree before the int64 coarse levels (build/oldtree,
# ABI 9) vs HEAD with every level binned, with the coarse levels as int64
# sums, and with them as fp32 atomics; C3 old vs new (the int32 path's
# issue code changed too)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
C5="--models 8 --scale 16 --rays 8192 --steps 20 --warmup 3"
C4="--models 4 --scale 16 --rays 4096 --steps 30 --warmup 3"
for r in 1 2; do
  $T 200 python build/oldtree/bench.py $Q $C5 > gpurun_out/abh_c5_old_$r.json 2> gpurun_out/abh_c5_old_$r.err || exit $?
  $T 200 python bench.py $Q $C5 --bin-int64-levels 0 > gpurun_out/abh_c5_new0_$r.json 2> gpurun_out/abh_c5_new0_$r.err || exit $?
  $T 200 python bench.py $Q $C5 --bin-int64-levels 9 > gpurun_out/abh_c5_i64_$r.json 2> gpurun_out/abh_c5_i64_$r.err || exit $?
  $T 200 python bench.py $Q $C5 --bin-int64-levels 0 --fx-f32-levels 0,1,2,3,4,5,6,7,8 > gpurun_out/abh_c5_f32_$r.json 2> gpurun_out/abh_c5_f32_$r.err || exit $?
  $T 200 python build/oldtree/bench.py $Q $C4 > gpurun_out/abh_c4_old_$r.json 2> gpurun_out/abh_c4_old_$r.err || exit $?
  $T 200 python bench.py $Q $C4 --bin-int64-levels 0 > gpurun_out/abh_c4_new0_$r.json 2> gpurun_out/abh_c4_new0_$r.err || exit $?
  $T 200 python bench.py $Q $C4 --bin-int64-levels 8 > gpurun_out/abh_c4_i64_$r.json 2> gpurun_out/abh_c4_i64_$r.err || exit $?
  $T 200 python bench.py $Q $C4 --bin-int64-levels 0 --fx-f32-levels 0,1,2,3,4,5,6,7 > gpurun_out/abh_c4_f32_$r.json 2> gpurun_out/abh_c4_f32_$r.err || exit $?
  $T 200 python build/oldtree/bench.py $Q --steps 40 --warmup 5 > gpurun_out/abh_c3_old_$r.json 2> gpurun_out/abh_c3_old_$r.err || exit $?
  $T 200 python bench.py $Q --steps 40 --warmup 5 > gpurun_out/abh_c3_new_$r.json 2> gpurun_out/abh_c3_new_$r.err || exit $?
done
echo done
