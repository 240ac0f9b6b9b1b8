#!/bin/bash
# scale-16 training with the round-6 default gradient (binned e5m17, coarse
# levels by fp32 atomics, fx_mode 5) vs fp32 atomics: C4's shape (K = 4) and
# a C5-shaped one (K = 8), 1000 steps each
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u tools/train_demo.py 1000 4096 4 16 > gpurun_out/train_s16_k4_r06n.json 2> gpurun_out/train_s16_k4_r06n.err || exit $?
$T 500 python -u tools/train_demo.py 1000 4096 8 16 > gpurun_out/train_s16_k8_r06n.json 2> gpurun_out/train_s16_k8_r06n.err || exit $?
# A/B: the even streams' fp32 issue without the unused vmax (librn_v1.so) vs HEAD
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
P=rad-nerf_amd/radnerf_amd
for r in 1 2; do
  for v in librn librn_v1; do
    RADNERF_LIB=$P/$v.so $T 200 python bench.py $Q --models 8 --scale 16 --rays 8192 --steps 20 --warmup 3 > gpurun_out/abn_c5_${v}_$r.json 2> gpurun_out/abn_c5_${v}_$r.err || exit $?
    RADNERF_LIB=$P/$v.so $T 200 python bench.py $Q --models 4 --scale 16 --rays 4096 --steps 30 --warmup 3 > gpurun_out/abn_c4_${v}_$r.json 2> gpurun_out/abn_c4_${v}_$r.err || exit $?
  done
done
echo done
