#!/bin/bash
# spread of the K = 8 scale-16 training demo: the round-6 default (coarse
# levels fp32) and every level binned (round 5), two ray streams each
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
for seed in 1234 77; do
  DEMO_SEED=$seed $T 300 python -u tools/train_demo.py 1000 4096 8 16 > gpurun_out/tk8_def_$seed.json 2> gpurun_out/tk8_def_$seed.err || exit $?
  BIN_F32_LEVELS=0 DEMO_SEED=$seed $T 300 python -u tools/train_demo.py 1000 4096 8 16 > gpurun_out/tk8_bin0_$seed.json 2> gpurun_out/tk8_bin0_$seed.err || exit $?
done
echo done
