#!/bin/bash
# where the scale-16 merged backward's time goes at the round-6 default
# (fx_mode 5): ablation tokens 0 (as is), 4096 (per-phase wave cycles),
# 4 (no grid scatter: the MLP phase + staging), 1 (no atomics / page stores),
# 2 (no dW) at C5 and C4 per GPU (librn_abl.so)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
ABL_K=8 ABL_SCALE=16 ABL_RAYS=8192 $T 400 python tools/ablate.py 0 4096 4 1 2 > gpurun_out/abl_c5_r06q.json 2> gpurun_out/abl_c5_r06q.err || exit $?
ABL_K=4 ABL_SCALE=16 ABL_RAYS=4096 $T 400 python tools/ablate.py 0 4096 4 1 2 > gpurun_out/abl_c4_r06q.json 2> gpurun_out/abl_c4_r06q.err || exit $?
ABL_K=2 ABL_SCALE=0.5 ABL_RAYS=8192 $T 400 python tools/ablate.py 0 4096 4 1 2 > gpurun_out/abl_c3_r06q.json 2> gpurun_out/abl_c3_r06q.err || exit $?
echo done
