#!/bin/bash
# round 5: per-phase wave cycles of the merged backward, base vs LDS-DMA
# window staging (ablation builds build/librn_abl_{base,dma}.so), C3 and C5
set -u
mkdir -p gpurun_out
TAG=${1:-l}
export TMPDIR=/tmp
T="timeout -k 10"
for v in base dma; do
  RADNERF_ABL_LIB=build/librn_abl_$v.so $T 300 python tools/ablate.py 0 4096 > gpurun_out/phase_c3_${v}_$TAG.json 2> gpurun_out/phase.err || exit $?
  ABL_K=8 ABL_SCALE=16 ABL_RAYS=8192 RADNERF_ABL_LIB=build/librn_abl_$v.so $T 300 python tools/ablate.py 0 4096 > gpurun_out/phase_c5_${v}_$TAG.json 2> gpurun_out/phase.err || exit $?
done
echo done
