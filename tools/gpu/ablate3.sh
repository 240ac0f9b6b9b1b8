#!/bin/bash
# field_bwd ablation (fixed-point build): phase cycles (flag 4096), barrier cost (512)
set -u
mkdir -p gpurun_out
TAG=${1:-a}
export TMPDIR=/tmp
timeout -k 10 200 python tools/ablate.py 0 4096 512 1 4097 > gpurun_out/ablate_$TAG.json 2> gpurun_out/ablate_$TAG.err || exit $?
ABL_K=8 ABL_SCALE=16 timeout -k 10 200 python tools/ablate.py 0 4096 1 > gpurun_out/ablate_c5_$TAG.json 2>> gpurun_out/ablate_$TAG.err || exit $?
