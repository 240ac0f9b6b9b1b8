#!/bin/bash
# round 5: where the merged backward's MLP phase goes (ablation build, C3):
# phase cycles with and without the grid scatter, MLP sub-phases
set -u
mkdir -p gpurun_out
TAG=${1:-e}
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u tools/ablate.py 0 4096 4 4100 > gpurun_out/abl_mlp_c3_$TAG.json 2> gpurun_out/abl_mlp_c3_$TAG.err || exit $?
ABL_K=8 ABL_SCALE=16 $T 300 python -u tools/ablate.py 0 4096 4 4100 > gpurun_out/abl_mlp_c5_$TAG.json 2> gpurun_out/abl_mlp_c5_$TAG.err || exit $?
echo done
