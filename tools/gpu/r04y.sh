#!/bin/bash
# C5 merged-backward phases, binned scatter: with and without the page stores
set -u
mkdir -p gpurun_out
TAG=${1:-y}
export TMPDIR=/tmp
ABL_K=8 ABL_SCALE=16 ABL_RAYS=8192 timeout -k 10 300 python3 tools/ablate.py 16 144 1 16 144 1 > gpurun_out/ablate_c5bin_$TAG.json 2> gpurun_out/ablate_c5bin_$TAG.err || exit $?
