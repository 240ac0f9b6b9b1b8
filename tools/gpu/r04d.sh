#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-d}
export TMPDIR=/tmp
T="timeout -k 10"
$T 200 python -u tools/bin_debug.py > gpurun_out/bin_debug_$TAG.log 2>&1 || exit $?
