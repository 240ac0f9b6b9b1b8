#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-a}
export TMPDIR=/tmp
timeout -k 10 200 python tools/ablate.py 0 4096 12288 256 4352 > gpurun_out/ablate_$TAG.json 2> gpurun_out/ablate_$TAG.err || exit $?
