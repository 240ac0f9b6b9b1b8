#!/bin/bash
# binned scatter pricing probe: bin + sum on C5's record volume
set -u
mkdir -p gpurun_out
TAG=${1:-a}
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u tools/bin_probe.py c5 10 > gpurun_out/binprobe_$TAG.json 2> gpurun_out/binprobe_$TAG.err || exit $?
