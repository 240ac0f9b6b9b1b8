#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-i}
export TMPDIR=/tmp
T="timeout -k 10"
$T 200 python3 tools/bin_probe.py c5 3 shuffled 0.125 > gpurun_out/binprobe_fp_$TAG.json 2> gpurun_out/binprobe_fp_$TAG.err || exit $?
$T 300 python3 tools/bin_probe.py c5 3 shuffled 1.0 > gpurun_out/binprobe_full_$TAG.json 2> gpurun_out/binprobe_full_$TAG.err || exit $?
