#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-e}
export TMPDIR=/tmp
T="timeout -k 10"
$T 200 python -u tools/bin_debug.py > gpurun_out/bin_debug_$TAG.log 2>&1 || exit $?
for v in "shuffled 1.0" "level 1.0" "shuffled 0.125" "level 0.125"; do
  set -- $v
  $T 300 python -u tools/bin_probe.py c5 5 $1 $2 >> gpurun_out/binprobe_$TAG.json 2>> gpurun_out/binprobe_$TAG.err || exit $?
done
