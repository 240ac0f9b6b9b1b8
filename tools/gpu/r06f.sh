#!/bin/bash
# per-level scatter form at the scale-16 shapes: levels
# [0, Lb) by atomics (the kernel's fp32 path), [Lb, 16) binned, vs all binned
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
STEP_K=8 STEP_B=8192 STEP_SCALE=16 $T 500 python tools/level_bin_probe.py 0 6 7 8 9 10 > gpurun_out/lvbin2_c5.json 2> gpurun_out/lvbin2_c5.err || exit $?
STEP_K=4 STEP_B=4096 STEP_SCALE=16 $T 400 python tools/level_bin_probe.py 0 6 7 8 9 10 > gpurun_out/lvbin2_c4.json 2> gpurun_out/lvbin2_c4.err || exit $?
echo done
