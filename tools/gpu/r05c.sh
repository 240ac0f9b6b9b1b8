#!/bin/bash
# round 5: per-entry agreement with the fp32-vs-fp32 floor
set -u
mkdir -p gpurun_out
TAG=${1:-c}
export TMPDIR=/tmp
T="timeout -k 10"
PT="python -u -m pytest -v -s --timeout 200 --timeout-method thread"
$T 300 $PT tests/test_gpu_fx.py::test_fx_per_entry_agreement > gpurun_out/r05_fx_floor_$TAG.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
