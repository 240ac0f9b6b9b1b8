#!/bin/bash
# round 6: the binned scatter's coarse levels as exact int64 sums (u64
# atomics): the binned / fixed-point GPU tests, then the per-level sweep at
# the C5 / C4 per-GPU shapes (int64 coarse levels vs fp32 coarse levels vs
# all binned)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_bin.py tests/test_gpu_fx.py tests/test_lib.py tests/test_lib_merged.py > gpurun_out/tests_i64_r06g.log 2>&1 || exit $?
STEP_K=8 STEP_B=8192 STEP_SCALE=16 $T 600 python tools/level_bin_probe.py bin0 i64:6 i64:8 i64:9 i64:10 i64:11 bin9 > gpurun_out/lvbin3_c5.json 2> gpurun_out/lvbin3_c5.err || exit $?
STEP_K=4 STEP_B=4096 STEP_SCALE=16 $T 500 python tools/level_bin_probe.py bin0 i64:6 i64:7 i64:8 i64:9 i64:10 bin8 > gpurun_out/lvbin3_c4.json 2> gpurun_out/lvbin3_c4.err || exit $?
echo done
