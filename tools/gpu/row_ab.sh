#!/bin/bash
# field_bwd row staging: sc1 buffer loads (default) vs the nt loads (flag
# 0x40000) interleaved in one process (tools/ablate.py), C3 and C5, then the
# merged-backward tests
set -o pipefail
tag=${1:-a}
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/ablate.py 0 262144 0 262144 > gpurun_out/rowab_c3_$tag.json 2> gpurun_out/rowab_c3_$tag.err || exit $?
ABL_K=8 ABL_SCALE=16 ABL_RAYS=8192 timeout -k 10 200 python3 tools/ablate.py 0 262144 > gpurun_out/rowab_c5_$tag.json 2> gpurun_out/rowab_c5_$tag.err || exit $?
cat gpurun_out/rowab_c3_$tag.json gpurun_out/rowab_c5_$tag.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_ml.py tests/test_gpu_fx.py tests/test_gpu_dist.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/rowab_tests_$tag.log 2>&1; rc=$?; tail -2 gpurun_out/rowab_tests_$tag.log; exit $rc
