#!/bin/bash
# GPU-box job for a forward-encoder change: GPU tests, field_fwd ablations
# (f0 full, f128 no memory, f256 no encoding, f4096 no MLP), launch-shape sweep, bench
set -u
mkdir -p gpurun_out
TAG=${1:-fw}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ablate.py ${ABL:-f0 f128 f256 f4096} > gpurun_out/ablate_$TAG.json 2> gpurun_out/ablate_$TAG.err || exit $?
timeout -k 10 300 python tools/fwd_blocks_sweep.py > gpurun_out/fwdsweep_$TAG.json 2> gpurun_out/fwdsweep_$TAG.err || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
