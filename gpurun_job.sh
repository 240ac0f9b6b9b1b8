#!/bin/bash
# GPU-box job: tests, bench, rocprof kernel-trace summary.  Stops at the first
# crash/timeout (rc not in {0,1}).
set -u
mkdir -p gpurun_out
TAG=${1:-r}
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --cpu-rays 0 --steps 10 --warmup 3 > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc" >> gpurun_out/prof_$TAG.log
exit $rc
