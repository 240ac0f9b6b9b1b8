#!/bin/bash
# quick GPU iteration: tests + ablation + bench (no profiler)
set -u
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ablate.py ${ABL:-0 1} > gpurun_out/ablate_$TAG.json 2> gpurun_out/ablate_$TAG.err || exit $?
timeout -k 10 300 python bench.py --cpu-rays 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
