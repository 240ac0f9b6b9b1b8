#!/bin/bash
# Round-4 closing evidence at HEAD (second pass): GPU tests, smoke, C3 / C4 / C5
# bench lines, kernel stats of C5
set -u
mkdir -p gpurun_out
TAG=${1:-fin}
export TMPDIR=/tmp
trap "find gpurun_out -name '*kernel_trace.csv' -delete" EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
timeout -k 10 300 python bench.py --models 4 --scale 16 --rays 4096 --cpu-rays 0 --dropin-step 0 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
timeout -k 10 300 python bench.py --models 8 --scale 16 --rays 8192 --cpu-rays 0 --dropin-step 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 10 --warmup 3 --models 8 --scale 16 --rays 8192 > gpurun_out/prof_c5_$TAG.log 2>&1 || exit $?
echo done
