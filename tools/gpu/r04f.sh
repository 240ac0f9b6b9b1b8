#!/bin/bash
# round 4: binned scatter debug + tests + layout probe + C5/C4 bench
set -u
mkdir -p gpurun_out
TAG=${1:-f}
export TMPDIR=/tmp
T="timeout -k 10"
$T 200 python -u tools/bin_debug.py > gpurun_out/bin_debug_$TAG.log 2>&1 || exit $?
$T 500 python -u -m pytest tests/test_gpu_bin.py tests/test_gpu_fx.py tests/test_gpu_render.py -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "bin or density or fx" > gpurun_out/tests_bin_$TAG.log 2>&1
echo "tests rc $?" >> gpurun_out/tests_bin_$TAG.log
for v in "shuffled 1.0" "level 1.0" "shuffled 0.125"; do
  set -- $v
  $T 300 python -u tools/bin_probe.py c5 5 $1 $2 >> gpurun_out/binprobe_$TAG.json 2>> gpurun_out/binprobe_$TAG.err || exit $?
done
$T 300 python bench.py --models 8 --scale 16 --rays 8192 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 300 python bench.py --models 4 --scale 16 --rays 4096 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
