#!/bin/bash
# binned scatter page size A/B at the scale-16 shapes: 64-KB pages (librn.so)
# vs 128-KB pages (librn_pg16k.so, -DGB_PAGE=16384): longer slice runs for
# the sum pass, half the pages for the bin pass; interleaved on one box
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
P=rad-nerf_amd/radnerf_amd
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
RADNERF_LIB=$P/librn_pg16k.so $T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bin.py -k "not layout" > gpurun_out/tests_pg16k.log 2>&1 || exit $?
for r in 1 2; do
  for v in librn librn_pg16k; do
    RADNERF_LIB=$P/$v.so $T 200 python bench.py $Q --steps 20 --warmup 3 --models 8 --scale 16 --rays 8192 > gpurun_out/pg_c5_${v}_$r.json 2> gpurun_out/pg_c5_${v}_$r.err || exit $?
    RADNERF_LIB=$P/$v.so $T 200 python bench.py $Q --steps 30 --warmup 3 --models 4 --scale 16 --rays 4096 > gpurun_out/pg_c4_${v}_$r.json 2> gpurun_out/pg_c4_${v}_$r.err || exit $?
  done
done
echo done
