#!/bin/bash
# round 4 combined: sum-pass probes + profile, binned / fx / density tests,
# MFMA counters, C5 / C4 bench with and without the binned scatter
set -u
mkdir -p gpurun_out
TAG=${1:-h}
export TMPDIR=/tmp
T="timeout -k 10"
trap "find gpurun_out -name '*counter_collection.csv' -size +20M -delete" EXIT
$T 200 python3 tools/bin_probe.py c5 3 shuffled 0.125 > gpurun_out/binprobe_fp_$TAG.json 2> gpurun_out/binprobe_fp_$TAG.err || exit $?
$T 300 python3 tools/bin_probe.py c5 3 shuffled 1.0 > gpurun_out/binprobe_full_$TAG.json 2> gpurun_out/binprobe_full_$TAG.err || exit $?
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_$TAG.txt 2>&1 || true
grep -i "utcl\|tlb\|mfma" gpurun_out/counters_$TAG.txt | head -80 > gpurun_out/counters_sel_$TAG.txt || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU -d gpurun_out/pmc_sum1_$TAG -o run --output-format csv -- python3 tools/bin_probe.py c5 1 shuffled 0.125 > gpurun_out/pmc_sum1_$TAG.log 2>&1 || exit $?
python3 tools/sq_reduce.py gpurun_out/pmc_sum1_$TAG k_grid > gpurun_out/sq_sum1_$TAG.json || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_sum2_$TAG -o run --output-format csv -- python3 tools/bin_probe.py c5 1 shuffled 0.125 > gpurun_out/pmc_sum2_$TAG.log 2>&1 || exit $?
python3 tools/sq_reduce.py gpurun_out/pmc_sum2_$TAG k_grid > gpurun_out/sq_sum2_$TAG.json || exit $?
$T 600 python -u -m pytest tests/test_gpu_bin.py tests/test_gpu_fx.py tests/test_gpu_render.py -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "bin or density or fx or ngp_render_train" > gpurun_out/tests_bin_$TAG.log 2>&1
echo "tests rc $?" >> gpurun_out/tests_bin_$TAG.log
bash tools/gpu/mfma_r04.sh $TAG || exit $?
for gb in 1 0; do
  $T 300 python bench.py --models 8 --scale 16 --rays 8192 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0 --grid-bin $gb > gpurun_out/bench_c5_gb${gb}_$TAG.json 2> gpurun_out/bench_c5_gb${gb}_$TAG.err || exit $?
  $T 300 python bench.py --models 4 --scale 16 --rays 4096 --cpu-rays 0 --dropin-step 0 --test-time-rays 0 --density-update 0 --train-step 0 --grid-bin $gb > gpurun_out/bench_c4_gb${gb}_$TAG.json 2> gpurun_out/bench_c4_gb${gb}_$TAG.err || exit $?
done
echo done
