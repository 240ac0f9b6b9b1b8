#!/bin/bash
# (first: the footprint probe)
# sum-pass profile: kernel trace + SQ / TCC counters of the probe (frac 0.125)
set -u
mkdir -p gpurun_out
TAG=${1:-g}
export TMPDIR=/tmp
trap "find gpurun_out -name '*counter_collection.csv' -size +20M -delete" EXIT
timeout -k 10 200 python3 tools/bin_probe.py c5 3 shuffled 0.125 > gpurun_out/binprobe_fp_$TAG.json 2> gpurun_out/binprobe_fp_$TAG.err || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sum_$TAG -o run --output-format csv -- python3 tools/bin_probe.py c5 2 shuffled 0.125 > gpurun_out/prof_sum_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU -d gpurun_out/pmc_sum1_$TAG -o run --output-format csv -- python3 tools/bin_probe.py c5 1 shuffled 0.125 > gpurun_out/pmc_sum1_$TAG.log 2>&1 || exit $?
python3 tools/sq_reduce.py gpurun_out/pmc_sum1_$TAG k_grid > gpurun_out/sq_sum1_$TAG.json || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_sum2_$TAG -o run --output-format csv -- python3 tools/bin_probe.py c5 1 shuffled 0.125 > gpurun_out/pmc_sum2_$TAG.log 2>&1 || exit $?
python3 tools/sq_reduce.py gpurun_out/pmc_sum2_$TAG k_grid > gpurun_out/sq_sum2_$TAG.json || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_TA_BUSY_sum -d gpurun_out/pmc_sum3_$TAG -o run --output-format csv -- python3 tools/bin_probe.py c5 1 shuffled 0.125 > gpurun_out/pmc_sum3_$TAG.log 2>&1
python3 tools/sq_reduce.py gpurun_out/pmc_sum3_$TAG k_grid > gpurun_out/sq_sum3_$TAG.json
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_$TAG.txt 2>&1 || true
grep -i "utcl\|tlb\|TCP_TCC\|TA_\|TCP_PENDING\|TCP_TCR" gpurun_out/counters_$TAG.txt | head -60 > gpurun_out/counters_tlb_$TAG.txt || true
grep -i mfma gpurun_out/counters_$TAG.txt | head -40 > gpurun_out/counters_mfma_$TAG.txt || true
echo done
