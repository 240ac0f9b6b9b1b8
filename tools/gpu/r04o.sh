#!/bin/bash
# sum-pass TCP / UTCL1 / TA counters (frac 0.125 probe) + the cached-run ablation
set -u
mkdir -p gpurun_out
TAG=${1:-o}
export TMPDIR=/tmp
T="timeout -k 10"
trap "find gpurun_out -name '*counter_collection.csv' -size +20M -delete" EXIT
$T 200 python3 tools/bin_probe.py c5 3 shuffled 0.125 > gpurun_out/binprobe_fp_$TAG.json 2> gpurun_out/binprobe_fp_$TAG.err || exit $?
i=0
for set in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum" \
           "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_THRASHING_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmc_tcp${i}_$TAG -o run --output-format csv -- python3 tools/bin_probe.py c5 1 shuffled 0.125 > gpurun_out/pmc_tcp${i}_$TAG.log 2>&1 || exit $?
  python3 tools/sq_reduce.py gpurun_out/pmc_tcp${i}_$TAG "k_grid" > gpurun_out/tcp${i}_$TAG.json || exit $?
done
echo done
