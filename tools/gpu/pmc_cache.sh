#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_hit -o run --output-format csv -- python3 bench.py --cpu-rays 0 --steps 2 --warmup 1 --train-step 0 > gpurun_out/pmc_hit.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_tcp -o run --output-format csv -- python3 bench.py --cpu-rays 0 --steps 2 --warmup 1 --train-step 0 > gpurun_out/pmc_tcp.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmc_acc -o run --output-format csv -- python3 bench.py --cpu-rays 0 --steps 2 --warmup 1 --train-step 0 > gpurun_out/pmc_acc.log 2>&1
echo done
