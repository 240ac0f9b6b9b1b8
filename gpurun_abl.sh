#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-a}
export TMPDIR=/tmp
timeout -k 10 300 python tools/ablate.py 0 1 2 4 s0 s1 s4 > gpurun_out/ablate_$TAG.json 2> gpurun_out/ablate_$TAG.err || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d gpurun_out/pmca_$TAG -o run --output-format csv -- python3 bench.py --cpu-rays 0 --steps 3 --warmup 1 --train-step 0 > gpurun_out/pmca_$TAG.log 2>&1
