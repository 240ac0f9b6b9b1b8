#!/bin/bash
# GPU-box job: SQ counters of the march (and the other kernels of a bench step)
set -u
mkdir -p gpurun_out
TAG=${1:-m}
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d gpurun_out/pmcm_$TAG -o run --output-format csv -- python3 bench.py --cpu-rays 0 --steps 2 --warmup 1 --train-step 0 > gpurun_out/pmcm_$TAG.log 2>&1
