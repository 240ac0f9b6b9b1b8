#!/bin/bash
# GPU-box job: SQ counters (instruction mix, waits) of field_fwd / field_bwd (merged) in one pass
set -u
mkdir -p gpurun_out
TAG=${1:-f}
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmcsq_$TAG -o run --output-format csv -- python3 tools/ablate.py f0 0 > gpurun_out/pmcsq_$TAG.log 2>&1
