#!/bin/bash
# fx record-sum fix check (diag + bench leg order), SQ counters of field_fwd
set -u
mkdir -p gpurun_out
TAG=${1:-d}
export TMPDIR=/tmp
trap "find gpurun_out -name '*counter_collection.csv' -delete" EXIT
timeout -k 10 200 python tools/fx_diag.py 8192 > gpurun_out/fx_diag_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python tools/api_probe.py bench 2 10 > gpurun_out/api_probe_$TAG.log 2>&1 || exit $?
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d gpurun_out/pmcsqf_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 > gpurun_out/pmcsqf_$TAG.log 2>&1 || exit $?
python3 tools/sq_reduce.py gpurun_out/pmcsqf_$TAG k_field_fwd_merged > gpurun_out/sqf_$TAG.json || exit $?
