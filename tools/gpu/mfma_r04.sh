#!/bin/bash
# MFMA utilisation: counter list, then SQ_VALU_MFMA_BUSY_CYCLES
# and a kernel trace of the C3 bench step and of the MLP-phase-only backward
# (tools/ablate.py flag 4: no grid scatter)
set -u
mkdir -p gpurun_out
TAG=${1:-m}
export TMPDIR=/tmp
trap "find gpurun_out -name '*counter_collection.csv' -size +20M -delete" EXIT
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_$TAG.txt 2>&1 || true
grep -i mfma gpurun_out/counters_$TAG.txt | head -40 > gpurun_out/counters_mfma_$TAG.txt || true
B="python3 bench.py --cpu-rays 0 --steps 3 --warmup 2 --train-step 0 --dropin-step 0 --test-time-rays 0 --density-update 0"
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/mfma_pmc_$TAG -o run --output-format csv -- $B > gpurun_out/mfma_pmc_$TAG.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace -d gpurun_out/mfma_tr_$TAG -o run --output-format csv -- $B > gpurun_out/mfma_tr_$TAG.log 2>&1 || exit $?
python3 tools/mfma_reduce.py gpurun_out/mfma_pmc_$TAG gpurun_out/mfma_tr_$TAG k_field_bwd_merged k_field_mlp_planes k_gate > gpurun_out/mfma_$TAG.json || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/mfma_pmc4_$TAG -o run --output-format csv -- python3 tools/ablate.py 4 > gpurun_out/mfma_pmc4_$TAG.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace -d gpurun_out/mfma_tr4_$TAG -o run --output-format csv -- python3 tools/ablate.py 4 > gpurun_out/mfma_tr4_$TAG.log 2>&1 || exit $?
python3 tools/mfma_reduce.py gpurun_out/mfma_pmc4_$TAG gpurun_out/mfma_tr4_$TAG k_field_bwd_merged > gpurun_out/mfma4_$TAG.json || exit $?
echo done
