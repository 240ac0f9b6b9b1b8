#!/bin/bash
# SQ counters of field_bwd (merged, production) and of two ablation builds
# (x4: no scatter = the MLP phase alone; x1: no atomics), one rocprofv3 run per
# token; reduced on the box to per-kernel means (tools/sq_reduce.py).
set -u
mkdir -p gpurun_out
TAG=${1:-s}
export TMPDIR=/tmp
trap "find gpurun_out -name '*counter_collection.csv' -delete" EXIT
for t in 0 x4 x1; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmcsq_${TAG}_$t -o run --output-format csv -- python3 tools/ablate.py $t > gpurun_out/pmcsq_${TAG}_$t.log 2>&1 || exit $?
  python3 tools/sq_reduce.py gpurun_out/pmcsq_${TAG}_$t k_field_bwd_merged > gpurun_out/sq_${TAG}_$t.json || exit $?
done
