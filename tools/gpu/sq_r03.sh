#!/bin/bash
# Round-3 SQ counters: field_bwd (production, MLP phase alone x4, no atomics x1)
# and the level-partitioned forward's encode and MLP-planes kernels (C3 and C5)
set -u
mkdir -p gpurun_out
TAG=${1:-r03}
export TMPDIR=/tmp
bash tools/gpu/pmc_sq2.sh $TAG || exit $?
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
export ENC_BLOCKS=4096 MLP_BLOCKS=256
for w in c3 c5; do
  if [ $w = c5 ]; then export ABL_K=8 ABL_SCALE=16 ABL_RAYS=8192; fi
  timeout -s KILL 150 rocprofv3 --pmc $SQ -d gpurun_out/pmcsq_${TAG}_enc_$w -o run --output-format csv -- python3 tools/enc_probe.py > gpurun_out/pmcsq_${TAG}_enc_$w.log 2>&1 || exit $?
  python3 tools/sq_reduce.py gpurun_out/pmcsq_${TAG}_enc_$w k_field_encode_levels > gpurun_out/sq_${TAG}_enc_$w.json || exit $?
  python3 tools/sq_reduce.py gpurun_out/pmcsq_${TAG}_enc_$w k_field_mlp_planes > gpurun_out/sq_${TAG}_mlpp_$w.json || exit $?
done
find gpurun_out -name '*counter_collection.csv' -delete
cat gpurun_out/sq_${TAG}_*.json
