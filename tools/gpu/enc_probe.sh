#!/bin/bash
# level-partitioned forward probe at C3 / C4 / C5
set -o pipefail
tag=${1:-e1}
export ENC_BLOCKS=${ENC_BLOCKS:-2048,4096} MLP_BLOCKS=${MLP_BLOCKS:-512,1024,2048}
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/enc_probe.py > gpurun_out/enc_c3_$tag.json 2> gpurun_out/enc_c3_$tag.err &&
ABL_K=4 ABL_SCALE=16 ABL_RAYS=4096 timeout -k 10 150 python -u tools/enc_probe.py > gpurun_out/enc_c4_$tag.json 2> gpurun_out/enc_c4_$tag.err &&
ABL_K=8 ABL_SCALE=16 ABL_RAYS=8192 timeout -k 10 150 python -u tools/enc_probe.py > gpurun_out/enc_c5_$tag.json 2> gpurun_out/enc_c5_$tag.err
rc=$?
cat gpurun_out/enc_c*_$tag.json
exit $rc
