#!/bin/bash
# level-forward probe (bit-exact vs the merged forward + timings) at C3 and C5,
# then the C3 / C5 bench lines without the side legs
set -o pipefail
tag=${1:-a}
mkdir -p gpurun_out
export ENC_BLOCKS=${ENC_BLOCKS:-4096} MLP_BLOCKS=256
Q="--dropin-step 0 --test-time-rays 0 --density-update 0 --cpu-rays 0 --train-step 0"
timeout -k 10 150 python3 tools/enc_probe.py > gpurun_out/encab_c3_$tag.json 2> gpurun_out/encab_c3_$tag.err &&
ABL_K=8 ABL_SCALE=16 ABL_RAYS=8192 timeout -k 10 150 python3 tools/enc_probe.py > gpurun_out/encab_c5_$tag.json 2> gpurun_out/encab_c5_$tag.err &&
timeout -k 10 150 python -u bench.py $Q --steps 30 --warmup 5 > gpurun_out/encab_b3_$tag.json 2> gpurun_out/encab_b3_$tag.err &&
timeout -k 10 150 python -u bench.py $Q --steps 20 --warmup 5 --models 8 --scale 16 --rays 8192 > gpurun_out/encab_b5_$tag.json 2> gpurun_out/encab_b5_$tag.err || exit $?
cat gpurun_out/encab_c3_$tag.json gpurun_out/encab_c5_$tag.json
python3 tools/bench_summary.py gpurun_out/encab_b*_$tag.json
