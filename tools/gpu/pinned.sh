#!/bin/bash
# GPU-box job: the sub-NeRF-per-GPU layout (radnerf_amd/pinned.py): its GPU
# tests, bench.py --pinned at one rank, and a 2-rank rehearsal on the one GPU
# over gloo (functional only: gloo stages the collectives through the host)
set -u
mkdir -p gpurun_out
TAG=${1:-pin}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pinned.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --pinned --cpu-rays 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
RADNERF_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --pinned --backend gloo --cpu-rays 0 --train-step 1 --steps 5 --warmup 2 > gpurun_out/bench_${TAG}_w2.json 2> gpurun_out/bench_${TAG}_w2.err
