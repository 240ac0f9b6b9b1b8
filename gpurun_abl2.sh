#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-a}
timeout -k 10 300 python tools/ablate.py ${ABL:-0 1 4 16 17 32} > gpurun_out/ablate_$TAG.json 2> gpurun_out/ablate_$TAG.err
