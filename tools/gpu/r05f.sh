#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-f}
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fx_entry_diag.py 2048 8 16 > gpurun_out/fxdiag_c5_$TAG.json 2> gpurun_out/fxdiag_c5_$TAG.err || exit $?
timeout -k 10 300 python -u tools/fx_entry_diag.py 2048 2 0.5 > gpurun_out/fxdiag_c3_$TAG.json 2> gpurun_out/fxdiag_c3_$TAG.err || exit $?
