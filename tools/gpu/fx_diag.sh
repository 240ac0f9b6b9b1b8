#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/fx_diag.py 8192 12 adam > gpurun_out/fx_diag_${1:-a}.log 2>&1
