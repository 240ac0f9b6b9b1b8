#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "$@" -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t1.log 2>&1
