#!/bin/bash
# Direct renderer vs ml_render() API step, in the bench's leg order
set -u
mkdir -p gpurun_out
TAG=${1:-a}
export TMPDIR=/tmp
timeout -k 10 200 python tools/api_probe.py bench 2 10 > gpurun_out/api_probe_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python tools/api_probe.py api 2 10 >> gpurun_out/api_probe_$TAG.log 2>&1 || exit $?
