#!/bin/bash
# A/B two builds of librn.so on the same box (box-to-box variance is ~5%):
#   cp <old build> rad-nerf_amd/radnerf_amd/librn_old.so, then gpurun this script
set -u
mkdir -p gpurun_out
for r in 1 2; do
for v in librn librn_old; do
  RADNERF_LIB=$PWD/rad-nerf_amd/radnerf_amd/$v.so timeout -k 10 200 python tools/ablate.py 0 > gpurun_out/ab_${v}_$r.json 2>/dev/null || exit 1
done; done
