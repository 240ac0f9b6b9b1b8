#!/bin/bash
# kernel stats of the level-partitioned forward probe (C3 and C5)
set -o pipefail
tag=${1:-p1}
export ENC_BLOCKS=4096 MLP_BLOCKS=256
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/encprof_c3_$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/enc_probe.py > $GRAFT_REPO_ROOT/gpurun_out/encprof_c3_$tag.log 2>&1 &&
ABL_K=8 ABL_SCALE=16 ABL_RAYS=8192 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/encprof_c5_$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/enc_probe.py > $GRAFT_REPO_ROOT/gpurun_out/encprof_c5_$tag.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
for f in $(find gpurun_out/encprof_c3_$tag gpurun_out/encprof_c5_$tag -name "*kernel_stats.csv"); do echo $f; cut -d, -f1-4 $f | head -12; done
exit $rc
