#!/bin/bash
# A/B of the level-partitioned forward through bench.py (C3, C4, C5, C2)
set -o pipefail
tag=${1:-a1}
mkdir -p gpurun_out
Q="--dropin-step 0 --test-time-rays 0 --density-update 0 --cpu-rays 0 --train-step 0"
run() {  # name, args...
  n=$1; shift
  timeout -k 10 150 python -u bench.py $Q --steps 30 --warmup 5 "$@" > gpurun_out/lv_${n}_$tag.json 2> gpurun_out/lv_${n}_$tag.err || return $?
}
for lv in 0 1; do
  run c3_$lv --level-fwd $lv &&
  run c4_$lv --models 4 --scale 16 --rays 4096 --level-fwd $lv &&
  run c5_$lv --models 8 --scale 16 --rays 8192 --level-fwd $lv &&
  run c2_$lv --models 1 --rays 8192 --level-fwd $lv || exit $?
done
python3 tools/bench_summary.py gpurun_out/lv_*_$tag.json
