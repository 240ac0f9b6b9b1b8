#!/bin/bash
# A/B of the working tree against an older tree copy under build/oldtree
# (bench.py + its package and librn.so; for ABI changes a RADNERF_LIB swap
# cannot cover) (dev tool): the field-kernel GPU tests on the working tree,
# then C3 and C5 alternating old / new.   usage: tools/gpu/ab_tree.sh <tag>
set -u
mkdir -p gpurun_out
TAG=$1
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fx.py tests/test_gpu_ml.py tests/test_gpu_bin.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for v in old new; do
    B=bench.py; [ $v = old ] && B=build/oldtree/bench.py
    timeout -k 10 200 python $B $Q --steps 40 --warmup 5 > gpurun_out/ab_${TAG}_c3_${v}_$r.json 2> gpurun_out/ab_${TAG}_c3_${v}_$r.err || exit $?
    timeout -k 10 200 python $B $Q --steps 20 --warmup 3 --models 8 --scale 16 --rays 8192 > gpurun_out/ab_${TAG}_c5_${v}_$r.json 2> gpurun_out/ab_${TAG}_c5_${v}_$r.err || exit $?
  done
done
python - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/ab_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["roofline"]["avg_launch_ms"],
          d.get("kernel_ms", {}).get("bwd_plan"))
PY
