#!/bin/bash
# A/B of two builds of librn.so on one box (dev tool): the field-kernel GPU
# tests on the new build, then the headline bench and the C5 per-GPU shape
# alternating old / new (RADNERF_LIB), so both see the same card and clocks.
# usage: tools/gpu/ab.sh <tag> [old_lib]   (VARIANTS="old new b": librn_<v>.so, new = librn.so)
# Every leg runs HEAD's Python binding: a library built from another revision
# of include/radnerf.h is refused at load (ABI 9 signature table), so an old
# leg must be built from a tree with the same C ABI (round 5's failed leg,
# DESIGN §5, called rn_gate_bwd with shifted arguments).
set -u
mkdir -p gpurun_out
TAG=${1:-ab}
OLD=${2:-rad-nerf_amd/radnerf_amd/librn_old.so}
NEW=rad-nerf_amd/radnerf_amd/librn.so
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fx.py tests/test_gpu_ml.py tests/test_gpu_bin.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for v in ${VARIANTS:-old new}; do
    L=rad-nerf_amd/radnerf_amd/librn_$v.so; [ $v = old ] && L=$OLD; [ $v = new ] && L=$NEW
    RADNERF_LIB=$L timeout -k 10 200 python bench.py $Q --steps 40 --warmup 5 > gpurun_out/ab_${TAG}_c3_${v}_$r.json 2> gpurun_out/ab_${TAG}_c3_${v}_$r.err || exit $?
    RADNERF_LIB=$L timeout -k 10 200 python bench.py $Q --steps 20 --warmup 3 --models 8 --scale 16 --rays 8192 > gpurun_out/ab_${TAG}_c5_${v}_$r.json 2> gpurun_out/ab_${TAG}_c5_${v}_$r.err || exit $?
  done
done
python - "$TAG" <<'EOF'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/ab_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["roofline"]["avg_launch_ms"],
          d.get("kernel_ms", {}).get("field_fwd"))
EOF
