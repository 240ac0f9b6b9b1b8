#!/bin/bash
# A/B (timing), second pass: ramped head chunks (librn_ramp.so) at C3 with two
# ramp heights, and at C2 / C1 (K = 1), interleaved with HEAD (no head chunks)
set -u
mkdir -p gpurun_out
TAG=${1:-r06s}
T="timeout -k 10"
L=rad-nerf_amd/radnerf_amd
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
for r in 1 2 3; do
  for v in base r1536 r768; do
    LIB=$L/librn_ramp.so; H=${v#r}; [ $v = base ] && { LIB=$L/librn.so; H=0; }
    RADNERF_LIB=$LIB $T 200 python bench.py $Q --steps 40 --warmup 5 --head-chunk $H > gpurun_out/hs_${TAG}_c3_${v}_$r.json 2> gpurun_out/hs_${TAG}_c3_${v}_$r.err || exit $?
  done
  for v in base r1024; do
    LIB=$L/librn_ramp.so; H=${v#r}; [ $v = base ] && { LIB=$L/librn.so; H=0; }
    RADNERF_LIB=$LIB $T 200 python bench.py $Q --steps 40 --warmup 5 --models 1 --rays 8192 --head-chunk $H > gpurun_out/hs_${TAG}_c2_${v}_$r.json 2> gpurun_out/hs_${TAG}_c2_${v}_$r.err || exit $?
  done
  for v in base r256; do
    LIB=$L/librn_ramp.so; H=${v#r}; [ $v = base ] && { LIB=$L/librn.so; H=0; }
    RADNERF_LIB=$LIB $T 200 python bench.py $Q --steps 60 --warmup 5 --models 1 --rays 1024 --head-chunk $H > gpurun_out/hs_${TAG}_c1_${v}_$r.json 2> gpurun_out/hs_${TAG}_c1_${v}_$r.err || exit $?
  done
done
python - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/hs_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["kernel_ms"].get("field_bwd"))
PY
