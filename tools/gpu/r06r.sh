#!/bin/bash
# A/B (timing): ramped head chunks (librn_ramp.so, -DRN_HEAD_RAMP=1: the first
# chunk of each block ramps 0 -> max_chunk, so the blocks' MLP / walk phases
# start staggered) vs HEAD (no head chunks), interleaved on one box
set -u
mkdir -p gpurun_out
TAG=${1:-r06r}
T="timeout -k 10"
L=rad-nerf_amd/radnerf_amd
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
for r in 1 2; do
  for v in base ramp; do
    if [ $v = base ]; then LIB=$L/librn.so; H3=0; H4=0; H5=0; else LIB=$L/librn_ramp.so; H3=1536; H4=2048; H5=6144; fi
    RADNERF_LIB=$LIB $T 200 python bench.py $Q --steps 40 --warmup 5 --head-chunk $H3 > gpurun_out/hr_${TAG}_c3_${v}_$r.json 2> gpurun_out/hr_${TAG}_c3_${v}_$r.err || exit $?
    RADNERF_LIB=$LIB $T 200 python bench.py $Q --steps 30 --warmup 5 --models 4 --scale 16 --rays 4096 --head-chunk $H4 > gpurun_out/hr_${TAG}_c4_${v}_$r.json 2> gpurun_out/hr_${TAG}_c4_${v}_$r.err || exit $?
    RADNERF_LIB=$LIB $T 200 python bench.py $Q --steps 20 --warmup 3 --models 8 --scale 16 --rays 8192 --head-chunk $H5 > gpurun_out/hr_${TAG}_c5_${v}_$r.json 2> gpurun_out/hr_${TAG}_c5_${v}_$r.err || exit $?
  done
done
python - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/hr_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["kernel_ms"].get("field_bwd"))
PY
