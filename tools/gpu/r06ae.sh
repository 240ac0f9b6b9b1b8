#!/bin/bash
# small head ramps at scale 16 (C5 to 1536 / 3072, C4 to 512 / 1024) vs none, interleaved
set -u
mkdir -p gpurun_out
TAG=${1:-r06ae}
T="timeout -k 10"
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
for r in 1 2; do
  for h in 0 1536 3072; do
    $T 200 python bench.py $Q --steps 20 --warmup 3 --models 8 --scale 16 --rays 8192 --head-chunk $h > gpurun_out/h2_${TAG}_c5_${h}_$r.json 2> gpurun_out/h2_${TAG}_c5_${h}_$r.err || exit $?
  done
  for h in 0 512 1024; do
    $T 200 python bench.py $Q --steps 30 --warmup 5 --models 4 --scale 16 --rays 4096 --head-chunk $h > gpurun_out/h2_${TAG}_c4_${h}_$r.json 2> gpurun_out/h2_${TAG}_c4_${h}_$r.err || exit $?
  done
done
python - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/h2_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["kernel_ms"].get("field_bwd"))
PY
