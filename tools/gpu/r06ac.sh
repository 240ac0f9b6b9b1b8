#!/bin/bash
# min_chunk re-sweep with the 1/16 tail (C3, C4, C5), interleaved on one box
set -u
mkdir -p gpurun_out
TAG=${1:-r06ac}
T="timeout -k 10"
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
for r in 1 2; do
  for mn in 384 512 640; do
    $T 200 python bench.py $Q --steps 40 --warmup 5 --min-chunk $mn > gpurun_out/m2_${TAG}_c3_${mn}_$r.json 2> gpurun_out/m2_${TAG}_c3_${mn}_$r.err || exit $?
  done
  for mn in 384 512 768 1024; do
    $T 200 python bench.py $Q --steps 30 --warmup 5 --models 4 --scale 16 --rays 4096 --min-chunk $mn > gpurun_out/m2_${TAG}_c4_${mn}_$r.json 2> gpurun_out/m2_${TAG}_c4_${mn}_$r.err || exit $?
  done
  for mn in 1024 1536 2048; do
    $T 200 python bench.py $Q --steps 20 --warmup 3 --models 8 --scale 16 --rays 8192 --min-chunk $mn > gpurun_out/m2_${TAG}_c5_${mn}_$r.json 2> gpurun_out/m2_${TAG}_c5_${mn}_$r.err || exit $?
  done
done
python - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/m2_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["kernel_ms"].get("field_bwd"))
PY
