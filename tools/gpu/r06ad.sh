#!/bin/bash
# max_chunk re-sweep at scale 0.5 with the head ramp and the 1/16 tail (C3, C2), interleaved
set -u
mkdir -p gpurun_out
TAG=${1:-r06ad}
T="timeout -k 10"
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
for r in 1 2; do
  for mx in 1280 1536 2048; do
    $T 200 python bench.py $Q --steps 40 --warmup 5 --max-chunk $mx --head-chunk $mx > gpurun_out/x2_${TAG}_c3_${mx}_$r.json 2> gpurun_out/x2_${TAG}_c3_${mx}_$r.err || exit $?
  done
  for mx in 768 1024 1536; do
    $T 200 python bench.py $Q --steps 40 --warmup 5 --models 1 --rays 8192 --max-chunk $mx --head-chunk $mx > gpurun_out/x2_${TAG}_c2_${mx}_$r.json 2> gpurun_out/x2_${TAG}_c2_${mx}_$r.err || exit $?
  done
done
python - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/x2_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["kernel_ms"].get("field_bwd"))
PY
