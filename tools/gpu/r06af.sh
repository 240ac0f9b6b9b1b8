#!/bin/bash
# max_chunk sweep for the pinned rank (K = 1 per rank, 65,536 rays, scale 16), interleaved
set -u
mkdir -p gpurun_out
TAG=${1:-r06af}
T="timeout -k 10"
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
for r in 1 2; do
  for mx in 1024 2048 4096; do
    $T 300 python bench.py --models 8 --scale 16 --rays 65536 --pinned-sim 8 $Q --steps 15 --warmup 3 --max-chunk $mx > gpurun_out/p2_${TAG}_${mx}_$r.json 2> gpurun_out/p2_${TAG}_${mx}_$r.err || exit $?
  done
done
python - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/p2_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["kernel_ms"].get("field_bwd"))
PY
