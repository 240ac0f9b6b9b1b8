#!/bin/bash
# max_chunk sweep at scale 16 with the new tail chunks (C5 3072, C4 1024), interleaved
set -u
mkdir -p gpurun_out
TAG=${1:-r06y}
T="timeout -k 10"
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
for r in 1 2; do
  for mx in 8192 12288 16384 24576; do
    $T 200 python bench.py $Q --steps 20 --warmup 3 --models 8 --scale 16 --rays 8192 --max-chunk $mx > gpurun_out/mx_${TAG}_c5_${mx}_$r.json 2> gpurun_out/mx_${TAG}_c5_${mx}_$r.err || exit $?
  done
  for mx in 3072 4096 6144 8192; do
    $T 200 python bench.py $Q --steps 30 --warmup 5 --models 4 --scale 16 --rays 4096 --max-chunk $mx > gpurun_out/mx_${TAG}_c4_${mx}_$r.json 2> gpurun_out/mx_${TAG}_c4_${mx}_$r.err || exit $?
  done
done
python - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/mx_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["kernel_ms"].get("field_bwd"))
PY
