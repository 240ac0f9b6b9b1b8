#!/bin/bash
# A/B (timing): a 1/32 tail (librn_t5.so, -DRN_TAIL_SHIFT=5) vs the default 1/16, interleaved
set -u
mkdir -p gpurun_out
TAG=${1:-r06ag}
T="timeout -k 10"
L=rad-nerf_amd/radnerf_amd
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
run() {   # name lib min_chunk shape-args...
  local n=$1 lib=$2 mn=$3; shift 3
  RADNERF_LIB=$L/$lib $T 200 python bench.py $Q --min-chunk $mn "$@" > gpurun_out/t5_${TAG}_${n}_$r.json 2> gpurun_out/t5_${TAG}_${n}_$r.err
}
C5="--steps 20 --warmup 3 --models 8 --scale 16 --rays 8192"
C4="--steps 30 --warmup 5 --models 4 --scale 16 --rays 4096"
C3="--steps 40 --warmup 5"
for r in 1 2; do
  run c3_t4_512 librn.so 512 $C3 || exit $?
  run c3_t5_512 librn_t5.so 512 $C3 || exit $?
  run c3_t5_256 librn_t5.so 256 $C3 || exit $?
  run c4_t4_512 librn.so 512 $C4 || exit $?
  run c4_t5_512 librn_t5.so 512 $C4 || exit $?
  run c4_t5_256 librn_t5.so 256 $C4 || exit $?
  run c5_t4_1536 librn.so 1536 $C5 || exit $?
  run c5_t5_1536 librn_t5.so 1536 $C5 || exit $?
  run c5_t5_768 librn_t5.so 768 $C5 || exit $?
done
python - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/t5_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["kernel_ms"].get("field_bwd"))
PY
