#!/bin/bash
# A/B (timing): the tail's share of the merged positions (librn_t<k>.so built
# with -DRN_TAIL_SHIFT=k: 2^-k of the work in min_chunk pieces; 31 = no tail;
# librn.so = 1/8), each with tail chunks near one per block or two, interleaved
set -u
mkdir -p gpurun_out
TAG=${1:-r06z}
T="timeout -k 10"
L=rad-nerf_amd/radnerf_amd
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
run() {   # name lib min_chunk shape-args...
  local n=$1 lib=$2 mn=$3; shift 3
  RADNERF_LIB=$L/$lib $T 200 python bench.py $Q --min-chunk $mn "$@" > gpurun_out/ts_${TAG}_${n}_$r.json 2> gpurun_out/ts_${TAG}_${n}_$r.err
}
C5="--steps 20 --warmup 3 --models 8 --scale 16 --rays 8192"
C4="--steps 30 --warmup 5 --models 4 --scale 16 --rays 4096"
C3="--steps 40 --warmup 5"
for r in 1 2; do
  run c5_t3_3072 librn.so 3072 $C5 || exit $?
  run c5_t2_6144 librn_t2.so 6144 $C5 || exit $?
  run c5_t2_3072 librn_t2.so 3072 $C5 || exit $?
  run c5_t4_1536 librn_t4.so 1536 $C5 || exit $?
  run c5_t4_3072 librn_t4.so 3072 $C5 || exit $?
  run c5_t31 librn_t31.so 3072 $C5 || exit $?
  run c4_t3_1024 librn.so 1024 $C4 || exit $?
  run c4_t4_512 librn_t4.so 512 $C4 || exit $?
  run c4_t31 librn_t31.so 1024 $C4 || exit $?
  run c3_t3_512 librn.so 512 $C3 || exit $?
  run c3_t4_512 librn_t4.so 512 $C3 || exit $?
  run c3_t4_256 librn_t4.so 256 $C3 || exit $?
  run c3_t2_512 librn_t2.so 512 $C3 || exit $?
done
python - "$TAG" <<'PY'
import json, sys, glob
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/ts_{tag}_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 1), d["ms_per_step"], d["kernel_ms"].get("field_bwd"))
PY
