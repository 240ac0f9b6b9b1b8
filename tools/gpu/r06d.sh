#!/bin/bash
# round 6: full GPU suite + smoke at HEAD (new int32 units, fp32-level option,
# sticky sum fault), C3 training demo with the new units and with levels 4-8
# on fp32 atomics, C3 bench A/B of the fp32-level option (interleaved)
set -u
mkdir -p gpurun_out
TAG=${1:-r06d}
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/gpu_suite_$TAG.log 2>&1 || exit $?
$T 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
$T 300 python -u tools/train_demo.py 1000 8192 2 0.5 > gpurun_out/tdemo_units_$TAG.json 2> gpurun_out/tdemo_units_$TAG.err || exit $?
FX_F32_LEVELS=3,4,5,6,7,8 $T 300 python -u tools/train_demo.py 1000 8192 2 0.5 > gpurun_out/tdemo_f32lv_$TAG.json 2> gpurun_out/tdemo_f32lv_$TAG.err || exit $?
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
for r in 1 2 3; do
  $T 200 python bench.py $Q --steps 40 --warmup 5 > gpurun_out/abf_c3_def_$r.json 2> gpurun_out/abf_c3_def_$r.err || exit $?
  $T 200 python bench.py $Q --steps 40 --warmup 5 --fx-f32-levels 3,4,5,6,7,8 > gpurun_out/abf_c3_f32_$r.json 2> gpurun_out/abf_c3_f32_$r.err || exit $?
done
echo done
