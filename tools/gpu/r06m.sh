#!/bin/bash
# round 6 final evidence at HEAD (fx_mode 5): full GPU suite, smoke, rocprofv3
# kernel stats of the C5 step, PMC traffic of C4 / C5, bench lines C3 / C4 /
# C5 / pinned (C1, C2 and C3's counters are unchanged from r06k: their code
# paths did not change)
set -u
mkdir -p gpurun_out
TAG=${1:-r06m}
trap "find gpurun_out -name '*kernel_trace.csv' -delete; find gpurun_out -name '*counter_collection.csv' -size +20M -delete" EXIT
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 250 --timeout-method thread > gpurun_out/gpu_suite_$TAG.log 2>&1 || exit $?
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
$T 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profc5_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 10 --warmup 3 --models 8 --scale 16 --rays 8192 > gpurun_out/profc5_$TAG.log 2>&1 || exit $?
cp profiles/traffic.json gpurun_out/traffic.json
pmc() {   # $1 = name, rest = bench args
  local n=$1; shift
  $T 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_${n}_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 "$@" > gpurun_out/pmcf_${n}_$TAG.log 2>&1 || return $?
  $T 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_${n}_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 "$@" > gpurun_out/pmcw_${n}_$TAG.log 2>&1 || return $?
  $T 300 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d gpurun_out/pmca_${n}_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 "$@" > gpurun_out/pmca_${n}_$TAG.log 2>&1 || return $?
  python tools/pmc_traffic.py gpurun_out/pmcf_${n}_$TAG gpurun_out/pmcw_${n}_$TAG gpurun_out/pmca_${n}_$TAG --merge gpurun_out/traffic.json > gpurun_out/traffic_${n}_$TAG.json
}
pmc c4 --models 4 --scale 16 --rays 4096 || exit $?
pmc c5 --models 8 --scale 16 --rays 8192 || exit $?
TJ="--traffic-json gpurun_out/traffic.json"
$T 500 python bench.py $TJ > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || exit $?
$T 300 python bench.py --models 4 --scale 16 --rays 4096 --cpu-rays 0 $TJ > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 8192 --cpu-rays 0 $TJ > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
$T 300 python bench.py --models 8 --scale 16 --rays 65536 --pinned-sim 8 --cpu-rays 0 $Q > gpurun_out/bench_c5pin_$TAG.json 2> gpurun_out/bench_c5pin_$TAG.err || exit $?
echo done
