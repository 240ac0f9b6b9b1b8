#!/bin/bash
# PMC passes (FETCH / WRITE / atomic requests) for C1 and C2 merged into
# gpurun_out/traffic.json (from profiles/traffic.json), then the C1 / C2 bench
# lines with that file in place
set -u
mkdir -p gpurun_out
TAG=${1:-r}
export TMPDIR=/tmp
trap "find gpurun_out -name '*counter_collection.csv' -delete" EXIT
cp profiles/traffic.json gpurun_out/traffic.json
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
pmc() {   # $1 = name, rest = bench args
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_${n}_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 "$@" > gpurun_out/pmcf_${n}_$TAG.log 2>&1 || return $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_${n}_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 "$@" > gpurun_out/pmcw_${n}_$TAG.log 2>&1 || return $?
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d gpurun_out/pmca_${n}_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 "$@" > gpurun_out/pmca_${n}_$TAG.log 2>&1 || return $?
  python tools/pmc_traffic.py gpurun_out/pmcf_${n}_$TAG gpurun_out/pmcw_${n}_$TAG gpurun_out/pmca_${n}_$TAG --merge gpurun_out/traffic.json > gpurun_out/traffic_${n}_$TAG.json
}
pmc c1 --models 1 --rays 1024 || exit $?
pmc c2 --models 1 --rays 8192 || exit $?
cp gpurun_out/traffic.json profiles/traffic.json
timeout -k 10 300 python bench.py --models 1 --rays 8192 --cpu-rays 0 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
timeout -k 10 300 python bench.py --models 1 --rays 1024 > gpurun_out/bench_c1_$TAG.json 2> gpurun_out/bench_c1_$TAG.err || exit $?
