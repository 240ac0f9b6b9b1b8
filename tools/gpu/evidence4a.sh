#!/bin/bash
# Round-4 evidence, part A: GPU tests, smoke, rocprofv3 kernel stats of the
# headline and of C5, PMC passes (FETCH / WRITE / atomic requests) for C3 and
# for C4 / C5 with the binned scatter (the default at scale 16) merged into
# gpurun_out/traffic.json.  Every GPU step has its own time limit; the script
# stops at the first failure.
set -u
mkdir -p gpurun_out
TAG=${1:-r}
PART=${2:-all}     # tests | pmc | all
Q="--cpu-rays 0 --dropin-step 0 --train-step 0 --density-update 0 --test-time-rays 0"
trap "find gpurun_out -name '*kernel_trace.csv' -delete; find gpurun_out -name '*counter_collection.csv' -size +20M -delete" EXIT
export TMPDIR=/tmp
if [ "$PART" != pmc ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 10 --warmup 3 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 10 --warmup 3 --models 8 --scale 16 --rays 8192 > gpurun_out/prof_c5_$TAG.log 2>&1 || exit $?
fi
[ "$PART" = tests ] && exit 0
cp profiles/traffic.json gpurun_out/traffic.json
pmc() {   # $1 = name, rest = bench args
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_${n}_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 "$@" > gpurun_out/pmcf_${n}_$TAG.log 2>&1 || return $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_${n}_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 "$@" > gpurun_out/pmcw_${n}_$TAG.log 2>&1 || return $?
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d gpurun_out/pmca_${n}_$TAG -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 "$@" > gpurun_out/pmca_${n}_$TAG.log 2>&1 || return $?
  python tools/pmc_traffic.py gpurun_out/pmcf_${n}_$TAG gpurun_out/pmcw_${n}_$TAG gpurun_out/pmca_${n}_$TAG --merge gpurun_out/traffic.json > gpurun_out/traffic_${n}_$TAG.json
}
pmc c3 || exit $?
pmc c4bin --models 4 --scale 16 --rays 4096 || exit $?
pmc c5bin --models 8 --scale 16 --rays 8192 || exit $?
echo done
