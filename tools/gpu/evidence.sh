#!/bin/bash
# GPU-box job for the round's evidence: GPU tests, smoke, full bench (with the
# CPU-oracle baseline), rocprofv3 kernel-trace summary, then separate PMC passes
# for HBM traffic (FETCH_SIZE / WRITE_SIZE / TCC_EA0_ATOMIC).  Every GPU step
# has its own time limit; the script stops at the first failure.
set -u
mkdir -p gpurun_out
TAG=${1:-r}
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --cpu-rays 0 --dropin-step 0 --steps 10 --warmup 3 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_$TAG -o run --output-format csv -- python3 bench.py --cpu-rays 0 --dropin-step 0 --steps 3 --warmup 1 > gpurun_out/pmcf_$TAG.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_$TAG -o run --output-format csv -- python3 bench.py --cpu-rays 0 --dropin-step 0 --steps 3 --warmup 1 > gpurun_out/pmcw_$TAG.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d gpurun_out/pmca_$TAG -o run --output-format csv -- python3 bench.py --cpu-rays 0 --dropin-step 0 --steps 3 --warmup 1 > gpurun_out/pmca_$TAG.log 2>&1
echo "atomic pass rc=$?" >> gpurun_out/pmca_$TAG.log
python tools/pmc_traffic.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG gpurun_out/pmca_$TAG > gpurun_out/traffic_$TAG.json
