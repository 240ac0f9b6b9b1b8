set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_ph1.log 2>&1 || { tail -30 gpurun_out/tests_ph1.log; exit 1; }
tail -2 gpurun_out/tests_ph1.log
Q="--dropin-step 0 --test-time-rays 0 --density-update 0 --cpu-rays 0 --train-step 0"
timeout -k 10 150 python -u bench.py $Q --steps 30 --warmup 5 --models 4 --scale 16 --rays 4096 > gpurun_out/ph1_c4.json 2> gpurun_out/ph1_c4.err &&
timeout -k 10 150 python -u bench.py $Q --steps 30 --warmup 5 --models 1 --rays 8192 > gpurun_out/ph1_c2.json 2> gpurun_out/ph1_c2.err || exit $?
python3 tools/bench_summary.py gpurun_out/ph1_c4.json gpurun_out/ph1_c2.json
