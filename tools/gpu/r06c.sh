#!/bin/bash
# fixed-point unit candidates at C3: per-entry agreement
# at the test's shape (2048 x 2) and the bench's (8192 x 2), and 1000 training
# steps each (PSNR vs fp32 atomics, steps redone in fp32)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
P=rad-nerf_amd/radnerf_amd
for v in d:librn.so a:librn_fxa.so b:librn_fxb.so c:librn_fxc.so; do
  n=${v%%:*}; l=${v#*:}
  RADNERF_LIB=$P/$l $T 300 python tools/fx_units_probe.py 2048 2 50 > gpurun_out/fxu2k_$n.json 2> gpurun_out/fxu2k_$n.err || exit $?
  RADNERF_LIB=$P/$l $T 300 python tools/fx_units_probe.py 8192 2 100 > gpurun_out/fxu8k_$n.json 2> gpurun_out/fxu8k_$n.err || exit $?
  RADNERF_LIB=$P/$l $T 400 python -u tools/train_demo.py 1000 8192 2 0.5 > gpurun_out/tdemo_$n.json 2> gpurun_out/tdemo_$n.err || exit $?
done
# per-level scatter form at C3
$T 400 python tools/level_bin_probe.py 0 6 8 10 12 14 > gpurun_out/lvbin_c3.json 2> gpurun_out/lvbin_c3.err || exit $?
# the new binned fault tests and the ABI load checks on the box
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bin.py tests/test_lib.py > gpurun_out/tests_bin_r06c.log 2>&1 || exit $?
echo done
