#!/bin/bash
# fixed-point unit study at C3: per-entry agreement,
# 3-step Adam difference and redo frequency for the default int32 units, finer
# units (variant builds) and fp32 atomics on the coarse / middle levels
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
P=rad-nerf_amd/radnerf_amd
run() {  # name lib [env]
  local n=$1 l=$2; shift 2
  env RADNERF_LIB=$P/$l "$@" $T 300 python tools/fx_units_probe.py 8192 2 200 > gpurun_out/fxu_$n.json 2> gpurun_out/fxu_$n.err || return $?
}
run d23 librn.so || exit $?
run v25 librn_fx25.so || exit $?
run v26 librn_fx26.so || exit $?
run v27 librn_fx27.so || exit $?
run m48 librn.so FX_F32_LEVELS=4,5,6,7,8 || exit $?
run m28 librn.so FX_F32_LEVELS=2,3,4,5,6,7,8 || exit $?
echo done
