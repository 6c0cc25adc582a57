#!/bin/bash
# PC sampling of the path kernel (rocprofv3, beta): which instructions the
# waves sit on.  Tries stochastic (hardware) sampling, then host-trap.
#   gpurun -- 'PCS_WL=c2 bash scripts/pcsample_box.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pcs_${PCS_WL:-c2}
mkdir -p $OUT
B="bench.py --workload ${PCS_WL:-c2} --steps 1 --warmup 1 --no-cpu-baseline --no-host-rate --spp ${PCS_SPP:-64}"
timeout -s KILL 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval ${PCS_INTERVAL:-1048576} --output-format csv -d $OUT/stoch -o run -- python3 $B > $OUT/stoch.log 2>&1
rc=$?; echo "stochastic rc=$rc"; tail -5 $OUT/stoch.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $rc -ne 0 ]; then
  timeout -s KILL 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval ${PCS_TIME_US:-100} --output-format csv -d $OUT/trap -o run -- python3 $B > $OUT/trap.log 2>&1
  rc=$?; echo "host_trap rc=$rc"; tail -5 $OUT/trap.log
fi
ls -R $OUT | head -30
