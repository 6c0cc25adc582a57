#!/bin/bash
# gpurun (round 2): GPU tests, host CPU facts, counter list, divergence and
# contraction A/B.  Each GPU step has its own time limit; a fault, abort or
# time-out ends the script (pytest failures do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/${R02_OUT:-r02a}
mkdir -p $OUT
{ nproc; cat /sys/fs/cgroup/cpu.max 2>&1; python3 -c "import os;print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; lscpu | head -20; } > $OUT/host.txt 2>&1
fatal() { case $1 in 0|1) return 1;; *) echo "fatal rc=$1 in $2"; return 0;; esac; }
if [ "${R02_TESTS:-1}" = 1 ]; then
  timeout -k 10 ${R02_TEST_TIMEOUT:-800} python3 -u -m pytest tests -m gpu -v -s ${R02_TEST_ARGS:-} ${R02_K:+-k "$R02_K"} --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -40 $OUT/pytest.log | grep -E "passed|failed|FAILED|Error" | tail -30
  if fatal $rc pytest; then exit 1; fi
fi
if [ "${R02_COUNTERS:-0}" = 1 ]; then
  timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "counters rc=$?"
fi
if [ -n "${R02_DIV:-}" ]; then
  timeout -k 10 400 python3 -u scripts/divergence.py ${R02_DIV} > $OUT/divergence.json 2> $OUT/divergence.err
  rc=$?; echo "divergence rc=$rc"; tail -3 $OUT/divergence.err
  if fatal $rc divergence; then exit 1; fi
fi
if [ -n "${R02_AB:-}" ]; then
  for wl in ${R02_AB_WL:-c2}; do
    AB_WORKLOAD=$wl timeout -k 10 400 python3 scripts/ab.py ${R02_AB_SPP:-128} ${R02_AB_REPS:-3} ${R02_AB} > $OUT/ab_$wl.json 2> $OUT/ab_$wl.err
    rc=$?; echo "ab $wl rc=$rc"; cat $OUT/ab_$wl.json | grep -E "kernel_ms_min|rmse" 
    if fatal $rc ab; then exit 1; fi
  done
fi
echo r02-check-done
