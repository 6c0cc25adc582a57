#!/bin/bash
# gpurun: round-4 checks in one box call.  Steps (env STEPS, default all):
#   tests  -- the GPU tests named in TESTS (default: the whole -m gpu suite)
#   ab     -- interleaved A/B of AB_VARIANTS on AB_WORKLOADS (scripts/ab.py)
#   bench  -- bench.py (default workload)
# Each GPU step runs under its own timeout; a fault / abort / timeout status
# (124, 134, 137, 139) ends the call, a plain test failure (1) does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/r04
mkdir -p $OUT
STEPS=${STEPS:-"tests ab"}
fatal() { case $1 in 124|134|137|139) echo "FATAL status $1 in $2"; exit $1;; esac; }
for step in $STEPS; do
  case $step in
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-900} python3 -u -m pytest ${TESTS:-tests -m gpu} -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -4 $OUT/pytest.log; fatal $rc tests ;;
    checktests)
      # the whole GPU suite on the check build (every decoded ref bounds-checked)
      RT_MI355X_LIB=raytracer-2025_amd/librt_mi355x_check.so timeout -k 10 ${TEST_TIMEOUT:-900} python3 -u -m pytest ${TESTS:-tests -m gpu} -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_check.log 2>&1
      rc=$?; echo "checktests rc=$rc"; tail -4 $OUT/pytest_check.log; fatal $rc checktests ;;
    ab)
      for wl in ${AB_WORKLOADS:-c2}; do
        AB_WORKLOAD=$wl timeout -k 10 ${AB_TIMEOUT:-400} python3 scripts/ab.py ${AB_SPP:-64} ${AB_REPS:-3} ${AB_VARIANTS:-base} > $OUT/ab_$wl.json 2> $OUT/ab_$wl.err
        rc=$?; echo "ab $wl rc=$rc"; fatal $rc ab
        python3 -c "import json,sys; d=json.load(open('$OUT/ab_$wl.json')); [print('$wl', k, round(v['kernel_ms_min'],2), v['kernel_ms'], v['rmse_vs_first']) for k,v in d.items()]"
      done ;;
    bench)
      timeout -k 10 ${BENCH_TIMEOUT:-400} python3 bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; echo "bench rc=$rc"; tail -c 1500 $OUT/bench.json; fatal $rc bench ;;
  esac
done
echo r04-done
