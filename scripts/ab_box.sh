#!/bin/bash
# gpurun: interleaved A/B of kernel variants (scripts/ab.py), then the GPU parity tests.
#   gpurun -- 'AB_SPP=128 AB_VARIANTS="a b" bash scripts/ab_box.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/ab
mkdir -p $OUT
timeout -k 10 400 python3 scripts/ab.py ${AB_SPP:-128} ${AB_REPS:-3} ${AB_VARIANTS} > $OUT/ab_${AB_WORKLOAD:-c2}.json 2> $OUT/ab.err || { echo "ab failed"; tail -5 $OUT/ab.err; exit 1; }
cat $OUT/ab_${AB_WORKLOAD:-c2}.json
if [ -n "${AB_TESTS:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
echo ab-done
