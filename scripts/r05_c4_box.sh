#!/bin/bash
# gpurun (round 5): C4 / C5 diagnostic runs (top-level node counters) and the
# C4 / C2 vector-memory counters (scripts/mem_box.sh, MEM_OUT=r05mem).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/r05c4
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 480 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
AB_WORKLOAD=c4 DIAG_LIB=librt_mi355x_diag_t1.so timeout -k 10 300 python3 scripts/diag.py 16 > $OUT/diag_c4.json 2> $OUT/diag_c4.err || { echo diag c4 failed; tail -5 $OUT/diag_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/diag_c4.json')); d.pop('raw'); print(d)"
AB_WORKLOAD=c5 DIAG_LIB=librt_mi355x_diag_t2.so timeout -k 10 300 python3 scripts/diag.py 16 > $OUT/diag_c5.json 2> $OUT/diag_c5.err || { echo diag c5 failed; tail -5 $OUT/diag_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/diag_c5.json')); d.pop('raw'); print(d)"
MEM_OUT=r05mem MEM_WORKLOADS="${MEM_WORKLOADS:-c4 c2}" bash scripts/mem_box.sh
