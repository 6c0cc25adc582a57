#!/bin/bash
# gpurun (round 5): diagnostic-build runs, one per "workload:lib:spp" in DIAG_RUNS.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/${DIAG_OUT:-r05diag}
mkdir -p $OUT
for d in ${DIAG_RUNS}; do
  w=${d%%:*}; rest=${d#*:}; lib=${rest%%:*}; spp=${rest##*:}
  AB_WORKLOAD=$w DIAG_LIB=$lib timeout -k 10 300 python3 scripts/diag.py $spp > $OUT/diag_$w.json 2> $OUT/diag_$w.err || { echo "diag $w failed"; tail -5 $OUT/diag_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/diag_$w.json')); d.pop('raw'); print(d)"
done
echo diag-done
