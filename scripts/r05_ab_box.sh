#!/bin/bash
# gpurun (round 5): interleaved A/B of kernel variants + optional diag runs.
#   AB_VARIANTS="base x y" AB_SPP=128 AB_REPS=3 [AB_WORKLOAD=c2] [DIAGS="lib1:name1 lib2:name2"] [DIAG_SPP=64] bash scripts/r05_ab_box.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/${AB_OUT:-r05ab}
mkdir -p $OUT
W=${AB_WORKLOAD:-c2}
timeout -k 10 ${AB_TIMEOUT:-500} python3 scripts/ab.py ${AB_SPP:-128} ${AB_REPS:-3} ${AB_VARIANTS} > $OUT/ab_$W.json 2> $OUT/ab_$W.err || { echo "ab failed"; tail -5 $OUT/ab_$W.err; exit 1; }
cat $OUT/ab_$W.json
for d in ${DIAGS:-}; do
  lib=${d%%:*}; name=${d##*:}
  AB_WORKLOAD=$W DIAG_LIB=$lib timeout -k 10 300 python3 scripts/diag.py ${DIAG_SPP:-64} > $OUT/diag_${W}_$name.json 2> $OUT/diag_${W}_$name.err || { echo "diag $name failed"; tail -5 $OUT/diag_${W}_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/diag_${W}_$name.json')); print('$name', {k: d[k] for k in ('kernel_ms','trace_lane_efficiency','wave_trace_iters_per_wave_bounce','trace_iters_per_ray','cycle_share')})"
done
echo ab-done
