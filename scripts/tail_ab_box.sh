#!/bin/bash
# gpurun: scripts/tail_ab.py per workload in TAB_WLS under the settings TAB_SETTINGS.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAB_OUT:-tail_ab}
mkdir -p $OUT
for wl in ${TAB_WLS:-c2}; do
  timeout -k 10 ${TAB_TIMEOUT:-400} python3 scripts/tail_ab.py $wl ${TAB_SPP:--} ${TAB_REPS:-3} $TAB_SETTINGS > $OUT/$wl.jsonl 2> $OUT/$wl.err || { echo "tail_ab $wl failed rc=$?"; tail -5 $OUT/$wl.err; exit 1; }
  tail -1 $OUT/$wl.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); [print(d["workload"][:3], k, round(v["full_min"],2), round(v["full_median"],2), round(v["worst8_min"],3), round(v["eff8"],4)) for k,v in d["settings"].items()]'
done
echo tail-ab-done
