#!/bin/bash
# gpurun: the tail-row queue split (rtk_tail_rows).  GPU tests named in TESTS,
# then per workload in TAIL_WLS the shard-scaling rehearsal
# (scripts/shard_scaling.py) under each RT_TAIL_PERMILLE of PERMILLES, then
# one WRITE_SIZE pass of the C2 bench (HBM write bytes per launch).  Every GPU
# step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAIL_OUT:-tailrows}
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for wl in ${TAIL_WLS:-c2}; do
  for pm in ${PERMILLES:-250}; do
    RT_TAIL_PERMILLE=$pm timeout -k 10 300 python3 scripts/shard_scaling.py $wl ${TAIL_SPP:--} 3 > $OUT/${wl}_$pm.jsonl 2> $OUT/${wl}_$pm.err || { echo "shard $wl $pm failed"; tail -5 $OUT/${wl}_$pm.err; exit 1; }
    echo "$wl permille $pm: $(tail -1 $OUT/${wl}_$pm.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print("full_ms", round(d["full_ms"],2), "eff8", d["eff8_worst_rank"], [ (r["n"], r["kernel_ms"]) for r in d["runs"] if r["rank"]==0])')"
  done
done
if [ "${WRITE_PASS:-1}" = 1 ]; then
  timeout -k 10 300 timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_c2 -o run -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate > $OUT/write_c2.log 2>&1 || { echo "write pass failed rc=$?"; tail -5 $OUT/write_c2.log; exit 1; }
  tail -1 $OUT/write_c2.log
fi
echo tailrows-done
