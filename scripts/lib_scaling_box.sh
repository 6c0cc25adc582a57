#!/bin/bash
# gpurun: shard-scaling rehearsal (scripts/shard_scaling.py) of kernel variants
# librt_ab_<name>.so (LIBS), interleaved REPEAT times; optional GPU tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/${LS_OUT:-libscale}
mkdir -p $OUT
if [ "${LS_TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for r in $(seq ${REPEAT:-2}); do
  for name in ${LIBS:-base}; do
    RT_LIB=librt_ab_$name.so timeout -k 10 200 python3 scripts/shard_scaling.py ${LS_WL:-c2} ${LS_SPP:-512} ${LS_REPS:-2} > $OUT/${name}_$r.jsonl 2> $OUT/${name}_$r.err || { echo "shard $name failed"; tail -5 $OUT/${name}_$r.err; exit 1; }
    echo "$name/$r: $(tail -1 $OUT/${name}_$r.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); r8=[x["kernel_ms"] for x in d["runs"] if x["n"]==8]; print("full_ms", round(d["full_ms"],2), "n8_max", max(r8), "n8_mean", round(sum(r8)/len(r8),2), "eff8", d["eff8_worst_rank"])')"
  done
done
echo libscale-done
