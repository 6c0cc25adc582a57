#!/bin/bash
# gpurun: GPU parity tests, then the shard-scaling rehearsal
# (scripts/shard_scaling.py) under queue settings name:RT_PART_SAMPLES:
# RT_CHUNK_MIN:RT_TAIL_SAMPLES (TAIL_CFGS).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAIL_OUT:-tail}
mkdir -p $OUT
if [ "${TAIL_TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for cfg in ${TAIL_CFGS:-old:0:64 d:6:0}; do
  IFS=: read name samples cmin tail <<< "$cfg"
  RT_PART_SAMPLES=$samples RT_CHUNK_MIN=$cmin RT_TAIL_SAMPLES=${tail:-48} timeout -k 10 200 python3 scripts/shard_scaling.py ${TAIL_WL:-c2} ${TAIL_SPP:-512} 3 > $OUT/${TAIL_WL:-c2}_$name.jsonl 2> $OUT/${TAIL_WL:-c2}_$name.err || { echo "shard $name failed"; tail -5 $OUT/${TAIL_WL:-c2}_$name.err; exit 1; }
  echo "$name: $(tail -1 $OUT/${TAIL_WL:-c2}_$name.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print("full_ms", round(d["full_ms"],2), "eff8", d["eff8_worst_rank"], [ (r["n"], r["kernel_ms"]) for r in d["runs"] if r["rank"]==0])')"
done
echo tail-box-done
