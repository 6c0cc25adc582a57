#!/bin/bash
# One gpurun call: GPU parity tests, smoke(), then the default bench line.
#   gpurun -- 'bash scripts/check_box.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/check
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 t=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; exit $rc; fi
}
run pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
run bench_c2 400 python3 bench.py ${BENCH_ARGS:-}
echo box-ok
