#!/bin/bash
# One gpurun call: the default bench line (C2, with cpu_baseline), the C4
# bench line, and rocprofv3 kernel-trace/--stats + separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) of both workloads.  Every GPU step has its own time
# limit and the script stops at the first failure.
#   gpurun -- 'bash scripts/bench_box.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/box
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 t=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; exit $rc; fi
}
run bench_c2 400 python3 bench.py
run bench_c4 600 python3 bench.py --workload c4 --steps 2 --warmup 1
run bench_c3 400 python3 bench.py --workload c3 --steps 3 --warmup 1
if [ -n "${BENCH_C5:-}" ]; then run bench_c5 900 python3 bench.py --workload c5 --steps 1 --warmup 1; fi
for w in ${PROFILE_WORKLOADS:-c2 c4 c3}; do
  B="bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline"
  if [ "$w" = c5 ]; then B="bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline"; fi  # ~51 s frames
  run trace_$w 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$w -o run -- python3 $B
  run fetch_$w 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$w -o run -- python3 $B
  run write_$w 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write_$w -o run -- python3 $B
done
echo box-ok
