#!/bin/bash
# One gpurun call: bench lines and rocprofv3 evidence per workload.
#   gpurun -- 'PROFILE_WORKLOADS="c2 c3 c4" bash scripts/prof_box.sh'
# Per workload: the bench line (C2 with its cpu_baseline and host rate), a
# --kernel-trace --stats run, and separate --pmc passes (never combined with
# trace domains): FETCH_SIZE; WRITE_SIZE; the L2->fabric read requests by
# size (32/64/128 B); executed f64 VALU instructions with the exec density;
# f32 VALU instructions with wave / busy cycles.  Every GPU step has its own
# time limit and the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_OUT:-prof}
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 t=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; exit $rc; fi
}
F64="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
F32="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
RDREQ="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
for w in ${PROFILE_WORKLOADS:-c2 c3 c4}; do
  case $w in
    c2) BL="--steps ${C2_STEPS:-5} --warmup 1"; P="--steps 2 --warmup 1";;
    c3) BL="--steps 3 --warmup 1"; P="--steps 2 --warmup 1";;
    c4) BL="--steps 2 --warmup 1"; P="--steps 2 --warmup 1";;
    c5) BL="--steps 1 --warmup 0"; P="--steps 1 --warmup 0 --spp ${C5_PROF_SPP:-256}";;
  esac
  if [ "${BENCH_LINES:-1}" = 1 ]; then run bench_$w 900 python3 bench.py --workload $w $BL; fi
  B="bench.py --workload $w $P --no-cpu-baseline --no-host-rate"
  run trace_$w 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$w -o run -- python3 $B
  if [ "${PMC:-1}" = 1 ]; then
    run fetch_$w 400 timeout -s KILL 390 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$w -o run -- python3 $B
    run write_$w 400 timeout -s KILL 390 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$w -o run -- python3 $B
    run rdreq_$w 400 timeout -s KILL 390 rocprofv3 --pmc $RDREQ --output-format csv -d $OUT/rdreq_$w -o run -- python3 $B
    run valu64_$w 400 timeout -s KILL 390 rocprofv3 --pmc $F64 --output-format csv -d $OUT/valu64_$w -o run -- python3 $B
    run valu32_$w 400 timeout -s KILL 390 rocprofv3 --pmc $F32 --output-format csv -d $OUT/valu32_$w -o run -- python3 $B
  fi
done
echo prof-ok
