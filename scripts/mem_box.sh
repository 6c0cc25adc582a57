#!/bin/bash
# One gpurun call: vector-memory pipeline counters (TA / TD / TCP) of the
# path kernel per workload, in separate --pmc passes within the per-block
# limits (2 TA, 2 TD, 4 TCP, 2 GRBM per pass).  Each GPU step has its own
# time limit and the script stops at the first failure.
#   gpurun -- 'MEM_WORKLOADS="c4 c2" bash scripts/mem_box.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/${MEM_OUT:-mem}
mkdir -p $OUT
P1="TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum"
P2="TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_COUNT TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum"
P3="TA_FLAT_READ_WAVEFRONTS_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_READ_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum"
for w in ${MEM_WORKLOADS:-c4 c2}; do
  B="bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline --no-host-rate"
  n=1
  for P in "$P1" "$P2" "$P3"; do
    echo "== $w pass $n"
    timeout -k 10 300 timeout -s KILL 290 rocprofv3 --pmc $P --output-format csv -d $OUT/${w}_p$n -o run -- python3 $B > $OUT/${w}_p$n.log 2>&1
    rc=$?
    tail -1 $OUT/${w}_p$n.log
    if [ $rc -ne 0 ]; then echo "pass failed rc=$rc"; exit $rc; fi
    n=$((n+1))
  done
done
echo mem-ok
