#!/bin/bash
# PMC passes (gpurun) for the latency / memory-pipe picture of the path kernel:
# VMEM and LDS in-flight levels (latency = LEVEL / INSTS), wait and issue
# shares, L1 (TCP) and TA activity.  One rocprofv3 run per counter set.
#   gpurun -- 'WORKLOADS="c2" bash scripts/lat_box.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/lat
mkdir -p $OUT
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU TA_BUSY_avr TA_TA_BUSY_avr"
      "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PERF_SEL_TOTAL_READ_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ_sum SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS_LOAD SQ_LDS_IDX_ACTIVE")
for w in ${WORKLOADS:-c2}; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    echo "== $w pass $i: $set"
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/${w}_p$i -o run -- python3 bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/${w}_p$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$w pass $i failed rc=$rc"; tail -5 $OUT/${w}_p$i.log; exit $rc; fi
  done
done
echo lat-done
