#!/bin/bash
# PMC passes (gpurun) for the instruction mix / stall split of the path
# kernel, one rocprofv3 run per counter set, per workload.
#   gpurun -- 'WORKLOADS="c2 c3" bash scripts/sq_box.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/${SQ_OUT:-sq}
mkdir -p $OUT
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
      "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VALU_TRANS_F64"
      "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_INT64 SQ_INSTS_VSKIPPED SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA")
for w in ${WORKLOADS:-c2}; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/${w}_p$i -o run -- python3 bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/${w}_p$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$w pass $i failed rc=$rc"; tail -5 $OUT/${w}_p$i.log; exit $rc; fi
  done
done
echo sq-done
