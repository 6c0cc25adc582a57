#!/bin/bash
# Second PMC round (gpurun): VALU utilisation, f64 instruction mix, waits, L2.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/prof2
mkdir -p $OUT
BENCH="bench.py --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline ${BENCH_EXTRA:-}"
i=0
for set in "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $BENCH > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; }
done
echo profile2-done
