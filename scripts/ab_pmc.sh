#!/bin/bash
# gpurun: PMC counters per A/B variant (scripts/ab.py under rocprofv3, one
# pass per counter set); scripts/ab_pmc_summary.py maps dispatches to variants.
#   gpurun -- 'AB_VARIANTS="a b" bash scripts/ab_pmc.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/abpmc
mkdir -p $OUT
SETS=("SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"
      "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_LDS SQ_INSTS_VMEM_RD")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 scripts/ab.py ${AB_SPP:-64} 1 ${AB_VARIANTS} > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; fi
done
echo "${AB_VARIANTS}" > $OUT/variants.txt
echo abpmc-done
