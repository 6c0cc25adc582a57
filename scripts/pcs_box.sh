#!/bin/bash
# gpurun: stochastic PC sampling (rocprofv3, beta) of the path kernel on one
# workload frame (scripts/ab.py on the product library: PCS_LIB, default base),
# summarised per instruction by scripts/pcs_summary.py.
#   gpurun -- 'PCS_WORKLOAD=c2 PCS_SPP=32 bash scripts/pcs_box.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pcs_${PCS_WORKLOAD:-c2}
mkdir -p $OUT
AB_WORKLOAD=${PCS_WORKLOAD:-c2} timeout -k 10 ${PCS_TIMEOUT:-300} rocprofv3 --pc-sampling-beta-enabled \
  --pc-sampling-method ${PCS_METHOD:-stochastic} --pc-sampling-unit ${PCS_UNIT:-cycles} \
  --pc-sampling-interval ${PCS_INTERVAL:-1048576} -d $OUT/raw -o pcs --output-format csv \
  -- python3 scripts/ab.py ${PCS_SPP:-32} 1 ${PCS_LIB:-base} > $OUT/run.log 2>&1
rc=$?
echo "pcs rc=$rc"
tail -5 $OUT/run.log
find $OUT/raw -name "*.csv" | head -20
[ $rc -eq 0 ] || exit $rc
python3 scripts/pcs_summary.py $OUT/raw > $OUT/summary.txt 2>&1
head -60 $OUT/summary.txt
echo pcs-done
