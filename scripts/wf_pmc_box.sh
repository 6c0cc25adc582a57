#!/bin/bash
# gpurun: counters of the full tier's megakernel and of its wavefront variant
# (RT_WAVEFRONT=1) on C5 at 1920 wide, PMC_SPP spp -- one --pmc pass per set.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/wf_pmc
mkdir -p $OUT
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU"
S2="FETCH_SIZE"
S3="WRITE_SIZE"
for mode in mega wf; do
  if [ $mode = wf ]; then V="prod@RT_WAVEFRONT=1"; else V="prod"; fi
  i=0
  for set in "$S1" "$S2" "$S3"; do
    i=$((i+1))
    AB_WORKLOAD=c5 timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $OUT/${mode}_$i -o run -- python3 scripts/ab.py ${PMC_SPP:-32} 1 $V > $OUT/${mode}_$i.log 2>&1
    rc=$?; echo "$mode pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
echo wf-pmc-done
