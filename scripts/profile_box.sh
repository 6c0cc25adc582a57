#!/bin/bash
# Runs on the GPU box (gpurun): rocprofv3 kernel trace + stats of bench.py,
# then separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ counters), each under
# its own time limit.  Output under gpurun_out/prof/; summarised into
# profiles/ by scripts/summarize_profiles.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
BENCH="bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $BENCH > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $BENCH > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq -o run -- python3 $BENCH > $OUT/pmc_sq.log 2>&1 || { echo "pmc sq failed rc=$?"; exit 1; }
echo profile-ok
